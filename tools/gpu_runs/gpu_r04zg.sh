#!/bin/bash
# round-4: 16-column colsum slabs -- full GPU suite, headline fp32 / bf16, WM step bf16 / fp32 (no profiler)
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r04zg}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/tests_$TAG.log | head; tail -20 gpurun_out/tests_$TAG.log; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
for P in fp32 bf16; do
  timeout -k 10 300 python bench.py --no-secondary --wm-steps 0 --no-cpu-baseline --precision $P > gpurun_out/bench_${TAG}_$P.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
  echo "$P: $(cut -c100-190 gpurun_out/bench_${TAG}_$P.json)"
  WM_B=256 WM_PREC=$P timeout -k 10 300 python tools/wm_prof.py 2>&1 | grep "WM step"
done
echo "gpu_$TAG done"
