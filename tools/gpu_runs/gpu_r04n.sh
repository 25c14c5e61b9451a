#!/bin/bash
# round-4: independent MFMA accumulator chains in the wave-K kernels (A/B), parity;
# does a CU-masked warm stream slow later work in the same process?
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r04n}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_baseline.py tests/test_gpu_determinism.py tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/tests_$TAG.log | head; tail -20 gpurun_out/tests_$TAG.log; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
timeout -k 10 300 python bench.py --no-secondary --wm-steps 0 --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
echo "main: $(cut -c100-200 gpurun_out/bench_$TAG.json)"
for v in noacc nowkacc2; do
  DREAMER_LIB_VARIANT=$v timeout -k 10 300 python bench.py --no-secondary --wm-steps 0 --no-cpu-baseline > gpurun_out/bench_${TAG}_$v.json 2> gpurun_out/bench_${TAG}_$v.err || { tail -30 gpurun_out/bench_${TAG}_$v.err; exit 1; }
  echo "variant $v: $(cut -c100-200 gpurun_out/bench_${TAG}_$v.json)"
done
timeout -k 10 300 python bench.py --no-secondary --wm-steps 0 --no-cpu-baseline --batch 64 > gpurun_out/bench_${TAG}_b64.json 2>> gpurun_out/bench_$TAG.err && echo "B64 main: $(cut -c100-200 gpurun_out/bench_${TAG}_b64.json)"
DREAMER_LIB_VARIANT=noacc timeout -k 10 300 python bench.py --no-secondary --wm-steps 0 --no-cpu-baseline --batch 64 > gpurun_out/bench_${TAG}_b64_noacc.json 2>> gpurun_out/bench_$TAG.err && echo "B64 noacc: $(cut -c100-200 gpurun_out/bench_${TAG}_b64_noacc.json)"
timeout -k 10 300 python bench.py --no-secondary --wm-steps 0 --no-cpu-baseline > gpurun_out/bench_${TAG}_again.json 2>> gpurun_out/bench_$TAG.err && echo "again: $(cut -c100-200 gpurun_out/bench_${TAG}_again.json)"
for c in after:0.875 after:1; do
  timeout -k 10 200 python tools/pipe_probe.py 10 $c 2>/tmp/pe.txt || { tail -20 /tmp/pe.txt; exit 1; }
done
for P in fp32 bf16; do WM_B=256 WM_PREC=$P timeout -k 10 200 python tools/wm_prof.py 2>&1 | grep "WM step"; done
echo "gpu_$TAG done"
