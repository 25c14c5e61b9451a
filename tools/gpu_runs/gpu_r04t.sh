#!/bin/bash
# round-4: split3 planes of h written by the GRU gates kernel for the grouped wave-K products (A/B + parity)
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r04t}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_baseline.py tests/test_gpu_determinism.py tests/test_gpu_parity.py tests/test_gpu_flips.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/tests_$TAG.log | head; tail -20 gpurun_out/tests_$TAG.log; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
for v in main noapl main noapl; do
  if [ $v = main ]; then VV=""; else VV=$v; fi
  DREAMER_LIB_VARIANT=$VV timeout -k 10 300 python bench.py --no-secondary --wm-steps 0 --no-cpu-baseline > gpurun_out/bench_${TAG}_$v.json 2> gpurun_out/bench_${TAG}.err || { tail -30 gpurun_out/bench_${TAG}.err; exit 1; }
  echo "$v: $(cut -c100-200 gpurun_out/bench_${TAG}_$v.json)"
done
echo "gpu_$TAG done"
