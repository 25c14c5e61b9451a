#!/bin/bash
# round-5: persistent BPTT (bptt.hip) -- parity at B = 16 / 64 / 128 + the engine
# parity suite, then the A/B at B = 64 / 128
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r05p}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_baseline.py tests/test_gpu_parity.py -m gpu -v -k "64 or 128 or 16 or parity or imagine or critic" \
  --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAILED|Error|assert|mismatch" gpurun_out/tests_$TAG.log | head -30; tail -40 gpurun_out/tests_$TAG.log | cut -c1-300; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
for cfg in "64 bf16" "64 fp32" "128 fp32" "128 bf16"; do
  set -- $cfg
  for P in 1 0; do
    DREAMER_PERSISTENT=$P timeout -k 10 200 python bench.py --batch $1 --precision $2 --steps 30 --no-cpu-baseline --no-secondary --wm-steps 0 > gpurun_out/ab_${TAG}_B$1_$2_p$P.json 2> gpurun_out/ab_${TAG}_B$1_$2_p$P.err || { tail -20 gpurun_out/ab_${TAG}_B$1_$2_p$P.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ab_${TAG}_B$1_$2_p$P.json'));print('B=$1 $2 persistent=$P', d['value'], d['ms_per_step'])"
  done
done
echo "gpu_$TAG done"
