#!/bin/bash
# round-5: scan at B = 256 as two interleaved B = 128 halves -- parity B = 256 / 128, A/B B = 256
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r05v}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_baseline.py -m gpu -v -k "256 or 128" \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/tests_$TAG.log | head -30; tail -30 gpurun_out/tests_$TAG.log | cut -c1-300; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
for cfg in "256 fp32" "256 bf16"; do
  set -- $cfg
  for P in 1 0; do
    DREAMER_PERSISTENT=$P timeout -k 10 200 python bench.py --batch $1 --precision $2 --steps 30 --no-cpu-baseline --no-secondary --wm-steps 0 > gpurun_out/ab_${TAG}_B$1_$2_p$P.json 2> gpurun_out/ab_${TAG}_B$1_$2_p$P.err || { tail -20 gpurun_out/ab_${TAG}_B$1_$2_p$P.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ab_${TAG}_B$1_$2_p$P.json'));print('B=$1 $2 persistent=$P', d['value'], d['ms_per_step'])"
  done
done
echo "gpu_$TAG done"
