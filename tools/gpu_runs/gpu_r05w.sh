#!/bin/bash
# round-5: k_gemm_wks3 with 64-row tiles (DR_WKS3_FM=4 variant) -- parity at B = 256, A/B B = 256 fp32 / bf16
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r05w}
mkdir -p gpurun_out
DREAMER_LIB_VARIANT=fm4 timeout -k 10 600 python -u -m pytest tests/test_gpu_baseline.py tests/test_gpu_bf16.py -m gpu -v -k "256" \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/tests_$TAG.log | head -30; tail -30 gpurun_out/tests_$TAG.log | cut -c1-300; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
for rep in 1 2; do
for cfg in "256 fp32" "256 bf16"; do
  set -- $cfg
  for V in fm4 base; do
    VV=$V; [ "$V" = base ] && VV=
    DREAMER_LIB_VARIANT=$VV timeout -k 10 200 python bench.py --batch $1 --precision $2 --steps 30 --no-cpu-baseline --no-secondary --wm-steps 0 > gpurun_out/ab_${TAG}_B$1_$2_$V.json 2> gpurun_out/ab_${TAG}_B$1_$2_$V.err || { tail -20 gpurun_out/ab_${TAG}_B$1_$2_$V.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ab_${TAG}_B$1_$2_$V.json'));print('B=$1 $2 variant=$V', d['value'], d['ms_per_step'])"
  done
done
done
echo "gpu_$TAG done"
