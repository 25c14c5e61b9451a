#!/bin/bash
# round-6 A/B: bf16 mode's world-model scan products (posterior scan forward / backward, grouped per step) as
# one-term products (default) vs the six-product form (head); fp32 WM digests (must be equal), WM step bf16 / fp32,
# then the WM and bf16 tests with their printed bf16-vs-oracle statistics
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r06z9}
mkdir -p gpurun_out
for v in "" head; do
  DREAMER_LIB_VARIANT=$v timeout -k 10 200 python tools/epoch_digest.py 256 fp32 3 wm 2>&1 | grep digest || exit 1
done
run() {  # variant precision
  DREAMER_LIB_VARIANT=$1 timeout -k 10 240 python bench.py --batch 256 --precision $2 --steps 3 --no-cpu-baseline \
    --no-secondary --wm-steps 12 > gpurun_out/b_${TAG}.json 2> gpurun_out/b_${TAG}.err || { tail -20 gpurun_out/b_${TAG}.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_${TAG}.json'));w=d.get('secondary',{}).get('wm_step',{});print('${1:-default} $2 wm', w.get('ms_per_step'), w.get('gpu_ms_per_step'), w.get('loss'))"
}
for rep in 1 2; do
  run "" bf16 && run head bf16 || exit 1
done
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_wm.py tests/test_gpu_bf16.py tests/test_gpu_determinism.py \
  > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/tests_$TAG.log | head -30; tail -30 gpurun_out/tests_$TAG.log | cut -c1-300; exit 1; }
grep -E "bf16 WM step" gpurun_out/tests_$TAG.log | cut -c1-600
tail -1 gpurun_out/tests_$TAG.log
echo "gpu_$TAG done"
