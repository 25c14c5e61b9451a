#!/bin/bash
# round-6 A/B: the 4-channel layers' weight gradients on the row-staged kernel
# (noc4w = the LDS-tiled k_conv_nhwc); WM tests
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r06z2}
mkdir -p gpurun_out
run() {  # variant precision
  DREAMER_LIB_VARIANT=$1 timeout -k 10 240 python bench.py --batch 256 --precision $2 --steps 3 --no-cpu-baseline \
    --no-secondary --wm-steps 12 > gpurun_out/b_${TAG}.json 2> gpurun_out/b_${TAG}.err || { tail -20 gpurun_out/b_${TAG}.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_${TAG}.json'));w=d.get('secondary',{}).get('wm_step',{});print('${1:-default} $2 wm', w.get('ms_per_step'), w.get('gpu_ms_per_step'), w.get('loss'))"
}
for rep in 1 2; do
  run "" fp32 && run noc4w fp32 && run "" bf16 && run noc4w bf16 || exit 1
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread -p no:cacheprovider tests/test_gpu_wm.py \
  > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/tests_$TAG.log | head -30; tail -30 gpurun_out/tests_$TAG.log | cut -c1-300; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
echo "gpu_$TAG done"
