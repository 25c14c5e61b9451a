#!/bin/bash
# round-6 A/B: the six-product upsampling convs (k_convT_split3 problems) on the LDS-DMA ping-pong kernel (default) vs head;
# convolutions) vs the committed tree (head: FWD on 128-channel tiles only); bitwise digests (agent epochs and
# WM steps), WM step fp32, its kernel trace, WM / bf16 / deep-VAE tests
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r06z8}
R=$(pwd)
mkdir -p gpurun_out
for v in "" head; do
  DREAMER_LIB_VARIANT=$v timeout -k 10 200 python tools/epoch_digest.py 256 fp32 3 2>&1 | grep digest || exit 1
  DREAMER_LIB_VARIANT=$v timeout -k 10 200 python tools/epoch_digest.py 256 fp32 3 wm 2>&1 | grep digest || exit 1
done
run() {  # variant precision
  DREAMER_LIB_VARIANT=$1 timeout -k 10 240 python bench.py --batch 256 --precision $2 --steps 3 --no-cpu-baseline \
    --no-secondary --wm-steps 12 > gpurun_out/b_${TAG}.json 2> gpurun_out/b_${TAG}.err || { tail -20 gpurun_out/b_${TAG}.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_${TAG}.json'));w=d.get('secondary',{}).get('wm_step',{});print('${1:-default} $2 wm', w.get('ms_per_step'), w.get('gpu_ms_per_step'), w.get('loss'))"
}
for rep in 1 2; do
  run "" fp32 && run head fp32 || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/wmprof_$TAG -o p -- python3 $R/bench.py --batch 256 --steps 1 --warmup 1 --no-cpu-baseline --no-secondary --wm-steps 8 > $R/gpurun_out/wmprof_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/wmprof_$TAG.log; exit 1; }
cd $R
python tools/prof_summary.py gpurun_out/wmprof_$TAG/p_results.db 24 > gpurun_out/wm_kernels_$TAG.txt && cat gpurun_out/wm_kernels_$TAG.txt
rm -rf gpurun_out/wmprof_$TAG
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_wm.py tests/test_gpu_bf16.py tests/test_gpu_deep_vae.py tests/test_gpu_determinism.py \
  > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/tests_$TAG.log | head -30; tail -30 gpurun_out/tests_$TAG.log | cut -c1-300; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
echo "gpu_$TAG done"
