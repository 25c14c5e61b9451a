#!/bin/bash
# round-6 A/B: gathered rows per batch in k_gru_gates (gb16 / gb32), wide wgrad column tiles for the 64-channel
# layers (wgnarrow = BN 128 / 256 as before), double-buffered six-product wgrad (wgsingle = the single-buffer
# kernel, wide tiles); then the tests of the touched paths
# (first run, r06l: a bf16 W_ih^T gather in k_gru_gates failed test_unguarded_flip_rate_B256[bf16] -- every row
#  diverged, flip rates warm 7.8e-3 / dream 1.16e-2 -- and was removed)
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r06l}
mkdir -p gpurun_out
run() {  # variant precision wm_steps
  DREAMER_LIB_VARIANT=$1 timeout -k 10 240 python bench.py --batch 256 --precision $2 --steps 30 --no-cpu-baseline \
    --no-secondary --wm-steps $3 > gpurun_out/b_${TAG}.json 2> gpurun_out/b_${TAG}.err || { tail -20 gpurun_out/b_${TAG}.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_${TAG}.json'));w=d.get('secondary',{}).get('wm_step',{});print('${1:-default} $2 B256', d['value'], d['ms_per_step'], 'wm', w.get('ms_per_step'), w.get('gpu_ms_per_step'))"
}
for rep in 1 2; do
  run "" bf16 0 && run gb16 bf16 0 && run gb32 bf16 0 && \
  run "" fp32 0 && run gb16 fp32 0 && run gb32 fp32 0 || exit 1
done
for rep in 1 2; do
  run "" fp32 10 && run wgsingle fp32 10 && run wgnarrow fp32 10 && run "" bf16 10 && run wgnarrow bf16 10 || exit 1
done
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_bf16.py tests/test_gpu_flips.py tests/test_gpu_wm.py tests/test_gpu_determinism.py \
  > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/tests_$TAG.log | head -30; tail -40 gpurun_out/tests_$TAG.log | cut -c1-300; exit 1; }
grep -cE "PASSED" gpurun_out/tests_$TAG.log; tail -1 gpurun_out/tests_$TAG.log
echo "gpu_$TAG done"
