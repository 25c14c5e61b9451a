#!/bin/bash
# round-6 A/B: fp32 encoder conv3 / conv4 (and the WM forward's) on the LDS-DMA split3 kernel k_conv_glds_s3
# (default) vs k_conv_split3 (nogs3); bitwise digests, B = 256 fp32 headline, WM step, kernel trace, tests
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r06z3}
R=$(pwd)
mkdir -p gpurun_out
for v in "" nogs3; do
  DREAMER_LIB_VARIANT=$v timeout -k 10 200 python tools/epoch_digest.py 256 fp32 3 2>&1 | grep digest || exit 1
done
run() {  # variant precision wm_steps
  DREAMER_LIB_VARIANT=$1 timeout -k 10 240 python bench.py --batch 256 --precision $2 --steps 30 --no-cpu-baseline \
    --no-secondary --wm-steps $3 > gpurun_out/b_${TAG}.json 2> gpurun_out/b_${TAG}.err || { tail -20 gpurun_out/b_${TAG}.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_${TAG}.json'));w=d.get('secondary',{}).get('wm_step',{});print('${1:-default} $2 B256', d['value'], d['ms_per_step'], 'wm', w.get('ms_per_step'))"
}
for rep in 1 2; do
  run "" fp32 0 && run nogs3 fp32 0 || exit 1
done
run "" fp32 10 && run nogs3 fp32 10 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o p -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --wm-steps 0 > $R/gpurun_out/prof_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/prof_$TAG.log; exit 1; }
cd $R
python tools/epoch_table.py gpurun_out/prof_$TAG/p_results.db 7 13 40 > gpurun_out/epoch_table_$TAG.txt && head -8 gpurun_out/epoch_table_$TAG.txt
rm -rf gpurun_out/prof_$TAG
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_bf16.py tests/test_gpu_wm.py tests/test_gpu_determinism.py \
  > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/tests_$TAG.log | head -30; tail -30 gpurun_out/tests_$TAG.log | cut -c1-300; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
echo "gpu_$TAG done"
