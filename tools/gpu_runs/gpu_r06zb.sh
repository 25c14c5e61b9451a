#!/bin/bash
# round-6 A/B: bf16 encoder conv3 / conv4 on a ping-pong one-term kernel with 512-row tiles (b16pp) vs
# k_conv_glds_bf16 (default); bf16 digests, B = 256 bf16 headline, kernel times
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r06zb}
R=$(pwd)
mkdir -p gpurun_out
for v in "" b16pp; do
  DREAMER_LIB_VARIANT=$v timeout -k 10 200 python tools/epoch_digest.py 256 bf16 3 2>&1 | grep digest || exit 1
done
run() {  # variant
  DREAMER_LIB_VARIANT=$1 timeout -k 10 240 python bench.py --batch 256 --precision bf16 --steps 30 --no-cpu-baseline \
    --no-secondary --wm-steps 0 > gpurun_out/b_${TAG}.json 2> gpurun_out/b_${TAG}.err || { tail -20 gpurun_out/b_${TAG}.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_${TAG}.json'));print('${1:-default} bf16 B256', d['value'], d['ms_per_step'])"
}
for rep in 1 2 3; do
  run "" && run b16pp || exit 1
done
for v in "" b16pp; do
  cd /tmp && export TMPDIR=/tmp
  DREAMER_LIB_VARIANT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o p -- python3 $R/bench.py --steps 3 --warmup 2 --precision bf16 --no-cpu-baseline --no-secondary --wm-steps 0 > $R/gpurun_out/prof_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/prof_$TAG.log; exit 1; }
  cd $R
  echo "variant ${v:-default}"; python tools/epoch_table.py gpurun_out/prof_$TAG/p_results.db 5 13 40 | grep -E "glds|enc12"
  rm -rf gpurun_out/prof_$TAG
done
DREAMER_LIB_VARIANT=b16pp timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_bf16.py > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/tests_$TAG.log | head; tail -5 gpurun_out/tests_$TAG.log; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
echo "gpu_$TAG done"
