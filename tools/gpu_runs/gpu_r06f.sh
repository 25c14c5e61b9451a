#!/bin/bash
# round-6: bf16 conv3 / conv4 on LDS-DMA staged operands (conv_glds.hip): bf16 tests, bench, kernel trace
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r06f}
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_bf16.py \
  > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/tests_$TAG.log | head -30; tail -40 gpurun_out/tests_$TAG.log | cut -c1-300; exit 1; }
grep -E "PASSED|FAILED|bf16 epoch|normwise" gpurun_out/tests_$TAG.log | cut -c1-250; tail -1 gpurun_out/tests_$TAG.log
for B in 64 256; do
  timeout -k 10 200 python bench.py --batch $B --precision bf16 --steps 30 --no-cpu-baseline --no-secondary --wm-steps 0 > gpurun_out/b_${TAG}.json 2> gpurun_out/b_${TAG}.err || { tail -20 gpurun_out/b_${TAG}.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_${TAG}.json'));print('B$B bf16', d['value'], d['ms_per_step'], 'enc', d['roofline']['encoder_ms'], d['roofline']['frac'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o p -- python3 $R/bench.py --batch 256 --precision bf16 --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --wm-steps 0 > $R/gpurun_out/prof_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/prof_$TAG.log; exit 1; }
cd $R && python tools/epoch_table.py gpurun_out/prof_$TAG/p_results.db 7 13 40 | grep -E "glds|conv|enc12|finish"
rm -rf gpurun_out/prof_$TAG
echo "gpu_$TAG done"
