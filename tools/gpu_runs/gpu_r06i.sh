#!/bin/bash
# round-6: persistent BPTT with Q5 merged into Q6: BPTT parity tests, configs[1] bench, kernel time
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r06i}
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_persistent.py "tests/test_gpu_baseline.py::test_epoch_vs_oracle_at_baseline_shape" \
  "tests/test_gpu_bf16.py::test_train_agent_bf16_epoch_vs_oracle" tests/test_gpu_determinism.py \
  > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/tests_$TAG.log | head -30; tail -40 gpurun_out/tests_$TAG.log | cut -c1-300; exit 1; }
grep -cE "PASSED" gpurun_out/tests_$TAG.log; tail -1 gpurun_out/tests_$TAG.log
for p in bf16 fp32; do
  timeout -k 10 200 python bench.py --batch 64 --precision $p --steps 30 --no-cpu-baseline --no-secondary --wm-steps 0 > gpurun_out/b_${TAG}.json 2> gpurun_out/b_${TAG}.err || { tail -20 gpurun_out/b_${TAG}.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_${TAG}.json'));print('B64 $p', d['value'], d['ms_per_step'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o p -- python3 $R/bench.py --batch 64 --precision bf16 --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --wm-steps 0 > $R/gpurun_out/prof_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/prof_$TAG.log; exit 1; }
cd $R && python tools/epoch_table.py gpurun_out/prof_$TAG/p_results.db 7 13 6 | head -7
rm -rf gpurun_out/prof_$TAG
echo "gpu_$TAG done"
