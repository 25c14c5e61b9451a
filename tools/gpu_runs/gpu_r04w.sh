#!/bin/bash
# round-4: the two B > 256 actor-gradient tests with the actor tail backward off, then the closing pass
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest "tests/test_gpu_vector.py::test_vector_epoch_vs_oracle_B4096" "tests/test_gpu_dp.py::test_eight_rank_configs2_matches_single" -m gpu -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_r04w.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/tests_r04w.log | head; tail -20 gpurun_out/tests_r04w.log; exit 1; }
tail -1 gpurun_out/tests_r04w.log
bash tools/gpu_runs/gpu_r04_final.sh ${1:-r04y}
