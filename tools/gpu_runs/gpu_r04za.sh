#!/bin/bash
# round-4: rows16 back on with the 32-column exclusion for the backward prologues
# (B = 512 DP comparison, B = 4096 vector epoch, pipelined = sequential), then
# AC_epochs = 2 pipeline probes (first warm start on the chain stream or fenced)
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest "tests/test_gpu_vector.py::test_vector_epoch_vs_oracle_B4096" "tests/test_gpu_dp.py::test_eight_rank_configs2_matches_single" tests/test_gpu_parity.py -m gpu -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_r05a.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/tests_r05a.log | head; tail -20 gpurun_out/tests_r05a.log; exit 1; }
tail -1 gpurun_out/tests_r05a.log
: > gpurun_out/pipe_r05a.txt
for c in "2 seq" "2 pipe:0.875:-1:0" "2 pipe:0.875:-1:1" "2 pipe:1:0:1" "2 pipe:0.75:-1:1" "10 seq" "10 pipe:0.875:-1:1"; do
  timeout -k 10 120 python -u tools/pipe_probe.py $c >> gpurun_out/pipe_r05a.txt 2>/dev/null || { echo "probe $c failed rc=$?"; exit 1; }
done
cat gpurun_out/pipe_r05a.txt
