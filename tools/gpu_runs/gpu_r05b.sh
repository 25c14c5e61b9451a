#!/bin/bash
# round-5: parity tests around the persistent posterior scan, the headline bench
# with it and with the launch form (DREAMER_PERSISTENT=0), kernel trace.
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r05b}
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_determinism.py tests/test_gpu_noise.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/tests_$TAG.log | head -30; tail -60 gpurun_out/tests_$TAG.log | cut -c1-300; exit 1; }
tail -3 gpurun_out/tests_$TAG.log
timeout -k 10 300 python bench.py --steps 30 --no-cpu-baseline --no-secondary --wm-steps 0 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cut -c1-300 gpurun_out/bench_$TAG.json
DREAMER_PERSISTENT=0 timeout -k 10 300 python bench.py --steps 30 --no-cpu-baseline --no-secondary --wm-steps 0 > gpurun_out/bench_${TAG}_launch.json 2> gpurun_out/bench_${TAG}_launch.err || { tail -30 gpurun_out/bench_${TAG}_launch.err; exit 1; }
cut -c1-300 gpurun_out/bench_${TAG}_launch.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o p -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --wm-steps 0 > $R/gpurun_out/prof_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/prof_$TAG.log; exit 1; }
cd $R
python tools/epoch_table.py gpurun_out/prof_$TAG/p_results.db 7 13 40 > gpurun_out/epoch_table_$TAG.txt && head -30 gpurun_out/epoch_table_$TAG.txt
rm -rf gpurun_out/prof_$TAG
echo "gpu_$TAG done"
