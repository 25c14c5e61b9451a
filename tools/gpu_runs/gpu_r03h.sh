#!/bin/bash
# GPU tests, then a profiled world-model step (kernel stats), then the
# profiled headline bench -> per-epoch kernel table.  Stops at the first failure.
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r03h}
R=$(pwd)
mkdir -p gpurun_out
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider \
    ${KEXPR:+-k "$KEXPR"} > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/tests_$TAG.log | head -20; tail -40 gpurun_out/tests_$TAG.log; exit 1; }
  tail -1 gpurun_out/tests_$TAG.log
fi
cd /tmp && export TMPDIR=/tmp
if [ "${WMPROF:-1}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/wmprof_$TAG -o p -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-secondary --wm-steps 5 > $R/gpurun_out/wmprof_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/wmprof_$TAG.log; exit 1; }
  (cd $R && python3 tools/prof_summary.py gpurun_out/wmprof_$TAG/p_results.db 60 > gpurun_out/wm_kernels_$TAG.txt 2>&1; head -40 gpurun_out/wm_kernels_$TAG.txt)
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o p -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --wm-steps 0 > $R/gpurun_out/prof_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/prof_$TAG.log; exit 1; }
cd $R && grep '"value"' gpurun_out/prof_$TAG.log | cut -c1-200
python tools/epoch_table.py gpurun_out/prof_$TAG/p_results.db 7 13 30 > gpurun_out/epoch_table_$TAG.txt && cat gpurun_out/epoch_table_$TAG.txt
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
  cut -c1-400 gpurun_out/bench_$TAG.json
fi
echo "gpu_r03h done"
