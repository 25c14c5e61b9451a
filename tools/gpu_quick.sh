#!/bin/bash
# quick iteration on the box: GPU tests, headline bench (no CPU leg / secondaries), kernel-trace profile
cd "$(dirname "$0")/.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-q}
shift
bash tools/gpu_tests.sh "$@" || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --wm-steps 0 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o p -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --wm-steps 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log; exit 1; }
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py gpurun_out/prof_$TAG/p_results.db 30
