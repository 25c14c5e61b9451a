#!/bin/bash
# One GPU-box pass: parity tests, bench line, kernel-trace profile.
#   tools/gpu_check.sh TAG   (run via gpurun from the repo root)
set -o pipefail
TAG=${1:-x}
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 240 python bench.py --steps 20 --warmup 3 --phases > gpurun_out/bench$TAG.json 2> gpurun_out/bench$TAG.err || { tail -20 gpurun_out/bench$TAG.err; exit 1; }
cat gpurun_out/bench$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof$TAG -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof$TAG.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof$TAG.log; exit 1; }
echo done
