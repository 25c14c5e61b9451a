#!/bin/bash
# HBM-side traffic of one short bench run, per kernel: two separate PMC passes
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950), kernel trace only.
#   bash tools/pmc_traffic.sh TAG [bench.py args]    (on the GPU box, from the repo root)
set -o pipefail
TAG=${1:-x}
shift
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $R/gpurun_out/pmc_$c$TAG -o p \
    -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --wm-steps 0 "$@" > $R/gpurun_out/pmc_$c$TAG.log 2>&1 \
    || { tail -20 $R/gpurun_out/pmc_$c$TAG.log; exit 1; }
done
cd $R && python3 tools/pmc_traffic.py gpurun_out/pmc_FETCH_SIZE$TAG gpurun_out/pmc_WRITE_SIZE$TAG --json gpurun_out/traffic$TAG.json > gpurun_out/traffic$TAG.txt
cat gpurun_out/traffic$TAG.txt
