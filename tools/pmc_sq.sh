#!/bin/bash
# SQ / TCC counters of one short bench run per kernel, two passes (8 SQ counters,
# then TCC hit / miss + GRBM), kernel trace only.  Counter list first (-L).
#   bash tools/pmc_sq.sh TAG [bench.py args]    (on the GPU box, from the repo root)
set -o pipefail
TAG=${1:-x}
shift
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/pmc_list$TAG.txt 2>&1 || true
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA"
P2="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $R/gpurun_out/pmcsq$i$TAG -o p \
    -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-secondary --wm-steps 0 "$@" > $R/gpurun_out/pmcsq$i$TAG.log 2>&1 \
    || { tail -20 $R/gpurun_out/pmcsq$i$TAG.log; exit 1; }
done
cd $R && python3 tools/pmc_sq.py gpurun_out/pmcsq1$TAG gpurun_out/pmcsq2$TAG > gpurun_out/pmcsq$TAG.txt && cat gpurun_out/pmcsq$TAG.txt
