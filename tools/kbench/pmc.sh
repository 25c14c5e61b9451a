#!/bin/bash
# PMC passes over selected microbenchmark cases (one counter group per pass)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export KB_REPS=5
i=0
for grp in "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAVES SQ_INSTS_VALU" "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_IFETCH" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $R/gpurun_out/pmc$i -o pmc -- $R/tools/kbench/kbench "$1" > $R/gpurun_out/pmc$i.log 2>&1 || { tail -5 $R/gpurun_out/pmc$i.log; exit 1; }
done
echo pmc-done
