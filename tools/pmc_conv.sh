#!/bin/bash
# SQ counter passes (one group per pass, kernel trace only) over tools/conv_ab.py:
# where the encoder conv kernels spend their wave cycles
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_ANY" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC" "SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $R/gpurun_out/pmcc$i -o pmc -- python3 $R/tools/conv_ab.py 0 > $R/gpurun_out/pmcc$i.log 2>&1 || { tail -5 $R/gpurun_out/pmcc$i.log; exit 1; }
done
echo pmc-done
