#!/bin/bash
# round-5: kernel trace of configs[1] (B = 64 bf16) and B = 64 fp32 through the
# bench command -- per-epoch table, and the trace database kept for an ordered
# per-launch listing of one epoch (what sits between the persistent kernels)
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r05za}
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for p in bf16 fp32; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG}_$p -o p -- python3 $R/bench.py --batch 64 --precision $p --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --wm-steps 0 > $R/gpurun_out/prof_${TAG}_$p.log 2>&1 || { tail -20 $R/gpurun_out/prof_${TAG}_$p.log; exit 1; }
  (cd $R && python tools/epoch_table.py gpurun_out/prof_${TAG}_$p/p_results.db 7 13 60 > gpurun_out/epoch_table_${TAG}_$p.txt && head -12 gpurun_out/epoch_table_${TAG}_$p.txt) || exit 1
done
echo "gpu_$TAG done"
