#!/bin/bash
# round-5: kernel trace of the headline bench command (B = 256 fp32) on the
# current tree; the trace database is kept for an ordered per-launch listing
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r05ze}
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG} -o p -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --wm-steps 0 > $R/gpurun_out/prof_${TAG}.log 2>&1 || { tail -20 $R/gpurun_out/prof_${TAG}.log; exit 1; }
cd $R && python tools/epoch_table.py gpurun_out/prof_${TAG}/p_results.db 7 13 60 > gpurun_out/epoch_table_${TAG}.txt && head -12 gpurun_out/epoch_table_${TAG}.txt
echo "gpu_$TAG done"
