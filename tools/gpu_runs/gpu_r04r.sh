#!/bin/bash
# round-4: bf16 WM step kernel trace (current build)
cd "$(dirname "$0")/../.." || exit 1
TAG=${1:-r04r}
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
WM_B=256 WM_PREC=bf16 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/wmprof_$TAG -o p -- python3 $R/tools/wm_prof.py > $R/gpurun_out/wmprof_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/wmprof_$TAG.log; exit 1; }
cd $R
grep "WM step" gpurun_out/wmprof_$TAG.log
python3 tools/prof_summary.py gpurun_out/wmprof_$TAG/p_results.db 60 > gpurun_out/wm_kernels_$TAG.txt && grep -E "wgrad|total" gpurun_out/wm_kernels_$TAG.txt
rm -rf gpurun_out/wmprof_$TAG
echo "gpu_$TAG done"
