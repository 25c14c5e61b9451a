#!/bin/bash
# round-6: world-model step kernel traces at the bench's B = 256, T = 15 (fp32 and bf16)
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r06h}
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for p in bf16 fp32; do
  WM_PREC=$p WM_B=256 WM_STEPS=6 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/wmprof_$TAG -o prof -- python3 $R/tools/wm_prof.py > $R/gpurun_out/wmprof_${TAG}_$p.log 2>&1 || { tail -20 $R/gpurun_out/wmprof_${TAG}_$p.log; exit 1; }
  grep "WM step" $R/gpurun_out/wmprof_${TAG}_$p.log
  (cd $R && python3 tools/prof_summary.py $(find gpurun_out/wmprof_$TAG -name '*.db' | head -1) 50 > gpurun_out/wm_kernels_${TAG}_$p.txt; head -40 gpurun_out/wm_kernels_${TAG}_$p.txt)
  rm -rf $R/gpurun_out/wmprof_$TAG
done
echo "gpu_$TAG done"
