#!/bin/bash
# round-4: unconditional repack loads + one launch for both TN operands -- full GPU suite, then WM-step kernels
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r04zd}
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/tests_$TAG.log | head; tail -20 gpurun_out/tests_$TAG.log; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
cd /tmp && export TMPDIR=/tmp
for P in bf16 fp32; do
  WM_B=256 WM_PREC=$P timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/wmprof_$TAG$P -o p -- python3 $R/tools/wm_prof.py > $R/gpurun_out/wmprof_$TAG$P.log 2>&1 || { tail -20 $R/gpurun_out/wmprof_$TAG$P.log; exit 1; }
  grep "WM step" $R/gpurun_out/wmprof_$TAG$P.log
  python3 $R/tools/prof_summary.py $R/gpurun_out/wmprof_$TAG$P/p_results.db 60 > $R/gpurun_out/wm_kernels_$TAG$P.txt && head -12 $R/gpurun_out/wm_kernels_$TAG$P.txt
  rm -rf $R/gpurun_out/wmprof_$TAG$P
done
echo "gpu_$TAG done"
