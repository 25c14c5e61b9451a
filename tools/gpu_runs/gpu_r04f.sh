#!/bin/bash
# round-4 profiles: the bf16 WM step's kernels (B = 256), epoch timelines of the
# headline (fp32) and of bf16 mode at B = 256.
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r04f}
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
WM_B=256 WM_PREC=bf16 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/wmprof_$TAG -o p -- python3 $R/tools/wm_prof.py > $R/gpurun_out/wmprof_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/wmprof_$TAG.log; exit 1; }
grep "WM step" $R/gpurun_out/wmprof_$TAG.log
for P in fp32 bf16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG}_$P -o p -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --wm-steps 0 --precision $P > $R/gpurun_out/prof_${TAG}_$P.log 2>&1 || { tail -20 $R/gpurun_out/prof_${TAG}_$P.log; exit 1; }
done
cd $R
python3 tools/prof_summary.py gpurun_out/wmprof_$TAG/p_results.db 50 > gpurun_out/wm_kernels_$TAG.txt && head -40 gpurun_out/wm_kernels_$TAG.txt
for P in fp32 bf16; do
  python tools/epoch_table.py gpurun_out/prof_${TAG}_$P/p_results.db 7 13 50 > gpurun_out/epoch_table_${TAG}_$P.txt
  python tools/epoch_timeline.py gpurun_out/prof_${TAG}_$P/p_results.db > gpurun_out/timeline_${TAG}_$P.txt
  head -3 gpurun_out/timeline_${TAG}_$P.txt
done
rm -rf gpurun_out/wmprof_$TAG gpurun_out/prof_${TAG}_fp32 gpurun_out/prof_${TAG}_bf16
echo "gpu_$TAG done"
