#!/bin/bash
# round-6 closing bench (bench.py defaults; roofline.traffic now groups the LDS-DMA conv kernels) and the WM step's
# kernel traces (fp32, bf16) on the final tree
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r06zz2}
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 900 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cut -c1-300 gpurun_out/bench_$TAG.json
for p in fp32 bf16; do
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/wmprof_$TAG -o p -- python3 $R/bench.py --batch 256 --precision $p --steps 1 --warmup 1 --no-cpu-baseline --no-secondary --wm-steps 8 > $R/gpurun_out/wmprof_${TAG}_$p.log 2>&1 || { tail -20 $R/gpurun_out/wmprof_${TAG}_$p.log; exit 1; }
  cd $R
  python tools/prof_summary.py gpurun_out/wmprof_$TAG/p_results.db 30 > gpurun_out/wm_kernels_${TAG}_$p.txt && head -12 gpurun_out/wm_kernels_${TAG}_$p.txt
  rm -rf gpurun_out/wmprof_$TAG
done
echo "gpu_$TAG done"
