#!/bin/bash
# round-5: kernel traces of the B = 64 bf16 epoch, persistent kernels on / off
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r05m}
mkdir -p gpurun_out
for P in 1 0; do
  DREAMER_PERSISTENT=$P timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_p$P -o run -- python3 bench.py --batch 64 --precision bf16 --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --wm-steps 0 > gpurun_out/prof_${TAG}_p$P.log 2>&1 || { tail -20 gpurun_out/prof_${TAG}_p$P.log; exit 1; }
done
find gpurun_out/prof_${TAG}_p1 -name "*kernel_stats.csv" | head
echo "gpu_$TAG done"
