#!/bin/bash
# round-5: A/B of the persistent kernels (scan + unroll) at B = 64 / 128, then a
# kernel trace of the B = 64 bf16 epoch
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r05n}
mkdir -p gpurun_out
for cfg in "64 bf16" "64 fp32" "128 fp32" "128 bf16"; do
  set -- $cfg
  for P in 1 0; do
    DREAMER_PERSISTENT=$P timeout -k 10 200 python bench.py --batch $1 --precision $2 --steps 30 --no-cpu-baseline --no-secondary --wm-steps 0 > gpurun_out/ab_${TAG}_B$1_$2_p$P.json 2> gpurun_out/ab_${TAG}_B$1_$2_p$P.err || { tail -20 gpurun_out/ab_${TAG}_B$1_$2_p$P.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ab_${TAG}_B$1_$2_p$P.json'));print('B=$1 $2 persistent=$P', d['value'], d['ms_per_step'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run -- python3 bench.py --batch 64 --precision bf16 --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --wm-steps 0 > gpurun_out/prof_${TAG}.log 2>&1 || { tail -20 gpurun_out/prof_${TAG}.log; exit 1; }
echo "gpu_$TAG done"
