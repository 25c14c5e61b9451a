#!/bin/bash
# round-5: persistent scan A/B -- headline fp32 B=256, bf16 B=256, configs[1] bf16 B=64,
# each with the persistent scan and with the launch form (DREAMER_PERSISTENT=0)
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r05j}
mkdir -p gpurun_out
for cfg in "256 fp32" "256 bf16" "64 bf16" "64 fp32"; do
  set -- $cfg
  for P in 1 0; do
    DREAMER_PERSISTENT=$P timeout -k 10 200 python bench.py --batch $1 --precision $2 --steps 30 --no-cpu-baseline --no-secondary --wm-steps 0 > gpurun_out/ab_${TAG}_B$1_$2_p$P.json 2> gpurun_out/ab_${TAG}_B$1_$2_p$P.err || { tail -20 gpurun_out/ab_${TAG}_B$1_$2_p$P.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ab_${TAG}_B$1_$2_p$P.json'));print('B=$1 $2 persistent=$P', d['value'], d['ms_per_step'])"
  done
done
echo "gpu_$TAG done"
