#!/bin/bash
# round-4: A/B of the staged backward prologues on 32-column skinny tiles (DR_BWD_WIDE, default 1) vs 16-column only
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r04zo}
mkdir -p gpurun_out
for v in main bwdnarrow main bwdnarrow main bwdnarrow; do
  if [ $v = main ]; then VV=""; else VV=$v; fi
  for P in fp32 bf16; do
    DREAMER_LIB_VARIANT=$VV timeout -k 10 300 python bench.py --no-secondary --wm-steps 0 --no-cpu-baseline --precision $P > gpurun_out/bench_${TAG}_${v}_$P.json 2> gpurun_out/bench_${TAG}.err || { tail -30 gpurun_out/bench_${TAG}.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/bench_${TAG}_${v}_$P.json').readline());print('$v $P', d['value'], d['ms_per_step'])"
  done
done
echo "gpu_$TAG done"
