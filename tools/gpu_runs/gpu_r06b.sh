#!/bin/bash
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r06b}
mkdir -p gpurun_out
for rep in 1 2; do
for v in on off nosync; do
for p in fp32 bf16; do
  export DREAMER_FAULT_AB=$v
  timeout -k 10 200 python bench.py --batch 256 --precision $p --steps 30 --no-cpu-baseline --no-secondary --wm-steps 0 > gpurun_out/b_${TAG}.json 2> gpurun_out/b_${TAG}.err || { tail -20 gpurun_out/b_${TAG}.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_${TAG}.json'));print('$rep $v $p', d['value'], d['ms_per_step'])"
done
done
done
echo "gpu_$TAG done"
