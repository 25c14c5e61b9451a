#!/bin/bash
# round-6 A/B: split-K of the tall split3 GEMM down to 2 / 4 K chunks per split (minch2 / minch4; default 8)
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r06y}
mkdir -p gpurun_out
run() {  # variant precision wm_steps
  DREAMER_LIB_VARIANT=$1 timeout -k 10 240 python bench.py --batch 256 --precision $2 --steps 20 --no-cpu-baseline \
    --no-secondary --wm-steps $3 > gpurun_out/b_${TAG}.json 2> gpurun_out/b_${TAG}.err || { tail -20 gpurun_out/b_${TAG}.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_${TAG}.json'));w=d.get('secondary',{}).get('wm_step',{});print('${1:-default} $2', d['value'], 'wm', w.get('ms_per_step'))"
}
for rep in 1 2; do
  run "" fp32 12 && run minch2 fp32 12 && run minch4 fp32 12 && run "" bf16 12 && run minch2 bf16 12 && run minch4 bf16 12 || exit 1
done
echo "gpu_$TAG done"
