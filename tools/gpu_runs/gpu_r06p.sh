#!/bin/bash
# round-6 A/B: k_gemm_wks3 unrolled form only past 5 chunks per wave (the BPTT's K = 1800 products; default)
# vs nounroll (the rolled loop everywhere) vs unrall (unrolled everywhere, 8-chunk trip count for short K)
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r06p}
mkdir -p gpurun_out
run() {  # variant precision batch
  DREAMER_LIB_VARIANT=$1 timeout -k 10 240 python bench.py --batch $3 --precision $2 --steps 30 --no-cpu-baseline \
    --no-secondary --wm-steps 0 > gpurun_out/b_${TAG}.json 2> gpurun_out/b_${TAG}.err || { tail -20 gpurun_out/b_${TAG}.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_${TAG}.json'));print('${1:-default} $2 B$3', d['value'], d['ms_per_step'])"
}
for rep in 1 2; do
  for cfg in "fp32 256" "bf16 256" "fp32 128" "bf16 128"; do
    run "" $cfg && run nounroll $cfg && run unrall $cfg || exit 1
  done
done
echo "gpu_$TAG done"
