#!/bin/bash
# round-6 A/B: k_gemm_wks3 column tiles: fn4 = 32 x 64 (fp32), fm1 = 16 x 64 (fp32), fn4b = 16 x 64 (bf16);
# default 32 x 32 (fp32) / 16 x 32 (bf16); bitwise digests of the fp32 variant
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r06w}
mkdir -p gpurun_out
for v in "" fn4; do
  DREAMER_LIB_VARIANT=$v timeout -k 10 200 python tools/epoch_digest.py 256 fp32 3 2>&1 | grep digest || exit 1
done
run() {  # variant precision batch
  DREAMER_LIB_VARIANT=$1 timeout -k 10 240 python bench.py --batch $3 --precision $2 --steps 30 --no-cpu-baseline \
    --no-secondary --wm-steps 0 > gpurun_out/b_${TAG}.json 2> gpurun_out/b_${TAG}.err || { tail -20 gpurun_out/b_${TAG}.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_${TAG}.json'));print('${1:-default} $2 B$3', d['value'], d['ms_per_step'])"
}
for rep in 1 2; do
  run "" fp32 256 && run fn4 fp32 256 && run fm1 fp32 256 && run "" bf16 256 && run fn4b bf16 256 || exit 1
done
echo "gpu_$TAG done"
