#!/bin/bash
# round-6 A/B: bf16 copies of the BPTT's gate gradients (GRU backward epilogue) and of base_net.0's g_pre for the
# one-term input-gradient products (head = previous commit); bitwise digests; bf16 / fp32 B = 256 headline
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r06v}
mkdir -p gpurun_out
for p in bf16 fp32; do
  for v in "" head; do
    DREAMER_LIB_VARIANT=$v timeout -k 10 200 python tools/epoch_digest.py 256 $p 3 2>&1 | grep digest || exit 1
  done
done
run() {  # variant precision batch
  DREAMER_LIB_VARIANT=$1 timeout -k 10 240 python bench.py --batch $3 --precision $2 --steps 30 --no-cpu-baseline \
    --no-secondary --wm-steps 0 > gpurun_out/b_${TAG}.json 2> gpurun_out/b_${TAG}.err || { tail -20 gpurun_out/b_${TAG}.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_${TAG}.json'));print('${1:-default} $2 B$3', d['value'], d['ms_per_step'])"
}
for rep in 1 2 3; do
  run "" bf16 256 && run head bf16 256 || exit 1
done
run "" fp32 256 && run head fp32 256 && run "" bf16 128 && run head bf16 128 || exit 1
echo "gpu_$TAG done"
