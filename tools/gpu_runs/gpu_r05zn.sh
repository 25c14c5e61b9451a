#!/bin/bash
# round-5: k_ln_gemm_sample loading its 16 weight rows in two halves of 8 (16 at
# once shipped) as a DREAMER_LIB_VARIANT build against the default, B = 256 fp32 /
# bf16 and B = 64 bf16, alternating, two rounds
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r05zn}
mkdir -p gpurun_out
for rep in 1 2; do
for pb in "fp32 256" "bf16 256" "bf16 64"; do set -- $pb; p=$1; bb=$2
for v in base ls8; do
  if [ $v = base ]; then unset DREAMER_LIB_VARIANT; else export DREAMER_LIB_VARIANT=$v; fi
  timeout -k 10 200 python bench.py --batch $bb --precision $p --steps 30 --no-cpu-baseline --no-secondary --wm-steps 0 > gpurun_out/b_${TAG}_${p}${bb}_${v}_$rep.json 2> gpurun_out/b_${TAG}_${p}${bb}_${v}_$rep.err || { tail -20 gpurun_out/b_${TAG}_${p}${bb}_${v}_$rep.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_${TAG}_${p}${bb}_${v}_$rep.json'));print('$p $bb $v', d['value'], d['ms_per_step'])"
done
done
done
unset DREAMER_LIB_VARIANT
echo "gpu_$TAG done"
