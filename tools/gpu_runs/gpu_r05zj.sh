#!/bin/bash
# round-5: k_gemm_wks3 with 8 waves per tile for the deep-K (>= 1024) products
# (the BPTT K = 1800 product) as a DREAMER_LIB_VARIANT build against the default,
# B = 256 fp32 / bf16, alternating, two rounds
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r05zj}
mkdir -p gpurun_out
for rep in 1 2; do
for p in fp32 bf16; do
for v in base k8; do
  if [ $v = base ]; then unset DREAMER_LIB_VARIANT; else export DREAMER_LIB_VARIANT=$v; fi
  timeout -k 10 200 python bench.py --batch 256 --precision $p --steps 30 --no-cpu-baseline --no-secondary --wm-steps 0 > gpurun_out/b_${TAG}_${p}_${v}_$rep.json 2> gpurun_out/b_${TAG}_${p}_${v}_$rep.err || { tail -20 gpurun_out/b_${TAG}_${p}_${v}_$rep.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_${TAG}_${p}_${v}_$rep.json'));print('$p $v', d['value'], d['ms_per_step'])"
done
done
done
unset DREAMER_LIB_VARIANT
echo "gpu_$TAG done"
