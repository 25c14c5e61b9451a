#!/bin/bash
# round-5: k_gemm_wks3 register-ring depth A/B (D = 2 shipped then; d3 / d4 builds, r05zf;
# VARIANTS="base d1" for r05zg) at B = 256 fp32 / bf16, alternating, two rounds
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r05zf}
mkdir -p gpurun_out
for rep in 1 2; do
for p in fp32 bf16; do
for v in ${VARIANTS:-base d3 d4}; do
  if [ $v = base ]; then unset DREAMER_LIB_VARIANT; else export DREAMER_LIB_VARIANT=$v; fi
  timeout -k 10 200 python bench.py --batch 256 --precision $p --steps 30 --no-cpu-baseline --no-secondary --wm-steps 0 > gpurun_out/b_${TAG}_${p}_${v}_$rep.json 2> gpurun_out/b_${TAG}_${p}_${v}_$rep.err || { tail -20 gpurun_out/b_${TAG}_${p}_${v}_$rep.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_${TAG}_${p}_${v}_$rep.json'));print('$p $v', d['value'], d['ms_per_step'])"
done
done
done
unset DREAMER_LIB_VARIANT
echo "gpu_$TAG done"
