#!/bin/bash
# round-5: the BPTT's actor input gradient (K = 200, N = 1624) on the wave-K
# split3 kernel with weight planes at B >= 128 -- full GPU suite, then A/B
# against the staged-skinny form (DR_A0_PLANES=0 variant 'a0old'), B = 256
# fp32 / bf16, alternating, two rounds
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r05zo}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/tests_$TAG.log | head -30; tail -30 gpurun_out/tests_$TAG.log | cut -c1-300; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
for rep in 1 2; do
for p in fp32 bf16; do
for v in base a0old; do
  if [ $v = base ]; then unset DREAMER_LIB_VARIANT; else export DREAMER_LIB_VARIANT=$v; fi
  timeout -k 10 200 python bench.py --batch 256 --precision $p --steps 30 --no-cpu-baseline --no-secondary --wm-steps 0 > gpurun_out/b_${TAG}_${p}_${v}_$rep.json 2> gpurun_out/b_${TAG}_${p}_${v}_$rep.err || { tail -20 gpurun_out/b_${TAG}_${p}_${v}_$rep.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_${TAG}_${p}_${v}_$rep.json'));print('$p $v', d['value'], d['ms_per_step'])"
done
done
done
unset DREAMER_LIB_VARIANT
echo "gpu_$TAG done"
