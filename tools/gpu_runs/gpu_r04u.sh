#!/bin/bash
# round-4: MFMA-cluster / static wave priority in the split-conv encoder kernels (A/B, fp32 and bf16 encoder)
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r04u}
mkdir -p gpurun_out
for v in main prio1 prio2 main prio1 prio2; do
  if [ $v = main ]; then VV=""; else VV=$v; fi
  for P in fp32 bf16; do
    DREAMER_LIB_VARIANT=$VV timeout -k 10 300 python bench.py --no-secondary --wm-steps 0 --no-cpu-baseline --precision $P > gpurun_out/bench_${TAG}_${v}_$P.json 2> gpurun_out/bench_${TAG}.err || { tail -30 gpurun_out/bench_${TAG}.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/bench_${TAG}_${v}_$P.json').readline());print('$v $P', d['value'], 'encoder_ms', d['roofline']['encoder_ms'])"
  done
done
echo "gpu_$TAG done"
