#!/bin/bash
# round-5: the next GRU hidden product forked to a side stream beside the
# current step's chain (launch-form scan / unroll at B >= 128) -- full GPU
# suite, then A/B (DREAMER_GH_FORK=1 / 0, alternating) at B = 256 fp32 / bf16
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r05zd}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/tests_$TAG.log | head -30; tail -30 gpurun_out/tests_$TAG.log | cut -c1-300; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
for rep in 1 2; do
for cfg in "256 fp32" "256 bf16"; do
for fk in 1 0; do
  set -- $cfg
  DREAMER_GH_FORK=$fk timeout -k 10 200 python bench.py --batch $1 --precision $2 --steps 30 --no-cpu-baseline --no-secondary --wm-steps 0 > gpurun_out/b_${TAG}_B$1_$2_f${fk}_$rep.json 2> gpurun_out/b_${TAG}_B$1_$2_f${fk}_$rep.err || { tail -20 gpurun_out/b_${TAG}_B$1_$2_f${fk}_$rep.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_${TAG}_B$1_$2_f${fk}_$rep.json'));print('B=$1 $2 fork=$fk', d['value'], d['ms_per_step'])"
done
done
done
echo "gpu_$TAG done"
