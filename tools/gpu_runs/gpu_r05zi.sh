#!/bin/bash
# round-5: k_gemm_wks3 ring depth 1, bf16 16-row tiles -- full GPU suite, then configs[1]
# and the headline bench (+ B = 256 bf16), x2
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r05zi}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/tests_$TAG.log | head -30; tail -30 gpurun_out/tests_$TAG.log | cut -c1-300; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
for rep in 1 2; do
for cfg in "64 bf16" "64 fp32" "256 fp32" "256 bf16"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --batch $1 --precision $2 --steps 30 --no-cpu-baseline --no-secondary --wm-steps 0 > gpurun_out/b_${TAG}_B$1_$2_$rep.json 2> gpurun_out/b_${TAG}_B$1_$2_$rep.err || { tail -20 gpurun_out/b_${TAG}_B$1_$2_$rep.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_${TAG}_B$1_$2_$rep.json'));print('B=$1 $2', d['value'], d['ms_per_step'])"
done
done
echo "gpu_$TAG done"
