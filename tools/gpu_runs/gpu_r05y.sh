#!/bin/bash
# round-5: BPTT with the heads' backward folded into the K = 1800 stage's action tile --
# parity (B = 16 / 64 / 128, engine suite), bench B = 64 bf16 / fp32 x2
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r05y}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_baseline.py tests/test_gpu_parity.py tests/test_gpu_persistent.py tests/test_gpu_bf16.py -m gpu -v -k "64 or 128 or 16 or parity or actor or persistent or epoch" \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/tests_$TAG.log | head -30; tail -30 gpurun_out/tests_$TAG.log | cut -c1-300; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
for rep in 1 2; do
for cfg in "64 bf16" "64 fp32"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --batch $1 --precision $2 --steps 30 --no-cpu-baseline --no-secondary --wm-steps 0 > gpurun_out/b_${TAG}_B$1_$2_$rep.json 2> gpurun_out/b_${TAG}_B$1_$2_$rep.err || { tail -20 gpurun_out/b_${TAG}_B$1_$2_$rep.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_${TAG}_B$1_$2_$rep.json'));print('B=$1 $2', d['value'], d['ms_per_step'])"
done
done
echo "gpu_$TAG done"
