#!/bin/bash
# round-5: bf16 one-term weight gradients -- bf16 / flips tests, bench B = 64 / 256 bf16
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r05s}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_flips.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/tests_$TAG.log | head -30; tail -30 gpurun_out/tests_$TAG.log | cut -c1-300; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
for cfg in "64 bf16" "256 bf16"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --batch $1 --precision $2 --steps 30 --no-cpu-baseline --no-secondary --wm-steps 0 > gpurun_out/b_${TAG}_B$1_$2.json 2> gpurun_out/b_${TAG}_B$1_$2.err || { tail -20 gpurun_out/b_${TAG}_B$1_$2.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_${TAG}_B$1_$2.json'));print('B=$1 $2', d['value'], d['ms_per_step'])"
done
echo "gpu_$TAG done"
