#!/bin/bash
# round-5: scan changes (all-thread gather, preloads, 16-lane LN; B = 256 tiling) --
# scan probe at B = 64, parity at B = 16..256, A/B at B = 256 / 64, kernel trace B = 64 bf16
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r05r}
mkdir -p gpurun_out
DREAMER_LIB_VARIANT=pscants timeout -k 10 150 python tools/pscan_probe.py --batch 64 --precision bf16 > gpurun_out/psprobe_64.txt 2>&1 || { tail -5 gpurun_out/psprobe_64.txt; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_baseline.py tests/test_gpu_parity.py -m gpu -v -k "64 or 128 or 16 or 256 or parity or warm" \
  --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/tests_$TAG.log | head -30; tail -30 gpurun_out/tests_$TAG.log | cut -c1-300; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
for cfg in "256 fp32" "256 bf16" "64 bf16"; do
  set -- $cfg
  for P in 1 0; do
    DREAMER_PERSISTENT=$P timeout -k 10 200 python bench.py --batch $1 --precision $2 --steps 30 --no-cpu-baseline --no-secondary --wm-steps 0 > gpurun_out/ab_${TAG}_B$1_$2_p$P.json 2> gpurun_out/ab_${TAG}_B$1_$2_p$P.err || { tail -20 gpurun_out/ab_${TAG}_B$1_$2_p$P.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ab_${TAG}_B$1_$2_p$P.json'));print('B=$1 $2 persistent=$P', d['value'], d['ms_per_step'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run -- python3 bench.py --batch 64 --precision bf16 --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --wm-steps 0 > gpurun_out/prof_$TAG.log 2>&1 || { tail -5 gpurun_out/prof_$TAG.log; exit 1; }
echo "gpu_$TAG done"
