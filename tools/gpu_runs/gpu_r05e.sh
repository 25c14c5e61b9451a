#!/bin/bash
# round-5: persistent scan iteration -- stage timeline (DR_PSCAN_TS variant),
# warm-start parity tests, headline bench persistent vs launch form
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r05e}
mkdir -p gpurun_out
DREAMER_LIB_VARIANT=pscants timeout -k 10 200 python tools/pscan_probe.py --batch 256 > gpurun_out/pscan_${TAG}_B256.txt 2>&1 || { tail -20 gpurun_out/pscan_${TAG}_B256.txt; exit 1; }
cat gpurun_out/pscan_${TAG}_B256.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_baseline.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "baseline or warm or graph or epoch_vs" \
  > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/tests_$TAG.log | head -30; tail -30 gpurun_out/tests_$TAG.log | cut -c1-300; exit 1; }
tail -2 gpurun_out/tests_$TAG.log
timeout -k 10 300 python bench.py --steps 30 --no-cpu-baseline --no-secondary --wm-steps 0 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cut -c1-250 gpurun_out/bench_$TAG.json
DREAMER_PERSISTENT=0 timeout -k 10 300 python bench.py --steps 30 --no-cpu-baseline --no-secondary --wm-steps 0 > gpurun_out/bench_${TAG}_launch.json 2> gpurun_out/bench_${TAG}_launch.err || { tail -30 gpurun_out/bench_${TAG}_launch.err; exit 1; }
cut -c1-250 gpurun_out/bench_${TAG}_launch.json
echo "gpu_$TAG done"
