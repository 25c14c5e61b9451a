#!/bin/bash
# round-5: fp32 encoder with split3-plane activations between the convolutions --
# encoder / parity tests, bench B = 256 fp32 x2, kernel trace of the headline command
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r05x}
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_baseline.py tests/test_gpu_parity.py tests/test_gpu_wm.py -m gpu -v -k "encoder or 256 or 16 or warm or blocks or deep or configs3 or wm" \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/tests_$TAG.log | head -30; tail -30 gpurun_out/tests_$TAG.log | cut -c1-300; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
for rep in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --no-cpu-baseline --no-secondary --wm-steps 0 > gpurun_out/b_${TAG}_$rep.json 2> gpurun_out/b_${TAG}_$rep.err || { tail -20 gpurun_out/b_${TAG}_$rep.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_${TAG}_$rep.json'));print('B=256 fp32', d['value'], d['ms_per_step'], d['roofline']['encoder_ms'], d['roofline']['frac'])"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o p -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --wm-steps 0 > $R/gpurun_out/prof_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/prof_$TAG.log; exit 1; }
cd $R
python tools/epoch_table.py gpurun_out/prof_$TAG/p_results.db 7 13 40 > gpurun_out/epoch_table_$TAG.txt && head -8 gpurun_out/epoch_table_$TAG.txt
echo "gpu_$TAG done"
