#!/bin/bash
# round-4: bf16 WM step with the 4-channel weight gradients on the one-term split kernel
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r04p}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_wm.py -m gpu -q -s --timeout 300 --timeout-method thread -p no:cacheprovider -k "bf16 or baseline_shape" > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/tests_$TAG.log | head; tail -20 gpurun_out/tests_$TAG.log; exit 1; }
grep -E "bf16 WM step|passed|failed" gpurun_out/tests_$TAG.log | cut -c1-700
for P in bf16 fp32; do WM_B=256 WM_PREC=$P timeout -k 10 200 python tools/wm_prof.py 2>&1 | grep "WM step"; done
echo "gpu_$TAG done"
