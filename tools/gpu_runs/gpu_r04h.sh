#!/bin/bash
# round-4: split-K finish fix (WM step), CU-masked warm stream probe for the pipelined epochs
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r04h}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_wm.py tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_$TAG.log 2>&1 || { tail -30 gpurun_out/tests_$TAG.log; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
for P in fp32 bf16; do
  WM_B=256 WM_PREC=$P timeout -k 10 200 python tools/wm_prof.py 2>&1 | grep "WM step"
done
timeout -k 10 400 python tools/pipe_probe.py 10 > gpurun_out/pipe_$TAG.txt 2>&1 || { tail -20 gpurun_out/pipe_$TAG.txt; exit 1; }
cat gpurun_out/pipe_$TAG.txt | grep -v amdgpu.ids
echo "gpu_$TAG done"
