#!/bin/bash
# round-4: bf16 world-model step (one-term split convs) -- WM tests incl. the
# bf16 bounds test, bf16 epoch tests, full bench (bf16 WM step line), the
# AC_epochs = 2 pipeline probe.  Stops at the first failure.
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r04e}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_wm.py tests/test_gpu_bf16.py -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/tests_$TAG.log 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed|bf16 WM|Error" gpurun_out/tests_$TAG.log | cut -c1-600 | head -60
[ $rc -ne 0 ] && { tail -40 gpurun_out/tests_$TAG.log; exit 1; }
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cut -c1-300 gpurun_out/bench_$TAG.json
timeout -k 10 300 python tools/pipe_probe.py 10 > gpurun_out/pipe_$TAG.txt 2>&1 || { tail -20 gpurun_out/pipe_$TAG.txt; exit 1; }
tail -3 gpurun_out/pipe_$TAG.txt
echo "gpu_$TAG done"
