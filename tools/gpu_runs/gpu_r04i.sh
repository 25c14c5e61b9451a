#!/bin/bash
# round-4: pipelined AC_epochs = 2 -- CU-masked warm stream x chain priority, one case per process
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r04i}
mkdir -p gpurun_out
: > gpurun_out/pipe_$TAG.txt
for c in seq pipe pipe:1:-1 pipe:0.9375:-1 pipe:0.875:-1 pipe:0.75:-1 pipe:0.875:0 seq pipe:0.875:-1; do
  timeout -k 10 200 python tools/pipe_probe.py 10 $c >> gpurun_out/pipe_$TAG.txt 2> gpurun_out/pipe_err_$TAG.txt || { tail -20 gpurun_out/pipe_err_$TAG.txt; exit 1; }
  tail -1 gpurun_out/pipe_$TAG.txt
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "pipelined" > gpurun_out/tests_$TAG.log 2>&1; tail -1 gpurun_out/tests_$TAG.log
echo "gpu_$TAG done"
