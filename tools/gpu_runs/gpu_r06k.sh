#!/bin/bash
# round-6 checkpoint: the whole GPU suite, smoke, default bench (the driver's command)
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r06k}
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/tests_$TAG.log | head -20; tail -30 gpurun_out/tests_$TAG.log | cut -c1-300; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 900 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cut -c1-300 gpurun_out/bench_$TAG.json
echo "gpu_$TAG done"
