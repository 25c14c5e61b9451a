#!/bin/bash
# round-5: full GPU test suite + smoke + default bench on the current tree
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r05k}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/tests_$TAG.log | head -20; tail -30 gpurun_out/tests_$TAG.log | cut -c1-300; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -2 gpurun_out/smoke_$TAG.log
echo "gpu_$TAG done"
