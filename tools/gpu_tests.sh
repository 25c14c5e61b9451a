#!/bin/bash
# GPU parity suite on the box: one pytest process, per-test timeout, log under gpurun_out/
cd "$(dirname "$0")/.." || exit 1
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider "$@" \
  > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -40 gpurun_out/gpu_tests.log
exit $rc
