#!/bin/bash
# round-6: the host-mapped fault word (no per-epoch copy): failure-path tests,
# then the headline / configs[1] bench (fp32, bf16)
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r06c}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_persistent.py "tests/test_gpu_parity.py::test_pipelined_engine_dropped_then_new_capture" \
  "tests/test_gpu_parity.py::test_pipelined_epochs_match_sequential" \
  > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/tests_$TAG.log | head -30; tail -40 gpurun_out/tests_$TAG.log | cut -c1-300; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/tests_$TAG.log | cut -c1-150; tail -1 gpurun_out/tests_$TAG.log
for rep in 1 2; do
for B in 256 64; do
for p in fp32 bf16; do
  timeout -k 10 200 python bench.py --batch $B --precision $p --steps 30 --no-cpu-baseline --no-secondary --wm-steps 0 > gpurun_out/b_${TAG}.json 2> gpurun_out/b_${TAG}.err || { tail -20 gpurun_out/b_${TAG}.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_${TAG}.json'));print('B$B $p', d['value'], d['ms_per_step'])"
done
done
done
echo "gpu_$TAG done"
