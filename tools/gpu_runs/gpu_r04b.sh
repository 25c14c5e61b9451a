#!/bin/bash
# round-4 iteration check: B = 256 parity + determinism + natural-noise flips,
# headline bench, kernel-trace epoch table.  Stops at the first failure.
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r04b}
TESTS=${TESTS:-"tests/test_gpu_baseline.py tests/test_gpu_determinism.py tests/test_gpu_flips.py tests/test_gpu_parity.py tests/test_gpu_rccl.py"}
VARIANTS=${VARIANTS:-""}
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest $TESTS -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/tests_$TAG.log 2>&1
rc=$?
if [ $rc -ne 0 ]; then
  grep -E "FAILED|Error|assert" gpurun_out/tests_$TAG.log | head -30; tail -30 gpurun_out/tests_$TAG.log
  # assertion failures only (pytest rc 1): localise with the single-knob-off variants; anything else ends the call
  if [ $rc -eq 1 ] && [ -n "$BISECT" ]; then
    for v in $BISECT; do
      DREAMER_LIB_VARIANT=$v timeout -k 10 300 python -u -m pytest "$BISECT_TEST" -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/bisect_${TAG}_$v.log 2>&1
      brc=$?
      echo "bisect $v: rc $brc $(tail -1 gpurun_out/bisect_${TAG}_$v.log)"
      [ $brc -gt 1 ] && exit 1
    done
  fi
  exit 1
fi
grep -E "PASSED|FAILED|passed|failed|flip|guarded|NATURAL" gpurun_out/tests_$TAG.log | cut -c1-400 | head -60
timeout -k 10 300 python bench.py --no-secondary --wm-steps 0 --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cut -c1-200 gpurun_out/bench_$TAG.json
for v in $VARIANTS; do
  DREAMER_LIB_VARIANT=$v timeout -k 10 300 python bench.py --no-secondary --wm-steps 0 --no-cpu-baseline > gpurun_out/bench_${TAG}_$v.json 2> gpurun_out/bench_${TAG}_$v.err || { tail -30 gpurun_out/bench_${TAG}_$v.err; exit 1; }
  echo "variant $v: $(cut -c1-160 gpurun_out/bench_${TAG}_$v.json)"
done
timeout -k 10 300 python bench.py --no-secondary --wm-steps 0 --no-cpu-baseline > gpurun_out/bench_${TAG}_again.json 2>> gpurun_out/bench_$TAG.err && echo "again: $(cut -c1-160 gpurun_out/bench_${TAG}_again.json)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o p -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --wm-steps 0 > $R/gpurun_out/prof_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/prof_$TAG.log; exit 1; }
cd $R
python tools/epoch_table.py gpurun_out/prof_$TAG/p_results.db 7 13 40 > gpurun_out/epoch_table_$TAG.txt && head -30 gpurun_out/epoch_table_$TAG.txt
python tools/prof_summary.py gpurun_out/prof_$TAG/p_results.db 40 > gpurun_out/kernel_stats_$TAG.txt
rm -rf gpurun_out/prof_$TAG
echo "gpu_$TAG done"
