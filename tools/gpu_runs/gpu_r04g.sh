#!/bin/bash
# round-4: wave-K split3 kernel variants (waves per tile, whole-wave prefetch):
# parity at B = 256 on the variant, headline A/B; the fp32 WM step's kernels
# and the call sites of its split-K finishes.
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r04g}
R=$(pwd)
mkdir -p gpurun_out
DREAMER_LIB_VARIANT=w8full timeout -k 10 400 python -u -m pytest "tests/test_gpu_baseline.py::test_epoch_vs_oracle_at_baseline_shape" -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_$TAG.log 2>&1 || { tail -30 gpurun_out/tests_$TAG.log; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
timeout -k 10 300 python bench.py --no-secondary --wm-steps 0 --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
echo "main: $(cut -c100-200 gpurun_out/bench_$TAG.json)"
for v in w8 full w8full; do
  DREAMER_LIB_VARIANT=$v timeout -k 10 300 python bench.py --no-secondary --wm-steps 0 --no-cpu-baseline > gpurun_out/bench_${TAG}_$v.json 2> gpurun_out/bench_${TAG}_$v.err || { tail -30 gpurun_out/bench_${TAG}_$v.err; exit 1; }
  echo "variant $v: $(cut -c100-200 gpurun_out/bench_${TAG}_$v.json)"
done
timeout -k 10 300 python bench.py --no-secondary --wm-steps 0 --no-cpu-baseline > gpurun_out/bench_${TAG}_again.json 2>> gpurun_out/bench_$TAG.err && echo "again: $(cut -c100-200 gpurun_out/bench_${TAG}_again.json)"
cd /tmp && export TMPDIR=/tmp
WM_B=256 WM_PREC=fp32 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/wmprof_$TAG -o p -- python3 $R/tools/wm_prof.py > $R/gpurun_out/wmprof_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/wmprof_$TAG.log; exit 1; }
cd $R
grep "WM step" gpurun_out/wmprof_$TAG.log
python3 tools/prof_summary.py gpurun_out/wmprof_$TAG/p_results.db 50 > gpurun_out/wm_kernels_$TAG.txt && head -14 gpurun_out/wm_kernels_$TAG.txt
python3 tools/trace_neighbors.py gpurun_out/wmprof_$TAG/p_results.db k_splitk_finish 4 1 3
rm -rf gpurun_out/wmprof_$TAG
echo "gpu_$TAG done"
