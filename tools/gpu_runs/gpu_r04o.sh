#!/bin/bash
# round-4: bf16 configs[1] (B = 64) regression A/B against the round-3 knob set; bf16 WM step kernels
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r04o}
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest "tests/test_gpu_api.py::test_train_dreamer_with_fake_env" -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_$TAG.log 2>&1; grep -E "PASSED|FAILED|Error|assert" gpurun_out/tests_$TAG.log | head -8
for v in main r03 norows16 notailbwd nogruepi main; do
  if [ $v = main ]; then VV=""; else VV=$v; fi
  DREAMER_LIB_VARIANT=$VV timeout -k 10 300 python bench.py --no-secondary --wm-steps 0 --no-cpu-baseline --batch 64 --precision bf16 > gpurun_out/bench_${TAG}_$v.json 2> gpurun_out/bench_${TAG}.err || { tail -30 gpurun_out/bench_${TAG}.err; exit 1; }
  echo "bf16 B64 $v: $(cut -c100-200 gpurun_out/bench_${TAG}_$v.json)"
done
DREAMER_LIB_VARIANT=r03 timeout -k 10 300 python bench.py --no-secondary --wm-steps 0 --no-cpu-baseline --precision bf16 > gpurun_out/bench_${TAG}_b256_r03.json 2>> gpurun_out/bench_${TAG}.err && echo "bf16 B256 r03: $(cut -c100-200 gpurun_out/bench_${TAG}_b256_r03.json)"
timeout -k 10 300 python bench.py --no-secondary --wm-steps 0 --no-cpu-baseline --precision bf16 > gpurun_out/bench_${TAG}_b256.json 2>> gpurun_out/bench_${TAG}.err && echo "bf16 B256 main: $(cut -c100-200 gpurun_out/bench_${TAG}_b256.json)"
cd /tmp && export TMPDIR=/tmp
WM_B=256 WM_PREC=bf16 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/wmprof_$TAG -o p -- python3 $R/tools/wm_prof.py > $R/gpurun_out/wmprof_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/wmprof_$TAG.log; exit 1; }
cd $R
grep "WM step" gpurun_out/wmprof_$TAG.log
python3 tools/prof_summary.py gpurun_out/wmprof_$TAG/p_results.db 50 > gpurun_out/wm_kernels_$TAG.txt && head -30 gpurun_out/wm_kernels_$TAG.txt
rm -rf gpurun_out/wmprof_$TAG
echo "gpu_$TAG done"
