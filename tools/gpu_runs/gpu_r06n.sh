#!/bin/bash
# round-6 A/B: (1) bf16 copies of h from the gates kernel for k_gemm_wks3<1> (noa16 = rounded in the GEMM) --
# bitwise-equal epochs checked by tools/epoch_digest.py, then the bf16 headline B = 256 / B = 128;
# (2) the all-parity-class 64 -> 32 upsampling conv (nocls = per-class kernels) in the WM step; WM / bf16 tests
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r06n}
R=$(pwd)
mkdir -p gpurun_out
for v in "" noa16; do
  DREAMER_LIB_VARIANT=$v timeout -k 10 200 python tools/epoch_digest.py 256 bf16 3 2>&1 | grep digest || exit 1
done
run() {  # variant precision batch wm_steps
  DREAMER_LIB_VARIANT=$1 timeout -k 10 240 python bench.py --batch $3 --precision $2 --steps 30 --no-cpu-baseline \
    --no-secondary --wm-steps $4 > gpurun_out/b_${TAG}.json 2> gpurun_out/b_${TAG}.err || { tail -20 gpurun_out/b_${TAG}.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_${TAG}.json'));w=d.get('secondary',{}).get('wm_step',{});print('${1:-default} $2 B$3', d['value'], d['ms_per_step'], 'wm', w.get('ms_per_step'))"
}
for rep in 1 2; do
  run "" bf16 256 0 && run noa16 bf16 256 0 && run "" bf16 128 0 && run noa16 bf16 128 0 || exit 1
done
for rep in 1 2; do
  run "" fp32 256 10 && run nocls fp32 256 10 && run "" bf16 256 10 && run nocls bf16 256 10 || exit 1
done
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_wm.py tests/test_gpu_bf16.py tests/test_gpu_flips.py tests/test_gpu_determinism.py \
  > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/tests_$TAG.log | head -30; tail -30 gpurun_out/tests_$TAG.log | cut -c1-300; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
cd /tmp && export TMPDIR=/tmp
for p in fp32 bf16; do
  WM_PREC=$p WM_B=256 WM_STEPS=6 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/wmprof_$TAG -o prof -- python3 $R/tools/wm_prof.py > $R/gpurun_out/wmprof_${TAG}_$p.log 2>&1 || { tail -20 $R/gpurun_out/wmprof_${TAG}_$p.log; exit 1; }
  grep "WM step" $R/gpurun_out/wmprof_${TAG}_$p.log
  (cd $R && python3 tools/prof_summary.py $(find gpurun_out/wmprof_$TAG -name '*.db' | head -1) 50 > gpurun_out/wm_kernels_${TAG}_$p.txt; head -16 gpurun_out/wm_kernels_${TAG}_$p.txt)
  rm -rf $R/gpurun_out/wmprof_$TAG
done
echo "gpu_$TAG done"
