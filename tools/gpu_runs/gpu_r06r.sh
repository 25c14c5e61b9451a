#!/bin/bash
# round-6 A/B: WM step -- tall NT products (heads' / upscaler's input gradients, encoder projection forward and
# backward) on split3 planes + the scan backward's K = 3 Hd products on k_gemm_wks3 (head = the previous commit);
# WM tests, kernel traces
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r06r}
R=$(pwd)
mkdir -p gpurun_out
run() {  # variant precision
  DREAMER_LIB_VARIANT=$1 timeout -k 10 240 python bench.py --batch 256 --precision $2 --steps 3 --no-cpu-baseline \
    --no-secondary --wm-steps 12 > gpurun_out/b_${TAG}.json 2> gpurun_out/b_${TAG}.err || { tail -20 gpurun_out/b_${TAG}.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_${TAG}.json'));w=d.get('secondary',{}).get('wm_step',{});print('${1:-default} $2 wm', w.get('ms_per_step'), w.get('gpu_ms_per_step'), w.get('loss'))"
}
for rep in 1 2; do
  run "" fp32 && run head fp32 && run "" bf16 && run head bf16 || exit 1
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread -p no:cacheprovider tests/test_gpu_wm.py tests/test_gpu_rccl.py tests/test_gpu_dp.py \
  > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/tests_$TAG.log | head -30; tail -30 gpurun_out/tests_$TAG.log | cut -c1-300; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
cd /tmp && export TMPDIR=/tmp
for p in fp32 bf16; do
  WM_PREC=$p WM_B=256 WM_STEPS=6 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/wmprof_$TAG -o prof -- python3 $R/tools/wm_prof.py > $R/gpurun_out/wmprof_${TAG}_$p.log 2>&1 || { tail -20 $R/gpurun_out/wmprof_${TAG}_$p.log; exit 1; }
  grep "WM step" $R/gpurun_out/wmprof_${TAG}_$p.log
  (cd $R && python3 tools/prof_summary.py $(find gpurun_out/wmprof_$TAG -name '*.db' | head -1) 60 > gpurun_out/wm_kernels_${TAG}_$p.txt; head -24 gpurun_out/wm_kernels_${TAG}_$p.txt)
  rm -rf $R/gpurun_out/wmprof_$TAG
done
echo "gpu_$TAG done"
