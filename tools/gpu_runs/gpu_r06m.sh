#!/bin/bash
# round-6: WM step -- posterior-scan products on split3 planes (wmscanf32 = the f32 wave-K route) A/B,
# kernel traces (fp32 / bf16), SQ / TCC counters of the fp32 step, WM tests
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r06m}
R=$(pwd)
mkdir -p gpurun_out
run() {  # variant precision
  DREAMER_LIB_VARIANT=$1 timeout -k 10 240 python bench.py --batch 256 --precision $2 --steps 3 --no-cpu-baseline \
    --no-secondary --wm-steps 12 > gpurun_out/b_${TAG}.json 2> gpurun_out/b_${TAG}.err || { tail -20 gpurun_out/b_${TAG}.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_${TAG}.json'));w=d.get('secondary',{}).get('wm_step',{});print('${1:-default} $2 wm', w.get('ms_per_step'), w.get('gpu_ms_per_step'), w.get('loss'))"
}
for rep in 1 2; do
  run "" fp32 && run wmscanf32 fp32 && run "" bf16 && run wmscanf32 bf16 || exit 1
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread -p no:cacheprovider tests/test_gpu_wm.py \
  > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/tests_$TAG.log | head -30; tail -30 gpurun_out/tests_$TAG.log | cut -c1-300; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
cd /tmp && export TMPDIR=/tmp
for p in fp32 bf16; do
  WM_PREC=$p WM_B=256 WM_STEPS=6 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/wmprof_$TAG -o prof -- python3 $R/tools/wm_prof.py > $R/gpurun_out/wmprof_${TAG}_$p.log 2>&1 || { tail -20 $R/gpurun_out/wmprof_${TAG}_$p.log; exit 1; }
  grep "WM step" $R/gpurun_out/wmprof_${TAG}_$p.log
  (cd $R && python3 tools/prof_summary.py $(find gpurun_out/wmprof_$TAG -name '*.db' | head -1) 50 > gpurun_out/wm_kernels_${TAG}_$p.txt; head -30 gpurun_out/wm_kernels_${TAG}_$p.txt)
  rm -rf $R/gpurun_out/wmprof_$TAG
done
cd $R && bash tools/pmc_sq.sh wm$TAG --wm-steps 2 --steps 1 || exit 1
echo "gpu_$TAG done"
