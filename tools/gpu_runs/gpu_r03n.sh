#!/bin/bash
# round-3 GPU pass: tests, profiled epoch (kernel table), profiled WM step,
# full bench, then library-variant A/B of the headline (tools/build_variant.py)
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r03n}
R=$(pwd)
mkdir -p gpurun_out
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider \
    ${KEXPR:+-k "$KEXPR"} > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/tests_$TAG.log | head -20; tail -40 gpurun_out/tests_$TAG.log; exit 1; }
  tail -1 gpurun_out/tests_$TAG.log
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o p -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --wm-steps 0 > $R/gpurun_out/prof_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/prof_$TAG.log; exit 1; }
(cd $R && python tools/epoch_table.py gpurun_out/prof_$TAG/p_results.db 7 13 30 > gpurun_out/epoch_table_$TAG.txt && head -12 gpurun_out/epoch_table_$TAG.txt)
if [ "${WMPROF:-1}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/wmprof_$TAG -o p -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-secondary --wm-steps 5 > $R/gpurun_out/wmprof_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/wmprof_$TAG.log; exit 1; }
  (cd $R && python3 tools/prof_summary.py gpurun_out/wmprof_$TAG/p_results.db 60 > gpurun_out/wm_kernels_$TAG.txt 2>&1; head -24 gpurun_out/wm_kernels_$TAG.txt)
fi
cd $R
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));print('bench', d['value'], d['roofline']['frac'], d['roofline']['encoder_ms'], 'wm', d['secondary']['wm_step']['ms_per_step'])"
fi
for v in ${VARIANTS:-}; do
  for lib in base $v; do
    if [ $lib = base ]; then unset DREAMER_LIB_VARIANT; else export DREAMER_LIB_VARIANT=$lib; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-secondary --wm-steps ${AB_WM:-0} ${AB_ARGS:-} > gpurun_out/ab_${TAG}_$lib.json 2> gpurun_out/ab_${TAG}_$lib.err || { tail -10 gpurun_out/ab_${TAG}_$lib.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ab_${TAG}_$lib.json'));print('ab $lib', d['value'], 'encoder_ms', d['roofline']['encoder_ms'], 'wm_ms', d.get('secondary', {}).get('wm_step', {}).get('ms_per_step'))"
  done
done
unset DREAMER_LIB_VARIANT
if [ "${DPPROBE:-0}" = 1 ]; then
  timeout -k 10 200 python tools/dp_probe.py 256 > gpurun_out/dpp1_$TAG.txt 2>&1 || { tail -20 gpurun_out/dpp1_$TAG.txt; exit 1; }
  grep epoch gpurun_out/dpp1_$TAG.txt
  DREAMER_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29519 tools/dp_probe.py 256 > gpurun_out/dpp2_$TAG.txt 2>&1 || { tail -20 gpurun_out/dpp2_$TAG.txt; exit 1; }
  grep epoch gpurun_out/dpp2_$TAG.txt
fi
echo "gpu_$TAG done"
