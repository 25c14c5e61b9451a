#!/bin/bash
# round-6 A/B: s_setprio 1 around the MFMA phase of k_conv_glds_s3's ping-pong (prio) vs none (default);
# digests, fp32 headline and WM step, conv kernel times
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r06za}
R=$(pwd)
mkdir -p gpurun_out
for v in "" prio; do
  DREAMER_LIB_VARIANT=$v timeout -k 10 200 python tools/epoch_digest.py 256 fp32 3 2>&1 | grep digest || exit 1
done
run() {  # variant wm_steps
  DREAMER_LIB_VARIANT=$1 timeout -k 10 240 python bench.py --batch 256 --precision fp32 --steps 30 --no-cpu-baseline \
    --no-secondary --wm-steps $2 > gpurun_out/b_${TAG}.json 2> gpurun_out/b_${TAG}.err || { tail -20 gpurun_out/b_${TAG}.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_${TAG}.json'));w=d.get('secondary',{}).get('wm_step',{});print('${1:-default} fp32 B256', d['value'], d['ms_per_step'], 'wm', w.get('ms_per_step'))"
}
for rep in 1 2; do
  run "" 10 && run prio 10 || exit 1
done
for v in "" prio; do
  cd /tmp && export TMPDIR=/tmp
  DREAMER_LIB_VARIANT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o p -- python3 $R/bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-secondary --wm-steps 0 > $R/gpurun_out/prof_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/prof_$TAG.log; exit 1; }
  cd $R
  echo "variant ${v:-default}"; python tools/epoch_table.py gpurun_out/prof_$TAG/p_results.db 5 13 40 | grep -E "glds_s3"
  rm -rf gpurun_out/prof_$TAG
done
echo "gpu_$TAG done"
