#!/bin/bash
# round-6 A/B: conv_glds stages (3: two workgroups per CU; 4; 6), bf16 B = 256 encoder and headline
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r06g}
R=$(pwd)
mkdir -p gpurun_out
for rep in 1 2; do
for st in 3 4 6; do
  export DREAMER_GLDS_STAGES=$st
  timeout -k 10 200 python bench.py --batch 256 --precision bf16 --steps 30 --no-cpu-baseline --no-secondary --wm-steps 0 > gpurun_out/b_${TAG}.json 2> gpurun_out/b_${TAG}.err || { tail -20 gpurun_out/b_${TAG}.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_${TAG}.json'));print('stages $st B256 bf16', d['value'], d['ms_per_step'], 'enc', d['roofline']['encoder_ms'], d['roofline']['frac'])"
done
done
cd /tmp && export TMPDIR=/tmp
for st in 3 6; do
export DREAMER_GLDS_STAGES=$st
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o p -- python3 $R/bench.py --batch 256 --precision bf16 --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --wm-steps 0 > $R/gpurun_out/prof_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/prof_$TAG.log; exit 1; }
(cd $R && python tools/epoch_table.py gpurun_out/prof_$TAG/p_results.db 7 13 12 | grep glds)
rm -rf $R/gpurun_out/prof_$TAG
done
echo "gpu_$TAG done"
