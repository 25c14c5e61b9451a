#!/bin/bash
# round-6: where the time goes -- phase times (fp32 / bf16, B = 64 / 128 / 256)
# and kernel-trace epoch tables of the bf16 headline and of configs[1] (B = 64 bf16)
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r06d}
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 300 python tools/phase_probe.py 64 128 256 > gpurun_out/phase_${TAG}_fp32.txt 2>&1 || { tail gpurun_out/phase_${TAG}_fp32.txt; exit 1; }
cat gpurun_out/phase_${TAG}_fp32.txt
PRECISION=bf16 timeout -k 10 300 python tools/phase_probe.py 64 128 256 > gpurun_out/phase_${TAG}_bf16.txt 2>&1 || { tail gpurun_out/phase_${TAG}_bf16.txt; exit 1; }
cat gpurun_out/phase_${TAG}_bf16.txt
cd /tmp && export TMPDIR=/tmp
for cfg in "256 bf16" "64 bf16"; do
  set -- $cfg
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_$TAG -o p -- python3 $R/bench.py --batch $1 --precision $2 --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --wm-steps 0 > $R/gpurun_out/prof_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/prof_$TAG.log; exit 1; }
  (cd $R && python tools/epoch_table.py gpurun_out/prof_$TAG/p_results.db 7 13 45 > gpurun_out/epoch_table_${TAG}_B$1_$2.txt && head -30 gpurun_out/epoch_table_${TAG}_B$1_$2.txt)
  rm -rf $R/gpurun_out/prof_$TAG
done
echo "gpu_$TAG done"
