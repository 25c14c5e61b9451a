#!/bin/bash
# round-4: conv K chunks in parity groups + convT parity class fastest -- headline fp32 / bf16,
# encoder traffic (PMC), epoch kernel stats, WM step bf16 / fp32
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r04zi}
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/tests_$TAG.log | head; tail -20 gpurun_out/tests_$TAG.log; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
for P in fp32 bf16; do
  timeout -k 10 300 python bench.py --no-secondary --wm-steps 0 --no-cpu-baseline --precision $P > gpurun_out/bench_${TAG}_$P.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
  echo "$P: $(cut -c100-190 gpurun_out/bench_${TAG}_$P.json)"
  WM_B=256 WM_PREC=$P timeout -k 10 300 python tools/wm_prof.py 2>&1 | grep "WM step"
done
bash tools/pmc_traffic.sh _${TAG}_fp32 > /dev/null && bash tools/pmc_traffic.sh _${TAG}_bf16 --precision bf16 > /dev/null || exit 1
head -8 gpurun_out/traffic_${TAG}_fp32.txt; head -8 gpurun_out/traffic_${TAG}_bf16.txt; grep "encoder group" gpurun_out/traffic_${TAG}_*.txt
rm -rf gpurun_out/pmc_*
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o p -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --wm-steps 0 > $R/gpurun_out/prof_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/prof_$TAG.log; exit 1; }
cd $R
python tools/epoch_table.py gpurun_out/prof_$TAG/p_results.db 7 13 40 > gpurun_out/epoch_table_$TAG.txt && head -8 gpurun_out/epoch_table_$TAG.txt
python tools/prof_summary.py gpurun_out/prof_$TAG/p_results.db 40 > gpurun_out/kernel_stats_$TAG.txt
rm -rf gpurun_out/prof_$TAG
echo "gpu_$TAG done"
