#!/bin/bash
# round-6 closing pass on one MI355X: GPU tests, smoke, kernel-trace profile of
# the headline bench command (kernel stats + per-epoch table + timeline), HBM
# traffic PMC passes of the shipped encoder kernels (fp32, bf16), then the
# default bench -- whose roofline.profile / traffic fields read the summaries
# this pass just wrote into profiles/ (box-local copies, merged back through
# gpurun_out/ and committed under the same names).  Stops at the first failure.
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r06z}
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/tests_$TAG.log | head -20; tail -30 gpurun_out/tests_$TAG.log; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -2 gpurun_out/smoke_$TAG.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o p -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --wm-steps 0 > $R/gpurun_out/prof_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/prof_$TAG.log; exit 1; }
cd $R
python tools/epoch_table.py gpurun_out/prof_$TAG/p_results.db 7 13 40 > gpurun_out/epoch_table_$TAG.txt && head -8 gpurun_out/epoch_table_$TAG.txt
python tools/epoch_timeline.py gpurun_out/prof_$TAG/p_results.db > gpurun_out/timeline_$TAG.txt
python tools/prof_summary.py gpurun_out/prof_$TAG/p_results.db 40 > gpurun_out/kernel_stats_$TAG.txt
cp gpurun_out/kernel_stats_$TAG.txt profiles/${TAG}_kernel_stats.txt
rm -rf gpurun_out/prof_$TAG
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o p -- python3 $R/bench.py --steps 5 --warmup 2 --precision bf16 --no-cpu-baseline --no-secondary --wm-steps 0 > $R/gpurun_out/prof_${TAG}_bf16.log 2>&1 || { tail -20 $R/gpurun_out/prof_${TAG}_bf16.log; exit 1; }
cd $R
python tools/epoch_table.py gpurun_out/prof_$TAG/p_results.db 7 13 40 > gpurun_out/epoch_table_${TAG}_bf16.txt && head -8 gpurun_out/epoch_table_${TAG}_bf16.txt
python tools/prof_summary.py gpurun_out/prof_$TAG/p_results.db 40 > gpurun_out/kernel_stats_${TAG}_bf16.txt
cp gpurun_out/kernel_stats_${TAG}_bf16.txt profiles/${TAG}_kernel_stats_bf16.txt
rm -rf gpurun_out/prof_$TAG
bash tools/pmc_traffic.sh _${TAG}_fp32 && bash tools/pmc_traffic.sh _${TAG}_bf16 --precision bf16 || exit 1
cp gpurun_out/traffic_${TAG}_fp32.json profiles/${TAG}_traffic_B256_r64_fp32.json
cp gpurun_out/traffic_${TAG}_bf16.json profiles/${TAG}_traffic_B256_r64_bf16.json
rm -rf gpurun_out/pmc_*
timeout -k 10 900 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cut -c1-400 gpurun_out/bench_$TAG.json
echo "gpu_$TAG done"
