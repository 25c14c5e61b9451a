#!/bin/bash
# round-3 closing pass on one MI355X: GPU tests, smoke, default bench,
# kernel-trace profile of the headline (kernel stats + per-epoch table), HBM
# traffic PMC passes of the shipped encoder kernels (fp32, bf16), and a
# 2-rank gloo rehearsal of the N > 1 bench path.  Stops at the first failure.
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r03z}
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/tests_$TAG.log | head -20; tail -30 gpurun_out/tests_$TAG.log; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -2 gpurun_out/smoke_$TAG.log
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cut -c1-300 gpurun_out/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o p -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --wm-steps 0 > $R/gpurun_out/prof_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/prof_$TAG.log; exit 1; }
cd $R
python tools/epoch_table.py gpurun_out/prof_$TAG/p_results.db 7 13 30 > gpurun_out/epoch_table_$TAG.txt && head -8 gpurun_out/epoch_table_$TAG.txt
python tools/prof_summary.py gpurun_out/prof_$TAG/p_results.db 40 > gpurun_out/kernel_stats_$TAG.txt
ls gpurun_out/prof_$TAG/ > gpurun_out/prof_files_$TAG.txt
bash tools/pmc_traffic.sh _${TAG}_fp32 && bash tools/pmc_traffic.sh _${TAG}_bf16 --precision bf16 || exit 1
grep encoder gpurun_out/traffic_${TAG}_fp32.txt gpurun_out/traffic_${TAG}_bf16.txt
DREAMER_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --wm-steps 3 --no-cpu-baseline > gpurun_out/dp2_$TAG.json 2> gpurun_out/dp2_$TAG.err \
  || { tail -30 gpurun_out/dp2_$TAG.err; exit 1; }
cut -c1-300 gpurun_out/dp2_$TAG.json
echo "gpu_$TAG done"
