#!/bin/bash
# round-4: train_Agent at AC_epochs = 1 returns one copy of the loss slots -- full GPU suite, headline x2, epoch timeline
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r04zn}
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/tests_$TAG.log | head; tail -20 gpurun_out/tests_$TAG.log; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-secondary --wm-steps 0 --no-cpu-baseline > gpurun_out/bench_${TAG}_$i.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
  echo "fp32 $i: $(cut -c100-190 gpurun_out/bench_${TAG}_$i.json)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o p -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --wm-steps 0 > $R/gpurun_out/prof_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/prof_$TAG.log; exit 1; }
cd $R
python tools/epoch_timeline.py gpurun_out/prof_$TAG/p_results.db > gpurun_out/timeline_$TAG.txt && head -3 gpurun_out/timeline_$TAG.txt
grep -E "copyBuffer|elementwise|Fill|cat|mean" gpurun_out/timeline_$TAG.txt | head
rm -rf gpurun_out/prof_$TAG
echo "gpu_$TAG done"
