#!/bin/bash
# kbench: chain tile-GEMM shape variants and the sampler kernel with phase stamps;
# rocprofv3 kernel trace of a short headline bench -> per-epoch kernel table
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd)
: > gpurun_out/kbench_${TAG:-r03d}.txt
for f in ${KB_FILTERS:-tv ts}; do
  KB_B=256 timeout -k 10 200 tools/kbench/kbench "$f" >> gpurun_out/kbench_${TAG:-r03d}.txt 2>&1 || { tail -20 gpurun_out/kbench_${TAG:-r03d}.txt; exit 1; }
done
grep -E "^ *(tv|ts)|phases ts" gpurun_out/kbench_${TAG:-r03d}.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG:-r03d} -o p -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --wm-steps 0 > $R/gpurun_out/prof_${TAG:-r03d}.log 2>&1 || { tail -20 $R/gpurun_out/prof_${TAG:-r03d}.log; exit 1; }
cd $R && grep '"value"' gpurun_out/prof_${TAG:-r03d}.log | cut -c1-200
python tools/epoch_table.py gpurun_out/prof_${TAG:-r03d}/p_results.db 7 13 45 > gpurun_out/epoch_table_${TAG:-r03d}.txt && cat gpurun_out/epoch_table_${TAG:-r03d}.txt
