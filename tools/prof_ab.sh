#!/bin/bash
# GPU box: rocprofv3 kernel stats of the bench with two builds of the library
#   bash tools/prof_ab.sh TAG   (dreamer_amd/libdreamer_hip_{prev,new}.so)
set -o pipefail
TAG=${1:-x}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
for v in prev new; do
  cp $R/dreamer_amd/libdreamer_hip_$v.so $R/dreamer_amd/libdreamer_hip.so
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof${TAG}_$v -o p -- python3 $R/bench.py --steps 5 --warmup 2 --wm-steps 0 --sequential > $R/gpurun_out/prof${TAG}_$v.log 2>&1 || exit 1
  python3 $R/tools/prof_summary.py $R/gpurun_out/prof${TAG}_$v/p_results.db | grep -m6 "k_conv_nhwc\|frames"
done
