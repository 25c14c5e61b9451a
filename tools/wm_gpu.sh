set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_wm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/wm.log 2>&1 || { tail -30 gpurun_out/wm.log; exit 1; }
tail -1 gpurun_out/wm.log
timeout -k 10 200 python tools/wm_prof.py > gpurun_out/wm_eager.txt 2>&1 || { tail -20 gpurun_out/wm_eager.txt; exit 1; }
cat gpurun_out/wm_eager.txt
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/wmprof -o prof -- python3 $R/tools/wm_prof.py > $R/gpurun_out/wmprof.log 2>&1 || { tail -20 $R/gpurun_out/wmprof.log; exit 1; }
cd $R && python3 tools/prof_summary.py $(find gpurun_out/wmprof -name '*.db' | head -1) 45
