cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_bf16v5 -o p -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --wm-steps 0 --precision bf16 > $GRAFT_REPO_ROOT/gpurun_out/prof_bf16v5.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_bf16v5.log; exit 1; }
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py gpurun_out/prof_bf16v5/p_results.db 12
