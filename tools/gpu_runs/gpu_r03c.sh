set -o pipefail
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "baseline or parity or test_gpu_wm or determinism or act_step or vector" > gpurun_out/tests_r03c.log 2>&1 || { tail -40 gpurun_out/tests_r03c.log; exit 1; }
tail -3 gpurun_out/tests_r03c.log
KB_B=256 timeout -k 10 120 tools/kbench/kbench ts > gpurun_out/kbench_r03c.txt 2>&1 || { tail -20 gpurun_out/kbench_r03c.txt; exit 1; }
grep -v "^ *phases" gpurun_out/kbench_r03c.txt
timeout -k 10 300 python tools/phase_probe.py 64 128 256 > gpurun_out/phase_probe.txt 2>&1 || { tail -20 gpurun_out/phase_probe.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/phase_probe.txt
