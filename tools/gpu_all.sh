#!/bin/bash
# GPU box: all -m gpu tests, then one bench line (with the WM-step secondary)
#   bash tools/gpu_all.sh TAG
set -o pipefail
TAG=${1:-x}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/gpu_tests$TAG.log 2>&1 || { tail -40 gpurun_out/gpu_tests$TAG.log; exit 1; }
tail -3 gpurun_out/gpu_tests$TAG.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench$TAG.json 2> gpurun_out/bench$TAG.err || { tail -20 gpurun_out/bench$TAG.err; exit 1; }
cat gpurun_out/bench$TAG.json
