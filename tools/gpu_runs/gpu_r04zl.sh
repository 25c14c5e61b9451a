#!/bin/bash
# round-4: code-path rehearsal of the driver's N > 1 bench (2 ranks, gloo standing in for RCCL, both on the
# one GPU -- time-sliced, so the numbers are not scaling figures): every secondary of the default bench at N = 2
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r04zl}
mkdir -p gpurun_out
DREAMER_DIST_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --wm-steps 2 > gpurun_out/dp_$TAG.json 2> gpurun_out/dp_$TAG.err || { grep -v "Training Agent" gpurun_out/dp_$TAG.err | tail -30; exit 1; }
cut -c1-600 gpurun_out/dp_$TAG.json
echo "gpu_$TAG done"
