#!/bin/bash
# GPU box: new parity tests + a 2-rank bench rehearsal (gloo, both ranks on
# the one GPU; the driver's N>1 runs use RCCL) + a north-star-shape line (B=256)
#   bash tools/gpu_dp_rehearsal.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-x}
K=${2:-update_S}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v -k "$K" --timeout 120 --timeout-method thread > gpurun_out/t$TAG.log 2>&1 || { tail -40 gpurun_out/t$TAG.log; exit 1; }
tail -3 gpurun_out/t$TAG.log
DREAMER_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --wm-steps 3 > gpurun_out/dp$TAG.json 2> gpurun_out/dp$TAG.err || { tail -30 gpurun_out/dp$TAG.err; exit 1; }
cat gpurun_out/dp$TAG.json
timeout -k 10 300 python bench.py --batch 256 --steps 10 --warmup 3 --no-cpu-baseline --wm-steps 5 > gpurun_out/b256$TAG.json 2> gpurun_out/b256$TAG.err || { tail -30 gpurun_out/b256$TAG.err; exit 1; }
cat gpurun_out/b256$TAG.json
