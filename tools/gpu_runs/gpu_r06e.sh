#!/bin/bash
# round-6: two half-batch chains on two streams vs one B = 256 chain (tools/half_probe.py)
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r06e}
mkdir -p gpurun_out
for p in fp32 bf16; do
  timeout -k 10 300 python tools/half_probe.py 256 $p > gpurun_out/half_${TAG}_$p.txt 2>&1 || { tail -30 gpurun_out/half_${TAG}_$p.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/half_${TAG}_$p.txt
done
echo "gpu_$TAG done"
