#!/bin/bash
# round-5: stage timeline of the persistent scan (DR_PSCAN_TS variant)
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r05c}
mkdir -p gpurun_out
for B in 256 64; do
  DREAMER_LIB_VARIANT=pscants timeout -k 10 200 python tools/pscan_probe.py --batch $B > gpurun_out/pscan_${TAG}_B$B.txt 2>&1 || { tail -20 gpurun_out/pscan_${TAG}_B$B.txt; exit 1; }
  cat gpurun_out/pscan_${TAG}_B$B.txt
done
echo "gpu_$TAG done"
