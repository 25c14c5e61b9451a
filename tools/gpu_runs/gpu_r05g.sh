#!/bin/bash
# round-5: persistent-scan stage timeline only (DR_PSCAN_TS variant)
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r05g}
mkdir -p gpurun_out
for B in ${BATCHES:-256}; do
DREAMER_LIB_VARIANT=pscants timeout -k 10 200 python tools/pscan_probe.py --batch $B > gpurun_out/pscan_${TAG}_B$B.txt 2>&1 || { tail -20 gpurun_out/pscan_${TAG}_B$B.txt; exit 1; }
cat gpurun_out/pscan_${TAG}_B$B.txt
done
