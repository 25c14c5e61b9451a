#!/bin/bash
# HBM traffic (FETCH_SIZE / WRITE_SIZE passes) of the shipped encoder kernels, fp32 and bf16, B=256 64x64
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
bash tools/pmc_traffic.sh _r03k_fp32 && bash tools/pmc_traffic.sh _r03k_bf16 --precision bf16 && echo "gpu_r03k done"
