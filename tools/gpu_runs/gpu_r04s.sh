#!/bin/bash
# round-4: SQ counter passes over the shipped chain kernels (k_gemm_wks3 default) of the headline bench
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r04s}
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAVES SQ_WAVE_CYCLES" \
           "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $R/gpurun_out/pmcc_${TAG}_$i -o p \
    -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --wm-steps 0 > $R/gpurun_out/pmcc_${TAG}_$i.log 2>&1 \
    || { tail -20 $R/gpurun_out/pmcc_${TAG}_$i.log; exit 1; }
done
cd $R
python tools/pmc_summary.py gpurun_out/pmcc_${TAG}_ > gpurun_out/pmc_chain_$TAG.txt
rm -rf gpurun_out/pmcc_${TAG}_*
grep -A22 "k_gemm_wks3\|k_gru_gates\|k_ln_gemm_sample" gpurun_out/pmc_chain_$TAG.txt | head -80
echo "gpu_$TAG done"
