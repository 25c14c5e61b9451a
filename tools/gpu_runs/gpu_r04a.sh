#!/bin/bash
# round-4 first probe: batch lanes on separate streams (tools/lanes_probe.py)
# and SQ counter passes over the shipped chain kernels of the headline bench.
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r04a}
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_noise.py tests/test_gpu_api.py -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/tests_$TAG.log | head -30; tail -30 gpurun_out/tests_$TAG.log; exit 1; }
grep -E "PASSED|FAILED|sampler|actor eps|corr|PIT|passed" gpurun_out/tests_$TAG.log | head -60
timeout -k 10 400 python -u tools/lanes_probe.py --reps 20 > gpurun_out/lanes_$TAG.txt 2>&1 || { tail -30 gpurun_out/lanes_$TAG.txt; exit 1; }
cat gpurun_out/lanes_$TAG.txt | grep -v '^{'
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
head -60 gpurun_out/pmc_chain_$TAG.txt
echo "gpu_$TAG done"
