#!/bin/bash
# Round-3 GPU session: selected parity tests, the full bench line, kbench
# timings of the chain GEMMs and SQ counter passes over them.  Every GPU step
# under its own time limit; the script stops at the first failure.
#   bash tools/gpu_runs/gpu_r03.sh TAG "pytest -k expression"
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r03}
KEXPR=${2:-}
R=$(pwd)
mkdir -p gpurun_out
if [ -n "$KEXPR" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider \
    -k "$KEXPR" > gpurun_out/tests_$TAG.log 2>&1 || { tail -60 gpurun_out/tests_$TAG.log; exit 1; }
  grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/tests_$TAG.log | tail -40
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
  cat gpurun_out/bench_$TAG.json
fi
if [ "${KB:-0}" = 1 ]; then
  KB_B=256 timeout -k 10 300 tools/kbench/kbench "${KB_FILTER:-tv}" > gpurun_out/kbench_$TAG.txt 2>&1 || { tail -20 gpurun_out/kbench_$TAG.txt; exit 1; }
  cat gpurun_out/kbench_$TAG.txt | grep -v "^ *phases" | head -60
fi
if [ "${PMC:-0}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  export KB_REPS=20 KB_B=256
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_ANY" \
             "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY" \
             "SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $R/gpurun_out/pmc_${TAG}_$i -o pmc \
      -- $R/tools/kbench/kbench "${PMC_FILTER:-tv0 GRU}" > $R/gpurun_out/pmc_${TAG}_$i.log 2>&1 || { tail -5 $R/gpurun_out/pmc_${TAG}_$i.log; exit 1; }
  done
  cd $R && python tools/pmc_summary.py gpurun_out/pmc_${TAG}_ > gpurun_out/pmc_${TAG}.txt && cat gpurun_out/pmc_${TAG}.txt
fi
echo "gpu_r03 done"
