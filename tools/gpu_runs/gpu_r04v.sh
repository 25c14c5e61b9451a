#!/bin/bash
# round-4: bisect the B = 4096 vector-epoch / B = 512 actor-gradient mismatch over the round-4 knobs
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r04v}
mkdir -p gpurun_out
for v in main r03 notailbwd norows16 nogruepi nowks3 nosreg; do
  if [ $v = main ]; then VV=""; else VV=$v; fi
  DREAMER_LIB_VARIANT=$VV timeout -k 10 300 python -u -m pytest "tests/test_gpu_vector.py::test_vector_epoch_vs_oracle_B4096" -m gpu -q --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/bisect_${TAG}_$v.log 2>&1
  rc=$?
  echo "$v: rc $rc $(grep -E 'out of tol|passed|failed' gpurun_out/bisect_${TAG}_$v.log | head -2 | cut -c1-200 | tr '\n' ' ')"
  [ $rc -gt 1 ] && exit 1
done
echo "gpu_$TAG done"
