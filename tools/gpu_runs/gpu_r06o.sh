#!/bin/bash
# round-6 A/B: k_gemm_wks3 with the K loop unrolled (a real register pipeline; nounroll = the rolled loop whose
# back edge waited for every load), ring depth du3 (fp32 3) / dub2 (bf16 2); bitwise digests; chain tests
cd "$(dirname "$0")/../.." || exit 1
export PYTHONUNBUFFERED=1
TAG=${1:-r06o}
mkdir -p gpurun_out
for p in fp32 bf16; do
  for v in "" nounroll; do
    DREAMER_LIB_VARIANT=$v timeout -k 10 200 python tools/epoch_digest.py 256 $p 3 2>&1 | grep digest || exit 1
  done
done
run() {  # variant precision batch
  DREAMER_LIB_VARIANT=$1 timeout -k 10 240 python bench.py --batch $3 --precision $2 --steps 30 --no-cpu-baseline \
    --no-secondary --wm-steps 0 > gpurun_out/b_${TAG}.json 2> gpurun_out/b_${TAG}.err || { tail -20 gpurun_out/b_${TAG}.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_${TAG}.json'));print('${1:-default} $2 B$3', d['value'], d['ms_per_step'])"
}
for rep in 1 2; do
  run "" fp32 256 && run nounroll fp32 256 && run du3 fp32 256 && \
  run "" bf16 256 && run nounroll bf16 256 && run dub2 bf16 256 || exit 1
done
run "" fp32 128 && run nounroll fp32 128 && run "" bf16 64 && run nounroll bf16 64 || exit 1
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_baseline.py tests/test_gpu_bf16.py tests/test_gpu_flips.py tests/test_gpu_determinism.py tests/test_gpu_parity.py \
  > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/tests_$TAG.log | head -30; tail -30 gpurun_out/tests_$TAG.log | cut -c1-300; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
echo "gpu_$TAG done"
