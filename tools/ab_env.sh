#!/bin/bash
# GPU box: bench A/B of a library knob read from the environment
#   bash tools/ab_env.sh TAG VAR   (runs VAR=0, VAR=1, VAR=0, VAR=1)
set -o pipefail
TAG=$1; VAR=$2
mkdir -p gpurun_out
for v in 0 1 0 1; do
  env $VAR=$v timeout -k 10 200 python bench.py --steps 20 --warmup 3 --wm-steps 10 > gpurun_out/ab${TAG}_$v.json 2>gpurun_out/ab$TAG.err || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/ab${TAG}_$v.json').read().strip().splitlines()[-1]); print('$VAR=$v', d['value'], d['epochs']['sequential_value'], d['roofline']['encoder_ms'], d['secondary']['wm_step']['ms_per_step'], d['losses'])"
done
