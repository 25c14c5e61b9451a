#!/bin/bash
# A/B of engine knobs: each line "ENV=.. ENV=.." runs one short bench
set -o pipefail
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  echo "== $line"
  env $line timeout -k 10 120 python bench.py --steps 20 --warmup 3 --phases --no-cpu-baseline > gpurun_out/ab$i.json 2> gpurun_out/ab$i.err || { tail -5 gpurun_out/ab$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab$i.json'));print(d['value'], d['ms_per_step'])"
  tail -1 gpurun_out/ab$i.err
done < "$1"
