cd $GRAFT_REPO_ROOT && export PYTHONUNBUFFERED=1
for c in 32 16 8; do
  DREAMER_WARM_CHUNK=$c timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --wm-steps 0 > gpurun_out/chunk_$c.json 2> gpurun_out/chunk_$c.err || exit 1
  echo "chunk $c: $(python -c "import json;d=json.load(open('gpurun_out/chunk_$c.json'));print(d['value'], d['ms_per_step'])")"
done
