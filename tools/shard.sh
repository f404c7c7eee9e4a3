# --shard tiles (one stream, phase by phase) vs the batch mode, C5 and C2, 1 GPU.
set -e
mkdir -p gpurun_out
for c in ${CFGS:-C5 C2}; do
  timeout -k 10 300 python bench.py --config $c --shard tiles --steps 3 --warmup 1 > gpurun_out/shard_$c.json 2> gpurun_out/shard_$c.err
  echo "$c tiles: $(python -c "import json;d=json.loads(open('gpurun_out/shard_$c.json').read().strip().split(chr(10))[-1]);print(d['value'], d['ms_per_step'], d['config']['exchange_bytes_per_phase'])")"
done
