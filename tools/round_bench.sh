# Default bench (as the driver runs it) + the other BASELINE.md configs, 1 GPU.
set -e
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/rb_default.json 2> gpurun_out/rb_default.err
tail -1 gpurun_out/rb_default.json
for c in ${CFGS:-C2 C4 C5}; do
  timeout -k 10 400 python bench.py --config $c --steps 3 --warmup 1 --cpu-seconds 5 > gpurun_out/rb_$c.json 2> gpurun_out/rb_$c.err
  echo "$c $(python -c "import json;d=json.loads(open('gpurun_out/rb_$c.json').read().strip().split(chr(10))[-1]);print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['cpu_baseline']['value'] if d['cpu_baseline'] else None)")"
done
