set -e
mkdir -p gpurun_out
for c in ${CFGS:-C3 C2 C4 C5}; do
  timeout -k 10 400 python bench.py --config $c --steps 3 --warmup 1 --cpu-seconds 5 > gpurun_out/cfg_$c.json 2> gpurun_out/cfg_$c.err
  echo "$c $(python -c "import json;d=json.loads(open('gpurun_out/cfg_$c.json').read().strip().split(chr(10))[-1]);print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['cpu_baseline']['value'] if d['cpu_baseline'] else None)")"
done
