#!/bin/bash
# short 1-GPU bench lines of several configs (no CPU legs). usage: tools/r04_bench.sh TAG CFG...
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
for c in "$@"; do
  st=10; [ $c = C5 ] && st=4
  timeout -k 10 300 python bench.py --config $c --steps $st --warmup 2 --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || { tail -5 $O/bench_$c.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_$c.json').read().strip().split(chr(10))[-1]);r=d['roofline'];print('$c', d['value'], d['ms_per_step'], d.get('verified_frames'), r['kernel'], r['avg_launch_us'], r['frac'])"
done
