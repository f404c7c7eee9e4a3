#!/bin/bash
# End-of-round bench lines on 1 GPU: the default bench (as the driver runs it, every CPU / e2e /
# hwaccel leg), then the other BASELINE.md configs. usage: tools/round_bench.sh TAG
# (CFGS: configs after the default, default "C2 C4 C5")
set -o pipefail
O=gpurun_out/${1:-rb}; mkdir -p $O
timeout -k 10 500 python bench.py > $O/bench_default_C3.json 2> $O/bench_default_C3.err || { tail -5 $O/bench_default_C3.err; exit 1; }
echo "C3 $(python -c "import json;d=json.loads(open('$O/bench_default_C3.json').read().strip().split(chr(10))[-1]);print(d['value'], d['ms_per_step'], d['verified_frames'], d['roofline']['frac'])")"
for c in ${CFGS:-C2 C4 C5}; do
  st=20; [ $c = C5 ] && st=6
  timeout -k 10 600 python bench.py --config $c --steps $st --warmup 2 > $O/bench_$c.json 2> $O/bench_$c.err || { tail -5 $O/bench_$c.err; exit 1; }
  echo "$c $(python -c "import json;d=json.loads(open('$O/bench_$c.json').read().strip().split(chr(10))[-1]);print(d['value'], d['ms_per_step'], d['verified_frames'], d['roofline']['frac'])")"
done
