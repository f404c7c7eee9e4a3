#!/bin/bash
# A/B of bench.py variants on one box: each "NAME=ENV..." argument runs the default bench
# (no CPU legs) with those environment settings; prints value / ms per step per variant.
# usage: tools/ab.sh "base=" "static0=VP9HIP_STATIC=0" ...   (BARGS: extra bench args)
mkdir -p gpurun_out/ab
for spec in "$@"; do
  name=${spec%%=*}; envs=${spec#*=}
  env $envs timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline ${BARGS:-} \
      > gpurun_out/ab/$name.json 2> gpurun_out/ab/$name.err || { echo "$name failed"; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab/$name.json').read().strip().split(chr(10))[-1]);print('$name', d['value'], d['ms_per_step'], d['verify']['frames'], len(d['verify']['mismatched']))"
done
