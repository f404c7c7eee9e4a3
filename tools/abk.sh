#!/bin/bash
# A/B like tools/ab.sh, printing the planner's event-timed kernel ms as well
mkdir -p gpurun_out/ab
for spec in "$@"; do
  name=${spec%%=*}; envs=${spec#*=}
  env $envs timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline ${BARGS:-} \
      > gpurun_out/ab/$name.json 2> gpurun_out/ab/$name.err || { echo "$name failed"; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/ab/$name.json').read().strip().split(chr(10))[-1]);km=d['roofline']['kernel_ms'];print('$name', d['value'], d['ms_per_step'], d['verify']['frames'], len(d['verify']['mismatched']), 'k_plan', km['k_plan'], 'k_plf', km['k_plf'])"
done
