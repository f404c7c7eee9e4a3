#!/bin/bash
# Bench variants per config on one box, no CPU legs, first 4 frames of every slot verified.
# usage: tools/cfg_ab.sh "NAME CONFIG INFLIGHT [ENV=VAL ...]" ...
#   e.g. tools/cfg_ab.sh "C5_if4 C5 4" "C5_if4_q8 C5 4 GPU_MAX_HW_QUEUES=8"
set -o pipefail
O=gpurun_out/cfg_ab; mkdir -p $O
for spec in "$@"; do
  set -- $spec; name=$1 cfg=$2 n=$3; shift 3
  env "$@" timeout -k 10 300 python bench.py --config $cfg --inflight $n --steps ${STEPS:-8} --warmup 2 --no-cpu-baseline --verify-frames 4 > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/$name.json').read().strip().split(chr(10))[-1]);print('$name', d['value'], d['ms_per_step'], d['verify']['frames'], d['verify']['of'], len(d['verify']['mismatched']))"
done
