#!/bin/bash
# Same-box ABAB of two builds on the default bench (or BARGS): A is either another tree
# (AB_TREE=dir: a `git worktree` of an earlier commit with its own library, run with its own
# bench.py) or ffmpeg-hybrid_amd/ab_base/libvp9hip.so swapped into this tree; B is this tree.
# Prints fps, ms per step, verified frames and the planner / k_psb / k_plf kernel ms.
# usage: tools/abso.sh [rounds]   (BARGS: extra bench args, STEPS)
set -o pipefail
O=$PWD/gpurun_out/abso; mkdir -p $O
L=ffmpeg-hybrid_amd/libvp9hip.so
[ -z "$AB_TREE" ] && cp $L $O/libvp9hip_B.so
run() {  # $1 = tag, $2 = dir
  (cd $2 && timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --verify-frames 4 ${BARGS:-}) > $O/$1.json 2> $O/$1.err || { echo "$1 failed"; tail -5 $O/$1.err; return 1; }
  python3 -c "import json;d=json.loads(open('$O/$1.json').read().strip().split(chr(10))[-1]);km=d['roofline'].get('kernel_ms',{});print('$1', d['value'], d['ms_per_step'], d['verify']['frames'], len(d['verify']['mismatched']), 'k_plan', km.get('k_plan'), 'k_psb', km.get('k_psb'), 'k_plf', km.get('k_plf'))"
}
for r in $(seq 1 ${1:-2}); do
  if [ -n "$AB_TREE" ]; then run A$r $AB_TREE || exit 1; else cp ffmpeg-hybrid_amd/ab_base/libvp9hip.so $L; run A$r . || { cp $O/libvp9hip_B.so $L; exit 1; }; fi
  [ -z "$AB_TREE" ] && cp $O/libvp9hip_B.so $L
  run B$r . || exit 1
done
