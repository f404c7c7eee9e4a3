#!/bin/bash
# A/B of two library builds on one box: ffmpeg-hybrid_amd/ab_base/libvp9hip.so (A) vs the
# tree's build (B), alternated ABAB; prints fps, ms per step and the planner / k_plf kernel ms.
# usage: tools/abso.sh [rounds]   (BARGS: extra bench args)
set -o pipefail
O=gpurun_out/abso; mkdir -p $O
L=ffmpeg-hybrid_amd/libvp9hip.so
cp $L $O/libvp9hip_B.so
for r in $(seq 1 ${1:-2}); do
  for v in A B; do
    if [ $v = A ]; then cp ffmpeg-hybrid_amd/ab_base/libvp9hip.so $L; else cp $O/libvp9hip_B.so $L; fi
    timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --verify-frames 4 ${BARGS:-} > $O/$v$r.json 2> $O/$v$r.err || { echo "$v$r failed"; tail -5 $O/$v$r.err; cp $O/libvp9hip_B.so $L; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/$v$r.json').read().strip().split(chr(10))[-1]);km=d['roofline']['kernel_ms'];print('$v$r', d['value'], d['ms_per_step'], d['verify']['frames'], len(d['verify']['mismatched']), 'k_plan', km.get('k_plan'), 'k_plf', km.get('k_plf'))"
  done
done
cp $O/libvp9hip_B.so $L
