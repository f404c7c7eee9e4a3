#!/bin/bash
# Same-box A/B/... of several trees on the default bench (or BARGS), interleaved round by
# round: each tree is a directory with its own library and bench.py (this tree is ".", other
# commits are `git worktree`s, e.g. ab_r03/). Prints fps, ms per step, verified frames and the
# serialised k_lf / k_plf / planner kernel ms of every run.
# usage: tools/abso.sh ROUNDS TREE...   (BARGS: extra bench args, STEPS)
# A TREE may carry one environment setting for its runs: .@VP9HIP_R4=0 (tag repo_VP9HIP_R4=0).
set -o pipefail
O=$PWD/gpurun_out/abso; mkdir -p $O
R=$1; shift
for r in $(seq 1 $R); do
  for spec in "$@"; do
    t=${spec%%@*}; ev=""; [ "$t" != "$spec" ] && ev=${spec#*@}
    tag=$(basename $(cd $t && pwd))${ev:+_$ev}_$r
    (cd $t && env $ev timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --verify-frames 4 ${BARGS:-}) > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/$tag.json').read().strip().split(chr(10))[-1]);km=d['roofline'].get('kernel_ms',{});print('$tag', d['value'], d['ms_per_step'], d['verify']['frames'], len(d['verify']['mismatched']), 'k_lf', km.get('k_lf'), 'k_plf', km.get('k_plf'), 'plan', km.get('k_plan'), 'k_mc', km.get('k_mc'), 'k_lfr', km.get('k_lfr'))"
  done
done
