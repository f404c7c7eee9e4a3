#!/bin/bash
# Planner-only kernel traces of several trees, same box (VP9HIP_PLAN_ONLY=1: the device
# planner alone, one batch in flight so no launches overlap): rocprofv3 --kernel-trace
# --stats per tree, then the per-kernel average durations side by side.
# usage: tools/plan_ab.sh TREE...   (a TREE may carry one env setting: .@VP9HIP_PLAN_DBG=4)
set -o pipefail
O=$PWD/gpurun_out/plan_ab; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for spec in "$@"; do
  t=${spec%%@*}; ev=""; [ "$t" != "$spec" ] && ev=${spec#*@}
  d=$(cd $OLDPWD && cd $t && pwd); tag=$(basename $d)${ev:+_$ev}
  (cd $d && env VP9HIP_PLAN_ONLY=1 $ev timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$tag -o run --output-format csv \
     -- python3 bench.py --inflight 1 --steps 6 --warmup 2 --no-cpu-baseline --verify-frames 0) > $O/$tag.log 2>&1 \
     || { echo "$tag failed"; tail -5 $O/$tag.log; exit 1; }
  echo "== $tag $(grep -o '"value": [0-9.]*' $O/$tag.log | head -1)"
  python3 - "$O/$tag" <<'PY'
import csv, glob, re, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    m = re.search(r"\b(k_\w+?)\s*[<(]", r["Name"])
    print("  %-14s %6s calls  avg %9.1f us  total %8.2f ms" % (m.group(1) if m else r["Name"][:14], r["Calls"],
          float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6))
PY
done
