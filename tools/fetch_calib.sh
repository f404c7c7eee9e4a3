#!/bin/bash
# FETCH_SIZE per launch of 256 MiB read once with 16-, 12- and 24-byte lane loads (GPU box).
# usage: tools/fetch_calib.sh   (tools/build/fetch_calib: hipcc ... tools/fetch_calib.hip)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/fetch_calib; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc -o run --output-format csv -- $ROOT/tools/build/fetch_calib > $OUT/run.log 2>&1
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/pmc/**/run_counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if r.get("Counter_Name") == "FETCH_SIZE":
        acc[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    print("%-40s FETCH_SIZE %.1f MiB per launch (%d launches) -> factor %.3f" % (k[:40], sum(v) / len(v) / 1024, len(v), 256.0 / (sum(v) / len(v) / 1024)))
PY
