#!/usr/bin/env python3
"""Per-kernel HBM traffic per launch from tools/profile.sh PMC passes.

FETCH_SIZE / WRITE_SIZE are kilobytes per dispatch (rocprofv3). On gfx950 FETCH_SIZE
counts 64 B per 128-B request of wide streaming reads (MI355X_MICROARCH.md, HBM
section), so `fetch_corrected` doubles it; both are reported.
Usage: traffic.py gpurun_out/prof_TAG [out.json]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    for k in ("k_plf", "k_resid", "k_pred", "k_lfr", "k_lf", "k_mc", "k_plan", "k_pllf", "k_psb"):
        if k in name:
            return k
    return None


def main(d, out=None):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if k and r["Counter_Name"] in ("FETCH_SIZE", "WRITE_SIZE"):
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]) * 1024.0)
    res = {}
    for k, c in acc.items():
        fe = sum(c["FETCH_SIZE"]) / max(1, len(c["FETCH_SIZE"]))
        wr = sum(c["WRITE_SIZE"]) / max(1, len(c["WRITE_SIZE"]))
        res[k] = {"fetch_bytes": fe, "fetch_corrected": 2 * fe, "write_bytes": wr,
                  "traffic_bytes": 2 * fe + wr, "launches": len(c["FETCH_SIZE"])}
    # the launch shape the counters were taken at (bench.py refuses a profile whose shape
    # differs from its own run): the bench line the profiled runs printed
    shape, bench = {}, None
    for f in sorted(glob.glob(os.path.join(d, "*.log"))):
        for line in open(f, errors="replace"):
            if line.startswith('{"metric"'):
                bench = json.loads(line)
        if bench:
            break
    if bench:
        kl = bench["roofline"]["kernel_launches"]
        for k in res:
            if k in kl:
                shape[k] = {"launches_per_step": kl[k], "streams_per_gpu": bench["config"]["streams_per_gpu"],
                            "frames_per_gpu": bench["config"]["frames_per_gpu"]}
    print(json.dumps({"per_launch": res, "shape": shape}, indent=1))
    if out:
        json.dump({"source": d, "per_launch": res, "shape": shape,
                   "bench_workload": bench["config"]["workload"] if bench else None}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:])
