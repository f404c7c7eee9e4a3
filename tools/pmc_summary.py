#!/usr/bin/env python3
"""Summarise tools/profile.sh output: per-kernel mean of each PMC counter and of the
kernel-trace duration. Usage: pmc_summary.py gpurun_out/prof_TAG"""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(name):
    """The kernel's identifier ("void k_plan<1, 1>(PlanDev)" -> "k_plan")."""
    n = name.strip()
    if n.startswith("void "):
        n = n[5:]
    n = n.replace("(anonymous namespace)::", "")
    for sep in "<(":
        n = n.split(sep)[0]
    return n.strip() or name[:40]


def main(d):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            acc[short(r["Kernel_Name"])]["duration_us"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, cs in sorted(acc.items()):
        if not k.startswith("k_"):
            continue
        print(k)
        for c, v in sorted(cs.items()):
            print("  %-24s n=%-5d mean=%.4g total=%.4g" % (c, len(v), sum(v) / len(v), sum(v)))


if __name__ == "__main__":
    main(sys.argv[1])
