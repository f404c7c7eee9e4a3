#!/usr/bin/env python3
"""GPU timeline of the last N graph-replayed steps in a rocprofv3 kernel trace: busy
fraction (union of kernel intervals), mean kernel concurrency, per-kernel busy time.
Usage: timeline.py gpurun_out/trace_TAG [steps]
With steps = 0: the kernels after bench.py's poison fill (the last fill-buffer kernel),
i.e. exactly the timed steps."""
import csv, glob, os, sys
from collections import defaultdict

d = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
rows = [r for r in csv.DictReader(open(f))]
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
# the last `steps` batches: split at the memset/fill or by count of k_lf... use time gaps > 1 ms
groups, cur = [], [ev[0]]
for e in ev[1:]:
    if e[0] - max(x[1] for x in cur[-50:]) > 1_000_000:
        groups.append(cur); cur = [e]
    else:
        cur.append(e)
groups.append(cur)
if steps == 0:
    fills = [x[0] for x in ev if "fill" in x[2].lower()]
    sel = [x for x in ev if x[0] > fills[-1] and "fill" not in x[2].lower()]
    groups = [sel]
    steps = 1
else:
    sel = [x for g in groups[-steps:] for x in g]
t0, t1 = min(x[0] for x in sel), max(x[1] for x in sel)
# union + concurrency
pts = sorted([(s, 1) for s, e, n in sel] + [(e, -1) for s, e, n in sel])
busy, conc_area, c, last = 0, 0, 0, pts[0][0]
for t, dlt in pts:
    if c > 0:
        busy += t - last
        conc_area += c * (t - last)
    c += dlt; last = t
per = defaultdict(int)
for s, e, n in sel:
    k = n.replace("(anonymous namespace)::", "").split("<")[0].split("(")[0].replace("void ", "")
    per[k] += e - s
span = t1 - t0
print("groups %d span %.3f ms busy %.1f%% mean concurrency %.2f" % (len(groups[-steps:]), span / 1e6, 100.0 * busy / span, conc_area / max(busy, 1)))
for k, v in sorted(per.items(), key=lambda x: -x[1]):
    print("  %-10s %.3f ms (sum of launch durations over the span / %d)" % (k, v / 1e6 / steps, steps))
