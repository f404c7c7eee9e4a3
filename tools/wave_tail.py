"""Wavefront-tail estimate for the intra launches (diagnostics, host only).

Per SB the cost proxy is the pixel rows its intra passes loop over (vp9hip_plan_sb_costs)
plus a fixed per-SB overhead C0 (tile loads + interior stores). For one frame group:
- launch schedule: launch t waits for every SB of diagonal t - 1 of every frame and tile,
  so the group takes sum_t max_{SB in diagonal t} cost;
- dataflow bound: each SB waits only for its left and top neighbours, so the group takes
  the longest path through any frame's tile DAG.
usage: python tools/wave_tail.py [frames] [C0]"""
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
v = importlib.import_module("ffmpeg-hybrid_amd")
bench = importlib.import_module("bench")

nf = int(sys.argv[1]) if len(sys.argv) > 1 else 60
c0 = float(sys.argv[2]) if len(sys.argv) > 2 else 48.0
frames, _, _ = bench.make_frames(v, "C3", nf, 0, "420")
W, H, tiles = 3840, 2160, 4
sbc, sbr = 60, 34
bounds = [(t * sbc // tiles, (t + 1) * sbc // tiles) for t in range(tiles)]   # SB columns per tile (approx.)
ndiag = max(hi - lo for lo, hi in bounds) + sbr - 1
dmax = np.zeros(ndiag)
crit = 0.0
tot = 0.0
allc = []
for f in frames:
    c = v.plan_sb_costs(f).reshape(sbr, sbc) + c0
    allc.append(c)
    tot += c.sum()
    for lo, hi in bounds:
        t = c[:, lo:hi]
        L = np.zeros_like(t)
        for y in range(sbr):
            for x in range(hi - lo):
                L[y, x] = t[y, x] + max(L[y - 1, x] if y else 0, L[y, x - 1] if x else 0)
                d = x + y
                dmax[d] = max(dmax[d], t[y, x])
        crit = max(crit, L[-1, -1])
allc = np.concatenate([a.ravel() for a in allc])
print("frames %d  SB cost (rows + %.0f): mean %.1f  p50 %.0f  p99 %.0f  max %.0f" %
      (nf, c0, allc.mean(), np.percentile(allc, 50), np.percentile(allc, 99), allc.max()))
print("launch schedule  sum_t max = %.0f   (%d diagonals, mean-SB chain %.0f)" % (dmax.sum(), ndiag, ndiag * allc.mean()))
print("dataflow bound   longest path = %.0f  (%.2fx)" % (crit, dmax.sum() / crit))
