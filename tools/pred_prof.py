"""Intra workgroup phase breakdown (profiling only): run bench.py in-process against the
PRED_PROF build (ffmpeg-hybrid_amd/prof/libvp9hip.so copied over the library on the GPU box)
and print the shader-clock cycles per intra SB workgroup (k_pred and the intra part of
k_plf): tile loads, passes (by the pass's largest transform), interior stores."""
import ctypes, runpy, sys, os
sys.argv = ["bench.py"] + sys.argv[1:]
try:
    runpy.run_path(os.path.join(os.path.dirname(__file__), "..", "bench.py"), run_name="__main__")
except SystemExit:
    pass
L = ctypes.CDLL(os.path.join(os.path.dirname(__file__), "..", "ffmpeg-hybrid_amd", "libvp9hip.so"))
out = (ctypes.c_ulonglong * 16)()
assert L.vp9hip_pred_prof_read(out) == 0
v = list(out)
nwg = max(v[4], 1)
print("intra workgroups %d, passes per workgroup %.1f" % (v[4], v[3] / nwg), file=sys.stderr)
for i, n in enumerate(["tile loads", "passes", "interior stores"]):
    print("  %-20s %8.0f cycles / workgroup" % (n, v[i] / nwg), file=sys.stderr)
for b in range(4):
    c = max(v[9 + b], 1)
    print("  pass MAXN %-2d        %8.0f cycles / pass  (%.2f passes / workgroup)" % (4 << b, v[5 + b] / c, v[9 + b] / nwg),
          file=sys.stderr)
c = max(v[14], 1)
print("  k_plf LF workgroup   %8.0f cycles / SB  (%d SBs)" % (v[13] / c, v[14]), file=sys.stderr)
print("  slowest intra wg     %8.0f cycles" % v[15], file=sys.stderr)

# k_plf workgroup timeline of the launches of one shape (the first with >= 2000 intra SBs):
# per launch its span, and per kind (intra / LF / residual) when the workgroups started and
# ended relative to the launch start, in microseconds (device real-time clock, 100 MHz)
cap = 65536
buf = (ctypes.c_ulonglong * (2 * cap))()
n = ctypes.c_int(0)
if hasattr(L, "vp9hip_plf_tl_read") and L.vp9hip_plf_tl_read(buf, cap, ctypes.byref(n)) == 0 and n.value:
    ev = sorted(((buf[2 * i] & ((1 << 62) - 1), buf[2 * i + 1], buf[2 * i] >> 62) for i in range(min(n.value, cap))))
    launches, cur, end = [], [], 0
    for e in ev:
        if cur and e[0] > end:
            launches.append(cur)
            cur = []
        cur.append(e)
        end = max(end, e[1]) if len(cur) > 1 else e[1]
    launches.append(cur)
    print("k_plf timeline: %d workgroups in %d launch clusters" % (len(ev), len(launches)), file=sys.stderr)
    names = ["intra", "LF", "resid"]
    for li, ln in enumerate(launches[:6]):
        t0 = min(e[0] for e in ln)
        t1 = max(e[1] for e in ln)
        print("launch %d: span %.1f us, %d workgroups" % (li, (t1 - t0) / 100.0, len(ln)), file=sys.stderr)
        for k in range(3):
            w = [e for e in ln if e[2] == k]
            if not w:
                continue
            st = sorted((e[0] - t0) / 100.0 for e in w)
            en = sorted((e[1] - t0) / 100.0 for e in w)
            du = sorted((e[1] - e[0]) / 100.0 for e in w)
            q = lambda a, f: a[min(len(a) - 1, int(f * len(a)))]
            print("  %-5s n=%5d start p50 %6.1f p90 %6.1f max %6.1f | end p50 %6.1f p90 %6.1f max %6.1f | dur p50 %6.1f p90 %6.1f max %6.1f"
                  % (names[k], len(w), q(st, .5), q(st, .9), st[-1], q(en, .5), q(en, .9), en[-1], q(du, .5), q(du, .9), du[-1]),
                  file=sys.stderr)
