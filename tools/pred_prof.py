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
