"""k_lfro wave-role breakdown (profiling only): run bench.py in-process with VP9HIP_LFRO=1
against the LFR_PROF build (ffmpeg-hybrid_amd/prof/libvp9hip.so copied over the library
on the GPU box) and print, per wave role, the cycles spent waiting on the workgroup's LDS
counters per SB step (busy = the R wave's lifetime - wait), summed over every k_lfro
workgroup of the run."""
import ctypes, runpy, sys, os
os.environ["VP9HIP_LFRO"] = "1"
sys.argv = ["bench.py"] + sys.argv[1:]
try:
    runpy.run_path(os.path.join(os.path.dirname(__file__), "..", "bench.py"), run_name="__main__")
except SystemExit:
    pass
L = ctypes.CDLL(os.path.join(os.path.dirname(__file__), "..", "ffmpeg-hybrid_amd", "libvp9hip.so"))
out = (ctypes.c_ulonglong * 16)()
assert L.vp9hip_lfr_prof_read(out) == 0
v = list(out)
nsb, nwg = max(v[10], 1), max(v[11], 1)
life = v[8] / nsb
print("workgroups", v[11], "SB steps", v[10], "R lifetime %.0f cycles / SB step" % life, file=sys.stderr)
for i, n in enumerate(["R (luma row edges)", "H0 (luma column edges, rows 0-31)", "H1 (luma column edges, rows 32-63)",
                       "C (chroma)", "L1 (interiors)", "L2 (top halos)", "S1 (bottom rows, hand-off)", "S2 (other rows)"]):
    print("  %-40s wait %8.0f  busy %8.0f cycles / SB step" % (n, v[i] / nsb, life - v[i] / nsb), file=sys.stderr)
print("  %-40s      %8.0f cycles / SB step" % ("L2: waits for the row above", v[9] / nsb), file=sys.stderr)
print("  %-40s      %8.0f cycles" % ("workgroup lifetime (R)", v[8] / nwg), file=sys.stderr)
