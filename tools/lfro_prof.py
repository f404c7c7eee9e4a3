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
print("  %-40s      %8.0f cycles / SB step" % ("R: waits for the top halo", v[15] / nsb), file=sys.stderr)
print("  %-40s      %8.0f cycles / SB step" % ("R: steady-state period (SBs n/4..3n/4)", v[12] / max(v[13], 1)), file=sys.stderr)
print("  %-40s      %8.0f cycles / workgroup" % ("L2: first SB's wait (pipeline fill)", v[14] / nwg), file=sys.stderr)
print("  %-40s      %8.0f cycles" % ("workgroup lifetime (R)", v[8] / nwg), file=sys.stderr)

tl = (ctypes.c_ulonglong * (24 * 8))()
if L.vp9hip_lfro_tl_read(tl) == 0 and any(tl):
    names = ["R ld_top ok", "R h0 ok", "R k0-3 done", "R h1 ok", "R rb", "H0 start", "H0 end", "H1 start", "H1 end",
             "C col start", "C col end", "C ld_top ok", "C end", "L1 stage start", "L1 ld_int", "L2 poll ok", "L2 ld_top",
             "S1 part0 start", "S1 progress", "S2 start", "S2 end"]
    t0 = min(x for x in tl if x)
    print("timeline of one row task (cycles from its first event; SBs 40..47):", file=sys.stderr)
    for e, nm in enumerate(names):
        print("  %-18s" % nm + "".join("%9d" % (tl[e * 8 + j] - t0 if tl[e * 8 + j] else -1) for j in range(8)), file=sys.stderr)
