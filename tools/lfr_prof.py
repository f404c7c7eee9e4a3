"""k_lfrd SB-step phase breakdown (profiling only): run bench.py in-process against the
LFR_PROF build (ffmpeg-hybrid_amd/prof/libvp9hip.so copied over the library on the GPU box)
and print the per-SB-step shader-clock cycles of each phase, summed over every k_lfr
workgroup of the run (lane 0 of the first filtering wave)."""
import ctypes, runpy, sys, os
sys.argv = ["bench.py"] + sys.argv[1:]
try:
    runpy.run_path(os.path.join(os.path.dirname(__file__), "..", "bench.py"), run_name="__main__")
except SystemExit:
    pass
L = ctypes.CDLL(os.path.join(os.path.dirname(__file__), "..", "ffmpeg-hybrid_amd", "libvp9hip.so"))
out = (ctypes.c_ulonglong * 16)()
assert L.vp9hip_lfr_prof_read(out) == 0
v = list(out)
nsb, nwg = max(v[6], 1), max(v[14], 1)
names = {8: "interior + left halo into the tile, progress probe", 0: "barrier A",
         9: "top-halo loads issued (store wave: previous tile stored)", 13: "column pass part 1 (edge x = 0) + barrier",
         2: "column pass part 2 (+ barrier)",
         12: "blocking wait for the row above, first SB (pipeline fill)",
         10: "blocking wait for the row above, later SBs", 11: "barrier after the wait (the store wave's spin: the blocking wait)",
         3: "top halo into the tile, next interior issued, barrier", 4: "row pass (+ barrier)"}
print("workgroups", v[14], "SB steps", v[6], "blocking waits", v[5], file=sys.stderr)
for i, n in names.items():
    print("  %-64s %8.0f cycles / SB step" % (n, v[i] / nsb), file=sys.stderr)
print("  %-64s %8.0f cycles / SB step" % ("sum", sum(v[i] for i in names) / nsb), file=sys.stderr)
print("  %-64s %8.0f cycles / workgroup" % ("workgroup lifetime", v[7] / nwg), file=sys.stderr)
