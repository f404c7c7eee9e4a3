"""FFHWAccel download consumer (transfer_data_from) vs device consumer on the C5 realistic-
density sample through tests/c/hwaccel_harness, with VP9HIP_DL_THREADS variants (profiling;
bench.py's hwaccel_path leg is the reported number). usage: hw_dl.py [reps] [threads...]"""
import os, subprocess, sys, tempfile
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
import bench
import importlib
v = importlib.import_module("ffmpeg-hybrid_amd")
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
threads = sys.argv[2:] or ["3"]
idx, W, H, BPP, l2t, gop, _ = bench.CONFIGS["C5"]
low = [v.SynthFrame(v.synth_params(W, H, BPP, seed=bench.frame_seed(0, i, idx), log2_tile_cols=l2t, inter=int(i % gop != 0),
                                   p_zero_eob=0.9, p_skip=0.7)) for i in range(32)]
pkts = [d for g in bench.encode_sample(v, low, gop, 32) for d in g]
with tempfile.TemporaryDirectory() as td:
    ivf = os.path.join(td, "s.ivf")
    with open(ivf, "wb") as f:
        f.write(v.ivf_write(pkts * reps, W, H))
    runs = [("device", "3")] + [("download", t) for t in threads]
    for mode, t in runs:
        env = dict(os.environ, VP9HIP_DL_THREADS=t)
        r = subprocess.run([os.path.join(ROOT, "tests", "c", "hwaccel_harness"), ivf, "-", str(BPP), "1", "1", "1", "16", mode, "0"],
                           capture_output=True, text=True, timeout=300, env=env)
        f = r.stdout.split()
        print(mode, "threads", t, "fps %.1f" % (int(f[1]) / float(f[3])) if len(f) >= 4 else r.stderr[-300:], flush=True)
