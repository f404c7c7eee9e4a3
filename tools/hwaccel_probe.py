#!/usr/bin/env python3
"""FFHWAccel adapter probe (GPU box): the bench's realistic-density C3 (or --config) sample
stream, repeated, through tests/c/hwaccel_harness with VP9HIP_HWACCEL_TRACE=1 (host time per
adapter step on stderr). Usage: hwaccel_probe.py [--config C3] [--reps 20] [--mode device]
[--lag 16] [--depth 0] [extra env NAME=VALUE ...]"""
import argparse, os, subprocess, sys, tempfile
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import importlib

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C3")
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--mode", default="device")
ap.add_argument("--lag", type=int, default=16)
ap.add_argument("--depth", type=int, default=0)          # 0: frame_params' default
ap.add_argument("env", nargs="*")
a = ap.parse_args()
v = importlib.import_module("ffmpeg-hybrid_amd")
cidx, W, H, BPP, L2, gop, nf = bench.CONFIGS[a.config]
n = max(gop, 16)
low = [v.SynthFrame(v.synth_params(W, H, BPP, seed=bench.frame_seed(0, i, cidx), log2_tile_cols=L2,
                                   inter=int(gop > 1 and i % gop != 0), p_zero_eob=0.9, p_skip=0.7)) for i in range(n)]
sample = bench.encode_sample(v, low, gop, n)
pkts = [d for g in sample for d in g]
env = dict(os.environ, VP9HIP_HWACCEL_TRACE="1")
for e in a.env:
    k, _, val = e.partition("=")
    env[k] = val
with tempfile.TemporaryDirectory() as td:
    ivf = os.path.join(td, "s.ivf")
    with open(ivf, "wb") as f:
        f.write(v.ivf_write(pkts * a.reps, W, H))
    r = subprocess.run([os.path.join(ROOT, "tests", "c", "hwaccel_harness"), ivf, "-", str(BPP), "1", "1", "1",
                        str(a.lag), a.mode, str(a.depth)], capture_output=True, text=True, timeout=300, env=env)
f = r.stdout.split()
print(a.config, a.mode, "lag", a.lag, "depth", a.depth, " ".join(a.env), "->",
      "%.1f fps" % (int(f[1]) / float(f[3])) if len(f) >= 4 else r.stdout.strip(), "rc", r.returncode)
for line in r.stderr.splitlines()[-6:]:
    print("  ", line)
