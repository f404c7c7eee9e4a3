"""FFHWAccel device-consumer rate, this build vs another build's library + harness
(ffmpeg-hybrid_amd/ab_r03/, e.g. the round-3 end), on the realistic-density sample of a
config, alternated ABAB (profiling). usage: hw_ab.py CONFIG [reps] [rounds]"""
import os, subprocess, sys, tempfile
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
import bench
import importlib
v = importlib.import_module("ffmpeg-hybrid_amd")
cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 2
idx, W, H, BPP, l2t, gop, _ = bench.CONFIGS[cfg]
n = max(gop, 16)
low = [v.SynthFrame(v.synth_params(W, H, BPP, seed=bench.frame_seed(0, i, idx), log2_tile_cols=l2t, inter=int(i % gop != 0),
                                   p_zero_eob=0.9, p_skip=0.7)) for i in range(n)]
pkts = [d for g in bench.encode_sample(v, low, gop, n) for d in g]
ab = os.path.join(ROOT, "ffmpeg-hybrid_amd", "ab_r03")
with tempfile.TemporaryDirectory() as td:
    ivf = os.path.join(td, "s.ivf")
    with open(ivf, "wb") as f:
        f.write(v.ivf_write(pkts * reps, W, H))
    head = os.path.join(ROOT, "tests", "c", "hwaccel_harness")
    variants = [("B(head)", head, dict(os.environ)), ("A(ab_r03)", os.path.join(ab, "hwaccel_harness"), dict(os.environ, LD_LIBRARY_PATH=ab))]
    for kv in os.environ.get("HW_AB_ENVS", "").split():      # extra head variants: NAME=VALUE
        k, val = kv.split("=", 1)
        variants.append(("B(%s)" % kv, head, dict(os.environ, **{k: val})))
    for xl in os.environ.get("HW_AB_X", "").split():          # harness:libdir pairs, relative to the repo
        x, l = xl.split(":", 1)
        variants.append(("X(%s)" % xl, os.path.join(ROOT, x), dict(os.environ, LD_LIBRARY_PATH=os.path.join(ROOT, l))))
    for r in range(rounds):
        for tag, exe, env in variants:
            p = subprocess.run([exe, ivf, "-", str(BPP), "1", "1", "1", "16", "device", "0"], capture_output=True, text=True,
                               timeout=300, env=env)
            f = p.stdout.split()
            print(cfg, tag, "fps %.1f" % (int(f[1]) / float(f[3])) if len(f) >= 4 else p.stderr[-300:], flush=True)
            for line in p.stderr.splitlines():
                if "hwaccel trace" in line:
                    print("   ", line, flush=True)
