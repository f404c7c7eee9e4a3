"""Write a config's realistic-density sample stream (bench.py's hwaccel-leg sample) as IVF,
repeated: mk_ivf.py CONFIG REPS OUT.ivf (profiling input for tests/c/hwaccel_harness)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench, importlib
v = importlib.import_module("ffmpeg-hybrid_amd")
cfg = sys.argv[1]; reps = int(sys.argv[2]); out = sys.argv[3]
idx, W, H, BPP, l2t, gop, _ = bench.CONFIGS[cfg]
n = max(gop, 16)
low = [v.SynthFrame(v.synth_params(W, H, BPP, seed=bench.frame_seed(0, i, idx), log2_tile_cols=l2t, inter=int(i % gop != 0),
                                   p_zero_eob=0.9, p_skip=0.7)) for i in range(n)]
pkts = [d for g in bench.encode_sample(v, low, gop, n) for d in g]
open(out, "wb").write(v.ivf_write(pkts * reps, W, H))
print(len(pkts) * reps, "frames")
