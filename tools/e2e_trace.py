"""e2e decoder on the low-density C3 sample with VP9HIP_STAGE_TRACE=1: where the caller
thread's time goes (staging setup / upload, device planning wall) per 16-frame batch."""
import importlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["VP9HIP_STAGE_TRACE"] = "1"
import bench  # noqa: E402

v = importlib.import_module("ffmpeg-hybrid_amd")
W, H = 3840, 2160
low = [v.SynthFrame(v.synth_params(W, H, 8, seed=bench.frame_seed(0, i, 2), log2_tile_cols=2, p_zero_eob=0.9,
                                   p_skip=0.7)) for i in range(16)]
sample = bench.encode_sample(v, low, 1, 16)
pkts = [d for g in sample for d in g]
dec = v.Decoder(0, max_batch=16, parse_threads=16)
for reps in (2, 40):
    t0 = time.perf_counter()
    n = 0
    for _, info in dec.decode(pkts * reps, download=False):
        dec.release(info.buf)
        n += 1
    dec.flush()
    print("frames %d fps %.1f" % (n, n / (time.perf_counter() - t0)), file=sys.stderr, flush=True)
dec.close()
