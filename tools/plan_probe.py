"""Device-planner probe: decode small synthetic frames through the device planner and the
host planner (VP9HIP_HOST_PLAN=1 in a child process) and compare both with the oracle.
Prints one line per case. Usage: python tools/plan_probe.py [host]"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import importlib  # noqa: E402

v = importlib.import_module("ffmpeg-hybrid_amd")
import oracle  # noqa: E402  (test infrastructure: the checker)

CASES = [
    (64, 64, 8, dict()),
    (352, 288, 8, dict()),
    (1024, 128, 8, dict(log2_tile_cols=2)),
    (352, 288, 8, dict(bitstream=1)),
    (200, 130, 10, dict()),
    (352, 288, 8, dict(inter=1)),
]


def run():
    for (w, h, bpp, kw) in CASES:
        inter = kw.get("inter", 0)
        key = v.SynthFrame(v.synth_params(w, h, bpp, seed=5, **{k: x for k, x in kw.items() if k not in ("inter", "bitstream")}))
        if kw.get("bitstream"):
            key = v.decode_frame(v.encode_frame(key, key.params.q_idx))
        dev = v.Device(0)
        dev.configure(w, h, bpp, nbufs=2)
        ok = True
        msg = ""
        try:
            dev.submit(key, 0)
            if inter:
                fi = v.SynthFrame(v.synth_params(w, h, bpp, seed=6, inter=1))
                dev.submit(fi, 1, (0, 0, 0))
            dev.sync()
            g = dev.download(1 if inter else 0)
        except Exception as e:  # noqa: BLE001
            ok = False
            msg = str(e)
        dev.close()
        if ok:
            r0 = v.alloc_planes(w, h, bpp)
            oracle.decode_frame(key.pkt, r0)
            r = r0
            if inter:
                r = v.alloc_planes(w, h, bpp)
                oracle.decode_frame(fi.pkt, r, [r0, r0, r0])
            bad = [int((a != b).sum()) for a, b in zip(v.visible(g, w, h), v.visible(r, w, h))]
            msg = "mismatched px per plane %s" % bad
            ok = not any(bad)
        print("%s %dx%d %d-bit %s: %s %s" % (os.environ.get("VP9HIP_HOST_PLAN", "dev"), w, h, bpp, kw,
                                            "OK" if ok else "FAIL", msg), flush=True)


if __name__ == "__main__":
    run()
    if len(sys.argv) > 1 and sys.argv[1] == "host":
        env = dict(os.environ, VP9HIP_HOST_PLAN="1")
        sys.exit(subprocess.call([sys.executable, os.path.abspath(__file__)], env=env))
