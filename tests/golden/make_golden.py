#!/usr/bin/env python3
"""Regenerate tests/golden/oracle_framemd5.json.

Per-frame MD5s (FATE framemd5 style, tests/fate-run.sh:172-174) of the oracle's
decode of seeded synthetic pass-1 packets. These are REGRESSION fixtures of the
oracle + generator (self-generated: the reference decoder could not be run here,
SURVEY.md §8c), not reference outputs.
"""
import hashlib
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

CASES = [
    ("key_352x288_8", 352, 288, 8, {}),
    ("key_200x130_8_skipzero", 200, 130, 8, {"p_zero_eob": 0.3, "p_skip": 0.5}),
    ("key_512x256_8_tiles2", 512, 256, 8, {"log2_tile_cols": 1}),
    ("key_176x144_8_lossless", 176, 144, 8, {"lossless": 1, "q_idx": 0}),
    ("key_352x288_8_stress", 352, 288, 8, {"coef_stress": 1}),
    ("key_352x288_8_sharp5", 352, 288, 8, {"sharpness": 5, "filter_level": 50}),
    ("key_176x144_10", 176, 144, 10, {}),
    ("key_96x80_12", 96, 80, 12, {}),
]
INTER = [
    ("inter_352x288_8_comp", 352, 288, 8, {"compound": 1}),
    ("inter_200x130_8_bilin", 200, 130, 8, {"bilinear": 1}),
    ("inter_176x144_10", 176, 144, 10, {"compound": 1}),
]


def md5_planes(v9, planes, w, h):
    return [hashlib.md5(p.tobytes()).hexdigest() for p in v9.visible(planes, w, h)]


def compute():
    v9 = importlib.import_module("ffmpeg-hybrid_amd")
    import oracle
    out = {}
    for name, w, h, bpp, kw in CASES:
        f = v9.SynthFrame(v9.synth_params(w, h, bpp, seed=0x56503900, **kw))
        pl = v9.alloc_planes(w, h, bpp)
        oracle.decode_frame(f.pkt, pl)
        out[name] = md5_planes(v9, pl, w, h)
    for name, w, h, bpp, kw in INTER:
        k = v9.SynthFrame(v9.synth_params(w, h, bpp, seed=0x56503901))
        ref = v9.alloc_planes(w, h, bpp)
        oracle.decode_frame(k.pkt, ref)
        f = v9.SynthFrame(v9.synth_params(w, h, bpp, seed=0x56503902, inter=1, **kw))
        pl = v9.alloc_planes(w, h, bpp)
        oracle.decode_frame(f.pkt, pl, [ref, ref, ref])
        out[name] = md5_planes(v9, pl, w, h)
    return out


if __name__ == "__main__":
    res = compute()
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "oracle_framemd5.json")
    with open(path, "w") as fh:
        json.dump(res, fh, indent=1, sort_keys=True)
    print("wrote", path, len(res), "cases")
