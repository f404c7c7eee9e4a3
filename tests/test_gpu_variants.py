"""The A/B switches of the pixel path stay bit-exact: k_lfrd instead of the band-overlapped
k_lfro (VP9HIP_LFRO=0), k_mcq's task slices per unit group (VP9HIP_MCQ_SLICES), one residual
launch per transform size (VP9HIP_RESID_MULTI=0), and intra SBs reading their left
neighbour's column from the frame rows instead of the saved SB edges (VP9HIP_EDGE=0, also on
the C3 keyframe shape); inter frames' intra levels as one k_pred launch per level instead of
k_predd (VP9HIP_PRED_DF=0); the k_predd work as a launch of its own instead of intra workers
inside the phase's k_lfro launch (VP9HIP_PRED_LF_FUSE=0; the default is fused), with its
default grid, on the 8K phases (VP9HIP_PRED_DF_MAX) and with a 3-workgroup grid that loops
over every ticket (VP9HIP_PRED_DF_WGS=3); the fused form on the 8K phases and with one
intra worker workgroup (DF_WGS=4). Each is switched (read when the context opens) on a key + P chain of
the C2 (1080p 8-bit) or C5 (8K 10-bit) shape, decoded through the bench's batch path and
compared with the CPU oracle. (The losing alternates of rounds 1-4 -- the single-tile row LF,
k_mc / k_mcp, MC tickets inside k_lfrd -- were removed in round 5; DESIGN.md §5 keeps
their measurements.)"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

pytestmark = pytest.mark.gpu

CASES = [
    ({"VP9HIP_LFRO": "0"}, "C2", 4),
    ({"VP9HIP_LFRO": "0"}, "C5", 2),
    ({"VP9HIP_MCQ_SLICES": "1"}, "C5", 2),
    ({"VP9HIP_MCQ_SLICES": "5"}, "C2", 4),
    ({"VP9HIP_RESID_MULTI": "0"}, "C2", 4),
    ({"VP9HIP_RESID_MULTI": "0"}, "C5", 2),
    ({"VP9HIP_EDGE": "0"}, "C3", 3),
    ({"VP9HIP_EDGE": "0"}, "C2", 3),
    ({"VP9HIP_PRED_DF": "0"}, "C2", 4),
    # the standalone k_predd launch (intra workers not fused into k_lfro), with its default
    # grid, on the 8K phases, and with a 3-workgroup grid that loops over every ticket
    ({"VP9HIP_PRED_LF_FUSE": "0"}, "C2", 4),
    ({"VP9HIP_PRED_LF_FUSE": "0", "VP9HIP_PRED_DF_MAX": "100000"}, "C5", 2),
    ({"VP9HIP_PRED_LF_FUSE": "0", "VP9HIP_PRED_DF_WGS": "3"}, "C2", 4),
    # the default fused form: on the 8K phases, and with one intra worker workgroup
    ({"VP9HIP_PRED_DF_MAX": "100000"}, "C5", 2),
    ({"VP9HIP_PRED_DF_WGS": "4"}, "C2", 4),
]


@pytest.mark.parametrize("env,config,n", CASES)
def test_switch_matches_oracle(v9, orc, env, config, n):
    frames, refs, geom = bench.make_frames(v9, config, n)
    W, H, BPP, log2, gop = geom
    os.environ.update(env)
    dev = v9.Device(0)
    try:
        dev.configure(W, H, BPP, nbufs=len(frames))
        dev.stage_batch(frames, list(range(len(frames))), refs)
        for _ in range(2):                       # the second run replays the captured graph
            dev.run_batch()
        dev.sync()
        bad = []
        for i, ref in bench.oracle_frames(v9, orc, frames, refs, (W, H, BPP, log2, gop)):
            d = bench.compare_frame(v9, dev.download(i), ref, geom)
            if d:
                bad.append((i, d))
        assert not bad, "%s %s: frames differing from the oracle: %s" % (env, config, bad)
    finally:
        dev.close()
        for k in env:
            del os.environ[k]
