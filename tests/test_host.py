"""CPU: the C-ABI library, the synthetic pass-1 generator and oracle regression fixtures."""
import ctypes
import json
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("header", ["vp9hip.h", "vp9hip_hwaccel.h"])
def test_library_exports_every_declared_symbol(v9, header):
    hdr = open(os.path.join(ROOT, "include", header)).read()
    declared = sorted(set(re.findall(r"\b(vp9h(?:ip)?_\w+)\s*\(", hdr)))
    assert declared, "no entry points found in include/" + header
    L = v9.lib()
    for sym in declared:
        assert hasattr(L, sym), sym
    nm = subprocess.run(["nm", "-D", "--defined-only", v9.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (vp9h(?:ip)?_\w+)", nm))
    assert set(declared) <= exported
    assert set(v9.ABI_SYMBOLS) <= exported


def test_struct_layouts_match_header(v9):
    # vp9h_block is 52 bytes (include/vp9hip.h); the Python mirror must agree
    assert ctypes.sizeof(v9.Block) == 52
    assert ctypes.sizeof(v9.SegParams) == 124             # 31 int32
    assert ctypes.sizeof(v9.SynthParams) == 200           # 72 + vp9h_seg_params + padding to the uint64 alignment
    assert ctypes.sizeof(v9.EncParams) == 88 + 124          # 22 int32 + vp9h_seg_params
    assert v9.SynthParams.seg.offset == 72 and v9.EncParams.seg.offset == 88


def test_no_device_is_an_error_not_a_fallback(v9):
    """Without a GPU the product path fails loudly (no CPU fallback)."""
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except ImportError:
        pass
    with pytest.raises(v9.Vp9HipError):
        v9.Device(0)


def _coverage(pkt, w, h):
    cols, rows = (w + 7) >> 3, (h + 7) >> 3
    cov = np.zeros((rows, cols), np.int32)
    bwh = [(8, 8), (8, 4), (4, 8), (4, 4), (4, 2), (2, 4), (2, 2), (2, 1), (1, 2), (1, 1), (1, 1), (1, 1), (1, 1)]
    for i in range(pkt.nblocks):
        b = pkt.blocks[i]
        bw, bh = bwh[b.bs]
        cov[b.row:min(b.row + bh, rows), b.col:min(b.col + bw, cols)] += 1
        # blocks never straddle a superblock (decode_sb, vp9.c:1115-1193)
        assert b.row // 8 == (b.row + bh - 1) // 8 and b.col // 8 == (b.col + bw - 1) // 8
    return cov


@pytest.mark.parametrize("w,h,kw", [(352, 288, {}), (200, 130, {}), (66, 66, {}),
                                    (512, 256, {"log2_tile_cols": 1}), (3840, 64, {"log2_tile_cols": 2})])
def test_synth_partition_covers_frame_once(v9, w, h, kw):
    f = v9.SynthFrame(v9.synth_params(w, h, 8, seed=5, **kw))
    cov = _coverage(f.pkt, w, h)
    assert (cov == 1).all()


def test_synth_deterministic_and_seeded(v9):
    a = v9.SynthFrame(v9.synth_params(352, 288, 8, seed=9))
    b = v9.SynthFrame(v9.synth_params(352, 288, 8, seed=9))
    c = v9.SynthFrame(v9.synth_params(352, 288, 8, seed=10))
    raw = lambda f: (ctypes.string_at(f.pkt.blocks, 52 * f.pkt.nblocks),
                     ctypes.string_at(f.pkt.coefs, f.nbytes_coefs))
    assert raw(a) == raw(b)
    assert raw(a) != raw(c)


def test_synth_rejects_illegal_tiling(v9):
    # 384 px -> 6 SB columns: only log2_tile_cols 0 is legal (vp9.c:800-810)
    with pytest.raises(v9.Vp9HipError):
        v9.SynthFrame(v9.synth_params(384, 64, 8, log2_tile_cols=1))


def test_synth_statistics_follow_survey(v9):
    """§8(d): skip 0.2, eob uniform in [1, min(n, 64)], q_idx 60 dequantization."""
    f = v9.SynthFrame(v9.synth_params(1920, 1080, 8, seed=3))
    bl = f.blocks()
    skip = np.mean([b.skip for b in bl])
    assert 0.15 < skip < 0.25
    eobs = np.ctypeslib.as_array(f.pkt.eobs, (f.pkt.neobs,))
    assert eobs.min() >= 1 and eobs.max() <= 64


def test_oracle_regression_framemd5(v9, orc):
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(ROOT, "tests", "golden", "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    want = json.load(open(os.path.join(ROOT, "tests", "golden", "oracle_framemd5.json")))
    got = mg.compute()
    assert got == want


def test_planner_stats_c3_frame(v9):
    """Host planner on a 4K frame (no GPU): every tx block becomes a job, passes pack
    ready jobs of any sizes into 64 lanes (never fewer passes than dependency levels),
    the wavefront step counts follow the SB grid (intra: x_in_tile + y, LF: x + 2y)."""
    f = v9.SynthFrame(v9.synth_params(3840, 2160, 8, seed=0x56503902, log2_tile_cols=2))
    st = v9.plan_stats(f)
    assert st["sbs"] == 60 * 34
    # keyframe: a prediction job per tx block (skip blocks too), a residual job per eob > 0
    eobs = np.ctypeslib.as_array(f.pkt.eobs, (f.pkt.neobs,))
    assert st["rjobs"] == int((eobs > 0).sum())
    assert st["pjobs"] >= f.pkt.neobs
    assert st["passes"] >= st["levels"] >= st["sbs"]   # a pass holds jobs of settled producers only
    assert st["passes"] <= 1.1 * st["levels"]          # list scheduling stays near that bound
    assert st["jobs_4x4"] + st["jobs_8x8"] + st["jobs_16x16"] + st["jobs_32x32"] == st["pjobs"]
    assert 0 < st["lane_use"] <= 1
    assert st["pred_steps"] == 15 + 34 - 1     # 4 tile columns of 15 SBs
    assert st["lf_steps"] == 60 + 2 * 33


def test_plan_sb_costs_sum_to_pass_rows(v9):
    """vp9hip_plan_sb_costs (the wavefront-tail diagnostic): per-SB pass rows of a 4K
    keyframe, every SB has intra work, and they sum to plan_stats' pass rows."""
    f = v9.SynthFrame(v9.synth_params(3840, 2160, 8, seed=0x56503902, log2_tile_cols=2))
    c = v9.plan_sb_costs(f)
    assert c.shape == (60 * 34,)
    assert (c >= 4).all()
    assert c.sum() == v9.plan_stats(f)["pass_rows"]


def test_planner_inter_level_schedule(v9):
    """Inter frames (no GPU): intra SBs are scheduled by dependency level. An SB waits only
    for the SBs whose intra pixels its intra blocks read, so a frame with ~10 % intra blocks
    needs far fewer intra steps than the x_in_tile + y diagonals; a keyframe (every block
    intra) keeps exactly the diagonals."""
    key = v9.SynthFrame(v9.synth_params(1920, 1080, 8, seed=0x56503901))
    st = v9.plan_stats(key)
    assert st["level_steps"] == st["pred_steps"] == 30 + 17 - 1
    inter = v9.SynthFrame(v9.synth_params(1920, 1080, 8, seed=0x56503911, inter=1))
    st = v9.plan_stats(inter)
    assert st["pred_steps"] <= 30 + 17 - 1        # diagonals holding an SB with intra blocks
    assert 1 <= st["level_steps"] < st["pred_steps"] / 3
