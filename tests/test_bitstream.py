"""Host bitstream side: VP9 frame bitstream <-> pass-1 packet.

vp9h_encode_frame writes a synthetic packet as a VP9 keyframe / intra-only bitstream, and
vp9h_decode_frame parses it back. The decoded packet must equal the original exactly:
- blocks (position, size, tx sizes, skip, modes);
- eobs;
- dequantized coefficients;
- LF levels and header fields.

That pins the encoder and decoder to each other. Against the reference libavcodec parse it
is **parity unpinned**: no VP9 bitstream or reference build is available here,
so the parse follows vp9.c / vp9block.c as restated in the C source, with no golden stream.
The GPU case decodes a bitstream on the host and reconstructs it on the MI355X, bit-exact
against the oracle's decode of the original packet.
"""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _arrays(p):
    csz = 2 if p.bpp == 8 else 4
    blocks = [(b.row, b.col, b.bs, b.tx, b.uvtx, b.skip, b.intra, tuple(b.mode), b.uvmode, b.seg_id)
              for b in (p.blocks[i] for i in range(p.nblocks))]
    eobs = np.ctypeslib.as_array(p.eobs, (p.neobs,)).copy() if p.neobs else np.zeros(0, np.uint16)
    coefs = ctypes.string_at(p.coefs, p.ncoefs * csz) if p.ncoefs else b""
    return blocks, eobs, coefs


def _same(a, b):
    A, B = _arrays(a), _arrays(b)
    assert A[0] == B[0], "blocks differ"
    assert np.array_equal(A[1], B[1]), "eobs differ"
    assert A[2] == B[2], "coefficients differ"
    assert bytes(a.lflvl) == bytes(b.lflvl)
    for k in ("width", "height", "bpp", "ss_h", "ss_v", "lossless", "filter_level", "sharpness", "log2_tile_cols", "keyframe", "intraonly"):
        assert getattr(a, k) == getattr(b, k), k


CASES = [
    (352, 288, 8, {}),
    (200, 130, 8, {}),
    (8, 8, 8, {}),
    (66, 66, 8, {}),
    (1024, 128, 8, {"log2_tile_cols": 2}),
    (130, 74, 8, {"p_zero_eob": 0.3, "p_skip": 0.5}),
    (352, 288, 8, {"sharpness": 3, "filter_level": 63}),
    (352, 288, 8, {"filter_level": 0}),
    (200, 136, 8, {"lossless": 1, "q_idx": 0}),
    (352, 288, 10, {}),
    (200, 130, 10, {"coef_stress": 1}),
    (176, 144, 12, {}),
    (176, 144, 10, {"lossless": 1, "q_idx": 0}),
]


@pytest.mark.parametrize("w,h,bpp,kw", CASES)
def test_keyframe_round_trip(v9, w, h, bpp, kw):
    for seed in (1, 2):
        f = v9.SynthFrame(v9.synth_params(w, h, bpp, seed=seed, **kw))
        data = v9.encode_frame(f, f.params.q_idx)
        assert data[0] >> 6 == 2                                   # frame marker
        assert data[1:4] == b"\x49\x83\x42" or bpp > 8             # sync code right after (profile 0)
        d = v9.decode_frame(data)
        _same(f.pkt, d.pkt)


@pytest.mark.parametrize("bpp", [8, 10, 12])
@pytest.mark.parametrize("ssh,ssv", [(1, 0), (0, 1), (0, 0)])
def test_profile_1_3_round_trip(v9, bpp, ssh, ssv):
    """Profiles 1 / 3: the colour config codes the subsampling
    (read_colorspace_details, vp9.c:457-517); chroma uvtx, nnz contexts and token
    counts follow it (vp9block.c:1291, 965-1130)."""
    for (w, h, kw) in [(200, 130, {}), (512, 136, {"log2_tile_cols": 1}), (66, 74, {"lossless": 1, "q_idx": 0})]:
        f = v9.SynthFrame(v9.synth_params(w, h, bpp, seed=61, ss_h=ssh, ss_v=ssv, **kw))
        data = v9.encode_frame(f, f.params.q_idx)
        profile = (data[0] >> 5 & 1) | (data[0] >> 4 & 1) << 1
        assert profile == (1 if bpp == 8 else 3)
        d = v9.decode_frame(data)
        assert (d.pkt.ss_h, d.pkt.ss_v) == (ssh, ssv)
        _same(f.pkt, d.pkt)


def _set_bits(data, pos, vals):
    b = bytearray(data)
    for i, v in enumerate(vals):
        k = pos + i
        b[k >> 3] = (b[k >> 3] & ~(0x80 >> (k & 7))) | (v << (7 - (k & 7)))
    return bytes(b)


def test_colour_config_refusals(v9):
    """read_colorspace_details (vp9.c:457-517): 8-bit 4:2:0 in profile 1, the reserved bit,
    and RGB in profile 0 are invalid data."""
    f = v9.SynthFrame(v9.synth_params(200, 130, 8, seed=62, ss_h=1, ss_v=0))
    data = v9.encode_frame(f, 60)
    # profile 1 keyframe: marker 2, profile 2, show_existing, type, show, error_res 4,
    # sync 24 -> colour space at bit 32, range 35, ss_h 36, ss_v 37, reserved 38
    assert v9.decode_frame(data).pkt.ss_v == 0
    for pos, vals in ((36, [1, 1]), (38, [1])):
        with pytest.raises(v9.Vp9HipError) as e:
            v9.decode_frame(_set_bits(data, pos, vals))
        assert e.value.code == v9.EINVALIDDATA
    k0 = v9.encode_frame(v9.SynthFrame(v9.synth_params(200, 130, 8, seed=63)), 60)
    with pytest.raises(v9.Vp9HipError) as e:
        v9.decode_frame(_set_bits(k0, 32, [1, 1, 1]))      # RGB in profile 0
    assert e.value.code == v9.EINVALIDDATA


def test_4k_tiles_round_trip(v9):
    f = v9.SynthFrame(v9.synth_params(3840, 2160, 8, seed=0x56503902, log2_tile_cols=2))
    d = v9.decode_frame(v9.encode_frame(f, f.params.q_idx))
    _same(f.pkt, d.pkt)


def test_intra_only_frame(v9):
    f = v9.SynthFrame(v9.synth_params(352, 288, 8, seed=9))
    f.pkt.keyframe, f.pkt.intraonly = 0, 1
    d = v9.decode_frame(v9.encode_frame(f, f.params.q_idx))
    assert d.pkt.intraonly == 1 and d.pkt.keyframe == 0
    _same(f.pkt, d.pkt)


def test_refusals(v9):
    inter = v9.SynthFrame(v9.synth_params(352, 288, 8, seed=3, inter=1))
    with pytest.raises(v9.Vp9HipError) as e:
        v9.encode_frame(inter, 60)
    assert e.value.code == v9.ENOSYS
    wrapped = v9.SynthFrame(v9.synth_params(200, 130, 8, seed=5, coef_stress=1))   # int16 wrap at 8-bit
    with pytest.raises(v9.Vp9HipError):
        v9.encode_frame(wrapped, wrapped.params.q_idx)
    with pytest.raises(v9.Vp9HipError):
        v9.decode_frame(b"\x00\x01")


def test_truncated_and_corrupt_streams_fail_cleanly(v9):
    """Truncation or flipped bytes either fail with an AVERROR or decode to some packet;
    the parser never reads outside the buffer (run in a child process)."""
    code = r"""
import importlib, random, sys
v9 = importlib.import_module("ffmpeg-hybrid_amd")
f = v9.SynthFrame(v9.synth_params(352, 288, 8, seed=4, log2_tile_cols=0))
data = v9.encode_frame(f, 60)
rng = random.Random(7)
ok = err = 0
for k in range(60):
    b = bytearray(data)
    if k < 20:
        b = b[: rng.randrange(1, len(b))]
    else:
        for _ in range(1 + k % 5):
            i = rng.randrange(len(b)); b[i] ^= 1 << rng.randrange(8)
    try:
        v9.decode_frame(bytes(b)); ok += 1
    except v9.Vp9HipError:
        err += 1
print(ok, err)
"""
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, PYTHONPATH=ROOT))
    assert r.returncode == 0, r.stderr[-2000:]
    ok, err = map(int, r.stdout.split())
    assert ok + err == 60 and err > 0


@pytest.mark.gpu
def test_bitstream_to_gpu_matches_oracle(v9, orc, gpu):
    """Host entropy decode of a VP9 bitstream, then the MI355X pixel path, bit-exact
    against the oracle's reconstruction of the original packet."""
    for (w, h, bpp, kw) in [(352, 288, 8, {}), (1024, 128, 8, {"log2_tile_cols": 2}), (200, 130, 10, {})]:
        f = v9.SynthFrame(v9.synth_params(w, h, bpp, seed=11, **kw))
        d = v9.decode_frame(v9.encode_frame(f, f.params.q_idx))
        gpu.configure(w, h, bpp, nbufs=1)
        gpu.submit(d, 0)
        gpu.sync()
        got = gpu.download(0)
        ref = v9.alloc_planes(w, h, bpp)
        orc.decode_frame(f.pkt, ref)
        for a, b in zip(v9.visible(got, w, h), v9.visible(ref, w, h)):
            assert np.array_equal(a, b)
