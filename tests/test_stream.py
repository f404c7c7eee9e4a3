"""Host bitstream side for whole streams: inter frames, MV prediction,
reference slots, probability contexts, backward adaptation, hidden frames,
show_existing_frame and superframes.

A vp9h_stream encoder writes synthetic pass-1 packets as a VP9 stream. It returns each
frame as coded, and a second vp9h_stream must decode exactly that packet. The coded
packet may differ from the synthetic one only as include/vp9hip.h documents:
- a predicted mode whose MV is not the packet's becomes NEWMV;
- a low-precision MV difference loses its odd 1/8-pel step;
- skipped inter blocks take the largest transform;
- coefficient-less inter blocks <= 8x8 become skip;
- fields the syntax does not carry are zero.

**Parity unpinned** against libavcodec, as for the keyframe tests (test_bitstream.py): no
VP9 stream or reference build exists here. The parse restates vp9.c,
vp9block.c, vp9mvs.c and vp9prob.c, cited in the C source. The GPU case reconstructs a
decoded inter stream on the MI355X and checks it against the oracle.
"""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NEARESTMV, NEARMV, ZEROMV, NEWMV = 10, 11, 12, 13
MAX_TX = [3, 3, 3, 3, 2, 2, 2, 1, 1, 1, 0, 0, 0]


def _mv(b, k, z, c):
    """mv[k][z][c] of a ctypes vp9h_block (flat int16[16])."""
    return b.mv[(k * 2 + z) * 2 + c]


def _blocks(p):
    return [p.blocks[i] for i in range(p.nblocks)]


def _btuple(b):
    return (b.row, b.col, b.bs, b.tx, b.uvtx, b.skip, b.intra, b.comp, b.seg_id, b.filter, tuple(b.mode), b.uvmode,
            tuple(b.ref), tuple(b.mv))


def _arrays(p):
    csz = 2 if p.bpp == 8 else 4
    eobs = np.ctypeslib.as_array(p.eobs, (p.neobs,)).copy() if p.neobs else np.zeros(0, np.uint16)
    coefs = ctypes.string_at(p.coefs, p.ncoefs * csz) if p.ncoefs else b""
    return eobs, coefs


def same_packet(a, b):
    """Decoded == coded, field by field."""
    for k in ("width", "height", "bpp", "ss_h", "ss_v", "keyframe", "intraonly", "lossless", "filter_level", "sharpness",
              "log2_tile_cols", "log2_tile_rows", "nblocks", "neobs", "ncoefs"):
        assert getattr(a, k) == getattr(b, k), k
    assert bytes(a.lflvl) == bytes(b.lflvl)
    assert list(a.ref_w) == list(b.ref_w) and list(a.ref_h) == list(b.ref_h)
    ba, bb = _blocks(a), _blocks(b)
    for i, (x, y) in enumerate(zip(ba, bb)):
        assert _btuple(x) == _btuple(y), "block %d: %s != %s" % (i, _btuple(x), _btuple(y))
    ea, ca = _arrays(a)
    eb, cb = _arrays(b)
    assert np.array_equal(ea, eb) and ca == cb


def check_legalized(orig, coded, stats, keep_modes=False):
    """The coded packet is the synthetic one up to what the syntax cannot carry."""
    bo, bc = _blocks(orig), _blocks(coded)
    assert len(bo) == len(bc)
    for o, c in zip(bo, bc):
        assert (o.row, o.col, o.bs, o.intra, o.seg_id) == (c.row, c.col, c.bs, c.intra, c.seg_id)
        if o.intra:
            assert (tuple(o.mode), o.uvmode, o.tx, o.uvtx) == (tuple(c.mode), c.uvmode, c.tx, c.uvtx)
            assert o.skip == c.skip
            continue
        assert c.comp == o.comp and c.ref[0] == o.ref[0] and (not o.comp or c.ref[1] == o.ref[1])
        assert c.filter == o.filter
        if o.skip:
            assert c.skip and c.tx == (0 if orig.lossless else MAX_TX[o.bs])
        else:
            assert c.tx == o.tx
            assert c.skip == o.skip or (c.skip and o.bs >= 9)
        for k in range(4):
            if keep_modes:
                assert c.mode[k] == o.mode[k]
                stats["kept"] += 1
                if o.mode[k] == ZEROMV:
                    assert all(_mv(c, k, z, q) == 0 for z in range(2) for q in range(2))
                continue
            for z in range(1 + o.comp):
                for comp in range(2):
                    d = _mv(c, k, z, comp) - _mv(o, k, z, comp)
                    assert abs(d) <= 1, (k, z, comp, d)
            if c.mode[k] == o.mode[k]:
                stats["kept"] += 1
                if c.mode[k] != NEWMV:
                    assert all(_mv(c, k, z, q) == _mv(o, k, z, q) for z in range(1 + o.comp) for q in range(2))
            else:
                assert c.mode[k] == NEWMV
                stats["to_new"] += 1


def _frames(v9, w, h, n, bpp=8, seed=700, **kw):
    """Keyframe + n - 1 inter frames (LAST = previous, GOLDEN = key, ALTREF = previous)."""
    key = {k: x for k, x in kw.items() if k in ("log2_tile_cols", "lossless", "q_idx", "ss_h", "ss_v")}
    fr = [v9.SynthFrame(v9.synth_params(w, h, bpp, seed=seed, **key))]
    for i in range(1, n):
        fr.append(v9.SynthFrame(v9.synth_params(w, h, bpp, seed=seed + i, inter=1, **kw)))
    return fr


def encode_stream(v9, frames, per_frame=None):
    """Encode a keyframe + inter stream: frame i > 0 refreshes slot i % 8 and references
    LAST = slot of frame i - 1, GOLDEN = slot 0, ALTREF = slot of frame i - 1."""
    enc = v9.Stream()
    datas, coded = [], []
    for i, f in enumerate(frames):
        kw = dict(per_frame(i) if per_frame else {})
        if i:
            prev = (i - 1) % 8
            kw.setdefault("ref_slot", (prev, 0, prev))
            kw.setdefault("refresh_mask", 1 << (i % 8))
        d, c = enc.encode(f, **kw)
        datas.append(d)
        coded.append(c)
    return datas, coded


def decode_stream(v9, datas):
    dec = v9.Stream()
    return [dec.decode(d) for d in datas]


STREAMS = [
    ("single_ref", dict(w=352, h=288, n=6), None),
    ("compound", dict(w=352, h=288, n=5, compound=1), None),
    ("bilinear", dict(w=200, h=130, n=4, bilinear=1), None),
    ("low_precision", dict(w=352, h=288, n=4), lambda i: {"allow_hp": 0}),
    ("tiles", dict(w=1024, h=136, n=3, log2_tile_cols=2), None),
    ("ten_bit", dict(w=176, h=144, n=4, bpp=10, compound=1), None),
    ("twelve_bit", dict(w=136, h=72, n=3, bpp=12), None),
    # profiles 1 / 3: subsampling coded in the colour config
    ("yuv422", dict(w=200, h=130, n=4, compound=1, ss_h=1, ss_v=0), None),
    ("yuv440", dict(w=200, h=130, n=4, ss_h=0, ss_v=1), lambda i: {"refresh_ctx": 1, "parallel": 0}),
    ("yuv444_10bit", dict(w=176, h=144, n=4, bpp=10, compound=1, ss_h=0, ss_v=0), None),
    ("yuv444_12bit", dict(w=136, h=72, n=3, bpp=12, ss_h=0, ss_v=0), None),
    ("prob_updates", dict(w=352, h=288, n=5, compound=1), lambda i: {"prob_updates": 11 + i}),
    ("backward_adaptation", dict(w=352, h=288, n=6, compound=1),
     lambda i: {"refresh_ctx": 1, "parallel": 0, "ctx_id": i % 4}),
    ("adaptation_and_updates", dict(w=264, h=200, n=6, compound=1),
     lambda i: {"refresh_ctx": 1, "parallel": i % 2, "ctx_id": (i * 3) % 4, "prob_updates": 5 + i}),
    ("error_res", dict(w=352, h=288, n=4), lambda i: {"error_res": int(i == 2)}),
    ("lossless", dict(w=200, h=136, n=3, lossless=1, q_idx=0), None),
    ("keep_modes", dict(w=352, h=288, n=5, compound=1), lambda i: {"keep_modes": 1}),
    ("keep_modes_adaptive", dict(w=200, h=200, n=5, compound=1),
     lambda i: {"keep_modes": 1, "refresh_ctx": 1, "parallel": 0, "allow_hp": i % 2}),
]


@pytest.mark.parametrize("name,shape,per_frame", STREAMS, ids=[s[0] for s in STREAMS])
def test_inter_stream_round_trip(v9, name, shape, per_frame):
    shape = dict(shape)
    frames = _frames(v9, shape.pop("w"), shape.pop("h"), shape.pop("n"), **shape)
    datas, coded = encode_stream(v9, frames, per_frame)
    stats = {"kept": 0, "to_new": 0}
    keep = bool(per_frame and per_frame(1).get("keep_modes"))
    for f, c in zip(frames, coded):
        check_legalized(f.pkt, c.pkt, stats, keep)
    for (p, info), c in zip(decode_stream(v9, datas), coded):
        assert info.show_frame == 1
        same_packet(p.pkt, c.pkt)
    assert stats["kept"] > stats["to_new"] / 4     # most predicted modes survive


def test_mv_prediction_modes_are_exercised(v9):
    """Every inter mode, the previous frame's MVs and sub-8x8 MVs appear in coded packets."""
    frames = _frames(v9, 352, 288, 5, compound=1)
    _, coded = encode_stream(v9, frames, lambda i: {"keep_modes": 1})
    modes = set()
    sub8 = 0
    for c in coded[1:]:
        for b in _blocks(c.pkt):
            if not b.intra:
                modes.update(b.mode)
                sub8 += b.bs > 9
    assert modes == {NEARESTMV, NEARMV, ZEROMV, NEWMV}
    assert sub8 > 10


def test_hidden_frames_show_existing_and_superframes(v9):
    """An ALTREF-style hidden frame packed with the next frame in a superframe, then
    shown later by show_existing_frame (vp9.c:1636-1653)."""
    frames = _frames(v9, 200, 130, 4)
    enc = v9.Stream()
    d0, c0 = enc.encode(frames[0])
    d1, c1 = enc.encode(frames[1], show_frame=0, ref_slot=(0, 0, 0), refresh_mask=1 << 2)   # hidden, slot 2
    d2, c2 = enc.encode(frames[2], ref_slot=(0, 0, 2), refresh_mask=1 << 1)
    d3, _ = enc.encode(None, show_existing_frame=1, show_slot=2)
    d4, c4 = enc.encode(frames[3], ref_slot=(1, 0, 2), refresh_mask=1 << 3)
    sf = v9.superframe_join([d1, d2])
    assert v9.superframe_split(sf) == [d1, d2]
    assert v9.superframe_split(d0) == [d0]
    assert len(d3) == 1
    dec = v9.Stream()
    out = []
    for pkt in (d0, sf, d3, d4):
        for fr in v9.superframe_split(pkt):
            out.append(dec.decode(fr))
    assert [i.show_frame for _, i in out] == [1, 0, 1, 1, 1]
    assert out[3][0] is None and out[3][1].show_existing_frame and out[3][1].show_slot == 2
    for (p, info), c in zip([out[0], out[1], out[2], out[4]], [c0, c1, c2, c4]):
        same_packet(p.pkt, c.pkt)
    assert list(out[4][1].ref_slot) == [1, 0, 2] and out[4][1].refresh_mask == 1 << 3


def test_intra_only_frame_mid_stream(v9):
    """A hidden intra-only frame resets one context (reset_ctx 2) and refreshes some slots;
    the inter frames after it reference it."""
    frames = _frames(v9, 264, 136, 4, compound=1)
    io = v9.SynthFrame(v9.synth_params(264, 136, 8, seed=77))
    io.pkt.keyframe, io.pkt.intraonly = 0, 1
    enc = v9.Stream()
    datas, coded = [], []
    for f, kw in [(frames[0], {}), (frames[1], dict(ref_slot=(0, 0, 0), refresh_mask=2, refresh_ctx=1, parallel=0)),
                  (io, dict(refresh_mask=0b1100, reset_ctx=2, ctx_id=1, refresh_ctx=1)),
                  (frames[2], dict(ref_slot=(2, 1, 3), refresh_mask=16, refresh_ctx=1, parallel=0, ctx_id=1)),
                  (frames[3], dict(ref_slot=(4, 0, 2), refresh_mask=32))]:
        d, c = enc.encode(f, **kw)
        datas.append(d)
        coded.append(c)
    res = decode_stream(v9, datas)
    assert res[2][1].show_frame == 0 and res[2][0].pkt.intraonly == 1
    for (p, _), c in zip(res, coded):
        same_packet(p.pkt, c.pkt)


def test_references_must_exist(v9):
    frames = _frames(v9, 200, 130, 2)
    with pytest.raises(v9.Vp9HipError):
        v9.Stream().encode(frames[1])                       # no keyframe: no slot written
    # a decoder that missed the keyframe refuses the inter frame
    enc2 = v9.Stream()
    d0, _ = enc2.encode(frames[0])
    d1, _ = enc2.encode(frames[1], ref_slot=(0, 0, 0))
    with pytest.raises(v9.Vp9HipError) as e:
        v9.Stream().decode(d1)
    assert e.value.code == v9.EINVALIDDATA
    with pytest.raises(v9.Vp9HipError):
        v9.Stream().decode(enc2.encode(None, show_existing_frame=1, show_slot=0)[0])


def test_corrupt_inter_streams_fail_cleanly(v9):
    """Flipped or truncated inter frames decode to some packet or fail with an AVERROR,
    never reading outside the buffer (child process)."""
    code = r"""
import importlib, random
v9 = importlib.import_module("ffmpeg-hybrid_amd")
fr = [v9.SynthFrame(v9.synth_params(200, 130, 8, seed=5))] + \
     [v9.SynthFrame(v9.synth_params(200, 130, 8, seed=6 + i, inter=1, compound=1)) for i in range(2)]
enc = v9.Stream()
ds = [enc.encode(fr[0])[0]] + [enc.encode(f, ref_slot=(0, 0, 0), refresh_mask=1, refresh_ctx=1, parallel=0)[0] for f in fr[1:]]
rng = random.Random(3)
ok = err = 0
for k in range(60):
    dec = v9.Stream()
    dec.decode(ds[0])
    b = bytearray(ds[1 + k % 2])
    if k < 20:
        b = b[: rng.randrange(1, len(b))]
    else:
        for _ in range(1 + k % 4):
            i = rng.randrange(len(b)); b[i] ^= 1 << rng.randrange(8)
    try:
        dec.decode(bytes(b)); ok += 1
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
@pytest.mark.parametrize("ssh,ssv", [(1, 1), (1, 0), (0, 0)])
def test_inter_bitstream_to_gpu_matches_oracle(v9, orc, gpu, ssh, ssv):
    """Host decode of an inter stream (compound, adaptation), then the MI355X pixel path
    with the decoded reference slots, bit-exact against the oracle's decode of the coded
    packets (4:2:0 and the profile 1 formats)."""
    w, h = 352, 288
    frames = _frames(v9, w, h, 5, compound=1, ss_h=ssh, ss_v=ssv)
    datas, coded = encode_stream(v9, frames, lambda i: {"refresh_ctx": 1, "parallel": 0})
    dec = v9.Stream()
    gpu.configure(w, h, 8, nbufs=8, ss_h=ssh, ss_v=ssv)
    slots = [None] * 8          # reference slot -> device buffer (frame index)
    oracle = []
    for i, d in enumerate(datas):
        p, info = dec.decode(d)
        refs = [slots[s] if slots[s] is not None else 0 for s in info.ref_slot]
        gpu.submit(p, i, refs)
        ref_planes = None if i == 0 else [oracle[r] for r in refs]
        out = v9.alloc_planes(w, h, 8, ssh, ssv)
        orc.decode_frame(coded[i].pkt, out, ref_planes)
        oracle.append(out)
        for s in range(8):
            if info.refresh_mask & (1 << s):
                slots[s] = i
    gpu.sync()
    for i in range(len(datas)):
        got = gpu.download(i)
        for a, b in zip(v9.visible(got, w, h, ssh, ssv), v9.visible(oracle[i], w, h, ssh, ssv)):
            assert np.array_equal(a, b), "frame %d" % i


TILE_STREAMS = [
    ("keyframes_8_cols", dict(w=2048, h=200, n=2, log2_tile_cols=3), None, 0),
    ("inter_4_cols", dict(w=1024, h=136, n=4, log2_tile_cols=2, compound=1), None, 0),
    ("adaptation_4_cols", dict(w=1024, h=200, n=4, log2_tile_cols=2, compound=1),
     lambda i: {"refresh_ctx": 1, "parallel": 0, "ctx_id": i % 4, "prob_updates": 3 + i}, 0),
    ("tile_rows", dict(w=1024, h=520, n=3, log2_tile_cols=2), lambda i: {"refresh_ctx": 1, "parallel": 0}, 1),
]


@pytest.mark.parametrize("name,shape,per_frame,log2_rows", TILE_STREAMS, ids=[s[0] for s in TILE_STREAMS])
@pytest.mark.parametrize("threads", [2, 3, 8])
def test_tile_threaded_parse_equals_serial(v9, name, shape, per_frame, log2_rows, threads):
    """vp9h_stream_set_threads (decode_tiles_mt, vp9.c:1441-1520): the tile columns parsed on
    `threads` threads give the serial walk's packet, field by field, including the symbol
    counts that backward adaptation sums over the columns (the next frame parses with the
    adapted probabilities) and tile rows (each column walks every tile row)."""
    shape = dict(shape)
    frames = _frames(v9, shape.pop("w"), shape.pop("h"), shape.pop("n"), **shape)
    for f in frames:
        f.pkt.log2_tile_rows = log2_rows
    datas, coded = encode_stream(v9, frames, per_frame)
    serial = v9.Stream()
    par = v9.Stream(threads=threads)
    for d, c in zip(datas, coded):
        (p0, i0), (p1, i1) = serial.decode(d), par.decode(d)
        same_packet(p0.pkt, c.pkt)
        same_packet(p1.pkt, p0.pkt)
        assert p1.pkt.log2_tile_rows == c.pkt.log2_tile_rows and (c.pkt.log2_tile_rows > 0) == (log2_rows > 0)


def test_tile_threaded_parse_rejects_truncated_tiles(v9):
    """A truncated tile fails the threaded parse with AVERROR_INVALIDDATA, as the serial one."""
    frames = _frames(v9, 1024, 136, 1, log2_tile_cols=2)
    datas, _ = encode_stream(v9, frames)
    d = datas[0][: len(datas[0]) * 3 // 4]
    for threads in (1, 4):
        with pytest.raises(v9.Vp9HipError) as e:
            v9.Stream(threads=threads).decode(d)
        assert e.value.code == v9.EINVALIDDATA


def test_header_peek_matches_the_parse(v9):
    """vp9h_frame_peek (no stream state) reads the same slot bookkeeping as the full parse:
    show_existing_frame / slot, show_frame, error_res, refresh mask, LAST / GOLDEN / ALTREF
    slots and sign bias; keyframes, inter, hidden, intra-only and show-existing headers."""
    import ctypes
    from test_ivf_decoder import _stream
    L = v9.lib()
    L.vp9h_frame_peek.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(v9.FrameInfo)]
    streams = [_stream(v9),
               encode_stream(v9, _frames(v9, 200, 130, 4), lambda i: {"error_res": int(i == 2)})[0]]
    enc = v9.Stream()
    key = enc.encode(_frames(v9, 176, 144, 1)[0])[0]
    intra = v9.SynthFrame(v9.synth_params(176, 144, 8, seed=77))
    intra.pkt.keyframe, intra.pkt.intraonly = 0, 1
    streams.append([key, enc.encode(intra, show_frame=0, refresh_mask=0x24)[0]])
    types = set()
    for pkts in streams:
        st = v9.Stream()
        for data in pkts:
            for fr in v9.superframe_split(data):
                peek = v9.FrameInfo()
                t = L.vp9h_frame_peek(fr, len(fr), ctypes.byref(peek))
                assert t >= 0
                types.add(t)
                _, info = st.decode(fr)
                assert (t == 2) == bool(info.show_existing_frame)
                for k in ("show_existing_frame", "show_frame", "refresh_mask", "error_res"):
                    assert getattr(peek, k) == getattr(info, k), k
                if info.show_existing_frame:
                    assert peek.show_slot == info.show_slot
                elif t == 1:
                    assert list(peek.ref_slot) == list(info.ref_slot)
                    assert list(peek.sign_bias) == list(info.sign_bias)
    assert types == {0, 1, 2, 3}
