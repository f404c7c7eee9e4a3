"""GPU parity: the HIP pixel path (through the C-ABI) vs the CPU oracle, bit-exact.

Each case decodes a synthetic pass-1 packet on the MI355X and with the oracle
(scalar restatement of libavcodec/vp9recon.c, vp9lpf.c, vp9_mc_template.c,
vp9dsp_template.c) and requires identical visible planes. Inter frames use the
oracle's keyframe output as reference (uploaded), so MC parity is tested
independently of intra parity.
"""
import numpy as np
import pytest

try:     # torch first: the zero-copy test shares its HIP runtime with libvp9hip.so (see _torch_first)
    import torch  # noqa: F401
except ImportError:
    pass

pytestmark = pytest.mark.gpu

# (w, h, bpp, extra synth params) — odd sizes exercise the frame-edge rules
# (vp9recon.c:103,192 n_px_have; vp9block.c:1442-1451 col_end/row_end).
CASES = [
    (352, 288, 8, {}),
    (200, 130, 8, {}),
    (66, 66, 8, {}),
    (8, 8, 8, {}),
    (130, 74, 8, {"p_zero_eob": 0.3, "p_skip": 0.5}),
    (512, 256, 8, {"log2_tile_cols": 1}),
    (1024, 128, 8, {"log2_tile_cols": 2}),
    (352, 288, 8, {"coef_stress": 1}),
    (200, 136, 8, {"lossless": 1, "q_idx": 0}),
    (352, 288, 8, {"sharpness": 3, "filter_level": 63}),
    (352, 288, 8, {"sharpness": 7, "filter_level": 20}),
    (352, 288, 8, {"filter_level": 0}),
    (352, 288, 10, {}),
    (200, 130, 10, {"coef_stress": 1}),
    (176, 144, 12, {}),
    (176, 144, 10, {"lossless": 1, "q_idx": 0}),
]


def _cmp(v9, got, ref, w, h, what):
    for p, (a, b) in enumerate(zip(v9.visible(got, w, h), v9.visible(ref, w, h))):
        if not np.array_equal(a, b):
            ys, xs = np.nonzero(a != b)
            raise AssertionError("%s plane %d: %d px differ, first at (x=%d, y=%d): gpu %d oracle %d"
                                 % (what, p, len(ys), xs[0], ys[0], a[ys[0], xs[0]], b[ys[0], xs[0]]))


@pytest.mark.parametrize("w,h,bpp,kw", CASES)
def test_keyframe_parity(v9, orc, gpu, w, h, bpp, kw):
    for seed in (1, 2):
        f = v9.SynthFrame(v9.synth_params(w, h, bpp, seed=seed, **kw))
        gpu.configure(w, h, bpp, nbufs=1)
        gpu.submit(f, 0)
        gpu.sync()
        got = gpu.download(0)
        ref = v9.alloc_planes(w, h, bpp)
        orc.decode_frame(f.pkt, ref)
        _cmp(v9, got, ref, w, h, "keyframe %dx%d@%d %s seed %d" % (w, h, bpp, kw, seed))


INTER = [
    (352, 288, 8, {}),
    (200, 130, 8, {"compound": 1}),
    (352, 288, 8, {"bilinear": 1}),
    (66, 66, 8, {"compound": 1, "p_zero_eob": 0.4}),
    (352, 288, 10, {"compound": 1}),
    (200, 130, 12, {"compound": 1}),
    (512, 256, 8, {"log2_tile_cols": 1, "coef_stress": 1}),
]


@pytest.mark.parametrize("w,h,bpp,kw", INTER)
def test_inter_parity(v9, orc, gpu, w, h, bpp, kw):
    """Inter frames through k_mcq (4-column tasks, packed dot products) and the in-place
    residuals, every MC variant of the INTER cases."""
    key_kw = {k: x for k, x in kw.items() if k in ("log2_tile_cols",)}
    key = v9.SynthFrame(v9.synth_params(w, h, bpp, seed=11, **key_kw))
    ref0 = v9.alloc_planes(w, h, bpp)
    orc.decode_frame(key.pkt, ref0)
    ref2 = v9.alloc_planes(w, h, bpp)   # a second, different reference for ALTREF
    key2 = v9.SynthFrame(v9.synth_params(w, h, bpp, seed=12, **key_kw))
    orc.decode_frame(key2.pkt, ref2)
    for seed in (3, 4):
        f = v9.SynthFrame(v9.synth_params(w, h, bpp, seed=seed, inter=1, **kw))
        gpu.configure(w, h, bpp, nbufs=3)
        gpu.upload(0, ref0)
        gpu.upload(1, ref2)
        gpu.submit(f, 2, (0, 0, 1))
        gpu.sync()
        got = gpu.download(2)
        out = v9.alloc_planes(w, h, bpp)
        orc.decode_frame(f.pkt, out, [ref0, ref0, ref2])
        _cmp(v9, got, out, w, h, "inter %dx%d@%d %s seed %d" % (w, h, bpp, kw, seed))


def test_batch_interleaved_keyframes(v9, orc, gpu):
    """Independent keyframes decoded in one batch (frames interleaved per wavefront launch)."""
    w, h, n = 512, 200, 5
    frames = [v9.SynthFrame(v9.synth_params(w, h, 8, seed=100 + i, log2_tile_cols=i % 2)) for i in range(n)]
    gpu.configure(w, h, 8, nbufs=n)
    gpu.stage_batch(frames, list(range(n)))
    for _ in range(2):          # re-running the staged batch is idempotent
        gpu.run_batch()
        gpu.sync()
    for i, f in enumerate(frames):
        ref = v9.alloc_planes(w, h, 8)
        orc.decode_frame(f.pkt, ref)
        _cmp(v9, gpu.download(i), ref, w, h, "batch frame %d" % i)


def test_wide_batch_separate_residual_launches(v9, orc, gpu):
    """A batch wide enough (>= 8 frames per phase) that residuals run as their own k_resid
    launches before the fused intra + LF wavefront (narrow phases fuse them too)."""
    w, h, n = 200, 136, 27
    frames = [v9.SynthFrame(v9.synth_params(w, h, 8, seed=300 + i)) for i in range(n)]
    gpu.configure(w, h, 8, nbufs=n)
    gpu.stage_batch(frames, list(range(n)))
    gpu.run_batch()
    gpu.sync()
    for i in (0, 7, 13, 26):
        ref = v9.alloc_planes(w, h, 8)
        orc.decode_frame(frames[i].pkt, ref)
        _cmp(v9, gpu.download(i), ref, w, h, "wide batch frame %d" % i)


@pytest.mark.parametrize("static", [1, 0])
def test_static_plan_keyframe_batch(v9, orc, monkeypatch, static):
    """Keyframe batches of wide phases run a launch list fixed at staging (runtime "static
    plan": no host wait between the device planner and the pixel launches; residual job
    ranges read from the planner's summary in HBM). Same pixels as the summary-read path
    (VP9HIP_STATIC=0), over 3 runs of the staged batch, mixed tile columns, lossless and
    lossy frames in one phase, and 10-bit."""
    monkeypatch.setenv("VP9HIP_STATIC", str(static))      # read when the context opens
    gpu = v9.Device(0)
    for bpp in (8, 10):
        w, h, n = 520, 136, 18
        frames = [v9.SynthFrame(v9.synth_params(w, h, bpp, seed=500 + i, log2_tile_cols=i % 2,
                                                **({"lossless": 1, "q_idx": 0} if i % 5 == 3 else {})))
                  for i in range(n)]
        gpu.configure(w, h, bpp, nbufs=n)
        gpu.stage_batch(frames, list(range(n)))
        for _ in range(3):
            gpu.run_batch()
        gpu.sync()
        assert sum(gpu.alg_bytes().values()) > 0
        for i in range(n):
            ref = v9.alloc_planes(w, h, bpp)
            orc.decode_frame(frames[i].pkt, ref)
            _cmp(v9, gpu.download(i), ref, w, h, "static=%d %d-bit batch frame %d" % (static, bpp, i))
    gpu.close()


@pytest.mark.parametrize("slot_streams", [1, 0])
def test_two_slots_cross_batch_dependency(v9, orc, monkeypatch, slot_streams):
    """The two batch slots run on streams of their own (VP9HIP_SLOT_STREAMS=1): a batch that
    references the other slot's frames waits for that slot's run on the device (dep_other),
    one that shares no buffer with it runs concurrently. Slot 1's P frames continue slot 0's
    GOP, run back to back without a host wait; then slot 0 again, overwriting buffers slot 1
    read (write-after-read across slots)."""
    monkeypatch.setenv("VP9HIP_SLOT_STREAMS", str(slot_streams))
    w, h = 352, 288
    key = v9.SynthFrame(v9.synth_params(w, h, 8, seed=900))
    ps = [v9.SynthFrame(v9.synth_params(w, h, 8, seed=901 + i, inter=1, compound=i % 2)) for i in range(5)]
    key2 = v9.SynthFrame(v9.synth_params(w, h, 8, seed=910))
    dev = v9.Device(0)
    try:
        dev.configure(w, h, 8, nbufs=8)
        dev.set_slot(0)
        dev.stage_batch([key, ps[0], ps[1]], [0, 1, 2], [None, (0, 0, 0), (1, 1, 0)])
        dev.set_slot(1)
        dev.stage_batch([ps[2], ps[3], key2], [3, 4, 5], [(2, 2, 0), (3, 3, 0), None])
        dev.set_slot(0)
        dev.run_batch()
        dev.set_slot(1)
        dev.run_batch()
        dev.sync()
        ref = {}
        seq = [(key, 0, None), (ps[0], 1, (0, 0, 0)), (ps[1], 2, (1, 1, 0)), (ps[2], 3, (2, 2, 0)),
               (ps[3], 4, (3, 3, 0)), (key2, 5, None)]
        for f, b, r in seq:
            out = v9.alloc_planes(w, h, 8)
            orc.decode_frame(f.pkt, out, None if r is None else [ref[r[0]], ref[r[1]], ref[r[2]]])
            ref[b] = out
            _cmp(v9, dev.download(b), out, w, h, "slot streams %d buffer %d" % (slot_streams, b))
        # slot 0 again, into buffers 3 / 4 that slot 1 read and wrote, from buffer 5 (slot 1's)
        dev.set_slot(0)
        dev.stage_batch([ps[4], key], [3, 4], [(5, 5, 5), None])
        dev.set_slot(1)
        dev.run_batch()          # slot 1's batch again (reads 2, 3; writes 3, 4, 5) ...
        dev.set_slot(0)
        dev.run_batch()          # ... then slot 0's, which must wait for it
        dev.sync()
        out = v9.alloc_planes(w, h, 8)
        orc.decode_frame(ps[4].pkt, out, [ref[5], ref[5], ref[5]])
        _cmp(v9, dev.download(3), out, w, h, "slot streams %d rewrite" % slot_streams)
        _cmp(v9, dev.download(4), ref[0], w, h, "slot streams %d key rewrite" % slot_streams)
    finally:
        dev.close()


@pytest.mark.parametrize("slot_streams", [1, 0])
def test_four_slots_chain_across_slots(v9, orc, monkeypatch, slot_streams):
    """VP9HIP_MAX_SLOTS batch slots: one GOP continued from slot to slot (each slot's batch
    reads the previous slot's last frame: dep_mask), plus an independent keyframe batch in
    every slot; all four run back to back without a host wait, then slot 3 wraps around
    onto slot 0's buffers (write-after-read across slots)."""
    monkeypatch.setenv("VP9HIP_SLOT_STREAMS", str(slot_streams))
    assert v9.Device.MAX_SLOTS == 4
    w, h = 352, 288
    key = v9.SynthFrame(v9.synth_params(w, h, 8, seed=930))
    ps = [v9.SynthFrame(v9.synth_params(w, h, 8, seed=931 + i, inter=1, compound=i % 2)) for i in range(8)]
    keys = [v9.SynthFrame(v9.synth_params(w, h, 8, seed=950 + i)) for i in range(4)]
    dev = v9.Device(0)
    try:
        dev.configure(w, h, 8, nbufs=12)
        # slot k: P frames into buffers 3k, 3k + 1 (chained from buffer 3k - 2), keyframe into 3k + 2
        seq = []
        for k in range(4):
            dev.set_slot(k)
            prev = 3 * k - 2 if k else None
            fr = ([key] if k == 0 else [ps[2 * k - 1]]) + [ps[2 * k], keys[k]]
            refs = [None if k == 0 else (prev, prev, prev), (3 * k, 3 * k, 3 * k), None]
            dev.stage_batch(fr, [3 * k, 3 * k + 1, 3 * k + 2], refs)
            seq += list(zip(fr, [3 * k, 3 * k + 1, 3 * k + 2], refs))
        for k in range(4):
            dev.set_slot(k)
            dev.run_batch()
        dev.sync()
        ref = {}
        for f, b, r in seq:
            out = v9.alloc_planes(w, h, 8)
            orc.decode_frame(f.pkt, out, None if r is None else [ref[r[0]], ref[r[1]], ref[r[2]]])
            ref[b] = out
            _cmp(v9, dev.download(b), out, w, h, "4 slots, slot streams %d, buffer %d" % (slot_streams, b))
        # slot 3 again (reads 7, writes 9..11), then slot 0 re-staged into buffers 0..2 from 11
        dev.set_slot(0)
        dev.stage_batch([ps[7], keys[0]], [0, 1], [(11, 11, 11), None])
        dev.set_slot(3)
        dev.run_batch()
        dev.set_slot(0)
        dev.run_batch()
        dev.sync()
        out = v9.alloc_planes(w, h, 8)
        orc.decode_frame(ps[7].pkt, out, [ref[11], ref[11], ref[11]])
        _cmp(v9, dev.download(0), out, w, h, "4 slots, slot streams %d, wrap-around" % slot_streams)
        _cmp(v9, dev.download(1), ref[2], w, h, "4 slots, slot streams %d, key rewrite" % slot_streams)
        with pytest.raises(v9.Vp9HipError):
            dev.set_slot(4)
    finally:
        dev.close()


def test_static_plan_rejects_inconsistent_packets(v9, orc, gpu):
    """A packet the device planner rejects (an intra mode > 9) in a static-plan batch: the
    planner neutralises the batch on the device (k_pguard) and the next wait reports
    AVERROR_INVALIDDATA; the context then decodes a clean batch bit-exact."""
    w, h, n = 352, 288, 16
    frames = [v9.SynthFrame(v9.synth_params(w, h, 8, seed=700 + i)) for i in range(n)]
    gpu.configure(w, h, 8, nbufs=n)
    b = frames[5].pkt.blocks[3]
    saved = b.mode[0]
    b.mode[0] = 20
    gpu.stage_batch(frames, list(range(n)))
    gpu.run_batch()
    with pytest.raises(v9.Vp9HipError) as e:
        gpu.sync()
    assert e.value.code == v9.EINVALIDDATA
    b.mode[0] = saved
    gpu.stage_batch(frames, list(range(n)))
    gpu.run_batch()
    gpu.sync()
    for i in (0, 5, 15):
        ref = v9.alloc_planes(w, h, 8)
        orc.decode_frame(frames[i].pkt, ref)
        _cmp(v9, gpu.download(i), ref, w, h, "clean batch frame %d" % i)


def test_decoder_api_sequence(v9, orc):
    """send_packet / receive_frame over a key + 3 inter frames."""
    w, h = 160, 96
    dec = v9.PacketDecoder(0, nbufs=3)
    pkts = [v9.SynthFrame(v9.synth_params(w, h, 8, seed=40))] + \
           [v9.SynthFrame(v9.synth_params(w, h, 8, seed=41 + i, inter=1)) for i in range(3)]
    prev = None
    for f in pkts:
        dec.send_packet(f)
        got = dec.receive_frame()
        ref = v9.alloc_planes(w, h, 8)
        orc.decode_frame(f.pkt, ref, None if prev is None else [prev, prev, prev])
        for a, b in zip(got, v9.visible(ref, w, h)):
            assert np.array_equal(a, b)
        prev = ref
    dec.dev.close()


def test_batch_gop_chains(v9, orc, gpu):
    """Two independent GOPs (key + 3 P frames, compound/bilinear refs to earlier frames)
    staged as ONE batch: chained frames run in order, the two chains concurrently."""
    w, h = 256, 136
    frames, outs, refs = [], [], []
    for c in range(2):
        base = 4 * c
        frames.append(v9.SynthFrame(v9.synth_params(w, h, 8, seed=500 + 10 * c)))
        outs.append(base)
        refs.append(None)
        for k in range(1, 4):
            kw = {"compound": 1} if k == 2 else {"bilinear": 1} if k == 3 else {}
            frames.append(v9.SynthFrame(v9.synth_params(w, h, 8, seed=501 + 10 * c + k, inter=1, **kw)))
            outs.append(base + k)
            refs.append((base + k - 1, base + k - 1, base))   # LAST = previous, ALTREF = keyframe
    order = [0, 4, 1, 5, 2, 6, 3, 7]                           # interleave the two chains
    gpu.configure(w, h, 8, nbufs=8)
    gpu.stage_batch([frames[i] for i in order], [outs[i] for i in order], [refs[i] for i in order])
    gpu.run_batch()
    gpu.sync()
    dec = {}
    for i in range(8):
        out = v9.alloc_planes(w, h, 8)
        r = refs[i]
        orc.decode_frame(frames[i].pkt, out, None if r is None else [dec[r[0]], dec[r[1]], dec[r[2]]])
        dec[outs[i]] = out
        _cmp(v9, gpu.download(outs[i]), out, w, h, "gop frame %d" % i)


SCALED = [
    # (reference size, frame size, bpp, extra params): down- and up-scaled references
    ((352, 288), (240, 200), 8, {}),
    ((176, 144), (352, 288), 8, {"compound": 1}),
    ((200, 130), (320, 208), 8, {"bilinear": 1}),
    ((256, 256), (200, 136), 10, {"compound": 1}),
]


@pytest.mark.parametrize("rs,fs,bpp,kw", SCALED)
def test_scaled_reference_parity(v9, orc, gpu, rs, fs, bpp, kw):
    """Reference scaling (vp9recon.c:492-628, vp9.c:845-880): a keyframe at one size,
    an inter frame at another size predicting from it (k_mcq's per-pixel scaled tasks)."""
    (rw, rh), (w, h) = rs, fs
    key = v9.SynthFrame(v9.synth_params(rw, rh, bpp, seed=900))
    gpu.configure(max(rw, w), max(rh, h), bpp, nbufs=2)
    gpu.stage_batch([key], [0])
    gpu.run_batch()
    kref = v9.alloc_planes(rw, rh, bpp)
    orc.decode_frame(key.pkt, kref)
    _cmp(v9, gpu.download(0), kref, rw, rh, "scaled-test keyframe")
    for seed in (901, 902):
        f = v9.SynthFrame(v9.synth_params(w, h, bpp, seed=seed, inter=1, **kw))
        for r in range(3):
            f.pkt.ref_w[r], f.pkt.ref_h[r] = rw, rh
        gpu.stage_batch([f], [1], [(0, 0, 0)])
        gpu.run_batch()
        gpu.sync()
        out = v9.alloc_planes(w, h, bpp)
        orc.decode_frame(f.pkt, out, [kref, kref, kref], [(rw, rh)] * 3)
        _cmp(v9, gpu.download(1), out, w, h, "scaled ref %dx%d -> %dx%d@%d %s seed %d" % (rw, rh, w, h, bpp, kw, seed))


@pytest.mark.parametrize("bpp", [8, 10])
def test_zero_copy_export_matches_download(v9, orc, gpu, bpp):
    """vp9hip_frame_device: torch views of the device planes hold the
    oracle's frame, at the buffer's own addresses (no copy)."""
    import torch
    w, h = 200, 130
    f = v9.SynthFrame(v9.synth_params(w, h, bpp, seed=77))
    gpu.configure(w, h, bpp, nbufs=2)
    gpu.submit(f, 1)
    gpu.sync()
    ptrs, ls, (vw, vh), stream = gpu.frame_device(1)
    assert (vw, vh) == (w, h) and stream
    views = gpu.frame_tensors(1, device="cuda:0")
    assert [t.data_ptr() for t in views] == ptrs
    ref = v9.alloc_planes(w, h, bpp)
    orc.decode_frame(f.pkt, ref)
    for t, r in zip(views, v9.visible(ref, w, h)):
        assert t.shape == r.shape
        assert np.array_equal(t.cpu().numpy().astype(r.dtype), r)


@pytest.mark.parametrize("mode,bpp", [("0", 8), ("2", 8), ("2", 10), ("1", 10)])
def test_loop_filter_schedules(v9, orc, monkeypatch, mode, bpp):
    """Both loop-filter schedules (vp9lpf.c:183-230 in raster SB order): VP9HIP_LFROW=0 runs
    x + 2y diagonal launches only; 2 runs the row-pipelined k_lfr for every phase (its rows
    start after the diagonals fused with the intra wavefront, workgroups hand the bottom SB
    rows to the next row through sc1 stores / loads); 1 (default) k_lfr for narrow phases.
    A wide keyframe batch and a narrow GOP, several SB rows and columns, 2 tile columns."""
    monkeypatch.setenv("VP9HIP_LFROW", mode)
    dev = v9.Device(0)
    try:
        w, h, n = 520, 300, 9
        frames = [v9.SynthFrame(v9.synth_params(w, h, bpp, seed=500 + i, log2_tile_cols=1)) for i in range(n)]
        dev.configure(w, h, bpp, nbufs=n)
        dev.stage_batch(frames, list(range(n)))
        for _ in range(2):      # graph replay: k_lfr counters reset by the launch itself
            dev.run_batch()
            dev.sync()
        for i in (0, 4, 8):
            ref = v9.alloc_planes(w, h, bpp)
            orc.decode_frame(frames[i].pkt, ref)
            _cmp(v9, dev.download(i), ref, w, h, "LFROW=%s keyframe batch frame %d" % (mode, i))
        # key + 2 inter frames, one chain (phases of one frame)
        key = v9.SynthFrame(v9.synth_params(w, h, bpp, seed=600))
        p1 = v9.SynthFrame(v9.synth_params(w, h, bpp, seed=601, inter=1))
        dev.configure(w, h, bpp, nbufs=2)
        dev.submit(key, 0)
        dev.submit(p1, 1, (0, 0, 0))
        dev.sync()
        r0 = v9.alloc_planes(w, h, bpp)
        orc.decode_frame(key.pkt, r0)
        r1 = v9.alloc_planes(w, h, bpp)
        orc.decode_frame(p1.pkt, r1, [r0, r0, r0])
        _cmp(v9, dev.download(0), r0, w, h, "LFROW=%s key" % mode)
        _cmp(v9, dev.download(1), r1, w, h, "LFROW=%s inter" % mode)
    finally:
        dev.close()


@pytest.mark.parametrize("levels,bpp,log2,df,fuse,nolf", [("1", 8, 0, "1", "0", 0), ("1", 8, 0, "0", "0", 0),
                                                           ("0", 8, 0, "1", "0", 0), ("1", 10, 1, "1", "0", 0),
                                                           ("1", 10, 1, "0", "0", 0), ("1", 8, 0, "1", "1", 0),
                                                           ("1", 10, 1, "1", "1", 0), ("1", 8, 0, "1", "1", 1)])
def test_inter_level_schedule(v9, orc, monkeypatch, levels, bpp, log2, df, fuse, nolf):
    """Inter frames' intra SBs scheduled by dependency level (VP9HIP_LEVELS=1, default):
    an SB runs once the intra SBs whose pixels its intra blocks read (left, top, top-left;
    vp9recon.c:71-121) have run; inter pixels (MC + residuals) are final before the first
    intra launch, and the loop filter is one k_lfr launch after them. A key + 4 P chain at a
    size with 15 x 9 SBs (many intra blocks next to other SBs' intra blocks) and 2 chains.
    VP9HIP_PRED_DF=1 (default): a phase's levels in one k_predd launch (per-SB done flags),
    0: one k_pred launch per level; VP9HIP_PRED_LF_FUSE=1: the k_predd work as intra worker
    workgroups inside the phase's k_lfro launch, whose loader waits per SB for their flags.
    Three runs: the graph replays reuse the counters and flags. nolf: chain 0's third frame
    is not loop-filtered (its phase takes the k_predd launch, the others the fused one)."""
    monkeypatch.setenv("VP9HIP_LEVELS", levels)
    monkeypatch.setenv("VP9HIP_PRED_DF", df)
    monkeypatch.setenv("VP9HIP_PRED_LF_FUSE", fuse)
    dev = v9.Device(0)
    try:
        w, h = 960, 544
        frames, outs, refs = [], [], []
        for c in range(2):
            base = 5 * c
            frames.append(v9.SynthFrame(v9.synth_params(w, h, bpp, seed=700 + 10 * c, log2_tile_cols=log2)))
            outs.append(base)
            refs.append(None)
            for k in range(1, 5):
                kw = {"compound": 1} if k == 3 else {}
                if nolf and c == 0 and k == 2:
                    kw["filter_level"] = 0
                frames.append(v9.SynthFrame(v9.synth_params(w, h, bpp, seed=701 + 10 * c + k, inter=1,
                                                            log2_tile_cols=log2, **kw)))
                outs.append(base + k)
                refs.append((base + k - 1, base + k - 1, base))
        order = [0, 5, 1, 6, 2, 7, 3, 8, 4, 9]
        dev.configure(w, h, bpp, nbufs=10)
        dev.stage_batch([frames[i] for i in order], [outs[i] for i in order], [refs[i] for i in order])
        for _ in range(3):
            dev.run_batch()
            dev.sync()
        dec = {}
        for i in range(10):
            out = v9.alloc_planes(w, h, bpp)
            r = refs[i]
            orc.decode_frame(frames[i].pkt, out, None if r is None else [dec[r[0]], dec[r[1]], dec[r[2]]])
            dec[outs[i]] = out
            _cmp(v9, dev.download(outs[i]), out, w, h, "LEVELS=%s chain frame %d" % (levels, i))
    finally:
        dev.close()
