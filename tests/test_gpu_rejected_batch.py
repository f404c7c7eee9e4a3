"""Errors are per frame: a frame the device rejects, or whose bitstream is corrupt, fails
alone (with the frames predicted from it); the other frames of its batch decode bit-exact.

The reference fails only the corrupt frame's decode: vp9_decode_frame returns
AVERROR_INVALIDDATA for that packet (/root/reference/libavcodec/vp9.c:1827-1832,
vp9recon.c:661-668) and the frames around it decode.

vp9hip_test_hooks(k | f << 16, 0) makes frame f of the k-th batch a context stages start
with an intra block whose mode the device planner rejects (a test hook in stage_dev, copied
by contexts opened afterwards); the bitstreams themselves are valid. Two planner paths:
  - keyframe batches run static launch plans: the verdict is read when the host next waits
    (finish_summary); k_pguard neutralises the rejected frame only, the others reconstruct
    in the same run (vp9hip_batch_frame_status: 0 / AVERROR_INVALIDDATA);
  - batches with inter frames are planned before their launches: run_batch reports the
    rejection, the valid frames are AVERROR(EAGAIN) (not run), and the front ends stage them
    again without the rejected frame and its dependents (vp9hip_pipeline.h).
A corrupt packet (truncated compressed header) fails in the host parse: the decoder reports
it on the call that consumes it (no reference slot refreshed, as vp9.c), the FFHWAccel
adapter on that frame's transfer; a GOP's later frames, predicted from it, fail with it.
"""
import numpy as np
import pytest

from test_ivf_decoder import _oracle_outputs
from test_stream import _frames

pytestmark = pytest.mark.gpu


def _keyframes(v9, w, h, n, seed=900):
    enc = v9.Stream()
    return [enc.encode(v9.SynthFrame(v9.synth_params(w, h, 8, seed=seed + i)))[0] for i in range(n)]


def _gops(v9, w, h, ngop, glen, seed=960):
    """ngop GOPs of key + glen - 1 P (LAST = previous frame, GOLDEN = the key)."""
    pkts = []
    for g in range(ngop):
        fr = _frames(v9, w, h, glen, seed=seed + 37 * g)
        enc = v9.Stream()
        pkts.append(enc.encode(fr[0])[0])
        for i, f in enumerate(fr[1:]):
            pkts.append(enc.encode(f, ref_slot=(i % 8, 0, i % 8), refresh_mask=1 << ((i + 1) % 8))[0])
    return pkts


def _truncated(v9, pkts, idx):
    """pkts with frame idx cut one byte into its compressed header: its uncompressed header
    (slot bookkeeping) parses, its entropy decode fails. header_size comes from parsing the
    intact stream from idx's keyframe."""
    k = max(i for i in range(idx + 1) if v9.vp9h_type(pkts[i]) == 0)
    st = v9.Stream()
    for d in pkts[k:idx + 1]:
        _, info = st.decode(d)
    return pkts[:idx] + [pkts[idx][:info.header_size + 1]] + pkts[idx + 1:]


def _decode_all(v9, dec, pkts):
    """send / receive loop that keeps going past errors: one entry per output frame or
    per error, in order (planes, or the error code)."""
    got = []

    def drain():
        while True:
            try:
                r = dec.receive_frame()
            except v9.Vp9HipError as e:
                if e.code == v9.EOF:
                    return
                got.append(e.code)
                continue
            if r is None:
                return
            got.append(r[0])

    for d in pkts:
        while True:
            try:
                dec.send_packet(d)
                break
            except v9.Vp9HipError as e:
                if e.code == v9.EAGAIN:
                    drain()
                    continue
                got.append(e.code)            # the packet's own decode failed
                break
        drain()
    dec.send_packet(None)
    while not dec.eof:
        try:
            r = dec.receive_frame()
        except v9.Vp9HipError as e:
            got.append(e.code)
            continue
        if r is not None:
            got.append(r[0])
    return got


def _check(v9, got, ref, bad, what):
    """got / ref in output order; bad: output indices that must fail with EINVALIDDATA."""
    assert len(got) == len(ref), (what, len(got), len(ref))
    for i, (g, o) in enumerate(zip(got, ref)):
        if i in bad:
            assert isinstance(g, int) and g == v9.EINVALIDDATA, "%s: frame %d: %r" % (what, i, g)
        else:
            assert not isinstance(g, int), "%s: frame %d failed with %r" % (what, i, g)
            for p in range(3):
                assert np.array_equal(g[p], o[p]), "%s: frame %d plane %d" % (what, i, p)


@pytest.fixture
def hooks(v9):
    yield v9.test_hooks
    v9.test_hooks()


def test_decoder_keyframes_fail_only_the_rejected_frame(v9, orc, hooks):
    """Static-plan batches of 16 keyframes: frame 3 of the second batch is rejected; the
    other 15 frames of that batch and the other batches decode bit-exact."""
    w, h, n, mb = 352, 288, 48, 16
    pkts = _keyframes(v9, w, h, n)
    ref = _oracle_outputs(v9, orc, pkts)
    hooks(reject_batch=2, reject_frame=3)
    dec = v9.Decoder(0, max_batch=mb, parse_threads=2)
    try:
        got = _decode_all(v9, dec, pkts)
    finally:
        dec.close()
    _check(v9, got, ref, {mb + 3}, "keyframes")


def test_decoder_gop_fails_the_rejected_frame_and_its_dependents(v9, orc, hooks):
    """Two GOPs of key + 11 P in batches of 8: frame 5 of the first batch is rejected at
    planning; frames 0-4 are staged again and decode, frames 5-11 (its chain: the rest of
    batch 1 and the first frames of batch 2) fail, the second GOP decodes."""
    w, h = 200, 130
    pkts = _gops(v9, w, h, 2, 12)
    ref = _oracle_outputs(v9, orc, pkts)
    hooks(reject_batch=1, reject_frame=5)
    dec = v9.Decoder(0, max_batch=8, parse_threads=2)
    try:
        got = _decode_all(v9, dec, pkts)
    finally:
        dec.close()
    _check(v9, got, ref, set(range(5, 12)), "GOPs")


def test_decoder_corrupt_packet_fails_alone(v9, orc):
    """A truncated keyframe in a keyframe stream: that packet's decode fails (send_packet /
    receive_frame reports it, no frame is output for it); every other frame decodes."""
    w, h, n = 352, 288, 20
    pkts = _keyframes(v9, w, h, n, seed=930)
    ref = _oracle_outputs(v9, orc, pkts)
    bad = 7
    pkts = _truncated(v9, pkts, bad)
    dec = v9.Decoder(0, max_batch=8, parse_threads=2)
    try:
        got = _decode_all(v9, dec, pkts)
    finally:
        dec.close()
    # the error surfaces on the call that consumes the packet's parse, which can come before
    # the earlier frames of its batch are output (the decoder delay)
    assert [g for g in got if isinstance(g, int)] == [v9.EINVALIDDATA]
    _check(v9, [g for g in got if not isinstance(g, int)], ref[:bad] + ref[bad + 1:], set(), "corrupt keyframe")


def test_batch_api_static_frame_status(v9, orc, hooks):
    """The batch API: the slot's status is sticky (every vp9hip_sync reports it), the
    per-frame status names the rejected frame, the batch's other frames and the other slot's
    batch are bit-exact, and restaging the slot clears it."""
    w, h, n = 352, 288, 16
    fr = [v9.SynthFrame(v9.synth_params(w, h, 8, seed=950 + i)) for i in range(2 * n)]
    hooks(reject_batch=2, reject_frame=4)
    dev = v9.Device(0)
    try:
        dev.configure(w, h, 8, nbufs=2 * n)
        dev.set_slot(0)
        dev.stage_batch(fr[:n], list(range(n)))          # static batch 1: clean
        dev.run_batch()
        dev.set_slot(1)
        dev.stage_batch(fr[n:], list(range(n, 2 * n)))   # static batch 2: frame 4 rejected
        dev.run_batch()
        for _ in range(2):
            with pytest.raises(v9.Vp9HipError) as e:
                dev.sync()
            assert e.value.code == v9.EINVALIDDATA
        assert dev.frame_status(1) == [0] * 4 + [v9.EINVALIDDATA] + [0] * (n - 5)
        assert dev.frame_status(0) == [0] * n
        for i in range(2 * n):
            if i == n + 4:
                continue
            ref = v9.alloc_planes(w, h, 8)
            orc.decode_frame(fr[i].pkt, ref)
            assert all(np.array_equal(a, b) for a, b in zip(v9.visible(dev.download(i), w, h), v9.visible(ref, w, h))), i
        dev.stage_batch(fr[n:], list(range(n, 2 * n)))   # static batch 3 in slot 1: clean again
        dev.run_batch()
        dev.sync()
        assert dev.frame_status(1) == [0] * n
        ref = v9.alloc_planes(w, h, 8)
        orc.decode_frame(fr[n + 4].pkt, ref)
        assert all(np.array_equal(a, b) for a, b in zip(v9.visible(dev.download(n + 4), w, h), v9.visible(ref, w, h)))
    finally:
        dev.close()


def test_batch_api_planned_batch_stops(v9, hooks):
    """A batch with inter frames is rejected by run_batch, before its pixel launches: the
    rejected frame is AVERROR_INVALIDDATA, the others AVERROR(EAGAIN) (stage them again)."""
    w, h = 200, 130
    fr = _frames(v9, w, h, 6, seed=975)
    refs = [None] + [(i - 1, 0, i - 1) for i in range(1, 6)]
    hooks(reject_batch=1, reject_frame=2)
    dev = v9.Device(0)
    try:
        dev.configure(w, h, 8, nbufs=6)
        dev.stage_batch(fr, list(range(6)), refs)
        with pytest.raises(v9.Vp9HipError) as e:
            dev.run_batch()
        assert e.value.code == v9.EINVALIDDATA
        assert dev.frame_status(0) == [v9.EAGAIN] * 2 + [v9.EINVALIDDATA] + [v9.EAGAIN] * 3
    finally:
        dev.close()


def _harness_check(v9, orc, tmp_path, pkts, w, h, bad, lag, depth, hooks=None):
    from test_hwaccel_harness import _read_frames, failed_frames, run_harness
    ivf = tmp_path / "s.ivf"
    ivf.write_bytes(v9.ivf_write(pkts, w, h))
    out = tmp_path / "out.yuv"
    rc, nout, _, err = run_harness(ivf, out, 8, 1, 1, 1, lag, "download", depth, hooks=hooks)
    assert rc == 3, err
    assert failed_frames(err) == {i: v9.EINVALIDDATA for i in bad}, err
    return _read_frames(str(out), w, h, 8, 1, 1), nout


def test_hwaccel_fails_only_the_rejected_frame(v9, orc, tmp_path):
    """The FFHWAccel path: batches of 16 keyframes read 32 behind; frame 3 of the second batch
    fails its transfer with AVERROR_INVALIDDATA, every other frame is the oracle's."""
    w, h, n = 352, 288, 48
    pkts = _keyframes(v9, w, h, n)
    ref = _oracle_outputs(v9, orc, pkts)
    got, nout = _harness_check(v9, orc, tmp_path, pkts, w, h, {19}, 32, 16, hooks=(2 | 3 << 16, 0))
    assert nout == n and len(got) == n
    for i in range(n):
        if i != 19:
            for p in range(3):
                assert np.array_equal(got[i][p], ref[i][p]), "frame %d plane %d" % (i, p)


def test_hwaccel_corrupt_packet_fails_it_and_its_dependents(v9, orc, tmp_path):
    """A P frame whose compressed header is truncated, in the first of three GOPs of key + 7
    P (batches of 8): it and the rest of its GOP (predicted from it) fail their transfer;
    the frames before it and the other GOPs are the oracle's."""
    w, h = 200, 130
    pkts = _gops(v9, w, h, 3, 8, seed=990)
    ref = _oracle_outputs(v9, orc, pkts)
    bad = 3
    pkts = _truncated(v9, pkts, bad)
    got, nout = _harness_check(v9, orc, tmp_path, pkts, w, h, set(range(bad, 8)), 8, 8)
    assert nout == len(pkts)
    for i in range(len(pkts)):
        if not bad <= i < 8:
            for p in range(3):
                assert np.array_equal(got[i][p], ref[i][p]), "frame %d plane %d" % (i, p)
