"""A keyframe batch the device planner rejects fails its own frames, and only those.

Keyframe batches run as static launch plans: the planner's verdict is read only when the
host next waits (finish_summary). A rejected batch is neutralised on the device (k_pguard)
and its status stays with the batch slot until the slot is restaged, so every later check of
that slot reports it, and the adapters remember the batch and fail its frames, not the next
batch's (the advisor's round-3 finding: the rejection used to be reported once and then
charged to whichever batch came next, or lost).

vp9hip_test_hooks(k, 0) makes the k-th static-plan batch a context stages carry an intra mode
the planner rejects (a test hook in stage_dev, copied by contexts opened afterwards); the
bitstreams themselves are valid.
"""
import numpy as np
import pytest

from test_ivf_decoder import _oracle_outputs

pytestmark = pytest.mark.gpu


def _keyframes(v9, w, h, n, seed=900):
    enc = v9.Stream()
    return [enc.encode(v9.SynthFrame(v9.synth_params(w, h, 8, seed=seed + i)))[0] for i in range(n)]


@pytest.fixture
def reject_second(v9):
    v9.test_hooks(reject_batch=2)
    yield
    v9.test_hooks()


def test_decoder_fails_only_the_rejected_batch(v9, orc, reject_second):
    w, h, n, mb = 352, 288, 48, 16        # batches of 16: static plans (8 frames per group)
    pkts = _keyframes(v9, w, h, n)
    ref = _oracle_outputs(v9, orc, pkts)
    dec = v9.Decoder(0, max_batch=mb, parse_threads=2)
    got = []
    try:
        for d in pkts:
            dec.send_packet(d)
        dec.send_packet(None)
        while not dec.eof:
            try:
                r = dec.receive_frame()
            except v9.Vp9HipError as e:
                got.append(e.code)
                continue
            if r is not None:
                got.append(r[0])
    finally:
        dec.close()
    assert len(got) == n
    for i, g in enumerate(got):
        if mb <= i < 2 * mb:                         # the second batch: rejected, each frame fails
            assert isinstance(g, int) and g == v9.EINVALIDDATA, "frame %d" % i
        else:
            assert not isinstance(g, int), "frame %d failed with %r" % (i, g)
            for p in range(3):
                assert np.array_equal(g[p], ref[i][p]), "frame %d plane %d" % (i, p)


def test_sync_reports_rejection_until_restaged(v9, orc, reject_second):
    """The batch API: the status is sticky for the slot (every vp9hip_sync reports it),
    the other slot's batch is unaffected, and restaging the slot clears it."""
    w, h, n = 352, 288, 16
    fr = [v9.SynthFrame(v9.synth_params(w, h, 8, seed=950 + i)) for i in range(2 * n)]
    dev = v9.Device(0)
    try:
        dev.configure(w, h, 8, nbufs=2 * n)
        dev.set_slot(0)
        dev.stage_batch(fr[:n], list(range(n)))          # static batch 1: clean
        dev.run_batch()
        dev.set_slot(1)
        dev.stage_batch(fr[n:], list(range(n, 2 * n)))   # static batch 2: rejected
        dev.run_batch()
        for _ in range(2):
            with pytest.raises(v9.Vp9HipError) as e:
                dev.sync()
            assert e.value.code == v9.EINVALIDDATA
        for i in (0, n - 1):                             # slot 0's frames are fine
            ref = v9.alloc_planes(w, h, 8)
            orc.decode_frame(fr[i].pkt, ref)
            assert all(np.array_equal(a, b) for a, b in zip(v9.visible(dev.download(i), w, h), v9.visible(ref, w, h)))
        dev.stage_batch(fr[n:], list(range(n, 2 * n)))   # static batch 3 in slot 1: clean again
        dev.run_batch()
        dev.sync()
        ref = v9.alloc_planes(w, h, 8)
        orc.decode_frame(fr[n].pkt, ref)
        assert all(np.array_equal(a, b) for a, b in zip(v9.visible(dev.download(n), w, h), v9.visible(ref, w, h)))
    finally:
        dev.close()


def test_hwaccel_fails_the_rejected_batch(v9, tmp_path):
    """The FFHWAccel path: the harness's wait on a frame of the rejected batch fails with
    AVERROR_INVALIDDATA after the first batch's 16 frames were read."""
    from test_hwaccel_harness import run_harness
    ivf = tmp_path / "k.ivf"
    ivf.write_bytes(v9.ivf_write(_keyframes(v9, 352, 288, 48), 352, 288))
    # the consumer reads 32 frames behind: batches of 16 fill up (static plans)
    rc, _, _, err = run_harness(ivf, "-", 8, 1, 1, 1, 32, "download", 16, hooks=(2, 0))
    # the harness counts the failed read too: 16 good frames + the first of the rejected batch
    assert rc == 1 and ("decode: %d after 17 frames" % v9.EINVALIDDATA) in err, err
