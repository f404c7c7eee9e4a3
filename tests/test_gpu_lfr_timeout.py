"""The row-pipelined loop filter's bounded hand-off waits never pass silently.

k_lfr bounds each wait for the SB row above (ctr[3] polls, 2^22 by default) and counts the
waits it gave up in its counter block (ctr[2]); such a frame was filtered with a stale top
halo. vp9hip_test_hooks(0, n) sets the bound for contexts opened afterwards, here to 1 poll, so the waits
of the first SBs of each row give up. The batch API must then fail vp9hip_sync with
VP9HIP_EBUG, and the decoder must fail the frames of that batch instead of handing them
out (the advisor's silent-corruption path: staging the next batch used to zero the words).
With the default bound the same stream decodes bit-exact.
"""
import pytest

from test_ivf_decoder import _oracle_outputs, _same
from test_stream import _frames

pytestmark = pytest.mark.gpu


def _gop(v9, n=4):
    """key + P chain at 1080p width (17 SB rows: k_lfr hand-offs on every row)."""
    fr = _frames(v9, 1920, 1080, n, seed=4242)
    enc = v9.Stream()
    return [enc.encode(fr[0])[0]] + [enc.encode(f, ref_slot=(0, 0, 0), refresh_mask=1)[0] for f in fr[1:]]


@pytest.fixture
def tiny_spin(v9):
    v9.test_hooks(lfr_spin=1)
    yield
    v9.test_hooks()


def test_decoder_fails_frames_of_a_timed_out_batch(v9, tiny_spin):
    pkts = _gop(v9)
    dec = v9.Decoder(0, max_batch=4, parse_threads=2)
    with pytest.raises(v9.Vp9HipError) as e:
        for _ in dec.decode(pkts, download=False):
            pass
    assert e.value.code == v9.EBUG
    dec.close()


def test_batch_sync_reports_timeout(v9, tiny_spin):
    fr = _frames(v9, 1920, 1080, 3, seed=4243)
    dev = v9.Device(0)
    try:
        dev.configure(1920, 1080, 8, nbufs=3)
        dev.stage_batch(fr, [0, 1, 2], [None, (0, 0, 0), (1, 1, 0)])
        dev.run_batch()
        with pytest.raises(v9.Vp9HipError) as e:
            dev.sync()
        assert e.value.code == v9.EBUG
    finally:
        dev.close()


def test_default_bound_decodes_bit_exact(v9, orc):
    pkts = _gop(v9)
    dec = v9.Decoder(0, max_batch=4, parse_threads=2)
    got = [pl for pl, _ in dec.decode(pkts)]
    dec.close()
    _same(got, _oracle_outputs(v9, orc, pkts), "default spin bound")


def test_hwaccel_fails_frames_of_a_timed_out_batch(v9, tmp_path):
    """The FFHWAccel path checks the same hand-off words before a frame is read
    (vp9hip_hwframe_sync / transfer). The consumer reads each frame at once (lag 0), so every
    read launches the batch holding just that frame: the keyframe's batch times out and the
    keyframe fails with VP9HIP_EBUG; the P frames, predicted from it, fail with
    AVERROR_INVALIDDATA without running. The harness reads them all and reports them."""
    from test_hwaccel_harness import failed_frames, run_harness
    ivf = tmp_path / "t.ivf"
    ivf.write_bytes(v9.ivf_write(_gop(v9), 1920, 1080))
    want = {0: v9.EBUG, 1: v9.EINVALIDDATA, 2: v9.EINVALIDDATA, 3: v9.EINVALIDDATA}
    for mode in ("download", "device"):
        rc, n, _, err = run_harness(ivf, "-", 8, 1, 1, 1, 0, mode, 4, hooks=(0, 1))
        assert rc == 3 and n == 4 and failed_frames(err) == want, (mode, err)
        # read 4 behind: one batch of 4 launches whole, and all of its frames time out
        rc, n, _, err = run_harness(ivf, "-", 8, 1, 1, 1, 4, mode, 4, hooks=(0, 1))
        assert rc == 3 and n == 4 and failed_frames(err) == {i: v9.EBUG for i in range(4)}, (mode, err)
