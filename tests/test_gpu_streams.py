"""Bitstreams through the whole decoder (host parse -> device pixel path) against the oracle's
decode loop, on the shapes and header features the reference's conformance suite drives:

- every frame size pair of FATE's vp90-2-02-size-WxH vectors, W, H in {8, 10, 16, 18, 32, 34,
  64, 66} (tests/fate/vpx.mak:113-116), and a subset of vp91-2-02-size-WxH, W, H in {196, 198,
  200, 202, 208, 210, 224, 226} (vpx.mak:117-121): each as a keyframe, an inter frame and a
  compound inter frame. The FATE bitstreams themselves are not in the container; these are
  synthetic streams of the same sizes (parity against the oracle, unpinned to the reference's
  MD5s);
- segmentation with per-segment alternate q and loop-filter levels (vp9.c:707-765), coded
  segment ids, temporally predicted ids (vp9block.c:101-141), a retained segmentation map,
  non-default loop-filter ref / mode deltas (vp9.c:692-702, lflvl vp9.c:767-791), a hidden
  intra-only frame and an error-resilient frame after it (which drop the retained map);
- the same at 10 bits.
"""
import pytest

from test_ivf_decoder import _decode_all, _oracle_outputs, _same

pytestmark = pytest.mark.gpu

SIZES = (8, 10, 16, 18, 32, 34, 64, 66)
SIZES2 = ((196, 196), (198, 226), (200, 210), (202, 224), (208, 200), (210, 198), (224, 208), (226, 202),
          (196, 226), (226, 196))


def _three(v9, w, h, bpp=8, seed=0):
    """keyframe, inter (LAST), compound inter (LAST + ALTREF) as one encoded stream."""
    enc = v9.Stream()
    key = v9.SynthFrame(v9.synth_params(w, h, bpp, seed=seed))
    p1 = v9.SynthFrame(v9.synth_params(w, h, bpp, seed=seed + 1, inter=1))
    p2 = v9.SynthFrame(v9.synth_params(w, h, bpp, seed=seed + 2, inter=1, compound=1))
    return [enc.encode(key)[0], enc.encode(p1, ref_slot=(0, 0, 0), refresh_mask=2)[0],
            enc.encode(p2, ref_slot=(1, 0, 0), refresh_mask=4)[0]]


@pytest.mark.parametrize("w", SIZES)
def test_fate_size_pairs(v9, orc, w):
    """vpx.mak:113-116: W x H for every H of the set, keyframe + inter + compound."""
    for h in SIZES:
        pkts = _three(v9, w, h, seed=1000 + 10 * w + h)
        _same(_decode_all(v9, pkts, max_batch=4), _oracle_outputs(v9, orc, pkts), "%dx%d" % (w, h))


@pytest.mark.parametrize("w,h", SIZES2)
def test_fate_size_pairs_large(v9, orc, w, h):
    """vpx.mak:117-121 (a subset of its 64 pairs)."""
    pkts = _three(v9, w, h, seed=2000 + w + h)
    _same(_decode_all(v9, pkts, max_batch=4), _oracle_outputs(v9, orc, pkts), "%dx%d" % (w, h))


SEG = dict(enabled=1, update_map=1, update_data=1, q_en=0b0110, lf_en=0b1011, q=[0, 8, -12, 0, 0, 0, 0, 0],
           lf=[3, 0, -5, 10, 0, 0, 0, 0], nseg=4, lf_delta_update=1, lf_ref=[2, 0, -2, -1], lf_mode=[1, -1])


def _seg_stream(v9, w, h, bpp, seed):
    """key (4 segments, alternate q / LF, LF deltas) -> inter with temporally predicted ids ->
    two inters keeping the map (alternate LF only; the second reads the first's kept map) ->
    hidden intra-only (features reset, the kept map dropped) -> inter on the intra-only frame
    -> error-resilient inter -> inter with LF deltas only (segmentation off)."""
    enc = v9.Stream()
    out = []

    def add(frame_kw, **enc_kw):
        io = frame_kw.pop("intraonly", 0)
        f = v9.SynthFrame(v9.synth_params(w, h, bpp, **frame_kw))
        if io:
            f.pkt.keyframe, f.pkt.intraonly = 0, 1
        out.append(enc.encode(f, **enc_kw)[0])

    temporal = dict(SEG, temporal=1)
    keep = dict(SEG, update_map=0, q_en=0)                # kept map: no alternate q (see below)
    deltas = dict(lf_delta_update=1, lf_ref=[0, -3, 2, 1], lf_mode=[-2, 3])
    add(dict(seed=seed, seg=SEG), seg=SEG)
    add(dict(seed=seed + 1, inter=1, seg=temporal), ref_slot=(0, 0, 0), refresh_mask=2, seg=temporal)
    add(dict(seed=seed + 2, inter=1, compound=1, seg=keep), ref_slot=(1, 0, 0), refresh_mask=4, seg=keep)
    add(dict(seed=seed + 3, inter=1, seg=keep), ref_slot=(2, 1, 2), refresh_mask=8, seg=keep)
    add(dict(seed=seed + 4, intraonly=1, seg=SEG), refresh_mask=16, show_frame=0, seg=SEG)
    add(dict(seed=seed + 5, inter=1, seg=temporal), ref_slot=(4, 3, 4), refresh_mask=32, seg=temporal)
    add(dict(seed=seed + 6, inter=1, seg=SEG), ref_slot=(5, 5, 5), refresh_mask=64, error_res=1, seg=SEG)
    add(dict(seed=seed + 7, inter=1, compound=1, seg=deltas), ref_slot=(6, 5, 6), refresh_mask=128, seg=deltas)
    return out


@pytest.mark.parametrize("bpp", [8, 10])
@pytest.mark.parametrize("w,h", [(352, 288), (200, 130)])
def test_segmentation_and_lf_deltas(v9, orc, bpp, w, h):
    """(The kept-map frame codes no alternate q: its blocks take the previous map's ids, and
    the synthetic coefficients are multiples of the base step only.)"""
    pkts = _seg_stream(v9, w, h, bpp, seed=3000 + bpp)
    ref = _oracle_outputs(v9, orc, pkts)
    assert len(ref) == 7                                 # the intra-only frame is hidden
    for mb in (1, 7):
        _same(_decode_all(v9, pkts, max_batch=mb), ref, "%dx%d %d-bit batch %d" % (w, h, bpp, mb))
