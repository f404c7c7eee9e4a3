"""GPU parity for VP9 profiles 1 / 3 chroma formats: 4:2:2, 4:4:0 and
4:4:4 at 8 / 10 / 12 bit, bit-exact against the oracle.

What differs from 4:2:0 on this path, and what each case exercises:
- chroma block / tx sizes: uvtx (vp9block.c:1291), chroma intra edges with the plane's
  subsampling (check_intra_mode, vp9recon.c:37-221);
- chroma MC: the 1/16-pel phase is mv * 2 on a non-subsampled axis
  (mc_chroma_unscaled, vp9recon.c:416-467); sub-8x8 chroma MVs per axis incl. the
  libvpx block-index bugs (vp9_mc_template.c:107-114, 296-305); scaled references
  (mc_chroma_scaled, vp9recon.c:543-628);
- loop filter: chroma uses mask[ss_h | ss_v] (vp9lpf.c:189), i.e. the luma masks at
  4:4:4, with 8-pixel edges plus inner 4-pixel edges on non-subsampled axes
  (filter_plane_cols / _rows, vp9lpf.c:31-181).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FORMATS = [(1, 0), (0, 1), (0, 0)]      # 4:2:2, 4:4:0, 4:4:4 (ss_h, ss_v)


def _cmp(v9, got, ref, w, h, ssh, ssv, what):
    for p, (a, b) in enumerate(zip(v9.visible(got, w, h, ssh, ssv), v9.visible(ref, w, h, ssh, ssv))):
        if not np.array_equal(a, b):
            ys, xs = np.nonzero(a != b)
            raise AssertionError("%s plane %d: %d px differ, first at (x=%d, y=%d): gpu %d oracle %d"
                                 % (what, p, len(ys), xs[0], ys[0], a[ys[0], xs[0]], b[ys[0], xs[0]]))


KEY = [
    (352, 288, 8, {}),
    (200, 130, 8, {}),
    (66, 74, 8, {"p_zero_eob": 0.3, "p_skip": 0.5}),
    (512, 256, 8, {"log2_tile_cols": 1}),
    (200, 136, 8, {"lossless": 1, "q_idx": 0}),
    (352, 288, 8, {"sharpness": 5, "filter_level": 63}),
    (200, 130, 10, {}),
    (176, 144, 12, {"coef_stress": 1}),
]


@pytest.mark.parametrize("ssh,ssv", FORMATS)
@pytest.mark.parametrize("w,h,bpp,kw", KEY)
def test_keyframe_parity_subsampling(v9, orc, gpu, ssh, ssv, w, h, bpp, kw):
    for seed in (21, 22):
        f = v9.SynthFrame(v9.synth_params(w, h, bpp, seed=seed, ss_h=ssh, ss_v=ssv, **kw))
        gpu.configure(w, h, bpp, nbufs=1, ss_h=ssh, ss_v=ssv)
        gpu.submit(f, 0)
        gpu.sync()
        ref = v9.alloc_planes(w, h, bpp, ssh, ssv)
        orc.decode_frame(f.pkt, ref)
        _cmp(v9, gpu.download(0), ref, w, h, ssh, ssv,
             "keyframe %dx%d@%d ss=%d%d %s seed %d" % (w, h, bpp, ssh, ssv, kw, seed))


INTER = [
    (352, 288, 8, {}),
    (200, 130, 8, {"compound": 1}),
    (130, 66, 8, {"bilinear": 1, "p_zero_eob": 0.4}),
    (200, 130, 10, {"compound": 1}),
]


@pytest.mark.parametrize("ssh,ssv", FORMATS)
@pytest.mark.parametrize("w,h,bpp,kw", INTER)
def test_inter_parity_subsampling(v9, orc, gpu, ssh, ssv, w, h, bpp, kw):
    refs = []
    for seed in (31, 32):
        k = v9.SynthFrame(v9.synth_params(w, h, bpp, seed=seed, ss_h=ssh, ss_v=ssv))
        r = v9.alloc_planes(w, h, bpp, ssh, ssv)
        orc.decode_frame(k.pkt, r)
        refs.append(r)
    for seed in (33, 34):
        f = v9.SynthFrame(v9.synth_params(w, h, bpp, seed=seed, inter=1, ss_h=ssh, ss_v=ssv, **kw))
        gpu.configure(w, h, bpp, nbufs=3, ss_h=ssh, ss_v=ssv)
        gpu.upload(0, refs[0])
        gpu.upload(1, refs[1])
        gpu.submit(f, 2, (0, 0, 1))
        gpu.sync()
        out = v9.alloc_planes(w, h, bpp, ssh, ssv)
        orc.decode_frame(f.pkt, out, [refs[0], refs[0], refs[1]])
        _cmp(v9, gpu.download(2), out, w, h, ssh, ssv,
             "inter %dx%d@%d ss=%d%d %s seed %d" % (w, h, bpp, ssh, ssv, kw, seed))


@pytest.mark.parametrize("ssh,ssv", FORMATS)
def test_scaled_reference_subsampling(v9, orc, gpu, ssh, ssv):
    """Scaled-reference chroma MC per subsampled / full axis (vp9recon.c:543-628)."""
    (rw, rh), (w, h) = (256, 200), (200, 136)
    key = v9.SynthFrame(v9.synth_params(rw, rh, 8, seed=930, ss_h=ssh, ss_v=ssv))
    gpu.configure(max(rw, w), max(rh, h), 8, nbufs=2, ss_h=ssh, ss_v=ssv)
    gpu.stage_batch([key], [0])
    gpu.run_batch()
    kref = v9.alloc_planes(rw, rh, 8, ssh, ssv)
    orc.decode_frame(key.pkt, kref)
    _cmp(v9, gpu.download(0), kref, rw, rh, ssh, ssv, "scaled-test keyframe")
    for seed, kw in ((931, {"compound": 1}), (932, {"bilinear": 1})):
        f = v9.SynthFrame(v9.synth_params(w, h, 8, seed=seed, inter=1, ss_h=ssh, ss_v=ssv, **kw))
        for r in range(3):
            f.pkt.ref_w[r], f.pkt.ref_h[r] = rw, rh
        gpu.stage_batch([f], [1], [(0, 0, 0)])
        gpu.run_batch()
        gpu.sync()
        out = v9.alloc_planes(w, h, 8, ssh, ssv)
        orc.decode_frame(f.pkt, out, [kref, kref, kref], [(rw, rh)] * 3)
        _cmp(v9, gpu.download(1), out, w, h, ssh, ssv, "scaled ss=%d%d seed %d" % (ssh, ssv, seed))


def test_gop_batch_444(v9, orc, gpu):
    """A key + 3 P GOP at 4:4:4 staged as one batch (chained phases)."""
    w, h = 256, 136
    frames = [v9.SynthFrame(v9.synth_params(w, h, 8, seed=940, ss_h=0, ss_v=0))]
    frames += [v9.SynthFrame(v9.synth_params(w, h, 8, seed=941 + k, inter=1, compound=int(k == 1), ss_h=0, ss_v=0))
               for k in range(3)]
    refs = [None, (0, 0, 0), (1, 1, 0), (2, 2, 0)]
    gpu.configure(w, h, 8, nbufs=4, ss_h=0, ss_v=0)
    gpu.stage_batch(frames, [0, 1, 2, 3], refs)
    gpu.run_batch()
    gpu.sync()
    dec = {}
    for i, f in enumerate(frames):
        out = v9.alloc_planes(w, h, 8, 0, 0)
        r = refs[i]
        orc.decode_frame(f.pkt, out, None if r is None else [dec[r[0]], dec[r[1]], dec[r[2]]])
        dec[i] = out
        _cmp(v9, gpu.download(i), out, w, h, 0, 0, "444 gop frame %d" % i)
