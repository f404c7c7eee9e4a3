"""CPU: pin the oracle's DSP restatement with the reference's own test generators.

The reference build could not be run here, so there are no golden
outputs of libavcodec; these tests pin the oracle with properties that any correct
restatement of vp9dsp_template.c must satisfy, using the input generators of the
reference's differential test tests/checkasm/vp9dsp.c:
  * itxfm: checkasm's double-precision forward transforms (vp9dsp.c:123-251) +
    lrint; the lossless WHT must invert exactly, DCT/ADST within rounding.
  * ipred: constant edges reproduce the constant for every directional mode;
    V/H/DC/TM known answers (vp9dsp_template.c:33-437).
  * loop filter: checkasm's crafted lines (vp9dsp.c:393-447): flat lines keep a flat
    profile, strong steps (fm false) stay untouched, 'off' lines never change.
  * MC: full-pel copy, constant sources, bilinear on ramps (vp9dsp_template.c:1971-2263).
"""
import math

import numpy as np
import pytest

RNG = np.random.default_rng(0x56503900)


# ---- checkasm forward transforms (tests/checkasm/vp9dsp.c:124-251) ----
def fwht_1d(x):
    t0 = x[0] + x[1]
    t3 = x[3] - x[2]
    t4 = math.trunc((t0 - t3) * 0.5)
    t1 = t4 - x[1]
    t2 = t4 - x[2]
    return [t0 - t2, t2, t3 + t1, t1]


def fdct_1d(x):
    n = len(x)
    out = [sum(x[m] * math.cos(math.pi * (2 * m + 1) * k / (n * 2.0)) for m in range(n)) for k in range(n)]
    out[0] *= math.sqrt(0.5)
    return out


def fadst4_1d(x):
    n = len(x)
    return [sum(x[m] * math.sin(math.pi * (m + 1) * (2 * k + 1) / (n * 2.0 + 1.0)) for m in range(n)) for k in range(n)]


def fadst_1d(x):
    n = len(x)
    return [sum(x[m] * math.sin(math.pi * (2 * m + 1) * (2 * k + 1) / (n * 4.0)) for m in range(n)) for k in range(n)]


SCALE = [[4.0, 16.0 * math.sqrt(0.5) / 3.0, 16.0 * math.sqrt(0.5) / 3.0, 32.0 / 9.0],
         [2.0] * 4, [1.0] * 4, [0.25], [4.0]]


def ftx(res, tx, txtp):
    sz = res.shape[0]
    if tx == 4:
        f = (fwht_1d, fwht_1d)
    elif tx == 0:
        f = [(fdct_1d, fdct_1d), (fadst4_1d, fdct_1d), (fdct_1d, fadst4_1d), (fadst4_1d, fadst4_1d)][txtp]
    else:
        f = [(fdct_1d, fdct_1d), (fadst_1d, fdct_1d), (fdct_1d, fadst_1d), (fadst_1d, fadst_1d)][txtp]
    sc = SCALE[tx][txtp]
    inp = res.astype(float).reshape(-1)
    temp = np.zeros(sz * sz)
    for i in range(sz):
        o = f[0](list(inp[i * sz:(i + 1) * sz]))
        for j in range(sz):
            temp[j * sz + i] = o[j] * sc
    out = np.zeros(sz * sz)
    for i in range(sz):
        out[i * sz:(i + 1) * sz] = f[1](list(temp[i * sz:(i + 1) * sz]))
    return np.array([int(np.rint(v)) for v in out])


def _dt(bpp):
    return np.uint8 if bpp == 8 else np.uint16


def fwht_int(res):
    """Integer forward WHT in libvpx's vp9_fwht4x4 order (the encoder side of VP9
    lossless): the butterfly of checkasm's fwht_1d (vp9dsp.c:124-136) on integers
    with a floor shift, first over columns, then rows, x4 (UNIT_QUANT_FACTOR) last."""
    def f(x):
        t0 = x[0] + x[1]
        t3 = x[3] - x[2]
        t4 = (t0 - t3) >> 1
        t1 = t4 - x[1]
        t2 = t4 - x[2]
        return [t0 - t2, t2, t3 + t1, t1]
    m = [[int(v) for v in row] for row in res]
    p1 = [[0] * 4 for _ in range(4)]
    for i in range(4):                       # columns
        o = f([m[k][i] for k in range(4)])
        for k in range(4):
            p1[k][i] = o[k]
    out = []
    for r in range(4):                       # rows
        out += [4 * v for v in f(p1[r])]
    # libavcodec stores coefficient (row, col) where libvpx stores (col, row): its scan
    # tables are the transposes of libvpx's (vp9data.c:454 {0,1,4,5,..} vs {0,4,1,5,..})
    return np.array(out).reshape(4, 4).T.reshape(-1)


@pytest.mark.parametrize("bpp", [8, 10])
def test_wht_lossless_roundtrip_exact(orc, bpp):
    mask = (1 << bpp) - 1
    for _ in range(50):
        src = RNG.integers(0, mask + 1, (4, 4))
        dst = RNG.integers(0, mask + 1, (4, 4))
        coef = fwht_int(src - dst)
        c = coef.astype(np.int16 if bpp == 8 else np.int32)
        d = dst.astype(_dt(bpp))
        orc.itxfm_add(bpp, d, c, 16, 4, 0)
        assert np.array_equal(d.astype(int), src), "WHT is lossless in VP9 (fwht/iwht, vp9dsp_template.c:1719-1750)"
        assert not c.any(), "itxfm_add must zero the coefficient block (checkasm vp9dsp.c:365-368)"


@pytest.mark.parametrize("tx", [0, 1, 2, 3])
@pytest.mark.parametrize("txtp", [0, 1, 2, 3])
def test_itxfm_inverts_checkasm_forward(orc, tx, txtp):
    if tx == 3 and txtp:
        pytest.skip("32x32 is DCT only")
    sz = 4 << tx
    bpp = 8
    worst = 0
    for _ in range(3 if tx < 3 else 1):
        src = RNG.integers(0, 256, (sz, sz))
        dst = RNG.integers(0, 256, (sz, sz))
        coef = ftx(src - dst, tx, txtp).astype(np.int16)
        d = dst.astype(np.uint8)
        orc.itxfm_add(bpp, d, coef, sz * sz, tx, txtp)
        assert not coef.any()
        worst = max(worst, int(np.abs(d.astype(int) - src).max()))
    # inverse(forward(residual)) reconstructs within rounding (both are ~orthonormal)
    assert worst <= 2, worst


@pytest.mark.parametrize("bpp", [8, 10])
def test_itxfm_dc_only_matches_full(orc, bpp):
    """eob==1 DC shortcut (vp9dsp_template.c:1165-1178) equals the 2-pass result for DC."""
    for tx in range(4):
        sz = 4 << tx
        for dc in (-700, -13, 0, 5, 999):
            dst = RNG.integers(0, 1 << bpp, (sz, sz)).astype(_dt(bpp))
            cdt = np.int16 if bpp == 8 else np.int32
            c1 = np.zeros(sz * sz, cdt); c1[0] = dc
            c2 = c1.copy()
            a, b = dst.copy(), dst.copy()
            orc.itxfm_add(bpp, a, c1, 1, tx, 0)
            orc.itxfm_add(bpp, b, c2, 2, tx, 0)    # eob 2: full path, same coefficients
            assert np.array_equal(a, b)


@pytest.mark.parametrize("bpp", [8, 10, 12])
def test_ipred_constant_edges(orc, bpp):
    for tx in range(4):
        n = 4 << tx
        for c in (0, 77, (1 << bpp) - 1):
            left = np.full(32, c, _dt(bpp))
            top = np.full(1 + 64, c, _dt(bpp))
            for mode in range(12):
                d = np.zeros((n, n), _dt(bpp))
                orc.intra_pred(bpp, d, left, top, tx, mode)
                assert (d == c).all(), (tx, mode, c)


def test_ipred_known_answers(orc):
    for tx in range(4):
        n = 4 << tx
        left = RNG.integers(0, 256, 32).astype(np.uint8)     # bottom-to-top
        top = RNG.integers(0, 256, 65).astype(np.uint8)      # top[0] = top-left
        T, L, tl = top[1:n + 1].astype(int), left[:n].astype(int), int(top[0])
        d = np.zeros((n, n), np.uint8)
        orc.intra_pred(8, d, left, top, tx, 0)
        assert (d == T[None, :]).all()
        orc.intra_pred(8, d, left, top, tx, 1)
        assert (d == L[::-1][:, None]).all()
        orc.intra_pred(8, d, left, top, tx, 2)
        assert (d == (T.sum() + L.sum() + n) // (2 * n)).all()
        orc.intra_pred(8, d, left, top, tx, 9)
        exp = np.clip(T[None, :] + L[::-1][:, None] - tl, 0, 255)
        assert (d == exp).all()
        for mode, val in ((12, 128), (13, 127), (14, 129)):
            orc.intra_pred(8, d, left, top, tx, mode)
            assert (d == val).all()


def _lf_line(kind, bpp, E, F, I, length=16):
    """One line of checkasm's randomize_loopfilter_buffers (vp9dsp.c:393-447); q0 at index 8."""
    mask = (1 << bpp) - 1
    sh = bpp - 8
    x = np.zeros(length, np.int64)
    q0 = int(RNG.integers(0, mask + 1))

    def sx(base, d):
        d <<= sh
        return int(np.clip(base - d + RNG.integers(0, 2 * d + 1), 0, mask))
    if kind == "flat16":
        x[8] = q0
        x[7] = p0 = sx(q0, E >> 2)
        for j in range(1, 8):
            x[7 - j] = sx(p0, F)
            x[8 + j] = sx(q0, F)
    elif kind == "off":
        x[:] = RNG.integers(0, mask + 1, length)
    return x


def test_loop_filter_checkasm_lines(orc):
    E, I, H, F = 20, 10, 7, 1
    for bpp in (8, 10):
        dt = _dt(bpp)
        for _ in range(50):
            line = _lf_line("flat16", bpp, E, F, I)
            buf = np.zeros((8, 16), dt)
            buf[:] = line.astype(dt)
            before = buf.astype(int).copy()
            orc.loop_filter(bpp, buf.reshape(-1), 8, 16, 0, 2, 0, 0, E, I, H)   # 16-wide, column edge
            after = buf.astype(int)
            # smoothing never widens the range of the line
            assert after.min() >= before.min() and after.max() <= before.max()
        # a step far above E: fm is false, nothing changes
        buf = np.zeros((8, 16), np.uint8)
        buf[:, 8:] = 200
        ref = buf.copy()
        orc.loop_filter(8, buf.reshape(-1), 8, 16, 0, 2, 0, 0, E, I, H)
        assert np.array_equal(buf, ref)
        # a constant line is a fixed point of every filter width
        for wd in range(3):
            buf = np.full((8, 16), 90, np.uint8)
            orc.loop_filter(8, buf.reshape(-1), 8, 16, 0, wd, 0, 0, E, I, H)
            assert (buf == 90).all()


@pytest.mark.parametrize("filt", [0, 1, 2, 3])
def test_mc_properties(orc, filt):
    for bpp in (8, 10):
        dt = _dt(bpp)
        src = RNG.integers(0, 1 << bpp, (72, 72)).astype(dt)
        dst = np.zeros((64, 64), dt)
        off = 3 * 72 + 3
        orc.mc(bpp, dst, src, off, 72, 16, 16, 0, 0, filt, 0)
        assert np.array_equal(dst[:16, :16], src[3:19, 3:19])
        const = np.full((72, 72), 300 if bpp > 8 else 100, dt)
        for mx, my in ((5, 0), (0, 9), (3, 14)):
            orc.mc(bpp, dst, const, off, 72, 8, 8, mx, my, filt, 0)
            assert (dst[:8, :8] == const[0, 0]).all()
    # bilinear interpolates a horizontal ramp exactly: src[x] = 8x -> value 8x + mx/2
    ramp = np.tile((np.arange(72) * 8).astype(np.uint16), (72, 1))
    d = np.zeros((64, 64), np.uint16)
    orc.mc(10, d, ramp, 3 * 72 + 3, 72, 8, 8, 4, 0, 3, 0)
    assert (d[:8, :8] == ramp[3:11, 3:11] + 2).all()


@pytest.mark.parametrize("filt", [0, 1, 2, 3])
def test_mc_scaled_unit_step_equals_unscaled(orc, filt):
    """do_scaled_8tap / do_scaled_bilin (vp9dsp_template.c:2363-2482) always run the 2-D
    filter; at step 16 (scale 1.0) they must equal the unscaled 1-D/2-D/copy paths
    (vp9dsp_template.c:1969-2361) -- the identity phase is exact."""
    for bpp in (8, 10):
        dt = _dt(bpp)
        src = RNG.integers(0, 1 << bpp, (96, 96)).astype(dt)
        for mx, my in ((0, 0), (6, 0), (0, 10), (3, 13), (15, 1)):
            for avg in (0, 1):
                a = RNG.integers(0, 1 << bpp, (64, 64)).astype(dt)
                b = a.copy()
                off = 8 * 96 + 8
                orc.mc(bpp, a, src, off, 96, 16, 8, mx, my, filt, avg)
                orc.mc_scaled(bpp, b, src, off, 96, 16, 8, mx, my, 16, 16, filt, avg)
                assert np.array_equal(a, b), (bpp, mx, my, filt, avg)


def test_mc_scaled_constant_and_step():
    """A constant reference stays constant at any scale; at step 32 (2x downscale) with
    phase 0 the full-pel source samples are every other pixel."""
    import oracle as orc
    for filt in range(4):
        src = np.full((160, 160), 77, np.uint8)
        d = np.zeros((64, 64), np.uint8)
        orc.mc_scaled(8, d, src, 8 * 160 + 8, 160, 16, 16, 5, 11, 24, 21, filt, 0)
        assert (d[:16, :16] == 77).all()
    src = RNG.integers(0, 256, (160, 160)).astype(np.uint8)
    d = np.zeros((64, 64), np.uint8)
    orc.mc_scaled(8, d, src, 8 * 160 + 8, 160, 16, 16, 0, 0, 32, 32, 1, 0)
    assert np.array_equal(d[:16, :16], src[8:40:2, 8:40:2])
