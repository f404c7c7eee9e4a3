/*
 * Planning rules of the pixel path, shared by the two planners: the host planner
 * (vp9hip_runtime.cpp, VP9HIP_HOST_PLAN=1 and vp9hip_plan_stats) and the device planner
 * (vp9hip_plan.hip, the default). One restatement of the reference, two executors: every
 * function is __host__ __device__ and takes its state through plain values or functors.
 *
 *   pl_intra_job       check_intra_mode (vp9recon.c:37-221): mode_conv, edge availability,
 *                      n_px_have clamps -> the PJob word; the edges the substituted mode
 *                      reads (vp9recon.c:71-97) -> its producer units
 *   pl_lf_mask_edges   mask_edges (vp9block.c:1142-1262)
 *   pl_lf_edge         filter_plane_cols / filter_plane_rows edge selection incl. the mix2
 *                      pairing (vp9lpf.c:31-181) -> LFRec.prog bytes
 *   pl_mc_block        inter_pred's prediction units (vp9_mc_template.c:30-464) with
 *                      mc_{luma,chroma}_{unscaled,scaled} positions (vp9recon.c:376-628)
 * Internal to libvp9hip.
 */
#ifndef VP9HIP_PLANLOGIC_H
#define VP9HIP_PLANLOGIC_H
#include <stdint.h>
#include "../../include/vp9hip.h"
#include "vp9hip_work.h"

#define PL_HD __host__ __device__ static inline

/* ff_vp9_bwh_tab (vp9data.c:25-38): [0] 4x4 units, [1] 8x8 units; [ss] also indexes chroma.
 * Bit-packed log2 sizes (3 bits per block size), so device code computes them in registers
 * instead of loading a table from memory. [1] = max([0] / 2, 1). */
PL_HD int pl_bwh(int i, int bs, int d)
{
    const uint64_t lw = 0x494936e4ull, lh = 0x20a29a71cull;     /* log2 of [0][bs][0] / [0][bs][1] */
    const int l = (int) (((d ? lh : lw) >> (3 * bs)) & 7) - i;
    return 1 << (l > 0 ? l : 0);
}

/* entry i of a table of n-bit fields packed into a 64-bit constant */
PL_HD int pl_field(uint64_t packed, int i, int bits) { return (int) ((packed >> (bits * i)) & ((1u << bits) - 1)); }

PL_HD int pl_min(int a, int b) { return a < b ? a : b; }
PL_HD int pl_max(int a, int b) { return a > b ? a : b; }
PL_HD int pl_clamp(int v, int lo, int hi) { return v < lo ? lo : v > hi ? hi : v; }
PL_HD int pl_rdiv(int a, int b) { return (a >= 0 ? a + (b >> 1) : a - (b >> 1)) / b; }   /* ROUNDED_DIV */

/* Tile column of SB column sbx: its first SB column (set_tile_offset, vp9.c:1244-1250). */
PL_HD int pl_tile_of(int sbx, int sb_cols, int log2, int *tile_sb0)
{
    int t = 0, s0 = 0;
    for (int ti = 0; ti < (1 << log2); ti++) {
        const int a = pl_min((ti * sb_cols) >> log2, sb_cols), b = pl_min(((ti + 1) * sb_cols) >> log2, sb_cols);
        if (sbx >= a && sbx < b) { t = ti; s0 = a; }
    }
    *tile_sb0 = s0;
    return t;
}

/* Packet-order index of SB (sbx, sby) in its frame. decode_tiles walks, per tile row, the
 * SB rows and within each row the tile columns left to right (vp9.c:1325-1395), so the
 * blocks of a packet come in SB raster order. */
PL_HD int pl_sb_dorder(int sbx, int sby, int sb_cols) { return sby * sb_cols + sbx; }

/* ff_vp9_intra_txfm_type (vp9data.c:437-452) */
PL_HD int pl_intra_txfm_type(int mode)
{
    return pl_field(0xd9b06ull, mode, 2);     /* { 2, 1, 0, 0, 3, 2, 1, 2, 1, 3, 0, 0, 0, 0 } */
}

/* The tx-block grid of one plane of a block (the end_x / end_y clipping of intra_recon /
 * inter_recon, vp9recon.c:243-244, 707-712): tx size, step and the ranges in 4x4 units. */
struct PlTxGrid {
    int txs, step;          /* tx size code, 4x4 units per tx block side */
    int ex, ey;             /* visible extent (4x4 units) of the block in this plane */
    int nx, ny;             /* tx blocks per row / column that start inside it */
    int pw4;                /* block width in this plane (4x4 units) */
    int bx, by;             /* plane pixel position of the block */
};
template <class B> PL_HD PlTxGrid pl_txgrid(const B &b, int p, int cols, int rows, int ss_h, int ss_v)
{
    PlTxGrid g;
    const int w4 = pl_bwh(1, b.bs, 0) << 1, h4 = pl_bwh(1, b.bs, 1) << 1;
    const int end_x = pl_min(2 * (cols - b.col), w4), end_y = pl_min(2 * (rows - b.row), h4);
    const int sh = p ? ss_h : 0, sv = p ? ss_v : 0;
    g.txs = p ? b.uvtx : b.tx;
    g.step = 1 << g.txs;
    g.pw4 = w4 >> sh;
    g.ex = end_x >> sh;
    g.ey = end_y >> sv;
    g.nx = g.ex > 0 ? (g.ex + g.step - 1) >> g.txs : 0;
    g.ny = g.ey > 0 ? (g.ey + g.step - 1) >> g.txs : 0;
    g.bx = b.col * 8 >> sh;
    g.by = b.row * 8 >> sv;
    return g;
}

/* One intra tx block: the PJob word (vp9hip_work.h) with check_intra_mode resolved, and the
 * edges the substituted mode reads (needs: 1 left, 2 top, 4 top-left, 8 top-right) and
 * whether the 4x4 top-right lies inside the block (trx). */
struct PlIntra { uint32_t a; int nd, trx; };
PL_HD PlIntra pl_intra_job(int p, int txs, int mode, int e, int gx, int gy, int x, int pw4, int tx0, int pw8, int ph8,
                           int ux0, int uy0)
{
    const int n = 4 << txs;
    const int have_top = gy > 0, have_left = gx > tx0, have_right = x < pw4 - 1;
    const int have_t = pw8 - gx, have_l = ph8 - gy;
    int m = mode;
    switch (m) {            /* mode_conv[mode][have_left][have_top] (vp9recon.c:49-87) */
    case 0: if (!have_top) m = 13; break;
    case 1: if (!have_left) m = 14; break;
    case 2: m = have_left ? (have_top ? 2 : 10) : (have_top ? 11 : 12); break;
    case 3: case 7: if (!have_top) m = 13; break;
    case 8: if (!have_left) m = 14; break;
    case 9: m = have_left ? (have_top ? 9 : 1) : (have_top ? 0 : 14); break;
    default: break;
    }
    /* slot_of = { 0, 1, 9, 2, 3, 4, 5, 6, 7, 8, 10, 11, 12, 13, 14 }; needs by slot (V H D45 D135
     * D117 D153 D63 D207 TM DC LEFT_DC TOP_DC DC_128/127/129) = { 2, 1, 2 | 8, 1 | 2 | 4, 1 | 2 | 4,
     * 1 | 2 | 4, 2 | 8, 1, 1 | 2 | 4, 1 | 2, 1, 2, 0, 0, 0 }, both packed 4 bits per entry */
    const uint64_t slot_of = 0xedcba8765432910ull, needs = 0x21371a777a12ull;
    const int slot = pl_field(slot_of, m, 4);
    const int ct = pl_min(n, have_t) - 1, cl = pl_min(n, have_l) - 1;
    const int trreal = txs == 0 && have_top && have_right && have_t >= 8;
    PlIntra r;
    r.a = (uint32_t) p | (uint32_t) txs << 2 | (uint32_t) (e ? 1 : 0) << 4 | (uint32_t) trreal << 5 |
          (uint32_t) have_top << 6 | (uint32_t) have_left << 7 | (uint32_t) slot << 8 | (uint32_t) ux0 << 12 |
          (uint32_t) uy0 << 16 | (uint32_t) ct << 20 | (uint32_t) cl << 25;
    r.nd = pl_field(needs, slot, 4);
    r.trx = (txs == 0 && (x < pw4 - 1) && (r.nd & 8)) ? 1 : 0;
    return r;
}

/* The 4x4 units of the job's own SB plane (16 units per map row) its substituted mode
 * reads: fn(unit). A level / pass order may only place the job after their producers. */
template <class F>
PL_HD void pl_local_reads(int ux0, int uy0, int n4, int nd, int trx, int units, int unitsv, F fn)
{
    if (uy0 > 0) {
        const int u0 = (nd & 4) ? ux0 - 1 : ux0, u1 = (nd & 2) ? ux0 + n4 + trx : ux0;
        for (int u = u0; u < u1; u++)
            if (u >= 0 && u < units) fn((uy0 - 1) * 16 + u);
    }
    if (ux0 > 0 && (nd & 1))
        for (int v = uy0; v < uy0 + n4; v++)
            if (v < unitsv) fn(v * 16 + ux0 - 1);
}

/* The units of OTHER SBs the job reads, in frame unit coordinates (fx, fy = the job's
 * first unit): left, top and top-left SBs (above-right reads stay inside the block's
 * columns, vp9recon.c:71-121). fn(ux, uy) with ux >= -1 / uy >= -1 unchecked. */
template <class F>
PL_HD void pl_cross_reads(int ux0, int uy0, int fx, int fy, int n4, int nd, int trx, F fn)
{
    if (uy0 == 0 && (nd & 6)) {
        const int u0 = (nd & 4) ? -1 : 0, u1 = (nd & 2) ? n4 + trx : 0;
        for (int u = u0; u < u1; u++) fn(fx + u, fy - 1);
    } else if (ux0 == 0 && (nd & 4)) {
        fn(fx - 1, fy - 1);
    }
    if (ux0 == 0 && (nd & 1))
        for (int v = 0; v < n4; v++) fn(fx - 1, fy + v);
}

/* ---------------------------------------------------------------- loop filter */
/* mask_edges (vp9block.c:1142-1262) for one plane class: or_(dir, row, kind, bits) ORs
 * bits into mask[dir][row][kind] (dir 0: column edges, 1: row edges). */
template <class OR>
PL_HD void pl_lf_mask_edges(OR or_, int ss_h, int ss_v, int row7, int col7, int w, int h, int col_end, int row_end,
                            int tx, int skip_inter)
{
    const unsigned wide_col[2] = { 0x11, 0x01 }, wide_row[2] = { 0x03, 0x07 };
    if (tx == 0 && (ss_v | ss_h)) {
        if (h == ss_v) { if (row7 & 1) return; if (!row_end) h += 1; }
        if (w == ss_h) { if (col7 & 1) return; if (!col_end) w += 1; }
    }
    const unsigned t = 1u << col7, m_col = (t << w) - t;
    if (tx == 0 && !skip_inter) {
        const unsigned m8 = m_col & wide_col[ss_h], m4 = m_col - m8;
        for (int y = row7; y < h + row7; y++) {
            const int id = 2 - !(y & wide_row[ss_v]);
            or_(0, y, 1, m8);
            or_(0, y, 2, m4);
            or_(1, y, id, ((ss_h & ss_v) && (col_end & 1) && (y & 1)) ? (t << (w - 1)) - t : m_col);
            if (!ss_h) or_(0, y, 3, m_col);
            if (!ss_v) or_(1, y, 3, (ss_h && (col_end & 1)) ? (t << (w - 1)) - t : m_col);
        }
        return;
    }
    if (!skip_inter) {
        const uint32_t masks = 0x011155ffu;        /* { 0xff, 0x55, 0x11, 0x01 }, a byte each */
        const int id = tx == 1;
        int l2 = tx + ss_h - 1;
        const unsigned m_row = m_col & ((masks >> (8 * l2)) & 255u);
        if (ss_h && tx > 1 && (w ^ (w - 1)) == 1) {
            const unsigned m16 = ((t << (w - 1)) - t) & ((masks >> (8 * l2)) & 255u), m8 = m_row - m16;
            for (int y = row7; y < h + row7; y++) { or_(0, y, 0, m16); or_(0, y, 1, m8); }
        } else {
            for (int y = row7; y < h + row7; y++) or_(0, y, id, m_row);
        }
        l2 = tx + ss_v - 1;
        const int step = 1 << l2;
        int y;
        if (ss_v && tx > 1 && (h ^ (h - 1)) == 1) {
            for (y = row7; y < h + row7 - 1; y += step) or_(1, y, 0, m_col);
            if (y - row7 == h - 1) or_(1, y, 1, m_col);
        } else {
            for (y = row7; y < h + row7; y += step) or_(1, y, id, m_col);
        }
    } else if (tx != 0) {
        or_(1, row7, (tx == 1) || (h == ss_v), m_col);
        const int id = (tx == 1) || (w == ss_h);
        for (int y = row7; y < h + row7; y++) or_(0, y, id, t);
    } else {
        const unsigned t8 = t & wide_col[ss_h], t4 = t - t8;
        for (int y = row7; y < h + row7; y++) { or_(0, y, 2, t4); or_(0, y, 1, t8); }
        or_(1, row7, 2 - !(row7 & wide_row[ss_v]), m_col);
    }
}

/* The LF level of one block (vp9block.c:1438-1441, levels vp9.c:767-791); 0 = not filtered. */
PL_HD int pl_lf_level(const vp9h_block &b, const uint8_t (*lflvl)[4][2], int filter_level)
{
    if (!filter_level || b.seg_id >= 8) return 0;
    return lflvl[b.seg_id][b.intra ? 0 : b.ref[0] + 1][b.mode[3] != VP9H_ZEROMV];
}

/* Both mask_edges calls of one block (vp9block.c:1442-1452): or_(cls, dir, row, kind, bits)
 * with cls 0 = luma masks, 1 = chroma masks. */
template <class OR>
PL_HD void pl_lf_block_masks(const vp9h_block &b, int cols, int rows, int ss_h, int ss_v, OR or_)
{
    const int bw8 = pl_bwh(1, b.bs, 0), bh8 = pl_bwh(1, b.bs, 1);
    const int x_end = pl_min(cols - b.col, bw8), y_end = pl_min(rows - b.row, bh8);
    const int skip_inter = !b.intra && b.skip, col7 = b.col & 7, row7 = b.row & 7;
    pl_lf_mask_edges([&](int d, int y, int k, unsigned v) { or_(0, d, y, k, v); }, 0, 0, row7, col7, x_end, y_end, 0, 0,
                     b.tx, skip_inter);
    pl_lf_mask_edges([&](int d, int y, int k, unsigned v) { or_(1, d, y, k, v); }, ss_h, ss_v, row7, col7, x_end, y_end,
                     (cols & 1) && b.col + bw8 >= cols ? cols & 7 : 0, (rows & 1) && b.row + bh8 >= rows ? rows & 7 : 0,
                     b.uvtx, skip_inter);
}

/* Filter width code | level of one edge (LFRec.prog) */
PL_HD uint8_t pl_lf_byte(int wd, int L)
{
    return wd ? (uint8_t) ((wd == 16 ? 3 : wd == 8 ? 2 : 1) << 6 | L) : 0;
}

/* Number of (plane class, direction, band, edge) items of an SB's LF program. */
PL_HD int pl_lf_items(int ss_h, int ss_v) { return 128 + 8 * (8 >> ss_v) + 8 * (8 >> ss_h); }

/* One item of the LF program (vp9lpf.c:31-181 per SB, loopfilter_sb 183-230): which filter
 * (width, level) edge e of band `band` gets, and its inner 4-wide edge, written through
 * put(byte offset, value). Item i: luma column edges 0..63, luma row edges 64..127, then the
 * chroma column and row edges. Chroma uses mask[ss_h | ss_v] (vp9lpf.c:189).
 * lvl(pos) = the level of 8x8 position pos (row * 8 + col); m(cls, dir, row, kind) = mask byte.
 * col0 / row0: the SB is at the frame's left / top edge (no outer edge there). */
template <class LVL, class M, class PUT>
PL_HD void pl_lf_item(int i, int ss_h, int ss_v, bool col0, bool row0, LVL lvl, M m, PUT put)
{
    int pl, dir, band, e;
    if (i < 128) { pl = 0; dir = i >> 6; band = (i >> 3) & 7; e = i & 7; }
    else {
        const int j = i - 128, nc = 8 * (8 >> ss_v);
        pl = 1;
        if (j < nc) { dir = 0; band = j >> 3; e = j & 7; }
        else { dir = 1; band = (j - nc) >> 3; e = (j - nc) & 7; }
    }
    const int sh = pl ? ss_h : 0, sv = pl ? ss_v : 0;
    const int cls = pl ? (ss_h | ss_v) : 0;
    const int dy = 1 << sv, dh = 1 << sh;
    if (dir == 0) {                     /* filter_plane_cols: band of pixel rows, edges left to right */
        const int cbase = pl ? LFP_CC : LFP_YC;
        const int half = band & 1, y = (band >> 1) * 2 * dy;
        const unsigned h10 = m(cls, 0, y, 0), h11 = m(cls, 0, y, 1), h12 = m(cls, 0, y, 2), h13 = m(cls, 0, y, 3);
        const unsigned h20 = m(cls, 0, y + dy, 0), h21 = m(cls, 0, y + dy, 1), h22 = m(cls, 0, y + dy, 2),
                       h23 = m(cls, 0, y + dy, 3);
        const unsigned h1 = h10 | h11 | h12, h2 = h21 | h22;
        const int k = e;
        const unsigned x = 1u << k;
        const int lc = sh ? k & ~1 : k;
        int wd = 0, L = 0;
        if (!col0 || k > 0) {
            if (!half) {
                if (h1 & x) { wd = (h10 & x) ? 16 : (h11 & x) ? 8 : 4; L = lvl(y * 8 + lc); }
            } else if (h1 & x) {
                if (h10 & x) { if (h20 & x) { wd = 16; L = lvl(y * 8 + lc); } }
                else if (h2 & x) { wd = (h21 & x) ? 8 : 4; L = lvl((y + dy) * 8 + lc); }
            } else if (h2 & x) { wd = (h21 & x) ? 8 : 4; L = lvl((y + dy) * 8 + lc); }
        }
        if (sh) { put(cbase + band * 8 + k, pl_lf_byte(wd, L)); return; }
        put(cbase + band * 16 + k * 2, pl_lf_byte(wd, L));
        const unsigned in = half ? h23 : h13;
        put(cbase + band * 16 + k * 2 + 1, (in & x) ? (uint8_t) (0x40 | lvl((half ? y + dy : y) * 8 + k)) : 0);
        return;
    }
    /* filter_plane_rows: band of pixel columns, edges top to bottom */
    const int rbase = pl ? LFP_CR(ss_h, ss_v) : LFP_YR;
    const int chunk = band >> 1, half = band & 1;
    const unsigned x = 1u << (chunk * 2 * dh), x2 = x << dh;
    const int lc1 = chunk * 2 * dh, lc2 = lc1 + dh;
    const int yy = e;
    const unsigned v0 = m(cls, 1, yy, 0), v1 = m(cls, 1, yy, 1), v2 = m(cls, 1, yy, 2), vm3 = m(cls, 1, yy, 3);
    const unsigned vm = v0 | v1 | v2;
    const int lr = sv ? yy & ~1 : yy;
    int wd = 0, L = 0;
    if (!row0 || yy) {
        if (!half) {
            if (vm & x) { wd = (v0 & x) ? 16 : (v1 & x) ? 8 : 4; L = lvl(lr * 8 + lc1); }
        } else if (vm & x) {
            if (v0 & x) { if (v0 & x2) { wd = 16; L = lvl(lr * 8 + lc1); } }
            else if (vm & x2) { wd = (v1 & x2) ? 8 : 4; L = lvl(lr * 8 + lc2); }
        } else if (vm & x2) { wd = (v1 & x2) ? 8 : 4; L = lvl(lr * 8 + lc2); }
    }
    if (sv) { put(rbase + band * 8 + yy, pl_lf_byte(wd, L)); return; }
    put(rbase + band * 16 + yy * 2, pl_lf_byte(wd, L));
    put(rbase + band * 16 + yy * 2 + 1,
        (!half ? (vm3 & x) : (vm3 & x2)) ? (uint8_t) (0x40 | lvl(yy * 8 + (half ? lc2 : lc1))) : 0);
}

/* ---------------------------------------------------------------- motion compensation */
/* What the MC position rules need of a frame: size in 8x8 units, subsampling and the
 * reference scale factors (vp9.c:845-880; 0 = unscaled). */
struct PlMcGeo {
    int32_t cols, rows, ss_h, ss_v;
    int32_t scale[3][2], step[3][2];
};
PL_HD int pl_scale_mv(int n, int scale) { return (int) (((int64_t) n * scale) >> 14); }

/* mc_luma_unscaled (vp9recon.c:376-414) or the scaled branch of mc_luma_scaled (492-541). */
PL_HD McRef pl_mc_luma_ref(const PlMcGeo &g, int rf, int x, int y, const int16_t *mv, int px, int py, int pw, int ph)
{
    McRef m;
    if (!g.scale[rf][0]) {
        m.ix = x + (mv[0] >> 3); m.iy = y + (mv[1] >> 3);
        m.mx = (uint8_t) ((mv[0] & 7) << 1); m.my = (uint8_t) ((mv[1] & 7) << 1);
        m.dx = m.dy = 16;
        return m;
    }
    const int mvx = pl_clamp(mv[0], -(x + pw - px + 4) * 8, (g.cols * 8 - x + px + 3) * 8);
    const int mvy = pl_clamp(mv[1], -(y + ph - py + 4) * 8, (g.rows * 8 - y + py + 3) * 8);
    const int mx = pl_scale_mv(mvx * 2, g.scale[rf][0]) + pl_scale_mv(x * 16, g.scale[rf][0]);
    const int my = pl_scale_mv(mvy * 2, g.scale[rf][1]) + pl_scale_mv(y * 16, g.scale[rf][1]);
    m.ix = mx >> 4; m.iy = my >> 4;
    m.mx = (uint8_t) (mx & 15); m.my = (uint8_t) (my & 15);
    m.dx = (uint8_t) g.step[rf][0]; m.dy = (uint8_t) g.step[rf][1];
    return m;
}

/* mc_chroma_unscaled (vp9recon.c:416-467; mv * 2 on a non-subsampled axis) or
 * mc_chroma_scaled with the libvpx rounding of webm issue 820 on subsampled axes (543-628). */
PL_HD McRef pl_mc_chroma_ref(const PlMcGeo &g, int rf, int x, int y, const int16_t *mv, int px, int py, int pw, int ph)
{
    McRef m;
    const int ssh = g.ss_h, ssv = g.ss_v;
    if (!g.scale[rf][0]) {
        const int mx = mv[0] * (1 << !ssh), my = mv[1] * (1 << !ssv);
        m.ix = x + (mx >> 4); m.iy = y + (my >> 4);
        m.mx = (uint8_t) (mx & 15); m.my = (uint8_t) (my & 15);
        m.dx = m.dy = 16;
        return m;
    }
    const int sx = g.scale[rf][0], sy = g.scale[rf][1];
    int mx, my;
    if (ssh) {
        const int mvx = pl_clamp(mv[0], -(x + pw - px + 4) * 16, (g.cols * 4 - x + px + 3) * 16);
        mx = pl_scale_mv(mvx, sx) + (pl_scale_mv(x * 16, sx) & ~15) + (pl_scale_mv(x * 32, sx) & 15);
    } else {
        const int mvx = pl_clamp(mv[0], -(x + pw - px + 4) * 8, (g.cols * 8 - x + px + 3) * 8);
        mx = pl_scale_mv(mvx * 2, sx) + pl_scale_mv(x * 16, sx);
    }
    if (ssv) {
        const int mvy = pl_clamp(mv[1], -(y + ph - py + 4) * 16, (g.rows * 4 - y + py + 3) * 16);
        my = pl_scale_mv(mvy, sy) + (pl_scale_mv(y * 16, sy) & ~15) + (pl_scale_mv(y * 32, sy) & 15);
    } else {
        const int mvy = pl_clamp(mv[1], -(y + ph - py + 4) * 8, (g.rows * 8 - y + py + 3) * 8);
        my = pl_scale_mv(mvy * 2, sy) + pl_scale_mv(y * 16, sy);
    }
    m.ix = mx >> 4; m.iy = my >> 4;
    m.mx = (uint8_t) (mx & 15); m.my = (uint8_t) (my & 15);
    m.dx = (uint8_t) g.step[rf][0]; m.dy = (uint8_t) g.step[rf][1];
    return m;
}

/* The prediction units of one inter block in inter_pred's order (vp9_mc_template.c:30-464):
 * emit(const McUnit &) per unit; returns the unit count. `frame` fills McUnit.frame.
 * Count-only callers pass an emit that ignores its argument. */
template <class EMIT>
PL_HD int pl_mc_block(const vp9h_block &b, const PlMcGeo &g, uint32_t frame, EMIT emit)
{
    const int ss_h = g.ss_h, ss_v = g.ss_v;
    const int r0 = b.ref[0], r1 = b.comp ? b.ref[1] : r0;
    /* the SCALED template when any reference is scaled (vp9recon.c:670-680) */
    const bool scaled_tpl = g.scale[r0][0] || (b.comp && g.scale[r1][0]);
    McUnit u;
    u.frame = frame;
    u.filter = b.filter;
    u.nref = b.comp ? 2 : 1;
    u.ref[0] = b.ref[0];
    u.ref[1] = b.ref[1];
    u.pad = 0;
    int cnt = 0;
    /* (x, y) plane position, (px, py, pw, ph) of mc_{luma,chroma}_dir */
    auto one = [&](int plane, int x, int y, int w, int hh, const int16_t (*mv)[2], int px, int py, int pw, int ph) {
        McUnit m = u;
        m.plane = (uint8_t) plane; m.x = (uint16_t) x; m.y = (uint16_t) y; m.w = (uint8_t) w; m.h = (uint8_t) hh;
        for (int k = 0; k < 2; k++) {
            if (k < m.nref) {
                const int rf = b.ref[k];
                m.r[k] = plane ? pl_mc_chroma_ref(g, rf, x, y, mv[k], px, py, pw, ph)
                               : pl_mc_luma_ref(g, rf, x, y, mv[k], px, py, pw, ph);
            } else {
                m.r[k].ix = m.r[k].iy = 0; m.r[k].mx = m.r[k].my = 0; m.r[k].dx = m.r[k].dy = 0;
            }
        }
        emit(m);
        cnt++;
    };
    auto chroma2 = [&](int x, int y, int w, int hh, const int16_t (*mv)[2], int px, int py, int pw, int ph) {
        one(1, x, y, w, hh, mv, px, py, pw, ph);
        one(2, x, y, w, hh, mv, px, py, pw, ph);
    };
    const int lx = b.col * 8, ly = b.row * 8, cx = b.col * (8 >> ss_h), cy = b.row * (8 >> ss_v);
    int16_t uv[2][2];
    /* ROUNDED_DIV_MVx2 / x4 chroma MVs of sub-8x8 blocks (vp9_mc_template.c:24-28) */
    auto avg2 = [&](int i0, int i1) -> const int16_t (*)[2] {
        for (int k = 0; k < 2; k++)
            for (int d = 0; d < 2; d++) uv[k][d] = (int16_t) pl_rdiv(b.mv[i0][k][d] + b.mv[i1][k][d], 2);
        return uv;
    };
    auto avg4 = [&]() -> const int16_t (*)[2] {
        for (int k = 0; k < 2; k++)
            for (int d = 0; d < 2; d++)
                uv[k][d] = (int16_t) pl_rdiv(b.mv[0][k][d] + b.mv[1][k][d] + b.mv[2][k][d] + b.mv[3][k][d], 4);
        return uv;
    };
    const int sub[4][2] = { { 0, 0 }, { 4, 0 }, { 0, 4 }, { 4, 4 } };
    if (b.bs > VP9H_BS_8x8 && scaled_tpl) {
        /* SCALED template: four 4x4 luma blocks; chroma 4x4 blocks with averaged MVs per
         * subsampled axis */
        for (int k = 0; k < 4; k++) one(0, lx + sub[k][0], ly + sub[k][1], 4, 4, b.mv[k], sub[k][0], sub[k][1], 8, 8);
        if (ss_v && ss_h) chroma2(cx, cy, 4, 4, avg4(), 0, 0, 4, 4);
        else if (ss_v) {
            chroma2(cx, cy, 4, 4, avg2(0, 2), 0, 0, 8, 4);
            chroma2(cx + 4, cy, 4, 4, avg2(1, 3), 4, 0, 8, 4);
        } else if (ss_h) {
            chroma2(cx, cy, 4, 4, avg2(0, 1), 0, 0, 4, 8);
            chroma2(cx, cy + 4, 4, 4, avg2(1, 2), 0, 4, 4, 8);      /* libvpx bug replica (296-305) */
        } else {
            for (int k = 0; k < 4; k++) chroma2(cx + sub[k][0], cy + sub[k][1], 4, 4, b.mv[k], sub[k][0], sub[k][1], 8, 8);
        }
    } else if (b.bs == VP9H_BS_8x4) {
        one(0, lx, ly, 8, 4, b.mv[0], 0, 0, 0, 0);
        one(0, lx, ly + 4, 8, 4, b.mv[2], 0, 0, 0, 0);
        if (ss_v) chroma2(cx, cy, 8 >> ss_h, 4, avg2(0, 2), 0, 0, 0, 0);
        else {
            chroma2(cx, cy, 8 >> ss_h, 4, b.mv[0], 0, 0, 0, 0);
            /* libvpx uses the wrong block index for 4:4:4 (vp9_mc_template.c:107-114) */
            chroma2(cx, cy + 4, 8 >> ss_h, 4, ss_h ? avg2(0, 2) : b.mv[2], 0, 0, 0, 0);
        }
    } else if (b.bs == VP9H_BS_4x8) {
        one(0, lx, ly, 4, 8, b.mv[0], 0, 0, 0, 0);
        one(0, lx + 4, ly, 4, 8, b.mv[1], 0, 0, 0, 0);
        if (ss_h) chroma2(cx, cy, 4, 8 >> ss_v, avg2(0, 1), 0, 0, 0, 0);
        else {
            chroma2(cx, cy, 4, 8 >> ss_v, b.mv[0], 0, 0, 0, 0);
            chroma2(cx + 4, cy, 4, 8 >> ss_v, b.mv[1], 0, 0, 0, 0);
        }
    } else if (b.bs > VP9H_BS_8x8) {
        for (int k = 0; k < 4; k++) one(0, lx + sub[k][0], ly + sub[k][1], 4, 4, b.mv[k], 0, 0, 0, 0);
        if (ss_v && ss_h) chroma2(cx, cy, 4, 4, avg4(), 0, 0, 0, 0);
        else if (ss_v) {
            chroma2(cx, cy, 4, 4, avg2(0, 2), 0, 0, 0, 0);
            chroma2(cx + 4, cy, 4, 4, avg2(1, 3), 0, 0, 0, 0);
        } else if (ss_h) {
            chroma2(cx, cy, 4, 4, avg2(0, 1), 0, 0, 0, 0);
            chroma2(cx, cy + 4, 4, 4, avg2(1, 2), 0, 0, 0, 0);      /* libvpx bug replica (296-305) */
        } else {
            for (int k = 0; k < 4; k++) chroma2(cx + sub[k][0], cy + sub[k][1], 4, 4, b.mv[k], 0, 0, 0, 0);
        }
    } else {
        const int bw = pl_bwh(0, b.bs, 0) * 4, bh = pl_bwh(0, b.bs, 1) * 4;
        const int uvbw = pl_bwh(ss_h, b.bs, 0) * 4, uvbh = pl_bwh(ss_v, b.bs, 1) * 4;
        one(0, lx, ly, bw, bh, b.mv[0], 0, 0, bw, bh);
        chroma2(cx, cy, uvbw, uvbh, b.mv[0], 0, 0, uvbw, uvbh);
    }
    return cnt;
}

/* ---------------------------------------------------------------- residual scratch */
/* Residual scratch offset (16-element units) of a tx block inside its SB's slot: luma
 * units first, then U and V. Each plane's 4x4-unit grid is laid out in Morton order over
 * its square part (so every size-aligned n x n tx block is one contiguous range of n^2
 * units, column-major n x n residuals fit exactly), the longer side's extra squares after. */
PL_HD uint32_t pl_morton(int x, int y, int s)
{
    uint32_t m = 0;
    for (int k = 0; (1 << k) < s; k++) m |= (uint32_t) ((x >> k) & 1) << (2 * k) | (uint32_t) ((y >> k) & 1) << (2 * k + 1);
    const int q = x >= s ? x / s : y / s;     /* index of the s x s square along the longer side */
    return m + (uint32_t) (q * s * s);
}
PL_HD int pl_rcap(int ss_h, int ss_v) { return 256 + 2 * ((16 >> ss_h) * (16 >> ss_v)); }
PL_HD uint32_t pl_resid_unit(int p, int ux, int uy, int ss_h, int ss_v)
{
    const int cw = 16 >> ss_h, ch = 16 >> ss_v, s = cw < ch ? cw : ch;
    if (p == 0) return pl_morton(ux, uy, 16);
    return 256 + (uint32_t) ((p - 1) * cw * ch) + pl_morton(ux, uy, s);
}

#endif
