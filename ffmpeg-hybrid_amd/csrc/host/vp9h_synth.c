/*
 * Synthetic pass-1 frame generator (bench / test input).
 *
 * Produces the same structures the reference's pass 1 leaves in memory for pass 2
 * (vp9.c:335-353): one block record per coded block in decode order, per-tx-block
 * eobs and dequantized coefficients. The block walk restates decode_sb's partition
 * rules at frame edges (vp9.c:1115-1193) and the tile/SB loop order of decode_tiles
 * (vp9.c:1325-1395); transform-size limits follow decode_mode (vp9block.c:88-91,
 * 171-215, 1291-1292); dequantization follows decode_coeffs_b_generic
 * (vp9block.c:905-917) with the qlookup tables (vp9.c:745-766); LF levels follow
 * vp9.c:767-791 with libvpx's default ref/mode deltas (vp9.c:659-668) or the given ones;
 * with segmentation (p->seg) the blocks draw segment ids, each segment with its alternate q
 * (the coefficients are multiples of that segment's step) and LF level.
 */
#include <stdlib.h>
#include <string.h>

#include "../../../include/vp9hip.h"
#include "../vp9_tables.h"

#define MIN(a, b) ((a) < (b) ? (a) : (b))

typedef struct Rng { uint64_t s; } Rng;
static uint64_t rng_u64(Rng *r)
{   /* splitmix64 */
    uint64_t z = (r->s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static double rng_f(Rng *r) { return (rng_u64(r) >> 11) * (1.0 / 9007199254740992.0); }
static int rng_int(Rng *r, int n) { return (int) (rng_u64(r) % (uint64_t) n); }

typedef struct Gen {
    const vp9h_synth_params *p;
    Rng rng;
    int cols, rows, sb_cols, sb_rows;
    int qmul[8][2][2];           /* [segment][y/uv][dc/ac] */
    int seg;                     /* the segment of the block being generated */
    /* growable outputs */
    vp9h_block *blocks; size_t nb, cb;
    uint16_t *eobs; size_t ne, ce;
    uint8_t *coefs; size_t nc, cc;    /* bytes */
    int err;
} Gen;

static void *grow(void *ptr, size_t *cap, size_t need, size_t elem, int *err)
{
    if (need <= *cap) return ptr;
    size_t nc = *cap ? *cap : 1024;
    while (nc < need) nc *= 2;
    void *n = realloc(ptr, nc * elem);
    if (!n) { *err = 1; return ptr; }
    *cap = nc;
    return n;
}

static const uint8_t max_tx_for_bs[VP9H_N_BS] = { 3, 3, 3, 3, 2, 2, 2, 1, 1, 1, 0, 0, 0 };

static int coef_mag(Gen *g)
{
    int m = 1;
    while (rng_f(&g->rng) > 0.6 && m < 64) m++;   /* geometric(0.6) */
    return m;
}

/* one tx block: eob + coefficients in scan order */
static void gen_txb(Gen *g, int tx, int uv)
{
    const vp9h_synth_params *p = g->p;
    int n = 16 << (2 * tx), i, eob;
    int hb = p->bpp > 8;
    if (rng_f(&g->rng) < p->p_zero_eob) eob = 0;
    else eob = 1 + rng_int(&g->rng, MIN(n, 64));
    g->eobs = grow(g->eobs, &g->ce, g->ne + 1, 2, &g->err);
    if (g->err) return;
    g->eobs[g->ne++] = eob;
    g->coefs = grow(g->coefs, &g->cc, g->nc + (size_t) eob * 4, 1, &g->err);
    if (g->err) return;
    for (i = 0; i < eob; i++) {
        int v;
        if (p->coef_stress) {
            /* raw token values over the whole codable range (vp9block.c:879-901) */
            int maxv = hb ? (p->bpp == 12 ? (1 << 18) : (1 << 16)) + 66 : (1 << 14) + 66;
            v = rng_int(&g->rng, maxv) + 1;
        } else {
            v = (i + 1 < eob && rng_f(&g->rng) < 0.3) ? 0 : coef_mag(g);
        }
        if (rng_u64(&g->rng) & 1) v = -v;
        int q = g->qmul[g->seg][uv][i > 0];
        int32_t stored;
        if (tx == 3)
            stored = (int32_t) ((int) ((unsigned) v * (unsigned) q) / 2);   /* vp9block.c:915 */
        else
            stored = (int32_t) ((unsigned) v * (unsigned) q);               /* vp9block.c:917 */
        if (!hb) {
            int16_t s16 = (int16_t) stored;
            memcpy(g->coefs + g->nc, &s16, 2);
            g->nc += 2;
        } else {
            memcpy(g->coefs + g->nc, &stored, 4);
            g->nc += 4;
        }
    }
}

static void gen_block(Gen *g, int row, int col, int bl, int bp)
{
    const vp9h_synth_params *p = g->p;
    int bs = bl * 3 + bp;
    int w4 = vp9t_bwh[1][bs][0], h4 = vp9t_bwh[1][bs][1];
    vp9h_block b;
    int i;

    memset(&b, 0, sizeof(b));
    b.row = row; b.col = col; b.bs = bs;
    if (p->seg.enabled && p->seg.nseg > 1) b.seg_id = (uint8_t) rng_int(&g->rng, MIN(8, p->seg.nseg));
    g->seg = b.seg_id;
    b.intra = !p->inter || rng_f(&g->rng) < 0.1;
    b.skip = rng_f(&g->rng) < p->p_skip;
    b.tx = p->lossless ? 0 : rng_int(&g->rng, max_tx_for_bs[bs] + 1);
    b.uvtx = b.tx - ((p->ss_h && w4 * 2 == (1 << b.tx)) || (p->ss_v && h4 * 2 == (1 << b.tx)));
    if (b.intra) {
        for (i = 0; i < 4; i++) b.mode[i] = rng_int(&g->rng, 10);
        /* sub-8x8 replication, vp9block.c:222-258 */
        if (bs == VP9H_BS_8x4) { b.mode[1] = b.mode[0]; b.mode[3] = b.mode[2]; }
        else if (bs == VP9H_BS_4x8) { b.mode[2] = b.mode[0]; b.mode[3] = b.mode[1]; }
        else if (bs <= VP9H_BS_8x8) { b.mode[1] = b.mode[2] = b.mode[3] = b.mode[0]; }
        b.uvmode = rng_int(&g->rng, 10);
    } else {
        int nref = 1 + (p->compound && rng_f(&g->rng) < 0.3);
        b.comp = nref == 2;
        b.ref[0] = 0;
        b.ref[1] = 2;
        b.filter = p->bilinear ? VP9H_FILTER_BILINEAR : rng_int(&g->rng, 3);
        for (i = 0; i < 4; i++) {
            int k, m = rng_f(&g->rng) < 0.5 ? VP9H_NEWMV : VP9H_NEARESTMV + rng_int(&g->rng, 3);
            b.mode[i] = m;
            for (k = 0; k < 2; k++) {
                if (m == VP9H_ZEROMV) { b.mv[i][k][0] = b.mv[i][k][1] = 0; }
                else {
                    b.mv[i][k][0] = rng_int(&g->rng, 1025) - 512;
                    b.mv[i][k][1] = rng_int(&g->rng, 1025) - 512;
                }
            }
        }
        if (bs == VP9H_BS_8x4) {
            b.mode[1] = b.mode[0]; b.mode[3] = b.mode[2];
            memcpy(b.mv[1], b.mv[0], sizeof(b.mv[0])); memcpy(b.mv[3], b.mv[2], sizeof(b.mv[0]));
        } else if (bs == VP9H_BS_4x8) {
            b.mode[2] = b.mode[0]; b.mode[3] = b.mode[1];
            memcpy(b.mv[2], b.mv[0], sizeof(b.mv[0])); memcpy(b.mv[3], b.mv[1], sizeof(b.mv[0]));
        } else if (bs <= VP9H_BS_8x8) {
            for (i = 1; i < 4; i++) { b.mode[i] = b.mode[0]; memcpy(b.mv[i], b.mv[0], sizeof(b.mv[0])); }
        }
    }

    if (!b.skip) {
        /* tx blocks inside the frame, reference loop order (vp9block.c:1005-1127) */
        int pl, x, y;
        size_t ne0 = g->ne;
        int any = 0;
        for (pl = 0; pl < 3; pl++) {
            int tx = pl ? b.uvtx : b.tx, step = 1 << tx;
            int end_x = MIN(2 * (g->cols - col), w4 * 2), end_y = MIN(2 * (g->rows - row), h4 * 2);
            if (pl) { end_x >>= p->ss_h; end_y >>= p->ss_v; }
            for (y = 0; y < end_y; y += step)
                for (x = 0; x < end_x; x += step) {
                    gen_txb(g, tx, pl > 0);
                    if (g->err) return;
                    any |= g->eobs[g->ne - 1] != 0;
                }
        }
        /* vp9block.c:1310-1314: an inter block <= 8x8 without coefficients becomes skip */
        if (!any && bs <= VP9H_BS_8x8 && !b.intra) {
            b.skip = 1;
            g->ne = ne0;   /* all eobs were 0: no coefficients were written */
        }
    }
    g->blocks = grow(g->blocks, &g->cb, g->nb + 1, sizeof(vp9h_block), &g->err);
    if (g->err) return;
    g->blocks[g->nb++] = b;
}

/* decode_sb's partition walk (vp9.c:1115-1193) */
static void gen_sb(Gen *g, int row, int col, int bl)
{
    static const double p_split[3] = { 0.5, 0.5, 0.3 };
    int hbs = 4 >> bl, bp;
    if (g->err) return;
    if (bl == 3) {
        bp = rng_f(&g->rng) < 0.1 ? 1 + rng_int(&g->rng, 3) : 0;
        gen_block(g, row, col, bl, bp);
    } else if (col + hbs < g->cols) {
        if (row + hbs < g->rows) {
            if (rng_f(&g->rng) < p_split[bl]) bp = 3;
            else { double u = rng_f(&g->rng); bp = u < 0.6 ? 0 : u < 0.8 ? 1 : 2; }
            switch (bp) {
            case 0: gen_block(g, row, col, bl, bp); break;
            case 1: gen_block(g, row, col, bl, bp); gen_block(g, row + hbs, col, bl, bp); break;
            case 2: gen_block(g, row, col, bl, bp); gen_block(g, row, col + hbs, bl, bp); break;
            default:
                gen_sb(g, row, col, bl + 1);
                gen_sb(g, row, col + hbs, bl + 1);
                gen_sb(g, row + hbs, col, bl + 1);
                gen_sb(g, row + hbs, col + hbs, bl + 1);
            }
        } else if (rng_f(&g->rng) < 0.7) {
            gen_sb(g, row, col, bl + 1);
            gen_sb(g, row, col + hbs, bl + 1);
        } else {
            gen_block(g, row, col, bl, 1);
        }
    } else if (row + hbs < g->rows) {
        if (rng_f(&g->rng) < 0.7) {
            gen_sb(g, row, col, bl + 1);
            gen_sb(g, row + hbs, col, bl + 1);
        } else {
            gen_block(g, row, col, bl, 2);
        }
    } else {
        gen_sb(g, row, col, bl + 1);
    }
}

static int clip_u6(int v) { return v < 0 ? 0 : v > 63 ? 63 : v; }

void vp9hip_synth_defaults(vp9h_synth_params *p, int width, int height, int bpp)
{
    memset(p, 0, sizeof(*p));
    p->width = width; p->height = height; p->bpp = bpp;
    p->ss_h = p->ss_v = 1;
    p->q_idx = 60;
    p->filter_level = 36;
    p->p_skip = 0.2f;
    p->seed = 0x56503900ull;
}

int vp9hip_synth_frame(vp9h_frame *out, const vp9h_synth_params *p)
{
    Gen g;
    int row, col, tc, i, s;
    int bidx = p->bpp == 8 ? 0 : p->bpp == 10 ? 1 : 2;
    if (!out || !p || p->width <= 0 || p->height <= 0 ||
        (p->bpp != 8 && p->bpp != 10 && p->bpp != 12))
        return VP9HIP_EINVAL;
    memset(&g, 0, sizeof(g));
    memset(out, 0, sizeof(*out));
    g.p = p;
    g.rng.s = p->seed;
    g.cols = (p->width + 7) >> 3;
    g.rows = (p->height + 7) >> 3;
    g.sb_cols = (p->width + 63) >> 6;
    g.sb_rows = (p->height + 63) >> 6;
    /* per-segment dequantization (vp9.c:745-766): the alternate-q feature of segment s */
    for (s = 0; s < 8; s++) {
        int q = p->lossless ? 0 : p->q_idx;
        if (p->seg.enabled && ((p->seg.q_en >> s) & 1)) q = p->seg.abs_delta ? p->seg.q[s] : q + p->seg.q[s];
        q = q < 0 ? 0 : q > 255 ? 255 : q;
        g.qmul[s][0][0] = vp9t_dc_q[bidx][q];
        g.qmul[s][0][1] = vp9t_ac_q[bidx][q];
        g.qmul[s][1][0] = vp9t_dc_q[bidx][q];
        g.qmul[s][1][1] = vp9t_ac_q[bidx][q];
    }
    /* legal tile-column range (vp9.c:800-810) */
    {
        int lmin = 0, lmax = 0;
        while (g.sb_cols > (64 << lmin)) lmin++;
        while ((g.sb_cols >> lmax) >= 4) lmax++;
        lmax = lmax > 0 ? lmax - 1 : 0;
        if (p->log2_tile_cols < lmin || p->log2_tile_cols > (lmax > lmin ? lmax : lmin))
            return VP9HIP_EINVAL;
    }
    /* decode_tiles' loop order (vp9.c:1325-1395), one tile row */
    for (row = 0; row < g.rows && !g.err; row += 8)
        for (tc = 0; tc < (1 << p->log2_tile_cols); tc++) {
            int s0 = MIN((tc * g.sb_cols) >> p->log2_tile_cols, g.sb_cols) << 3;
            int s1 = MIN(((tc + 1) * g.sb_cols) >> p->log2_tile_cols, g.sb_cols) << 3;
            for (col = s0; col < s1; col += 8) gen_sb(&g, row, col, 0);
        }
    if (g.err) {
        free(g.blocks); free(g.eobs); free(g.coefs);
        return VP9HIP_ENOMEM;
    }
    out->width = p->width;
    out->height = p->height;
    out->bpp = p->bpp;
    out->ss_h = p->ss_h;
    out->ss_v = p->ss_v;
    out->keyframe = !p->inter;
    out->lossless = p->lossless;
    out->filter_level = p->lossless ? 0 : p->filter_level;
    out->sharpness = p->sharpness;
    out->log2_tile_cols = p->log2_tile_cols;
    /* lflvl (vp9.c:767-791): the segment's alternate LF level, then the ref / mode deltas
     * in effect (libvpx's defaults ref {1,0,-1,-1}, mode {0,0} unless given) */
    {
        static const int ref_def[4] = { 1, 0, -1, -1 }, mode_def[2] = { 0, 0 };
        const int *ref_delta = p->seg.lf_delta_update ? p->seg.lf_ref : ref_def;
        const int *mode_delta = p->seg.lf_delta_update ? p->seg.lf_mode : mode_def;
        const int sh = out->filter_level >= 32;
        for (s = 0; s < 8; s++) {
            int lvl = out->filter_level;
            if (p->seg.enabled && ((p->seg.lf_en >> s) & 1)) lvl = p->seg.abs_delta ? p->seg.lf[s] : lvl + p->seg.lf[s];
            lvl = clip_u6(lvl);
            out->lflvl[s][0][0] = out->lflvl[s][0][1] = clip_u6(lvl + ref_delta[0] * (1 << sh));
            for (i = 1; i < 4; i++)
                for (int m = 0; m < 2; m++)
                    out->lflvl[s][i][m] = clip_u6(lvl + (ref_delta[i] + mode_delta[m]) * (1 << sh));
        }
    }
    for (i = 0; i < 3; i++) { out->ref_w[i] = p->width; out->ref_h[i] = p->height; }
    out->nblocks = (uint32_t) g.nb;
    out->neobs = (uint32_t) g.ne;
    out->ncoefs = g.nc / (p->bpp > 8 ? 4 : 2);
    out->blocks = g.blocks;
    out->eobs = g.eobs;
    out->coefs = g.coefs;
    return 0;
}

void vp9hip_synth_free(vp9h_frame *f)
{
    if (!f) return;
    free((void *) f->blocks);
    free((void *) f->eobs);
    free((void *) f->coefs);
    f->blocks = NULL; f->eobs = NULL; f->coefs = NULL;
}
