/*
 * VP9 bitstream <-> pass-1 packet on the host (the entropy / bool
 * decoder and frame-level parse that stay on the host, in C).
 *
 * One syntax walker serves both directions. Decoding reads every syntax element from the
 * bool decoder and fills a vp9h_frame. Encoding walks a vp9h_frame and writes the same
 * elements, so a synthetic packet becomes a real bitstream (the IVF generator of SURVEY
 * 8(d)). The walker restates the reference's parse:
 *   uncompressed header      vp9.c:519-760 (decode_frame_header), get_sbits_inv :383
 *   compressed header        vp9.c:790-900 (tx mode, coefficient / skip updates),
 *                            update_prob + inv_recenter_nonneg vp9.c:389-457
 *   tiles                    vp9.c:1325-1395 (tile sizes, per-tile bool coders, SB order)
 *   partition                decode_sb, vp9.c:1115-1193
 *   block syntax             decode_mode, vp9block.c:80-290 (keyframe / intra-only path)
 *   contexts                 vp9block.c:700-735 (SET_CTXS), vp9.c:1720-1730 (per frame)
 *   coefficient tokens       decode_coeffs_b_generic vp9block.c:806-923, decode_coeffs
 *                            vp9block.c:965-1130 (non-zero contexts, merge / splat)
 *   bool coder               vpx_rac.h:34-135; the encoder is the RFC 6386 section 7 one
 * Scope of this version: keyframes and intra-only frames, profiles 0 and 2 (4:2:0,
 * 8/10/12-bit), segmentation parsed, forward probability updates parsed. Inter frames
 * and backward adaptation (refresh_frame_context with frame_parallel = 0) return
 * AVERROR(ENOSYS).
 */
#include <stdlib.h>
#include <string.h>

#include "../../../include/vp9hip.h"
#include "../vp9_tables.h"

#define MIN(a, b) ((a) < (b) ? (a) : (b))
#define MAX(a, b) ((a) > (b) ? (a) : (b))

/* ------------------------------------------------------------------ bool coder */
typedef struct BoolDec {
    const uint8_t *start, *p, *end;
    uint64_t value;      /* the next bits of the stream, left-aligned (bit 63 first) */
    int bits;            /* valid bits in value */
    uint32_t range;
    int pad;             /* zero bytes filled in past the end */
} BoolDec;

/* top the window up to >= 57 valid bits: 8 bytes at a time while the stream lasts */
static void bd_fill(BoolDec *d)
{
    if (d->end - d->p >= 8) {
        uint64_t be;
        memcpy(&be, d->p, 8);
        be = __builtin_bswap64(be);
        const int nbytes = (64 - d->bits) >> 3;
        if (nbytes < 8) be &= ~0ull << (64 - 8 * nbytes);
        d->value |= be >> d->bits;
        d->p += nbytes;
        d->bits += 8 * nbytes;
        return;
    }
    while (d->bits <= 56) {
        uint64_t byte = 0;
        if (d->p < d->end) byte = *d->p++;
        else d->pad++;
        d->value |= byte << (56 - d->bits);
        d->bits += 8;
    }
}

static void bd_init(BoolDec *d, const uint8_t *p, size_t n)
{
    d->start = d->p = p; d->end = p + n;
    d->value = 0; d->bits = 0; d->pad = 0;
    d->range = 255;
    bd_fill(d);
}

/* bytes the byte-serial coder of RFC 6386 7.3 (2-byte window, one byte per 8 shifts) would
 * have requested past the end: the vpx_rac_is_end test (vpx_rac.h:47-52) */
static int bd_overrun(const BoolDec *d)
{
    const int64_t shifted = 8 * ((int64_t) (d->p - d->start) + d->pad) - d->bits;
    const int64_t over = 2 + shifted / 8 - (int64_t) (d->end - d->start);
    return over > 0 ? (int) over : 0;
}

/* one bool (vpx_rac_get_prob, vpx_rac.h:87-110): compare the top byte with the split,
 * renormalise by the leading zeros of the range */
static inline __attribute__((always_inline)) int bd_read(BoolDec *d, int prob)
{
    if (d->bits < 16) bd_fill(d);
    const uint32_t split = 1 + (((d->range - 1) * (uint32_t) prob) >> 8);
    const uint64_t big = (uint64_t) split << 56;
    const int bit = d->value >= big;                 /* selects, not a branch: bits are noisy */
    d->range = bit ? d->range - split : split;
    d->value -= bit ? big : 0;
    const int sh = __builtin_clz(d->range) - 24;
    d->range <<= sh;
    d->value <<= sh;
    d->bits -= sh;
    return bit;
}

typedef struct BoolEnc {
    uint8_t *buf; size_t pos, cap;
    uint32_t range, bottom;
    int bit_count;
    int err;
} BoolEnc;

static void be_put(BoolEnc *e, uint8_t v)
{
    if (e->pos == e->cap) {
        size_t nc = e->cap ? 2 * e->cap : 4096;
        uint8_t *n = realloc(e->buf, nc);
        if (!n) { e->err = 1; return; }
        e->buf = n; e->cap = nc;
    }
    e->buf[e->pos++] = v;
}

static void be_init(BoolEnc *e) { memset(e, 0, sizeof(*e)); e->range = 255; e->bit_count = 24; }

static void be_carry(BoolEnc *e)
{
    size_t q = e->pos;
    while (q > 0 && e->buf[q - 1] == 255) e->buf[--q] = 0;
    if (q > 0) e->buf[q - 1]++;
}

static void be_write(BoolEnc *e, int prob, int bit)
{
    const uint32_t split = 1 + (((e->range - 1) * (uint32_t) prob) >> 8);
    if (bit) { e->bottom += split; e->range -= split; }
    else e->range = split;
    while (e->range < 128) {
        e->range <<= 1;
        if (e->bottom & (1u << 31)) be_carry(e);
        e->bottom <<= 1;
        if (!--e->bit_count) {
            be_put(e, (uint8_t) (e->bottom >> 24));
            e->bottom &= (1u << 24) - 1;
            e->bit_count = 8;
        }
    }
}

static void be_flush(BoolEnc *e)
{
    int c = e->bit_count;
    uint32_t v = e->bottom;
    if (c < 32 && (v & (1u << (32 - c)))) be_carry(e);
    v <<= c & 7;
    c >>= 3;
    while (--c >= 0) v <<= 8;
    for (c = 0; c < 4; c++) { be_put(e, (uint8_t) (v >> 24)); v <<= 8; }
}

/* one coder, either direction: bc_bool returns the bit read, or writes `bit` */
typedef struct BC { int enc; BoolDec d; BoolEnc e; } BC;

static inline __attribute__((always_inline)) int bc_bool(BC *c, int prob, int bit)
{
    if (c->enc) { be_write(&c->e, prob, bit); return bit; }
    return bd_read(&c->d, prob);
}
static inline __attribute__((always_inline)) int bc_bool_e(BC *c, const int enc, int prob, int bit)
{
    if (enc) { be_write(&c->e, prob, bit); return bit; }
    return bd_read(&c->d, prob);
}
static int bc_uint(BC *c, int bits, int v)
{
    int r = 0;
    while (bits--) r = (r << 1) | bc_bool(c, 128, (v >> bits) & 1);
    return r;
}

/* trees: node i has children t[i][0..1]; a child <= 0 is the leaf -symbol */
static int tree_path(const int8_t (*t)[2], int node, int sym, int *bits, int depth)
{
    for (int b = 0; b < 2; b++) {
        const int ch = t[node][b];
        bits[depth] = b;
        if (ch <= 0 ? -ch == sym : tree_path(t, ch, sym, bits, depth + 1) > 0)
            return ch <= 0 ? depth + 1 : tree_path(t, ch, sym, bits, depth + 1);
    }
    return -1;
}
static int bc_tree(BC *c, const int8_t (*t)[2], const uint8_t *probs, int sym)
{
    if (c->enc) {
        int bits[16], n = tree_path(t, 0, sym, bits, 0), i = 0;
        for (int k = 0; k < n; k++) { be_write(&c->e, probs[i], bits[k]); i = t[i][bits[k]]; }
        return sym;
    }
    int i = 0;
    do i = t[i][bd_read(&c->d, probs[i])]; while (i > 0);
    return -i;
}

/* VP9 trees (spec constants): partition NONE/H/V/SPLIT; intra modes V=0 H=1 DC=2 D45=3
 * D135=4 D117=5 D153=6 D63=7 D207=8 TM=9; segment ids 0..7 */
static const int8_t partition_tree[3][2] = { { -0, 1 }, { -1, 2 }, { -2, -3 } };
static const int8_t intramode_tree[9][2] = {
    { -2, 1 }, { -9, 2 }, { -0, 3 }, { 4, 6 }, { -1, 5 }, { -4, -5 }, { -3, 7 }, { -7, 8 }, { -6, -8 },
};
static const int8_t segment_tree[7][2] = { { 1, 2 }, { 3, 4 }, { 5, 6 }, { -0, -1 }, { -2, -3 }, { -4, -5 }, { -6, -7 } };

/* ------------------------------------------------------------------ bit writer / reader */
typedef struct Bits { uint8_t *buf; size_t cap; size_t bit; const uint8_t *in; size_t in_bits; int enc, err; } Bits;

static int bits_rw(Bits *b, int n, int v)
{
    int r = 0;
    for (int i = n - 1; i >= 0; i--) {
        int bit;
        if (b->enc) {
            const size_t byte = b->bit >> 3;
            if (byte >= b->cap) {
                size_t nc = b->cap ? 2 * b->cap : 64;
                uint8_t *p = realloc(b->buf, nc);
                if (!p) { b->err = 1; return 0; }
                memset(p + b->cap, 0, nc - b->cap);
                b->buf = p; b->cap = nc;
            }
            bit = (v >> i) & 1;
            if (bit) b->buf[byte] |= (uint8_t) (0x80 >> (b->bit & 7));
        } else {
            if (b->bit >= b->in_bits) { b->err = 1; return 0; }
            bit = (b->in[b->bit >> 3] >> (7 - (b->bit & 7))) & 1;
        }
        b->bit++;
        r = (r << 1) | bit;
    }
    return r;
}
/* get_sbits_inv (vp9.c:383): magnitude, then the sign bit */
static int bits_sinv(Bits *b, int n, int v)
{
    int m = bits_rw(b, n, v < 0 ? -v : v);
    return bits_rw(b, 1, v < 0) ? -m : m;
}

/* ------------------------------------------------------------------ frame state */
enum { P_TX32 = 179, P_TX16 = 185, P_TX8 = 189, P_SKIP = 191 };   /* ProbContext offsets (vp9dec.h:56-81) */
enum { TX_SEL = 4 };

typedef struct Probs {
    uint8_t p[311];                      /* ProbContext, flat */
    uint8_t coef[4][2][2][6][6][11];     /* 3 coded + 8 from the pareto model */
} Probs;

typedef struct Hdr {
    int profile, keyframe, intraonly, show, errorres, w, h, bpp, ss_h, ss_v;
    int refreshctx, parallel, ctxid, resetctx;
    int filter_level, sharpness, lf_delta_enabled, lf_ref[4], lf_mode[2];
    int qidx, ydc, uvdc, uvac, lossless;
    int seg_enabled, seg_update_map, seg_temporal, seg_abs, seg_pred[3];
    uint8_t seg_prob[7];
    int seg_q_en[8], seg_q[8], seg_lf_en[8], seg_lf[8], seg_ref_en[8], seg_ref[8], seg_skip[8];
    int log2_tile_cols, log2_tile_rows;
    int txmode;
    int qmul[8][2][2];                   /* [seg][y/uv][dc/ac] */
    uint8_t lflvl[8][4][2];
} Hdr;

typedef struct Walk {
    Hdr h;
    Probs pr;
    int cols, rows, sb_cols, sb_rows;
    /* above contexts, per frame (vp9.c:1720-1730) */
    uint8_t *a_part, *a_skip, *a_tx, *a_mode, *a_ynnz, *a_unnz, *a_vnnz;
    /* left contexts, per SB row of a tile */
    uint8_t l_part[8], l_skip[8], l_tx[8], l_mode[16], l_ynnz[16], l_unnz[16], l_vnnz[16];
    int tile_col_start;
    BC *c;
    /* packet being read (enc) or written (dec) */
    const vp9h_frame *in;
    uint32_t bi, ei;  uint64_t ci;       /* read cursors (enc) */
    vp9h_block *blocks; size_t nb, cb;
    uint16_t *eobs; size_t ne, ce;
    uint8_t *coefs; size_t nc, cc;       /* bytes */
    int err;
} Walk;

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

static void probs_default(Probs *pr)
{
    memcpy(pr->p, vp9t_default_probs, 311);
    for (int t = 0; t < 4; t++)
        for (int i = 0; i < 2; i++)
            for (int j = 0; j < 2; j++)
                for (int b = 0; b < 6; b++)
                    for (int k = 0; k < 6; k++) {
                        uint8_t *q = pr->coef[t][i][j][b][k];
                        memcpy(q, vp9t_default_coef_probs[t][i][j][b][k], 3);
                        memcpy(q + 3, vp9t_model_pareto8[q[2]], 8);
                    }
}

/* update_prob (vp9.c:399-457): sub-exponential delta, decoded or (encoder) never sent */
static int inv_recenter(int v, int m)
{
    if (v > 2 * m) return v;
    return (v & 1) ? m - ((v + 1) >> 1) : m + (v >> 1);
}
static const uint8_t inv_map[255] = {
    7, 20, 33, 46, 59, 72, 85, 98, 111, 124, 137, 150, 163, 176, 189, 202, 215, 228, 241, 254,
};
static uint8_t inv_map_at(int d)
{
    /* inv_map_table: the 20 coarse entries, then 1..253 without them (vp9.c:401-419) */
    if (d < 20) return inv_map[d];
    int v = 0, k = 19;
    for (int x = 1; x <= 253; x++) {
        if (x % 13 == 7 && x <= 254) continue;      /* 7, 20, 33, ... are the coarse values */
        if (++k == d) { v = x; break; }
    }
    return (uint8_t) (d == 254 ? 253 : v);
}
static int read_update_prob(BC *c, int p)
{
    int d;
    if (!bc_bool(c, 128, 0)) d = bc_uint(c, 4, 0);
    else if (!bc_bool(c, 128, 0)) d = bc_uint(c, 4, 0) + 16;
    else if (!bc_bool(c, 128, 0)) d = bc_uint(c, 5, 0) + 32;
    else {
        d = bc_uint(c, 7, 0);
        if (d >= 65) d = (d << 1) - 65 + bc_bool(c, 128, 0);
        d += 64;
    }
    if (d > 254) d = 254;
    const int m = inv_map_at(d);
    return p <= 128 ? 1 + inv_recenter(m, p - 1) : 255 - inv_recenter(m, 255 - p);
}
/* a probability that may be updated: flag with prob 252 (the encoder never updates) */
static void maybe_update(Walk *w, uint8_t *p)
{
    if (bc_bool(w->c, 252, 0)) *p = (uint8_t) read_update_prob(w->c, *p);
}

/* ------------------------------------------------------------------ coefficients */
static const int16_t *scan_of(int tx, int txtp)
{
    if (tx == 4) return vp9t_scan_default_4x4;
    switch (tx) {
    case 0: return txtp == 1 ? vp9t_scan_col_4x4 : txtp == 2 ? vp9t_scan_row_4x4 : vp9t_scan_default_4x4;
    case 1: return txtp == 1 ? vp9t_scan_col_8x8 : txtp == 2 ? vp9t_scan_row_8x8 : vp9t_scan_default_8x8;
    case 2: return txtp == 1 ? vp9t_scan_col_16x16 : txtp == 2 ? vp9t_scan_row_16x16 : vp9t_scan_default_16x16;
    default: return vp9t_scan_default_32x32;
    }
}
static const int16_t (*nb_of(int tx, int txtp))[2]
{
    if (tx == 4) return vp9t_nb_default_4x4;
    switch (tx) {
    case 0: return txtp == 1 ? vp9t_nb_col_4x4 : txtp == 2 ? vp9t_nb_row_4x4 : vp9t_nb_default_4x4;
    case 1: return txtp == 1 ? vp9t_nb_col_8x8 : txtp == 2 ? vp9t_nb_row_8x8 : vp9t_nb_default_8x8;
    case 2: return txtp == 1 ? vp9t_nb_col_16x16 : txtp == 2 ? vp9t_nb_row_16x16 : vp9t_nb_default_16x16;
    default: return vp9t_nb_default_32x32;
    }
}
/* ff_vp9_intra_txfm_type (vp9data.c:437-452), inter modes 10-13 -> DCT_DCT */
static const uint8_t intra_txtp[14] = { 2, 1, 0, 0, 3, 2, 1, 2, 1, 3, 0, 0, 0, 0 };

/* the CAT3-CAT6 extra-bit probabilities (decode_coeffs_b_generic) */
static const uint8_t cat6_probs[18] = { 255, 255, 255, 255, 254, 254, 254, 252, 249, 243, 230, 196, 177, 153, 140, 133, 130, 129 };

/* token magnitude + sign of coefficient i (encoder side: from the stored dequantized value) */
static int enc_value(const Walk *w, int stored, int q, int tx32)
{
    const int a = stored < 0 ? -stored : stored;
    if (!tx32) return q ? a / q : 0;
    /* stored = (val * q) / 2 truncated: val * q is 2a or 2a + 1 */
    if ((2 * a) % q == 0) return 2 * a / q;
    return (2 * a + 1) / q;
}

/* one tx block's tokens (decode_coeffs_b_generic, vp9block.c:806-923): returns the eob */
static inline __attribute__((always_inline)) int
walk_tokens_t(Walk *w, int n_coeffs, int tx32, const uint8_t (*p)[6][11], int nnz, const int16_t *scan,
              const int16_t (*nb)[2], const int16_t *band_counts, const int *qmul, int eob_in,
              const uint8_t *cin, int csz, const int enc)
{
    BC *c = w->c;
    const int bpp = w->h.bpp;
    int i = 0, band = 0, band_left = band_counts[0];
    const uint8_t *tp = p[0][nnz];
    uint8_t cache[1024];
    /* encoder: the values to send */
    int vals[1024];
    if (enc)
        for (int k = 0; k < eob_in; k++) {
            int32_t s;
            if (csz == 2) { int16_t t; memcpy(&t, cin + 2 * k, 2); s = t; } else memcpy(&s, cin + 4 * k, 4);
            const int v = enc_value(w, s, qmul[k > 0], tx32);
            vals[k] = s < 0 ? -v : v;
            /* the value must come back from the decoder's dequantization (8-bit packets
             * whose int16 coefficients wrapped are not representable) */
            const int32_t back = tx32 ? (int32_t) ((int) ((unsigned) vals[k] * (unsigned) qmul[k > 0]) / 2)
                                      : (int32_t) ((unsigned) vals[k] * (unsigned) qmul[k > 0]);
            if ((csz == 2 ? (int32_t) (int16_t) back : back) != s) { w->err = 1; return 0; }
        }
    const size_t c0 = w->nc;
    if (!enc) {
        w->coefs = grow(w->coefs, &w->cc, w->nc + (size_t) n_coeffs * csz, 1, &w->err);
        if (w->err) return 0;
    }
    do {
        /* more coefficients? */
        if (!bc_bool_e(c, enc, tp[0], i < eob_in)) break;
    skip_eob:
        {
            const int v = enc ? vals[i] : 0, av = v < 0 ? -v : v;
            if (!bc_bool_e(c, enc, tp[1], av != 0)) {                       /* ZERO */
                if (!--band_left) band_left = band_counts[++band];
                cache[scan[i]] = 0;
                nnz = (1 + cache[nb[i][0]] + cache[nb[i][1]]) >> 1;
                tp = p[band][nnz];
                if (!enc) {
                    if (csz == 2) { const int16_t z = 0; memcpy(w->coefs + c0 + (size_t) i * 2, &z, 2); }
                    else { const int32_t z = 0; memcpy(w->coefs + c0 + (size_t) i * 4, &z, 4); }
                }
                if (++i == n_coeffs) break;
                goto skip_eob;
            }
            const int rc = scan[i];
            int val;
            if (!bc_bool_e(c, enc, tp[2], av > 1)) { val = 1; cache[rc] = 1; }
            else if (!bc_bool_e(c, enc, tp[3], av > 4)) {
                if (!bc_bool_e(c, enc, tp[4], av > 2)) { val = 2; cache[rc] = 2; }
                else { val = 3 + bc_bool_e(c, enc, tp[5], av == 4); cache[rc] = 3; }
            } else if (!bc_bool_e(c, enc, tp[6], av > 10)) {
                cache[rc] = 4;
                if (!bc_bool_e(c, enc, tp[7], av > 6)) val = 5 + bc_bool_e(c, enc, 159, av == 6);
                else {
                    const int e = av - 7;
                    val = 7 + (bc_bool_e(c, enc, 165, (e >> 1) & 1) << 1);
                    val += bc_bool_e(c, enc, 145, e & 1);
                }
            } else {
                cache[rc] = 5;
                if (!bc_bool_e(c, enc, tp[8], av > 34)) {
                    if (!bc_bool_e(c, enc, tp[9], av > 18)) {
                        const int e = av - 11;
                        val = 11 + (bc_bool_e(c, enc, 173, (e >> 2) & 1) << 2);
                        val += bc_bool_e(c, enc, 148, (e >> 1) & 1) << 1;
                        val += bc_bool_e(c, enc, 140, e & 1);
                    } else {
                        const int e = av - 19;
                        val = 19 + (bc_bool_e(c, enc, 176, (e >> 3) & 1) << 3);
                        val += bc_bool_e(c, enc, 155, (e >> 2) & 1) << 2;
                        val += bc_bool_e(c, enc, 140, (e >> 1) & 1) << 1;
                        val += bc_bool_e(c, enc, 135, e & 1);
                    }
                } else if (!bc_bool_e(c, enc, tp[10], av > 66)) {
                    const int e = av - 35;
                    val = 35 + (bc_bool_e(c, enc, 180, (e >> 4) & 1) << 4);
                    val += bc_bool_e(c, enc, 157, (e >> 3) & 1) << 3;
                    val += bc_bool_e(c, enc, 141, (e >> 2) & 1) << 2;
                    val += bc_bool_e(c, enc, 134, (e >> 1) & 1) << 1;
                    val += bc_bool_e(c, enc, 130, e & 1);
                } else {
                    /* CAT6: 14 extra bits at 8-bit, 16 at 10-bit, 18 at 12-bit */
                    const int nbits = bpp == 12 ? 18 : bpp == 10 ? 16 : 14, e = av - 67;
                    val = 67;
                    for (int k = nbits - 1; k >= 0; k--) val += bc_bool_e(c, enc, cat6_probs[17 - k], (e >> k) & 1) << k;
                }
            }
            if (!--band_left) band_left = band_counts[++band];
            const int neg = bc_bool_e(c, enc, 128, v < 0);
            if (!enc) {
                const int32_t sv = neg ? -val : val;
                int32_t st = tx32 ? (int32_t) ((int) ((unsigned) sv * (unsigned) qmul[i > 0]) / 2)
                                  : (int32_t) ((unsigned) sv * (unsigned) qmul[i > 0]);
                if (csz == 2) { int16_t t = (int16_t) st; memcpy(w->coefs + c0 + (size_t) i * 2, &t, 2); }
                else memcpy(w->coefs + c0 + (size_t) i * 4, &st, 4);
            }
            nnz = (1 + cache[nb[i][0]] + cache[nb[i][1]]) >> 1;
            tp = p[band][nnz];
        }
    } while (++i < n_coeffs);
    if (!enc) w->nc += (size_t) i * csz;
    return i;
}

/* the walker's direction as a constant, so the decode loop carries no encoder branches */
static int walk_tokens(Walk *w, int n_coeffs, int tx32, const uint8_t (*p)[6][11], int nnz, const int16_t *scan,
                       const int16_t (*nb)[2], const int16_t *band_counts, const int *qmul, int eob_in,
                       const uint8_t *cin, int csz)
{
    if (w->c->enc)
        return walk_tokens_t(w, n_coeffs, tx32, p, nnz, scan, nb, band_counts, qmul, eob_in, cin, csz, 1);
    return walk_tokens_t(w, n_coeffs, tx32, p, nnz, scan, nb, band_counts, qmul, eob_in, cin, csz, 0);
}

static const int16_t band_counts[4][6] = {
    { 1, 2, 3, 4, 3, 16 - 13 }, { 1, 2, 3, 4, 11, 64 - 21 }, { 1, 2, 3, 4, 11, 256 - 21 }, { 1, 2, 3, 4, 11, 1024 - 21 },
};

/* merge (before) / splat (after) of the non-zero contexts of an n x n (step) tx grid */
static void nnz_merge(uint8_t *la, int end, int step)
{
    for (int n = 0; n < end; n += step) {
        int any = 0;
        for (int k = 0; k < step; k++) any |= la[n + k];
        la[n] = !!any;
    }
}
static void nnz_splat(uint8_t *la, int end, int full, int step)
{
    for (int n = 0; n < end; n += step) {
        const int m = full ? step - 1 : MIN(end - n - 1, step - 1);
        for (int k = 1; k <= m; k++) la[n + k] = la[n];
    }
}

/* decode_coeffs (vp9block.c:965-1130) for a keyframe / intra block */
static int walk_coeffs(Walk *w, vp9h_block *b, int row, int col)
{
    const int csz = w->h.bpp > 8 ? 4 : 2;
    const int lossless = w->h.lossless;
    const int tx = b->tx;
    const int w4 = vp9t_bwh[1][b->bs][0] << 1, h4 = vp9t_bwh[1][b->bs][1] << 1;
    const int end_x = MIN(2 * (w->cols - col), w4), end_y = MIN(2 * (w->rows - row), h4);
    const int (*qmul)[2] = w->h.qmul[b->seg_id];
    int total = 0;
    for (int pl = 0; pl < 3; pl++) {
        const int t = pl ? b->uvtx : tx, step = 1 << t;
        const int sh = pl ? w->h.ss_h : 0, sv = pl ? w->h.ss_v : 0;
        const int ex = end_x >> sh, ey = end_y >> sv, full_x = ex == (w4 >> sh), full_y = ey == (h4 >> sv);
        uint8_t *a = pl == 0 ? w->a_ynnz + col * 2 : (pl == 1 ? w->a_unnz : w->a_vnnz) + (col << !w->h.ss_h);
        uint8_t *l = pl == 0 ? w->l_ynnz + ((row & 7) << 1) : (pl == 1 ? w->l_unnz : w->l_vnnz) + ((row & 7) << !w->h.ss_v);
        const uint8_t (*p)[6][11] = (const uint8_t (*)[6][11]) w->pr.coef[t][pl > 0][!b->intra];
        if (step > 1) { nnz_merge(l, ey, step); nnz_merge(a, ex, step); }
        int n = 0;
        for (int y = 0; y < ey; y += step)
            for (int x = 0; x < ex; x += step, n += step * step) {
                const int mode = pl ? 0 : b->mode[b->bs > VP9H_BS_8x8 && t == 0 ? n : 0];
                const int txtp = pl ? 0 : intra_txtp[mode];
                const int tcode = lossless ? 4 : t;
                int eob_in = 0;
                const uint8_t *cin = NULL;
                if (w->c->enc) {
                    if (w->ei >= w->in->neobs) { w->err = 1; return 0; }
                    eob_in = w->in->eobs[w->ei++];
                    cin = (const uint8_t *) w->in->coefs + w->ci * csz;
                    w->ci += (uint64_t) eob_in;
                }
                const int eob = walk_tokens(w, 16 << (2 * t), t == 3, p, a[x] + l[y], scan_of(tcode, txtp),
                                            nb_of(tcode, txtp), band_counts[t], qmul[pl > 0], eob_in, cin, csz);
                if (!w->c->enc) {
                    w->eobs = grow(w->eobs, &w->ce, w->ne + 1, 2, &w->err);
                    if (w->err) return 0;
                    w->eobs[w->ne++] = (uint16_t) eob;
                }
                a[x] = l[y] = !!eob;
                total |= !!eob;
            }
        if (step > 1) { nnz_splat(a, ex, full_x, step); nnz_splat(l, ey, full_y, step); }
    }
    return total;
}

/* ------------------------------------------------------------------ block / partition */
static const uint8_t left_ctx_of[13] = { 0x0, 0x8, 0x0, 0x8, 0xc, 0x8, 0xc, 0xe, 0xc, 0xe, 0xf, 0xe, 0xf };
static const uint8_t above_ctx_of[13] = { 0x0, 0x0, 0x8, 0x8, 0x8, 0xc, 0xc, 0xc, 0xe, 0xe, 0xe, 0xf, 0xf };
static const uint8_t max_tx_of[13] = { 3, 3, 3, 3, 2, 2, 2, 1, 1, 1, 0, 0, 0 };

static void walk_block(Walk *w, int row, int col, int bl, int bp)
{
    BC *c = w->c;
    const Hdr *h = &w->h;
    vp9h_block b;
    const int bs = bl * 3 + bp;
    if (c->enc) {
        if (w->bi >= w->in->nblocks) { w->err = 1; return; }
        b = w->in->blocks[w->bi++];
        if (b.row != row || b.col != col || b.bs != bs) { w->err = 1; return; }
    } else {
        memset(&b, 0, sizeof(b));
        b.row = (uint16_t) row; b.col = (uint16_t) col; b.bs = (uint8_t) bs;
    }
    const int row7 = row & 7, max_tx = max_tx_of[bs];
    const int bw4 = vp9t_bwh[1][bs][0], bh4 = vp9t_bwh[1][bs][1];
    const int have_a = row > 0, have_l = col > w->tile_col_start;

    /* segment id (keyframe / intra-only: coded only with update_map) */
    b.seg_id = h->seg_enabled && h->seg_update_map ? (uint8_t) bc_tree(c, segment_tree, h->seg_prob, b.seg_id) : 0;
    /* skip */
    if (h->seg_enabled && h->seg_skip[b.seg_id]) b.skip = 1;
    else b.skip = (uint8_t) bc_bool(c, w->pr.p[P_SKIP + w->l_skip[row7] + w->a_skip[col]], b.skip);
    b.intra = 1;
    /* tx size */
    if (h->txmode == TX_SEL) {
        int cx;
        if (have_a) {
            if (have_l)
                cx = (w->a_skip[col] ? max_tx : w->a_tx[col]) + (w->l_skip[row7] ? max_tx : w->l_tx[row7]) > max_tx;
            else
                cx = w->a_skip[col] ? 1 : (w->a_tx[col] * 2 > max_tx);
        } else if (have_l) {
            cx = w->l_skip[row7] ? 1 : (w->l_tx[row7] * 2 > max_tx);
        } else {
            cx = 1;
        }
        int t = 0;
        const uint8_t *pp = w->pr.p;
        switch (max_tx) {
        case 3:
            t = bc_bool(c, pp[P_TX32 + cx * 3], b.tx > 0);
            if (t) { t += bc_bool(c, pp[P_TX32 + cx * 3 + 1], b.tx > 1); if (t == 2) t += bc_bool(c, pp[P_TX32 + cx * 3 + 2], b.tx > 2); }
            break;
        case 2:
            t = bc_bool(c, pp[P_TX16 + cx * 2], b.tx > 0);
            if (t) t += bc_bool(c, pp[P_TX16 + cx * 2 + 1], b.tx > 1);
            break;
        case 1: t = bc_bool(c, pp[P_TX8 + cx], b.tx > 0); break;
        default: t = 0;
        }
        b.tx = (uint8_t) t;
    } else {
        b.tx = (uint8_t) MIN(max_tx, h->txmode);
    }
    /* intra modes with above / left 4x4 mode contexts (keyframe probabilities) */
    uint8_t *a = w->a_mode + col * 2, *l = w->l_mode + (row7 << 1);
    if (bs > VP9H_BS_8x8) {
        b.mode[0] = a[0] = (uint8_t) bc_tree(c, intramode_tree, vp9t_kf_ymode_probs[a[0]][l[0]], b.mode[0]);
        if (bs != VP9H_BS_8x4) {
            b.mode[1] = (uint8_t) bc_tree(c, intramode_tree, vp9t_kf_ymode_probs[a[1]][b.mode[0]], b.mode[1]);
            l[0] = a[1] = b.mode[1];
        } else {
            l[0] = a[1] = b.mode[1] = b.mode[0];
        }
        if (bs != VP9H_BS_4x8) {
            b.mode[2] = a[0] = (uint8_t) bc_tree(c, intramode_tree, vp9t_kf_ymode_probs[a[0]][l[1]], b.mode[2]);
            if (bs != VP9H_BS_8x4) {
                b.mode[3] = (uint8_t) bc_tree(c, intramode_tree, vp9t_kf_ymode_probs[a[1]][b.mode[2]], b.mode[3]);
                l[1] = a[1] = b.mode[3];
            } else {
                l[1] = a[1] = b.mode[3] = b.mode[2];
            }
        } else {
            b.mode[2] = b.mode[0];
            l[1] = a[1] = b.mode[3] = b.mode[1];
        }
    } else {
        b.mode[0] = (uint8_t) bc_tree(c, intramode_tree, vp9t_kf_ymode_probs[*a][*l], b.mode[0]);
        b.mode[3] = b.mode[2] = b.mode[1] = b.mode[0];
        memset(a, b.mode[0], vp9t_bwh[0][bs][0]);
        memset(l, b.mode[0], vp9t_bwh[0][bs][1]);
    }
    b.uvmode = (uint8_t) bc_tree(c, intramode_tree, vp9t_kf_uvmode_probs[b.mode[3]], b.uvmode);
    b.uvtx = (uint8_t) (b.tx - ((h->ss_h && bw4 * 2 == (1 << b.tx)) || (h->ss_v && bh4 * 2 == (1 << b.tx))));

    /* contexts (SET_CTXS, vp9block.c:718-735) */
    memset(w->a_skip + col, b.skip, bw4); memset(w->l_skip + row7, b.skip, bh4);
    memset(w->a_tx + col, b.tx, bw4); memset(w->l_tx + row7, b.tx, bh4);
    memset(w->a_part + col, above_ctx_of[bs], bw4); memset(w->l_part + row7, left_ctx_of[bs], bh4);

    if (!c->enc) {
        w->blocks = grow(w->blocks, &w->cb, w->nb + 1, sizeof(vp9h_block), &w->err);
        if (w->err) return;
        w->blocks[w->nb++] = b;
    }
    if (!b.skip) {
        walk_coeffs(w, &b, row, col);
    } else {
        /* SPLAT_ZERO_YUV (vp9block.c:1313-1345): the whole block, unclipped */
        memset(w->a_ynnz + col * 2, 0, 2 * bw4); memset(w->l_ynnz + row7 * 2, 0, 2 * bh4);
        const int ux = w->h.ss_h ? bw4 : 2 * bw4, uy = w->h.ss_v ? bh4 : 2 * bh4;
        memset(w->a_unnz + (col << !w->h.ss_h), 0, ux); memset(w->a_vnnz + (col << !w->h.ss_h), 0, ux);
        memset(w->l_unnz + (row7 << !w->h.ss_v), 0, uy); memset(w->l_vnnz + (row7 << !w->h.ss_v), 0, uy);
    }
}

/* decode_sb (vp9.c:1115-1193) */
static void walk_sb(Walk *w, int row, int col, int bl)
{
    BC *c = w->c;
    if (w->err) return;
    const int ctx = ((w->a_part[col] >> (3 - bl)) & 1) | (((w->l_part[row & 7] >> (3 - bl)) & 1) << 1);
    const uint8_t *p = (w->h.keyframe || w->h.intraonly) ? vp9t_kf_partition_probs[bl][ctx]
                                                          : w->pr.p + 263 + (bl * 4 + ctx) * 3;
    const int hbs = 4 >> bl;
    int bp = 0;
    if (c->enc) {   /* the packet's next block says which partition this node takes */
        if (w->bi >= w->in->nblocks) { w->err = 1; return; }
        const vp9h_block *nb = &w->in->blocks[w->bi];
        const int nbl = nb->bs == VP9H_BS_4x4 ? 3 : nb->bs / 3;
        bp = (nb->row == row && nb->col == col && nbl == bl) ? nb->bs - 3 * bl : 3;
    }
    if (bl == 3) {
        bp = bc_tree(c, partition_tree, p, bp);
        walk_block(w, row, col, bl, bp);
    } else if (col + hbs < w->cols) {
        if (row + hbs < w->rows) {
            bp = bc_tree(c, partition_tree, p, bp);
            switch (bp) {
            case 0: walk_block(w, row, col, bl, bp); break;
            case 1: walk_block(w, row, col, bl, bp); walk_block(w, row + hbs, col, bl, bp); break;
            case 2: walk_block(w, row, col, bl, bp); walk_block(w, row, col + hbs, bl, bp); break;
            default:
                walk_sb(w, row, col, bl + 1); walk_sb(w, row, col + hbs, bl + 1);
                walk_sb(w, row + hbs, col, bl + 1); walk_sb(w, row + hbs, col + hbs, bl + 1);
            }
        } else if (bc_bool(c, p[1], bp == 3)) {
            walk_sb(w, row, col, bl + 1); walk_sb(w, row, col + hbs, bl + 1);
        } else {
            walk_block(w, row, col, bl, 1);
        }
    } else if (row + hbs < w->rows) {
        if (bc_bool(c, p[2], bp == 3)) { walk_sb(w, row, col, bl + 1); walk_sb(w, row + hbs, col, bl + 1); }
        else walk_block(w, row, col, bl, 2);
    } else {
        walk_sb(w, row, col, bl + 1);
    }
}

/* ------------------------------------------------------------------ headers */
static void set_qmul_lf(Walk *w)
{
    Hdr *h = &w->h;
    const int bidx = (h->bpp - 8) >> 1;
    for (int i = 0; i < (h->seg_enabled ? 8 : 1); i++) {
        int qyac = h->qidx, lvl = h->filter_level;
        if (h->seg_enabled && h->seg_q_en[i]) qyac = h->seg_abs ? h->seg_q[i] : h->qidx + h->seg_q[i];
        qyac = MAX(0, MIN(255, qyac));
        const int qydc = MAX(0, MIN(255, qyac + h->ydc)), quvdc = MAX(0, MIN(255, qyac + h->uvdc)),
                  quvac = MAX(0, MIN(255, qyac + h->uvac));
        h->qmul[i][0][0] = vp9t_dc_q[bidx][qydc];
        h->qmul[i][0][1] = vp9t_ac_q[bidx][qyac];
        h->qmul[i][1][0] = vp9t_dc_q[bidx][quvdc];
        h->qmul[i][1][1] = vp9t_ac_q[bidx][quvac];
        /* LF levels (vp9.c:767-791) */
        const int sh = h->filter_level >= 32;
        if (h->seg_enabled && h->seg_lf_en[i]) lvl = h->seg_abs ? h->seg_lf[i] : h->filter_level + h->seg_lf[i];
        lvl = MAX(0, MIN(63, lvl));
        for (int r = 0; r < 4; r++)
            for (int m = 0; m < 2; m++) {
                int v = lvl;
                if (h->lf_delta_enabled) v = lvl + (h->lf_ref[r] + (r ? h->lf_mode[m] : 0)) * (1 << sh);
                h->lflvl[i][r][m] = (uint8_t) MAX(0, MIN(63, v));
            }
    }
    for (int i = h->seg_enabled ? 8 : 1; i < 8; i++) {
        memcpy(h->qmul[i], h->qmul[0], sizeof(h->qmul[0]));
        memcpy(h->lflvl[i], h->lflvl[0], sizeof(h->lflvl[0]));
    }
}

/* uncompressed header (vp9.c:519-800), both directions. Returns the bit position of the
 * 16-bit compressed-header size, or -1. */
static long walk_uncompressed(Walk *w, Bits *b)
{
    Hdr *h = &w->h;
    if (bits_rw(b, 2, 2) != 2) return -1;                        /* frame marker */
    int prof = bits_rw(b, 1, h->profile & 1);
    prof |= bits_rw(b, 1, h->profile >> 1) << 1;
    if (prof == 3) prof += bits_rw(b, 1, 0);
    h->profile = prof;
    if (prof == 1 || prof == 3) return -2;                       /* 4:2:2 / 4:4:4: not here */
    if (bits_rw(b, 1, 0)) return -2;                             /* show_existing_frame */
    h->keyframe = !bits_rw(b, 1, !h->keyframe);
    h->show = bits_rw(b, 1, h->show);
    h->errorres = bits_rw(b, 1, h->errorres);
    if (h->keyframe) {
        if (bits_rw(b, 24, 0x498342) != 0x498342) return -1;     /* sync code */
        /* color config (read_colorspace_details): bit depth, color space, range */
        int bits = 0;
        if (prof >= 2) { bits = 1 + bits_rw(b, 1, h->bpp == 12); }
        h->bpp = 8 + 2 * bits;
        const int cs = bits_rw(b, 3, 2);                          /* BT709 */
        if (cs == 7) return -2;                                   /* sRGB: profile 1/3 only */
        bits_rw(b, 1, 0);                                         /* color range */
        h->ss_h = h->ss_v = 1;
        h->w = bits_rw(b, 16, h->w - 1) + 1;
        h->h = bits_rw(b, 16, h->h - 1) + 1;
        if (bits_rw(b, 1, 0)) bits_rw(b, 32, 0);                   /* render size */
    } else {
        h->intraonly = h->show ? 0 : bits_rw(b, 1, h->intraonly);
        h->resetctx = h->errorres ? 0 : bits_rw(b, 2, h->resetctx);
        if (!h->intraonly) return -2;                            /* inter frames: not in this version */
        if (bits_rw(b, 24, 0x498342) != 0x498342) return -1;
        if (prof >= 1) {
            int bits = 1 + bits_rw(b, 1, h->bpp == 12);
            h->bpp = 8 + 2 * bits;
            if (bits_rw(b, 3, 2) == 7) return -2;
            bits_rw(b, 1, 0);
        } else {
            h->bpp = 8;
        }
        h->ss_h = h->ss_v = 1;
        bits_rw(b, 8, 0xff);                                      /* refresh mask */
        h->w = bits_rw(b, 16, h->w - 1) + 1;
        h->h = bits_rw(b, 16, h->h - 1) + 1;
        if (bits_rw(b, 1, 0)) bits_rw(b, 32, 0);
    }
    h->refreshctx = h->errorres ? 0 : bits_rw(b, 1, h->refreshctx);
    h->parallel = h->errorres ? 1 : bits_rw(b, 1, h->parallel);
    h->ctxid = bits_rw(b, 2, 0);
    if (h->keyframe || h->intraonly) h->ctxid = 0;
    if (h->keyframe || h->errorres || h->intraonly) {
        h->lf_ref[0] = 1; h->lf_ref[1] = 0; h->lf_ref[2] = -1; h->lf_ref[3] = -1;
        h->lf_mode[0] = h->lf_mode[1] = 0;
    }
    h->filter_level = bits_rw(b, 6, h->filter_level);
    h->sharpness = bits_rw(b, 3, h->sharpness);
    if ((h->lf_delta_enabled = bits_rw(b, 1, h->lf_delta_enabled))) {
        if (bits_rw(b, 1, 0)) {                                  /* delta update */
            for (int i = 0; i < 4; i++) if (bits_rw(b, 1, 0)) h->lf_ref[i] = bits_sinv(b, 6, 0);
            for (int i = 0; i < 2; i++) if (bits_rw(b, 1, 0)) h->lf_mode[i] = bits_sinv(b, 6, 0);
        }
    }
    h->qidx = bits_rw(b, 8, h->qidx);
    h->ydc = bits_rw(b, 1, 0) ? bits_sinv(b, 4, 0) : 0;
    h->uvdc = bits_rw(b, 1, 0) ? bits_sinv(b, 4, 0) : 0;
    h->uvac = bits_rw(b, 1, 0) ? bits_sinv(b, 4, 0) : 0;
    h->lossless = h->qidx == 0 && !h->ydc && !h->uvdc && !h->uvac;
    if ((h->seg_enabled = bits_rw(b, 1, 0))) {
        if ((h->seg_update_map = bits_rw(b, 1, 0))) {
            for (int i = 0; i < 7; i++) h->seg_prob[i] = (uint8_t) (bits_rw(b, 1, 0) ? bits_rw(b, 8, 0) : 255);
            if ((h->seg_temporal = bits_rw(b, 1, 0)))
                for (int i = 0; i < 3; i++) h->seg_pred[i] = bits_rw(b, 1, 0) ? bits_rw(b, 8, 0) : 255;
        }
        if (bits_rw(b, 1, 0)) {
            h->seg_abs = bits_rw(b, 1, 0);
            for (int i = 0; i < 8; i++) {
                if ((h->seg_q_en[i] = bits_rw(b, 1, 0))) h->seg_q[i] = bits_sinv(b, 8, 0);
                if ((h->seg_lf_en[i] = bits_rw(b, 1, 0))) h->seg_lf[i] = bits_sinv(b, 6, 0);
                if ((h->seg_ref_en[i] = bits_rw(b, 1, 0))) h->seg_ref[i] = bits_rw(b, 2, 0);
                h->seg_skip[i] = bits_rw(b, 1, 0);
            }
        }
    }
    /* tiling (vp9.c:845-867) */
    w->cols = (h->w + 7) >> 3; w->rows = (h->h + 7) >> 3;
    w->sb_cols = (w->cols + 7) >> 3; w->sb_rows = (w->rows + 7) >> 3;
    int lmin = 0, lmax = 0;
    while (w->sb_cols > (64 << lmin)) lmin++;
    while ((w->sb_cols >> lmax) >= 4) lmax++;
    lmax = MAX(0, lmax - 1);
    int l2 = lmin;
    if (b->enc && (h->log2_tile_cols < lmin || h->log2_tile_cols > MAX(lmin, lmax))) return -1;
    while (lmax > l2) {
        if (bits_rw(b, 1, l2 < h->log2_tile_cols)) l2++;
        else break;
    }
    h->log2_tile_cols = l2;
    h->log2_tile_rows = bits_rw(b, 1, h->log2_tile_rows > 0);
    if (h->log2_tile_rows) h->log2_tile_rows += bits_rw(b, 1, h->log2_tile_rows > 1);
    set_qmul_lf(w);
    const long pos = (long) b->bit;
    bits_rw(b, 16, 0);                                            /* compressed header size */
    return pos;
}

/* compressed header (vp9.c:885-990, keyframe / intra-only part) */
static void walk_compressed(Walk *w)
{
    BC *c = w->c;
    Hdr *h = &w->h;
    bc_bool(c, 128, 0);                                           /* marker bit */
    if (h->lossless) h->txmode = 0;
    else {
        int m = bc_uint(c, 2, MIN(h->txmode, 3));
        if (m == 3) m += bc_bool(c, 128, h->txmode == TX_SEL);
        h->txmode = m;
        if (m == TX_SEL) {
            for (int i = 0; i < 2; i++) maybe_update(w, &w->pr.p[P_TX8 + i]);
            for (int i = 0; i < 4; i++) maybe_update(w, &w->pr.p[P_TX16 + i]);
            for (int i = 0; i < 6; i++) maybe_update(w, &w->pr.p[P_TX32 + i]);
        }
    }
    for (int t = 0; t < 4; t++) {
        if (bc_bool(c, 128, 0))
            for (int i = 0; i < 2; i++)
                for (int j = 0; j < 2; j++)
                    for (int k = 0; k < 6; k++)
                        for (int l = 0; l < 6; l++) {
                            if (l >= 3 && k == 0) break;          /* dc band: 3 contexts */
                            uint8_t *p = w->pr.coef[t][i][j][k][l];
                            for (int n = 0; n < 3; n++) maybe_update(w, &p[n]);
                            memcpy(p + 3, vp9t_model_pareto8[p[2]], 8);
                        }
        if (h->txmode == t) break;
    }
    for (int i = 0; i < 3; i++) maybe_update(w, &w->pr.p[P_SKIP + i]);
}

/* ------------------------------------------------------------------ frame walk */
static void tile_offsets(int idx, int log2n, int n, int *start, int *end)
{
    const int s0 = MIN((idx * n) >> log2n, n), s1 = MIN(((idx + 1) * n) >> log2n, n);
    *start = s0 * 8; *end = MIN(s1 * 8, 0x7fffffff);
}

static int alloc_ctx(Walk *w)
{
    const size_t n = (size_t) w->sb_cols * 8 + 16;
    w->a_part = calloc(n, 1); w->a_skip = calloc(n, 1); w->a_tx = calloc(n, 1);
    w->a_mode = calloc(2 * n, 1); w->a_ynnz = calloc(2 * n, 1); w->a_unnz = calloc(2 * n, 1); w->a_vnnz = calloc(2 * n, 1);
    if (!w->a_part || !w->a_skip || !w->a_tx || !w->a_mode || !w->a_ynnz || !w->a_unnz || !w->a_vnnz) return -1;
    memset(w->a_mode, 2 /* DC_PRED */, 2 * n);
    return 0;
}
static void free_ctx(Walk *w)
{
    free(w->a_part); free(w->a_skip); free(w->a_tx); free(w->a_mode); free(w->a_ynnz); free(w->a_unnz); free(w->a_vnnz);
}

/* Walk every tile (vp9.c:1325-1395): per tile row, SB rows, tile columns, SBs. */
static int walk_tiles(Walk *w, BC *coders)
{
    const int ntc = 1 << w->h.log2_tile_cols, ntr = 1 << w->h.log2_tile_rows;
    for (int tr = 0; tr < ntr; tr++) {
        int r0, r1;
        tile_offsets(tr, w->h.log2_tile_rows, w->sb_rows, &r0, &r1);
        for (int row = r0; row < r1; row += 8)
            for (int tc = 0; tc < ntc; tc++) {
                int c0, c1;
                tile_offsets(tc, w->h.log2_tile_cols, w->sb_cols, &c0, &c1);
                w->tile_col_start = c0;
                memset(w->l_part, 0, sizeof(w->l_part)); memset(w->l_skip, 0, sizeof(w->l_skip));
                memset(w->l_mode, 2, sizeof(w->l_mode));
                memset(w->l_ynnz, 0, sizeof(w->l_ynnz)); memset(w->l_unnz, 0, sizeof(w->l_unnz));
                memset(w->l_vnnz, 0, sizeof(w->l_vnnz)); memset(w->l_tx, 0, sizeof(w->l_tx));
                w->c = &coders[tr * ntc + tc];
                for (int col = c0; col < c1; col += 8) {
                    /* a tile whose data ran out is invalid (vp9.c:1383-1385) */
                    if (!w->c->enc && bd_overrun(&w->c->d) > 10) { w->err = 1; return -1; }
                    walk_sb(w, row, col, 0);
                    if (w->err) return -1;
                }
            }
    }
    return 0;
}

/* ------------------------------------------------------------------ API */
int vp9h_encode_frame(const vp9h_frame *pkt, int base_q_idx, uint8_t **out, size_t *out_size)
{
    if (!pkt || !out || !out_size || base_q_idx < 0 || base_q_idx > 255) return VP9HIP_EINVAL;
    if (!pkt->keyframe && !pkt->intraonly) return VP9HIP_ENOSYS;
    if (pkt->ss_h != 1 || pkt->ss_v != 1 || (pkt->bpp != 8 && pkt->bpp != 10 && pkt->bpp != 12)) return VP9HIP_ENOSYS;
    Walk w;
    memset(&w, 0, sizeof(w));
    Hdr *h = &w.h;
    h->profile = pkt->bpp > 8 ? 2 : 0;
    h->keyframe = pkt->keyframe; h->intraonly = pkt->intraonly && !pkt->keyframe;
    h->show = h->keyframe ? 1 : 0;
    h->w = pkt->width; h->h = pkt->height; h->bpp = pkt->bpp;
    h->refreshctx = 0; h->parallel = 1;
    h->resetctx = 3;                 /* intra-only: every decoder starts from the default probabilities */
    h->lf_delta_enabled = 1;         /* libvpx's default ref / mode deltas, as the packet's levels assume */
    h->filter_level = pkt->filter_level; h->sharpness = pkt->sharpness;
    h->qidx = pkt->lossless ? 0 : base_q_idx;
    h->log2_tile_cols = pkt->log2_tile_cols; h->log2_tile_rows = pkt->log2_tile_rows;
    h->txmode = pkt->lossless ? 0 : TX_SEL;
    w.in = pkt;
    probs_default(&w.pr);

    Bits b;
    memset(&b, 0, sizeof(b));
    b.enc = 1;
    const long szpos = walk_uncompressed(&w, &b);
    if (szpos < 0 || b.err) return szpos == -2 ? VP9HIP_ENOSYS : VP9HIP_EINVAL;
    if (h->lossless != !!pkt->lossless) return VP9HIP_EINVAL;
    /* compressed header */
    BC ch;
    memset(&ch, 0, sizeof(ch));
    ch.enc = 1;
    be_init(&ch.e);
    w.c = &ch;
    walk_compressed(&w);
    be_flush(&ch.e);
    /* tiles */
    const int ntc = 1 << h->log2_tile_cols, ntr = 1 << h->log2_tile_rows, nt = ntc * ntr;
    BC *coders = calloc((size_t) nt, sizeof(BC));
    int r = 0;
    if (!coders || alloc_ctx(&w) < 0) r = VP9HIP_ENOMEM;
    if (!r) {
        for (int i = 0; i < nt; i++) { coders[i].enc = 1; be_init(&coders[i].e); bc_bool(&coders[i], 128, 0); }
        if (walk_tiles(&w, coders) < 0 || w.bi != pkt->nblocks || w.ei != pkt->neobs || w.ci != pkt->ncoefs)
            r = VP9HIP_EINVALIDDATA;
    }
    size_t total = 0;
    if (!r) {
        for (int i = 0; i < nt; i++) { be_flush(&coders[i].e); if (coders[i].e.err) r = VP9HIP_ENOMEM; }
        if (ch.e.err || ch.e.pos > 0xffff) r = r ? r : VP9HIP_EINVAL;
    }
    if (!r) {
        /* the compressed header size, then byte alignment */
        const size_t hbytes = (size_t) ((szpos + 16 + 7) >> 3);
        b.bit = (size_t) szpos;
        bits_rw(&b, 16, (int) ch.e.pos);
        b.bit = hbytes * 8;
        total = hbytes + ch.e.pos;
        for (int i = 0; i < nt; i++) total += coders[i].e.pos + (i + 1 < nt ? 4 : 0);
        uint8_t *o = malloc(total);
        if (!o || b.err) r = VP9HIP_ENOMEM;
        else {
            size_t pos = 0;
            memcpy(o, b.buf, hbytes); pos = hbytes;
            memcpy(o + pos, ch.e.buf, ch.e.pos); pos += ch.e.pos;
            for (int i = 0; i < nt; i++) {
                const size_t n = coders[i].e.pos;
                if (i + 1 < nt) { o[pos] = (uint8_t) (n >> 24); o[pos + 1] = (uint8_t) (n >> 16); o[pos + 2] = (uint8_t) (n >> 8); o[pos + 3] = (uint8_t) n; pos += 4; }
                memcpy(o + pos, coders[i].e.buf, n); pos += n;
            }
            *out = o;
            *out_size = total;
        }
    }
    free(b.buf);
    free(ch.e.buf);
    if (coders) for (int i = 0; i < nt; i++) free(coders[i].e.buf);
    free(coders);
    free_ctx(&w);
    return r;
}

int vp9h_decode_frame(const uint8_t *data, size_t size, vp9h_frame *out)
{
    if (!data || !out || size < 3) return VP9HIP_EINVAL;
    memset(out, 0, sizeof(*out));
    Walk w;
    memset(&w, 0, sizeof(w));
    Bits b;
    memset(&b, 0, sizeof(b));
    b.in = data; b.in_bits = size * 8;
    const long szpos = walk_uncompressed(&w, &b);
    if (szpos == -2) return VP9HIP_ENOSYS;
    if (szpos < 0 || b.err) return VP9HIP_EINVALIDDATA;
    const Hdr *h = &w.h;
    if (h->refreshctx && !h->parallel) return VP9HIP_ENOSYS;    /* backward adaptation: not in this version */
    b.bit = (size_t) szpos;
    const size_t csize = (size_t) bits_rw(&b, 16, 0);
    const size_t hbytes = (size_t) ((szpos + 16 + 7) >> 3);
    if (hbytes + csize > size || !csize) return VP9HIP_EINVALIDDATA;
    probs_default(&w.pr);
    BC ch;
    memset(&ch, 0, sizeof(ch));
    bd_init(&ch.d, data + hbytes, csize);
    w.c = &ch;
    walk_compressed(&w);
    /* tiles */
    const int ntc = 1 << h->log2_tile_cols, ntr = 1 << h->log2_tile_rows, nt = ntc * ntr;
    BC *coders = calloc((size_t) nt, sizeof(BC));
    if (!coders || alloc_ctx(&w) < 0) { free(coders); free_ctx(&w); return VP9HIP_ENOMEM; }
    const uint8_t *p = data + hbytes + csize, *end = data + size;
    int r = 0;
    for (int i = 0; i < nt && !r; i++) {
        size_t n = (size_t) (end - p);
        if (i + 1 < nt) {
            if (end - p < 4) { r = VP9HIP_EINVALIDDATA; break; }
            n = (size_t) p[0] << 24 | (size_t) p[1] << 16 | (size_t) p[2] << 8 | p[3];
            p += 4;
            if (n > (size_t) (end - p)) { r = VP9HIP_EINVALIDDATA; break; }
        }
        bd_init(&coders[i].d, p, n);
        if (bc_bool(&coders[i], 128, 0)) r = VP9HIP_EINVALIDDATA;   /* marker bit */
        p += n;
    }
    if (!r && walk_tiles(&w, coders) < 0) r = w.err ? VP9HIP_EINVALIDDATA : VP9HIP_ENOMEM;
    free(coders);
    free_ctx(&w);
    if (r) { free(w.blocks); free(w.eobs); free(w.coefs); return r; }
    out->width = h->w; out->height = h->h; out->bpp = (uint8_t) h->bpp;
    out->ss_h = (uint8_t) h->ss_h; out->ss_v = (uint8_t) h->ss_v;
    out->keyframe = (uint8_t) h->keyframe; out->intraonly = (uint8_t) h->intraonly;
    out->lossless = (uint8_t) h->lossless;
    out->filter_level = (uint8_t) h->filter_level; out->sharpness = (uint8_t) h->sharpness;
    out->log2_tile_cols = (uint8_t) h->log2_tile_cols; out->log2_tile_rows = (uint8_t) h->log2_tile_rows;
    memcpy(out->lflvl, h->lflvl, sizeof(out->lflvl));
    out->nblocks = (uint32_t) w.nb; out->neobs = (uint32_t) w.ne;
    out->ncoefs = w.nc / (h->bpp > 8 ? 4 : 2);
    out->blocks = w.blocks; out->eobs = w.eobs; out->coefs = w.coefs;
    return 0;
}

void vp9h_frame_free(vp9h_frame *f)
{
    if (!f) return;
    free((void *) f->blocks); free((void *) f->eobs); free((void *) f->coefs);
    f->blocks = NULL; f->eobs = NULL; f->coefs = NULL;
}

void vp9h_buffer_free(uint8_t *p) { free(p); }
