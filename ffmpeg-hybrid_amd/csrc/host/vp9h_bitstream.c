/*
 * VP9 bitstream <-> pass-1 packet on the host (the entropy / bool
 * decoder, mode / MV decode and frame-level parse that stay on the host, in C).
 *
 * One syntax walker serves both directions. Decoding reads every syntax element from the
 * bool decoder and fills a vp9h_frame. Encoding walks a vp9h_frame and writes the same
 * elements, so a synthetic packet becomes a real bitstream (the IVF generator of SURVEY
 * 8(d)). A vp9h_stream carries what passes from frame to frame: the 4 saved probability
 * contexts, the 8 reference slots, the last frame's MV pairs and segmentation map, and the
 * persistent header fields. The walker restates the reference's parse:
 *   uncompressed header      vp9.c:519-880 (decode_frame_header), get_sbits_inv :383
 *   compressed header        vp9.c:903-1110 (tx mode, coefficient / mode / MV updates),
 *                            update_prob + inv_recenter_nonneg vp9.c:389-457
 *   frame state              vp9.c:1616-1686 (segmentation-map / MV-pair references),
 *                            1738-1752 (context save), 1821-1823 (adaptation)
 *   tiles                    vp9.c:1302-1395 (tile sizes, per-tile bool coders, SB order)
 *   partition                decode_sb, vp9.c:1115-1193
 *   block syntax             decode_mode, vp9block.c:80-803 (segment ids, skip, intra /
 *                            inter, tx size, intra modes, references, inter modes,
 *                            filters, contexts, MV pairs)
 *   motion vectors           find_ref_mvs / read_mv_component / ff_vp9_fill_mv, vp9mvs.c
 *   coefficient tokens       decode_coeffs_b_generic vp9block.c:806-923, decode_coeffs
 *                            vp9block.c:965-1130 (non-zero contexts, merge / splat)
 *   backward adaptation      ff_vp9_adapt_probs, vp9prob.c:25-290
 *   bool coder               vpx_rac.h:34-135; the encoder is the RFC 6386 section 7 one
 *   superframes              bsf/vp9_superframe_split.c:40-95
 * Scope: profiles 0-3 (4:2:0 / 4:2:2 / 4:4:0 / 4:4:4, 8/10/12-bit; RGB parses as 4:4:4).
 * The encoder never sends loop-filter delta updates or segmentation.
 */
#include <pthread.h>
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
        if (n < 0) c->e.err = 1;                      /* not a symbol of this tree */
        for (int k = 0; k < n; k++) { be_write(&c->e, probs[i], bits[k]); i = t[i][bits[k]]; }
        return sym;
    }
    int i = 0;
    do i = t[i][bd_read(&c->d, probs[i])]; while (i > 0);
    return -i;
}

/* bc_tree with the direction a constant (the walkers' _t forms): the decoder's tree walk inline */
static inline __attribute__((always_inline)) int bc_tree_e(BC *c, const int enc, const int8_t (*t)[2], const uint8_t *probs,
                                                           int sym)
{
    if (enc) return bc_tree(c, t, probs, sym);
    int i = 0;
    do i = t[i][bd_read(&c->d, probs[i])]; while (i > 0);
    return -i;
}

/* small context fills (SET_CTXS, vp9block.c:718-745, and the SPLAT / segment-map fills):
 * sizes 1, 2, 4, 8, 16 as one or two stores, as the reference's setctx_2d / AV_WN64A splats do;
 * a libc memset call per fill cost ~30 % of the single-thread parse (tools/parse_bench.c) */
typedef uint16_t __attribute__((may_alias, aligned(1))) u16_ua;
typedef uint32_t __attribute__((may_alias, aligned(1))) u32_ua;
typedef uint64_t __attribute__((may_alias, aligned(1))) u64_ua;
static inline __attribute__((always_inline)) void fill_ctx(uint8_t *p, int v, int n)
{
    const uint64_t x = 0x0101010101010101ull * (uint8_t) v;
    switch (n) {
    case 1: p[0] = (uint8_t) v; return;
    case 2: *(u16_ua *) p = (uint16_t) x; return;
    case 4: *(u32_ua *) p = (uint32_t) x; return;
    case 8: *(u64_ua *) p = x; return;
    default: memset(p, v, (size_t) n);
    }
}
/* the same for the non-zero contexts, whose fills reach 16 bytes */
static inline __attribute__((always_inline)) void fill_ctx16(uint8_t *p, int v, int n)
{
    if (n == 16) {
        const uint64_t x = 0x0101010101010101ull * (uint8_t) v;
        ((u64_ua *) p)[0] = x;
        ((u64_ua *) p)[1] = x;
    } else {
        fill_ctx(p, v, n);
    }
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


/* inter trees (vp9data.c): inter modes NEAREST=10 NEAR=11 ZERO=12 NEW=13; switchable
 * filter ids (0 regular, 1 smooth, 2 sharp); MV joint / class / fraction */
static const int8_t inter_mode_tree[3][2] = { { -12, 1 }, { -10, 2 }, { -11, -13 } };
static const int8_t filter_tree[2][2] = { { -0, 1 }, { -1, -2 } };
static const int8_t mv_joint_tree[3][2] = { { -0, 1 }, { -1, 2 }, { -2, -3 } };
static const int8_t mv_class_tree[10][2] = {
    { -0, 1 }, { -1, 2 }, { 3, 4 }, { -2, -3 }, { 5, 6 }, { -4, -5 }, { -6, 7 }, { 8, 9 }, { -7, -8 }, { -9, -10 },
};
static const int8_t mv_fp_tree[3][2] = { { -0, 1 }, { -1, 2 }, { -2, -3 } };
/* switchable filter id -> FilterMode (ff_vp9_filter_lut) and back */
static const uint8_t filter_of_id[3] = { VP9H_FILTER_REGULAR, VP9H_FILTER_SMOOTH, VP9H_FILTER_SHARP };
static const uint8_t id_of_filter[3] = { 1, 0, 2 };

/* ------------------------------------------------------------------ probabilities */
/* ProbContext (vp9dec.h:56-81); vp9t_default_probs is this struct's bytes */
typedef struct MvProbs {
    uint8_t sign, classes[10], class0, bits[10], class0_fp[2][3], fp[3], class0_hp, hp;
} MvProbs;
typedef struct PC {
    uint8_t y_mode[4][9], uv_mode[10][9], filter[4][2], mv_mode[7][3], intra[4], comp[5];
    uint8_t single_ref[5][2], comp_ref[5], tx32p[2][3], tx16p[2][2], tx8p[2], skip[3], mv_joint[3];
    MvProbs mv_comp[2];
    uint8_t partition[4][4][3];
} PC;
_Static_assert(sizeof(PC) == sizeof(vp9t_default_probs), "ProbContext layout");

/* the probabilities one frame decodes with: coefficient probabilities with the 8
 * pareto-model entries appended */
typedef struct Probs { PC p; uint8_t coef[4][2][2][6][6][11]; } Probs;
/* one of the 4 saved frame contexts (s->prob_ctx) */
typedef struct SavedCtx { PC p; uint8_t coef[4][2][2][6][6][3]; } SavedCtx;

/* symbol counts for backward adaptation (VP9TileData.counts, vp9dec.h:190-218) */
typedef struct Counts {
    unsigned y_mode[4][10], uv_mode[10][10], filter[4][3], mv_mode[7][4], intra[4][2], comp[5][2];
    unsigned single_ref[5][2][2], comp_ref[5][2], tx32p[2][4], tx16p[2][3], tx8p[2][2], skip[3][2];
    unsigned mv_joint[4];
    struct {
        unsigned sign[2], classes[11], class0[2], bits[10][2], class0_fp[2][4], fp[4], class0_hp[2], hp[2];
    } mv_comp[2];
    unsigned partition[4][4][4];
    unsigned coef[4][2][2][6][6][3];
    unsigned eob[4][2][2][6][6][2];
} Counts;

/* ------------------------------------------------------------------ frame / stream state */
typedef struct Mv { int16_t x, y; } Mv;
static inline uint32_t mv_bits(Mv m) { return (uint16_t) m.x | (uint32_t) (uint16_t) m.y << 16; }
/* VP9mvrefPair: per 8x8 of a frame, for MV prediction in this frame and the next */
typedef struct MvPair { Mv mv[2]; int8_t ref[2]; } MvPair;

/* a frame's side buffers (VP9Frame.extradata: segmentation map + MV pairs), shared by
 * reference between CUR_FRAME / REF_FRAME_MVPAIR / REF_FRAME_SEGMAP (vp9.c:110-165).
 * Row progress, as the reference's frame threads report it (ff_thread_report_progress,
 * vp9.c:1434; awaited at vp9mvs.c:177-178 and vp9block.c:116-117): rows_done[r] counts the
 * tile columns that have walked SB row r; the row is final at ntc. A frame whose walk
 * failed marks its side failed, so a frame reading it does not wait forever. */
typedef struct Side {
    int refs;                            /* atomic: frames of a pipelined parse share sides */
    int w, h, sb_cols, sb_rows;
    uint8_t *seg;
    MvPair *mv;
    int ntc;                             /* tile columns of the frame that writes it */
    int *rows_done;
    int failed;
    pthread_mutex_t mu;
    pthread_cond_t cv;
} Side;

static Side *side_new(int w, int h)
{
    Side *s = calloc(1, sizeof(*s));
    if (!s) return NULL;
    s->refs = 1; s->w = w; s->h = h;
    s->sb_cols = (w + 63) >> 6; s->sb_rows = (h + 63) >> 6;
    const size_t n = (size_t) s->sb_cols * s->sb_rows * 64;
    s->seg = calloc(n, 1);
    s->mv = calloc(n, sizeof(MvPair));
    s->rows_done = calloc((size_t) s->sb_rows, sizeof(int));
    s->ntc = 1;
    if (!s->seg || !s->mv || !s->rows_done) { free(s->seg); free(s->mv); free(s->rows_done); free(s); return NULL; }
    pthread_mutex_init(&s->mu, NULL);
    pthread_cond_init(&s->cv, NULL);
    return s;
}
static Side *side_ref(Side *s) { if (s) __atomic_add_fetch(&s->refs, 1, __ATOMIC_RELAXED); return s; }
static void side_unref(Side **p)
{
    Side *s = *p;
    *p = NULL;
    if (s && !__atomic_sub_fetch(&s->refs, 1, __ATOMIC_ACQ_REL)) {
        pthread_mutex_destroy(&s->mu);
        pthread_cond_destroy(&s->cv);
        free(s->seg); free(s->mv); free(s->rows_done); free(s);
    }
}
/* one tile column has walked SB row r (its MV pairs and segment ids are written) */
static void side_publish(Side *s, int r)
{
    if (__atomic_add_fetch(&s->rows_done[r], 1, __ATOMIC_ACQ_REL) >= s->ntc) {
        pthread_mutex_lock(&s->mu);
        pthread_cond_broadcast(&s->cv);
        pthread_mutex_unlock(&s->mu);
    }
}
static void side_fail(Side *s)
{
    if (!s) return;
    pthread_mutex_lock(&s->mu);
    __atomic_store_n(&s->failed, 1, __ATOMIC_RELEASE);
    pthread_cond_broadcast(&s->cv);
    pthread_mutex_unlock(&s->mu);
}
/* wait until SB row r is final; -1 if its frame failed */
static int side_wait(Side *s, int r)
{
    if (r >= s->sb_rows) r = s->sb_rows - 1;
    if (__atomic_load_n(&s->rows_done[r], __ATOMIC_ACQUIRE) >= s->ntc) return 0;
    pthread_mutex_lock(&s->mu);
    while (__atomic_load_n(&s->rows_done[r], __ATOMIC_ACQUIRE) < s->ntc && !__atomic_load_n(&s->failed, __ATOMIC_ACQUIRE))
        pthread_cond_wait(&s->cv, &s->mu);
    const int ok = __atomic_load_n(&s->rows_done[r], __ATOMIC_ACQUIRE) >= s->ntc;
    pthread_mutex_unlock(&s->mu);
    return ok ? 0 : -1;
}

enum { P_SINGLE = 0, P_COMP = 1, P_SWITCH = 2 };     /* comppredmode */
enum { TX_SEL = 4 };
enum { FILTER_SWITCHABLE = 4 };

typedef struct SegFeat { int q_en, q, lf_en, lf, ref_en, ref, skip; } SegFeat;

/* the frame header (s->s.h), persistent across frames like the reference's */
typedef struct Hdr {
    int profile, keyframe, intraonly, invisible, errorres, w, h, bpp, ss_h, ss_v;
    int resetctx, refreshmask, refidx[3], signbias[3];
    int hp, filtermode, allowcomp, fixcompref, varcompref[2];
    int refreshctx, parallel, ctxid, ctxid_raw;
    int filter_level, sharpness, lf_delta_enabled, lf_ref[4], lf_mode[2];
    int qidx, ydc, uvdc, uvac, lossless;
    int seg_enabled, seg_update_map, seg_temporal, seg_update_data, seg_abs;
    uint8_t seg_prob[7], seg_pred[3];
    SegFeat seg[8];
    int log2_tile_cols, log2_tile_rows;
    int txmode, comppred;
    int use_last_mvs;
    int qmul[8][2][2];                   /* [seg][y/uv][dc/ac] */
    uint8_t lflvl[8][4][2];
} Hdr;

struct vp9h_stream {
    int tile_threads;                    /* decode: tile columns walked concurrently (1: serial) */
    Hdr h;
    SavedCtx ctx[4];
    struct { int valid, w, h, bpp, ss_h, ss_v; } slot[8];
    int last_keyframe;
    Side *cur;                           /* CUR_FRAME: the last decoded frame */
    Side *segref;                        /* REF_FRAME_SEGMAP */
};

static void ctx_reset(SavedCtx *c)
{
    memcpy(&c->p, vp9t_default_probs, sizeof(c->p));
    memcpy(c->coef, vp9t_default_coef_probs, sizeof(c->coef));
}

int vp9h_stream_open(vp9h_stream **out)
{
    if (!out) return VP9HIP_EINVAL;
    vp9h_stream *s = calloc(1, sizeof(*s));
    if (!s) return VP9HIP_ENOMEM;
    for (int i = 0; i < 4; i++) ctx_reset(&s->ctx[i]);
    s->h.sharpness = -1;
    s->tile_threads = 1;
    *out = s;
    return 0;
}

void vp9h_stream_close(vp9h_stream *s)
{
    if (!s) return;
    side_unref(&s->cur);
    side_unref(&s->segref);
    free(s);
}

/* ------------------------------------------------------------------ walk state */
typedef struct Walk {
    vp9h_stream *st;
    Hdr *h;
    Probs pr;
    Counts cnt;
    int cols, rows, sb_cols, sb_rows;
    /* above contexts, per frame (vp9.c:1720-1730, vp9dec.h above_*_ctx) */
    uint8_t *a_part, *a_skip, *a_tx, *a_mode, *a_ynnz, *a_unnz, *a_vnnz;
    uint8_t *a_segpred, *a_intra, *a_comp, *a_ref, *a_filter;
    Mv (*a_mv)[2];
    /* left contexts, per SB row of a tile */
    uint8_t l_part[8], l_skip[8], l_tx[8], l_mode[16], l_ynnz[16], l_unnz[16], l_vnnz[16];
    uint8_t l_segpred[8], l_intra[8], l_comp[8], l_ref[8], l_filter[8];
    Mv l_mv[16][2];
    int tile_col_start;
    int minx, miny, maxx, maxy;          /* MV clamp of the current block (vp9block.c:1281-1284) */
    BC *c;
    Side *side;                          /* this frame's seg map + MV pairs */
    Side *mvref;                         /* REF_FRAME_MVPAIR */
    Side *segref;                        /* REF_FRAME_SEGMAP */
    /* encoder: the packet being written, its read cursors, the update policy */
    const vp9h_frame *in;
    uint32_t bi, ei;  uint64_t ci;
    uint64_t rng;
    int prob_updates, keep_modes;
    const vp9h_seg_params *eseg;         /* segment features / LF deltas to write */
    int last_keyframe, last_invisible;   /* the previous frame's header flags */
    Hdr hs;                              /* pipelined parse: the header as of this frame */
    int32_t ref_w[3], ref_h[3];          /* reference sizes at this frame's header */
    /* output packet (decoded, or as coded by the encoder) */
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

static uint32_t rng_next(Walk *w)
{   /* splitmix64 (encoder update policy only) */
    uint64_t z = (w->rng += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return (uint32_t) ((z ^ (z >> 31)) >> 32);
}

/* ------------------------------------------------------------------ forward updates */
/* update_prob (vp9.c:389-457): a sub-exponential index d, remapped through inv_map_table
 * and recentred on the old probability */
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
static int prob_of_delta(int p, int d)
{
    const int m = inv_map_at(d);
    return p <= 128 ? 1 + inv_recenter(m, p - 1) : 255 - inv_recenter(m, 255 - p);
}
/* the index d the encoder sends for `target`, or -1 */
static int delta_of_prob(int p, int target)
{
    for (int d = 0; d <= 253; d++)
        if (prob_of_delta(p, d) == target) return d;
    return -1;
}
static int walk_update_prob(BC *c, int p, int target)
{
    const int d0 = c->enc ? delta_of_prob(p, target) : 0;
    int d;
    if (!bc_bool(c, 128, d0 >= 16)) d = bc_uint(c, 4, d0);
    else if (!bc_bool(c, 128, d0 >= 32)) d = bc_uint(c, 4, d0 - 16) + 16;
    else if (!bc_bool(c, 128, d0 >= 64)) d = bc_uint(c, 5, d0 - 32) + 32;
    else {
        const int e = d0 - 64;
        d = bc_uint(c, 7, e < 65 ? e : (e + 65) >> 1);
        if (d >= 65) d = (d << 1) - 65 + bc_bool(c, 128, (e + 65) & 1);
        d += 64;
    }
    if (d > 254) d = 254;
    return prob_of_delta(p, d);
}
/* the encoder's update decision: a new probability, or -1 for none */
static int want_update(Walk *w, int p)
{
    if (!w->c->enc || !w->prob_updates || (rng_next(w) & 7)) return -1;
    for (int tries = 0; tries < 8; tries++) {
        const int t = 1 + (int) (rng_next(w) % 255);
        if (t != p && delta_of_prob(p, t) >= 0) return t;
    }
    return -1;
}
/* a probability that may be updated: flag with prob 252 (vpx_rac_get_prob_branchy) */
static void maybe_update(Walk *w, uint8_t *p)
{
    const int t = want_update(w, *p);
    if (bc_bool(w->c, 252, t >= 0)) *p = (uint8_t) walk_update_prob(w->c, *p, t);
}
/* MV probabilities: a literal 7-bit value (vp9.c:1063-1106) */
static void maybe_update_mv(Walk *w, uint8_t *p)
{
    int t = want_update(w, *p);
    if (t >= 0) t |= 1;
    if (bc_bool(w->c, 252, t >= 0)) *p = (uint8_t) ((bc_uint(w->c, 7, t >> 1) << 1) | 1);
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

/* token magnitude of a stored (dequantized) coefficient, encoder side */
static int enc_value(int stored, int q, int tx32)
{
    const int a = stored < 0 ? -stored : stored;
    if (!tx32) return q ? a / q : 0;
    /* stored = (val * q) / 2 truncated: val * q is 2a or 2a + 1 */
    if ((2 * a) % q == 0) return 2 * a / q;
    return (2 * a + 1) / q;
}

/* one tx block's tokens (decode_coeffs_b_generic, vp9block.c:806-923): returns the eob.
 * cnt / eobc are the coefficient / more-coefficients counts of this tx size and plane. */
static inline __attribute__((always_inline)) int
walk_tokens_t(Walk *w, int n_coeffs, int tx32, const uint8_t (*p)[6][11], int nnz, const int16_t *scan,
              const int16_t (*nb)[2], const int16_t *band_counts, const int *qmul, int eob_in,
              const uint8_t *cin, int csz, unsigned (*cnt)[6][3], unsigned (*eobc)[6][2], const int enc)
{
    BC *c = w->c;
    const int bpp = w->h->bpp;
    int i = 0, band = 0, band_left = band_counts[0];
    const uint8_t *tp = p[0][nnz];
    uint8_t cache[1024];
    /* encoder: the values to send */
    int vals[1024];
    if (enc)
        for (int k = 0; k < eob_in; k++) {
            int32_t s;
            if (csz == 2) { int16_t t; memcpy(&t, cin + 2 * k, 2); s = t; } else memcpy(&s, cin + 4 * k, 4);
            const int v = enc_value(s, qmul[k > 0], tx32);
            vals[k] = s < 0 ? -v : v;
            /* the value must come back from the decoder's dequantization (8-bit packets
             * whose int16 coefficients wrapped are not representable) */
            const int32_t back = tx32 ? (int32_t) ((int) ((unsigned) vals[k] * (unsigned) qmul[k > 0]) / 2)
                                      : (int32_t) ((unsigned) vals[k] * (unsigned) qmul[k > 0]);
            if ((csz == 2 ? (int32_t) (int16_t) back : back) != s) { w->err = 1; return 0; }
        }
    /* the first "more coefficients?" before the output is grown: most tx blocks of a
     * realistic stream stop here (eob 0) */
    const int more0 = bc_bool_e(c, enc, tp[0], 0 < eob_in);
    eobc[0][nnz][more0]++;
    if (!more0) return 0;
    const size_t c0 = w->nc;
    w->coefs = grow(w->coefs, &w->cc, w->nc + (size_t) n_coeffs * csz, 1, &w->err);
    if (w->err) return 0;
    goto skip_eob;
    do {
        /* more coefficients? */
        const int more = bc_bool_e(c, enc, tp[0], i < eob_in);
        eobc[band][nnz][more]++;
        if (!more) break;
    skip_eob:
        {
            const int v = enc ? vals[i] : 0, av = v < 0 ? -v : v;
            if (!bc_bool_e(c, enc, tp[1], av != 0)) {                       /* ZERO */
                cnt[band][nnz][0]++;
                if (!--band_left) band_left = band_counts[++band];
                cache[scan[i]] = 0;
                nnz = (1 + cache[nb[i][0]] + cache[nb[i][1]]) >> 1;
                tp = p[band][nnz];
                if (csz == 2) { const int16_t z = 0; memcpy(w->coefs + c0 + (size_t) i * 2, &z, 2); }
                else { const int32_t z = 0; memcpy(w->coefs + c0 + (size_t) i * 4, &z, 4); }
                if (++i == n_coeffs) break;
                goto skip_eob;
            }
            const int rc = scan[i];
            int val;
            if (!bc_bool_e(c, enc, tp[2], av > 1)) { val = 1; cache[rc] = 1; cnt[band][nnz][1]++; }
            else {
                cnt[band][nnz][2]++;
                if (!bc_bool_e(c, enc, tp[3], av > 4)) {
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
            }
            if (!--band_left) band_left = band_counts[++band];
            const int neg = bc_bool_e(c, enc, 128, v < 0);
            const int32_t sv = neg ? -val : val;
            int32_t st = tx32 ? (int32_t) ((int) ((unsigned) sv * (unsigned) qmul[i > 0]) / 2)
                              : (int32_t) ((unsigned) sv * (unsigned) qmul[i > 0]);
            if (csz == 2) { int16_t t = (int16_t) st; memcpy(w->coefs + c0 + (size_t) i * 2, &t, 2); }
            else memcpy(w->coefs + c0 + (size_t) i * 4, &st, 4);
            nnz = (1 + cache[nb[i][0]] + cache[nb[i][1]]) >> 1;
            tp = p[band][nnz];
        }
    } while (++i < n_coeffs);
    w->nc += (size_t) i * csz;
    return i;
}
/* the walker's direction as a constant, so the decode loop carries no encoder branches */
static int walk_tokens(Walk *w, int n_coeffs, int tx32, const uint8_t (*p)[6][11], int nnz, const int16_t *scan,
                       const int16_t (*nb)[2], const int16_t *band_counts, const int *qmul, int eob_in,
                       const uint8_t *cin, int csz, unsigned (*cnt)[6][3], unsigned (*eobc)[6][2])
{
    if (w->c->enc)
        return walk_tokens_t(w, n_coeffs, tx32, p, nnz, scan, nb, band_counts, qmul, eob_in, cin, csz, cnt, eobc, 1);
    return walk_tokens_t(w, n_coeffs, tx32, p, nnz, scan, nb, band_counts, qmul, eob_in, cin, csz, cnt, eobc, 0);
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

/* decode_coeffs (vp9block.c:965-1130): returns whether any tx block has coefficients */
static inline __attribute__((always_inline)) int walk_coeffs_t(Walk *w, vp9h_block *b, int row, int col, const int enc)
{
    const int csz = w->h->bpp > 8 ? 4 : 2;
    const int lossless = w->h->lossless;
    const int tx = b->tx;
    const int w4 = vp9t_bwh[1][b->bs][0] << 1, h4 = vp9t_bwh[1][b->bs][1] << 1;
    const int end_x = MIN(2 * (w->cols - col), w4), end_y = MIN(2 * (w->rows - row), h4);
    const int (*qmul)[2] = w->h->qmul[b->seg_id];
    int total = 0;
    for (int pl = 0; pl < 3; pl++) {
        const int t = pl ? b->uvtx : tx, step = 1 << t;
        const int sh = pl ? w->h->ss_h : 0, sv = pl ? w->h->ss_v : 0;
        const int ex = end_x >> sh, ey = end_y >> sv, full_x = ex == (w4 >> sh), full_y = ey == (h4 >> sv);
        uint8_t *a = pl == 0 ? w->a_ynnz + col * 2 : (pl == 1 ? w->a_unnz : w->a_vnnz) + (col << !w->h->ss_h);
        uint8_t *l = pl == 0 ? w->l_ynnz + ((row & 7) << 1) : (pl == 1 ? w->l_unnz : w->l_vnnz) + ((row & 7) << !w->h->ss_v);
        const uint8_t (*p)[6][11] = (const uint8_t (*)[6][11]) w->pr.coef[t][pl > 0][!b->intra];
        unsigned (*cnt)[6][3] = w->cnt.coef[t][pl > 0][!b->intra];
        unsigned (*eobc)[6][2] = w->cnt.eob[t][pl > 0][!b->intra];
        if (step > 1) { nnz_merge(l, ey, step); nnz_merge(a, ex, step); }
        int n = 0;
        for (int y = 0; y < ey; y += step)
            for (int x = 0; x < ex; x += step, n += step * step) {
                const int mode = pl ? 0 : b->mode[b->bs > VP9H_BS_8x8 && t == 0 ? n : 0];
                const int txtp = pl ? 0 : intra_txtp[mode];
                const int tcode = lossless ? 4 : t;
                int eob_in = 0;
                const uint8_t *cin = NULL;
                if (enc) {
                    if (w->ei >= w->in->neobs) { w->err = 1; return 0; }
                    eob_in = w->in->eobs[w->ei++];
                    cin = (const uint8_t *) w->in->coefs + w->ci * csz;
                    w->ci += (uint64_t) eob_in;
                }
                const int eob = walk_tokens_t(w, 16 << (2 * t), t == 3, p, a[x] + l[y], scan_of(tcode, txtp),
                                            nb_of(tcode, txtp), band_counts[t], qmul[pl > 0], eob_in, cin, csz,
                                            cnt, eobc, enc);
                if (w->err) return 0;
                w->eobs = grow(w->eobs, &w->ce, w->ne + 1, 2, &w->err);
                if (w->err) return 0;
                w->eobs[w->ne++] = (uint16_t) eob;
                a[x] = l[y] = !!eob;
                total |= !!eob;
            }
        if (step > 1) { nnz_splat(a, ex, full_x, step); nnz_splat(l, ey, full_y, step); }
    }
    return total;
}

/* ------------------------------------------------------------------ motion vectors */
/* find_ref_mvs (vp9mvs.c:37-275): candidate idx (0 nearest, 1 near) of reference `ref`
 * for sub-block sb (-1: the whole block) of b, whose MVs of earlier sub-blocks are set */
static const int8_t mv_ref_blk_off[13][8][2] = {
    { { 3, -1 }, { -1, 3 }, { 4, -1 }, { -1, 4 }, { -1, -1 }, { 0, -1 }, { -1, 0 }, { 6, -1 } },
    { { 0, -1 }, { -1, 0 }, { 4, -1 }, { -1, 2 }, { -1, -1 }, { 0, -3 }, { -3, 0 }, { 2, -1 } },
    { { -1, 0 }, { 0, -1 }, { -1, 4 }, { 2, -1 }, { -1, -1 }, { -3, 0 }, { 0, -3 }, { -1, 2 } },
    { { 1, -1 }, { -1, 1 }, { 2, -1 }, { -1, 2 }, { -1, -1 }, { 0, -3 }, { -3, 0 }, { -3, -3 } },
    { { 0, -1 }, { -1, 0 }, { 2, -1 }, { -1, -1 }, { -1, 1 }, { 0, -3 }, { -3, 0 }, { -3, -3 } },
    { { -1, 0 }, { 0, -1 }, { -1, 2 }, { -1, -1 }, { 1, -1 }, { -3, 0 }, { 0, -3 }, { -3, -3 } },
    { { 0, -1 }, { -1, 0 }, { 1, -1 }, { -1, 1 }, { -1, -1 }, { 0, -3 }, { -3, 0 }, { -3, -3 } },
    { { 0, -1 }, { -1, 0 }, { 1, -1 }, { -1, -1 }, { 0, -2 }, { -2, 0 }, { -2, -1 }, { -1, -2 } },
    { { -1, 0 }, { 0, -1 }, { -1, 1 }, { -1, -1 }, { -2, 0 }, { 0, -2 }, { -1, -2 }, { -2, -1 } },
    { { 0, -1 }, { -1, 0 }, { -1, -1 }, { 0, -2 }, { -2, 0 }, { -1, -2 }, { -2, -1 }, { -2, -2 } },
    { { 0, -1 }, { -1, 0 }, { -1, -1 }, { 0, -2 }, { -2, 0 }, { -1, -2 }, { -2, -1 }, { -2, -2 } },
    { { 0, -1 }, { -1, 0 }, { -1, -1 }, { 0, -2 }, { -2, 0 }, { -1, -2 }, { -2, -1 }, { -2, -2 } },
    { { 0, -1 }, { -1, 0 }, { -1, -1 }, { 0, -2 }, { -2, 0 }, { -1, -2 }, { -2, -1 }, { -2, -2 } },
};
#define MV_INVALID 0x80008000u

typedef struct Cand { int idx, sb; uint32_t mem, mem8; Mv out; } Cand;

static Mv clamp_mv(const Walk *w, Mv m)
{
    m.x = (int16_t) MAX(w->minx, MIN(w->maxx, m.x));
    m.y = (int16_t) MAX(w->miny, MIN(w->maxy, m.y));
    return m;
}
/* an MV of an earlier sub-block of this block (RETURN_DIRECT_MV): 1 = found */
static int cand_direct(Cand *c, Mv mv)
{
    const uint32_t m = mv_bits(mv);
    if (!c->idx) { c->out = mv; return 1; }
    if (c->mem == MV_INVALID) { c->mem = m; return 0; }
    if (m != c->mem) { c->out = mv; return 1; }
    return 0;
}
/* a neighbour's MV (RETURN_MV), clamped to the block's range */
static int cand_add(const Walk *w, Cand *c, Mv mv)
{
    if (c->sb > 0) {
        if (c->mem8 == MV_INVALID) {
            const Mv t = clamp_mv(w, mv);
            if (mv_bits(t) != c->mem) { c->out = t; return 1; }
            c->mem8 = mv_bits(mv);
        } else if (c->mem8 != mv_bits(mv)) {
            const Mv t = clamp_mv(w, mv);
            if (mv_bits(t) != c->mem) c->out = t;
            else c->out.x = c->out.y = 0;            /* libvpx's quirk, kept by vp9mvs.c:131-133 */
            return 1;
        }
        return 0;
    }
    const uint32_t m = mv_bits(mv);
    if (!c->idx) { c->out = clamp_mv(w, mv); return 1; }
    if (c->mem == MV_INVALID) { c->mem = m; return 0; }
    if (m != c->mem) { c->out = clamp_mv(w, mv); return 1; }
    return 0;
}
static int cand_scaled(const Walk *w, Cand *c, Mv mv, int flip)
{
    if (flip) { mv.x = (int16_t) -mv.x; mv.y = (int16_t) -mv.y; }
    return cand_add(w, c, mv);
}

static Mv find_ref_mv(const Walk *w, const vp9h_block *b, int row, int col, int ref, int z, int idx, int sb)
{
    const int8_t (*p)[2] = mv_ref_blk_off[b->bs];
    const int stride = w->sb_cols * 8, row7 = row & 7;
    const Hdr *h = w->h;
    const MvPair *cur = w->side->mv;
    Cand c = { idx, sb, MV_INVALID, MV_INVALID, { 0, 0 } };
    Mv m0 = { b->mv[0][z][0], b->mv[0][z][1] }, m1 = { b->mv[1][z][0], b->mv[1][z][1] },
       m2 = { b->mv[2][z][0], b->mv[2][z][1] };
    int i;
    if (sb >= 0) {
        if (sb == 1 || sb == 2) {
            if (cand_direct(&c, m0)) return c.out;
        } else if (sb == 3) {
            if (cand_direct(&c, m2) || cand_direct(&c, m1) || cand_direct(&c, m0)) return c.out;
        }
        if (row > 0) {
            const MvPair *mv = &cur[(row - 1) * stride + col];
            if (mv->ref[0] == ref) { if (cand_add(w, &c, w->a_mv[2 * col + (sb & 1)][0])) return c.out; }
            else if (mv->ref[1] == ref) { if (cand_add(w, &c, w->a_mv[2 * col + (sb & 1)][1])) return c.out; }
        }
        if (col > w->tile_col_start) {
            const MvPair *mv = &cur[row * stride + col - 1];
            if (mv->ref[0] == ref) { if (cand_add(w, &c, w->l_mv[2 * row7 + (sb >> 1)][0])) return c.out; }
            else if (mv->ref[1] == ref) { if (cand_add(w, &c, w->l_mv[2 * row7 + (sb >> 1)][1])) return c.out; }
        }
        i = 2;
    } else {
        i = 0;
    }
    /* neighbours coded with the same reference */
    for (; i < 8; i++) {
        const int cc = p[i][0] + col, r = p[i][1] + row;
        if (cc >= w->tile_col_start && cc < w->cols && r >= 0 && r < w->rows) {
            const MvPair *mv = &cur[r * stride + cc];
            if (mv->ref[0] == ref) { if (cand_add(w, &c, mv->mv[0])) return c.out; }
            else if (mv->ref[1] == ref) { if (cand_add(w, &c, mv->mv[1])) return c.out; }
        }
    }
    /* this position in the previous frame, same reference */
    if (h->use_last_mvs) {
        const MvPair *mv = &w->mvref->mv[row * stride + col];
        if (mv->ref[0] == ref) { if (cand_add(w, &c, mv->mv[0])) return c.out; }
        else if (mv->ref[1] == ref) { if (cand_add(w, &c, mv->mv[1])) return c.out; }
    }
    /* neighbours with another reference, negated across a sign-bias change */
    for (i = 0; i < 8; i++) {
        const int cc = p[i][0] + col, r = p[i][1] + row;
        if (cc >= w->tile_col_start && cc < w->cols && r >= 0 && r < w->rows) {
            const MvPair *mv = &cur[r * stride + cc];
            if (mv->ref[0] != ref && mv->ref[0] >= 0 &&
                cand_scaled(w, &c, mv->mv[0], h->signbias[mv->ref[0]] != h->signbias[ref]))
                return c.out;
            if (mv->ref[1] != ref && mv->ref[1] >= 0 && mv_bits(mv->mv[0]) != mv_bits(mv->mv[1]) &&
                cand_scaled(w, &c, mv->mv[1], h->signbias[mv->ref[1]] != h->signbias[ref]))
                return c.out;
        }
    }
    if (h->use_last_mvs) {
        const MvPair *mv = &w->mvref->mv[row * stride + col];
        if (mv->ref[0] != ref && mv->ref[0] >= 0 &&
            cand_scaled(w, &c, mv->mv[0], h->signbias[mv->ref[0]] != h->signbias[ref]))
            return c.out;
        if (mv->ref[1] != ref && mv->ref[1] >= 0 && mv_bits(mv->mv[0]) != mv_bits(mv->mv[1]) &&
            cand_scaled(w, &c, mv->mv[1], h->signbias[mv->ref[1]] != h->signbias[ref]))
            return c.out;
    }
    Mv zero = { 0, 0 };
    return clamp_mv(w, zero);
}

/* the prediction ff_vp9_fill_mv starts from (vp9mvs.c:295-345): the candidate, lowered
 * to 1/4 pel when high precision is off or the candidate is large. *hp: precision used */
static Mv mv_pred(const Walk *w, const vp9h_block *b, int row, int col, int z, int mode, int sb, int *hp)
{
    Mv m = find_ref_mv(w, b, row, col, b->ref[z], z, mode == VP9H_NEARMV, mode == VP9H_NEWMV ? -1 : sb);
    *hp = 1;
    if (mode == VP9H_NEWMV || sb == -1) {
        *hp = w->h->hp && abs(m.x) < 64 && abs(m.y) < 64;
        if (!*hp) {
            if (m.y & 1) m.y = (int16_t) (m.y < 0 ? m.y + 1 : m.y - 1);
            if (m.x & 1) m.x = (int16_t) (m.x < 0 ? m.x + 1 : m.x - 1);
        }
    }
    return m;
}

/* read_mv_component (vp9mvs.c:277-330): one component of an MV difference, idx 0 = y */
static inline __attribute__((always_inline)) int walk_mv_comp_t(Walk *w, int idx, int hp, int v, const int enc)
{
    BC *c = w->c;
    MvProbs *mp = &w->pr.p.mv_comp[idx];
    typeof(w->cnt.mv_comp[0]) *ct = &w->cnt.mv_comp[idx];
    /* encoder: v = +-(n + 1); n = class0 (n < 16) or (8 << cls) + bits << 3 | fp << 1 | hp */
    const int an = (v < 0 ? -v : v) - 1;
    int cls0 = 0;
    if (enc && an >= 16) { cls0 = 1; while ((8 << (cls0 + 1)) <= an) cls0++; }
    const int sign = bc_bool_e(c, enc, mp->sign, v < 0);
    const int cls = bc_tree_e(c, enc, mv_class_tree, mp->classes, enc ? (an >= 16 ? cls0 : 0) : 0);
    ct->sign[sign]++;
    ct->classes[cls]++;
    int n;
    if (cls) {
        const int r = an - (8 << cls);
        n = 0;
        for (int m = 0; m < cls; m++) {
            const int bit = bc_bool_e(c, enc, mp->bits[m], (r >> (3 + m)) & 1);
            n |= bit << m;
            ct->bits[m][bit]++;
        }
        n <<= 3;
        const int fp = bc_tree_e(c, enc, mv_fp_tree, mp->fp, (r >> 1) & 3);
        n |= fp << 1;
        ct->fp[fp]++;
        if (hp) {
            const int bit = bc_bool_e(c, enc, mp->hp, r & 1);
            ct->hp[bit]++;
            n |= bit;
        } else {
            n |= 1;
            ct->hp[1]++;                   /* counted although not coded, as libvpx does */
        }
        n += 8 << cls;
    } else {
        const int c0 = bc_bool_e(c, enc, mp->class0, (an >> 3) & 1);
        ct->class0[c0]++;
        const int fp = bc_tree_e(c, enc, mv_fp_tree, mp->class0_fp[c0], (an >> 1) & 3);
        ct->class0_fp[c0][fp]++;
        n = (c0 << 3) | (fp << 1);
        if (hp) {
            const int bit = bc_bool_e(c, enc, mp->class0_hp, an & 1);
            ct->class0_hp[bit]++;
            n |= bit;
        } else {
            n |= 1;
            ct->class0_hp[1]++;
        }
    }
    return sign ? -(n + 1) : (n + 1);
}

/* ff_vp9_fill_mv (vp9mvs.c:295-365) for sub-block sb (-1: whole block). Encoder: `t` is
 * the packet's MV pair for this sub-block; the coded MV can differ from it only by the
 * odd 1/8-pel step a low-precision difference cannot carry. */
static inline __attribute__((always_inline)) void walk_fill_mv_t(Walk *w, vp9h_block *b, int row, int col, int mode, int sb, Mv out[2], const Mv t[2], const int enc)
{
    for (int z = 0; z < 1 + b->comp; z++) {
        if (mode == VP9H_ZEROMV) { out[z].x = out[z].y = 0; continue; }
        int hp;
        Mv m = mv_pred(w, b, row, col, z, mode, sb, &hp);
        if (mode == VP9H_NEWMV) {
            int dx = 0, dy = 0;
            if (enc) {
                dx = t[z].x - m.x; dy = t[z].y - m.y;
                if (!hp) { dx -= (dx & 1) ? (dx > 0 ? 1 : -1) : 0; dy -= (dy & 1) ? (dy > 0 ? 1 : -1) : 0; }
            }
            const int j = bc_tree_e(w->c, enc, mv_joint_tree, w->pr.p.mv_joint, (dx != 0) | (dy != 0) << 1);
            w->cnt.mv_joint[j]++;
            if (j >= 2) m.y = (int16_t) (m.y + walk_mv_comp_t(w, 0, hp, dy, enc));
            if (j & 1) m.x = (int16_t) (m.x + walk_mv_comp_t(w, 1, hp, dx, enc));
        }
        out[z] = m;
    }
    if (!b->comp) out[1].x = out[1].y = 0;
}

/* encoder: the inter mode that reproduces the packet's MVs, preferring the packet's mode
 * (keep_modes: the packet's mode, whatever MV it predicts) */
static int choose_mode(const Walk *w, const vp9h_block *b, int row, int col, int sb, int want, const Mv t[2])
{
    const int nz = 1 + b->comp;
    if (w->keep_modes && want >= VP9H_NEARESTMV && want <= VP9H_NEWMV) return want;
    if (want == VP9H_ZEROMV) {
        int ok = 1;
        for (int z = 0; z < nz; z++) ok &= !t[z].x && !t[z].y;
        if (ok) return VP9H_ZEROMV;
    } else if (want == VP9H_NEARESTMV || want == VP9H_NEARMV) {
        int ok = 1, hp;
        for (int z = 0; z < nz; z++) ok &= mv_bits(mv_pred(w, b, row, col, z, want, sb, &hp)) == mv_bits(t[z]);
        if (ok) return want;
    }
    return VP9H_NEWMV;
}

/* ------------------------------------------------------------------ block / partition */
static const uint8_t left_ctx_of[13] = { 0x0, 0x8, 0x0, 0x8, 0xc, 0x8, 0xc, 0xe, 0xc, 0xe, 0xf, 0xe, 0xf };
static const uint8_t above_ctx_of[13] = { 0x0, 0x0, 0x8, 0x8, 0x8, 0xc, 0xc, 0xc, 0xe, 0xe, 0xe, 0xf, 0xf };
static const uint8_t max_tx_of[13] = { 3, 3, 3, 3, 2, 2, 2, 1, 1, 1, 0, 0, 0 };
static const uint8_t inter_mode_ctx[14][14] = {
    { 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 5, 5, 5, 5 }, { 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 5, 5, 5, 5 },
    { 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 5, 5, 5, 5 }, { 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 5, 5, 5, 5 },
    { 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 5, 5, 5, 5 }, { 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 5, 5, 5, 5 },
    { 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 5, 5, 5, 5 }, { 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 5, 5, 5, 5 },
    { 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 5, 5, 5, 5 }, { 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 5, 5, 5, 5 },
    { 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 2, 2, 1, 3 }, { 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 2, 2, 1, 3 },
    { 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 1, 1, 0, 3 }, { 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 3, 3, 3, 4 },
};

/* the segment id (decode_mode, vp9block.c:101-141) */
static inline __attribute__((always_inline)) void walk_seg_id_t(Walk *w, vp9h_block *b, const vp9h_block *t, int row, int col, int w4, int h4, const int enc)
{
    const Hdr *h = w->h;
    BC *c = w->c;
    const int row7 = row & 7;
    if (!h->seg_enabled) {
        b->seg_id = 0;
    } else if (h->keyframe || h->intraonly) {
        b->seg_id = h->seg_update_map ? (uint8_t) bc_tree_e(c, enc, segment_tree, h->seg_prob, t->seg_id) : 0;
    } else {
        /* the temporal prediction: the smallest id under the block in the reference map */
        int pred = 0;
        if (!h->errorres && w->segref) {
            const uint8_t *map = w->segref->seg;
            pred = 8;
            for (int y = 0; y < h4; y++)
                for (int x = 0; x < w4; x++) pred = MIN(pred, map[(y + row) * 8 * w->sb_cols + col + x]);
        }
        if (!h->seg_update_map ||
            (h->seg_temporal && bc_bool_e(c, enc, h->seg_pred[w->a_segpred[col] + w->l_segpred[row7]], t->seg_id == pred))) {
            b->seg_id = (uint8_t) pred;
            fill_ctx(w->a_segpred + col, 1, w4);
            fill_ctx(w->l_segpred + row7, 1, h4);
        } else {
            b->seg_id = (uint8_t) bc_tree_e(c, enc, segment_tree, h->seg_prob, t->seg_id);
            fill_ctx(w->a_segpred + col, 0, w4);
            fill_ctx(w->l_segpred + row7, 0, h4);
        }
    }
    if (h->seg_enabled && (h->seg_update_map || h->keyframe || h->intraonly)) {
        const int bw4 = vp9t_bwh[1][b->bs][0], bh4 = vp9t_bwh[1][b->bs][1];
        for (int y = 0; y < bh4; y++) fill_ctx(w->side->seg + (row + y) * 8 * w->sb_cols + col, b->seg_id, bw4);
    }
}

/* the reference frames of an inter block (vp9block.c:333-574) */
static inline __attribute__((always_inline)) void walk_refs_t(Walk *w, vp9h_block *b, const vp9h_block *t, int have_a, int have_l, int col, int row7, const int enc)
{
    const Hdr *h = w->h;
    BC *c = w->c;
    const uint8_t ai = w->a_intra[col], li = w->l_intra[row7], ac = w->a_comp[col], lc = w->l_comp[row7];
    const uint8_t ar = w->a_ref[col], lr = w->l_ref[row7];
    const int fix = h->fixcompref;
    int ctx;
    if (h->seg_enabled && h->seg[b->seg_id].ref_en) {
        b->comp = 0;
        b->ref[0] = (uint8_t) (h->seg[b->seg_id].ref - 1);
        return;
    }
    if (h->comppred != P_SWITCH) {
        b->comp = h->comppred == P_COMP;
    } else {
        if (have_a) {
            if (have_l) {
                if (ac && lc) ctx = 4;
                else if (ac) ctx = 2 + (li || lr == fix);
                else if (lc) ctx = 2 + (ai || ar == fix);
                else ctx = (!ai && ar == fix) ^ (!li && lr == fix);
            } else {
                ctx = ac ? 3 : (!ai && ar == fix);
            }
        } else if (have_l) {
            ctx = lc ? 3 : (!li && lr == fix);
        } else {
            ctx = 1;
        }
        b->comp = (uint8_t) bc_bool_e(c, enc, w->pr.p.comp[ctx], t->comp);
        w->cnt.comp[ctx][b->comp]++;
    }
    if (b->comp) {
        const int fix_idx = h->signbias[fix], var_idx = !fix_idx, v1 = h->varcompref[1], v0 = h->varcompref[0];
        b->ref[fix_idx] = (uint8_t) fix;
        if (have_a) {
            if (have_l) {
                if (ai) ctx = li ? 2 : 1 + 2 * (lr != v1);
                else if (li) ctx = 1 + 2 * (ar != v1);
                else if (lr == ar && ar == v1) ctx = 0;
                else if (!lc && !ac) {
                    if ((ar == fix && lr == v0) || (lr == fix && ar == v0)) ctx = 4;
                    else ctx = ar == lr ? 3 : 1;
                } else if (!lc) {
                    if (ar == v1 && lr != v1) ctx = 1;
                    else ctx = (lr == v1 && ar != v1) ? 2 : 4;
                } else if (!ac) {
                    if (lr == v1 && ar != v1) ctx = 1;
                    else ctx = (ar == v1 && lr != v1) ? 2 : 4;
                } else {
                    ctx = lr == ar ? 4 : 2;
                }
            } else {
                ctx = ai ? 2 : ac ? 4 * (ar != v1) : 3 * (ar != v1);
            }
        } else if (have_l) {
            ctx = li ? 2 : lc ? 4 * (lr != v1) : 3 * (lr != v1);
        } else {
            ctx = 2;
        }
        const int bit = bc_bool_e(c, enc, w->pr.p.comp_ref[ctx], t->ref[var_idx] == v1);
        b->ref[var_idx] = (uint8_t) h->varcompref[bit];
        w->cnt.comp_ref[ctx][bit]++;
        return;
    }
    /* single reference: LAST, or GOLDEN / ALTREF */
    if (have_a && !ai) {
        if (have_l && !li) {
            if (lc) ctx = ac ? 1 + (!fix || !lr || !ar) : 3 * !ar + (!fix || !lr);
            else if (ac) ctx = 3 * !lr + (!fix || !ar);
            else ctx = 2 * !lr + 2 * !ar;
        } else if (ai) {
            ctx = 2;
        } else if (ac) {
            ctx = 1 + (!fix || !ar);
        } else {
            ctx = 4 * !ar;
        }
    } else if (have_l && !li) {
        ctx = lc ? 1 + (!fix || !lr) : 4 * !lr;
    } else {
        ctx = 2;
    }
    int bit = bc_bool_e(c, enc, w->pr.p.single_ref[ctx][0], t->ref[0] != 0);
    w->cnt.single_ref[ctx][0][bit]++;
    if (!bit) { b->ref[0] = 0; return; }
    if (have_a) {
        if (have_l) {
            if (li) {
                if (ai) ctx = 2;
                else if (ac) ctx = 1 + 2 * (fix == 1 || ar == 1);
                else if (!ar) ctx = 3;
                else ctx = 4 * (ar == 1);
            } else if (ai) {
                if (lc) ctx = 1 + 2 * (fix == 1 || lr == 1);
                else if (!lr) ctx = 3;
                else ctx = 4 * (lr == 1);
            } else if (ac) {
                if (lc) ctx = lr == ar ? 3 * (fix == 1 || lr == 1) : 2;
                else if (!lr) ctx = 1 + 2 * (fix == 1 || ar == 1);
                else ctx = 3 * (lr == 1) + (fix == 1 || ar == 1);
            } else if (lc) {
                if (!ar) ctx = 1 + 2 * (fix == 1 || lr == 1);
                else ctx = 3 * (ar == 1) + (fix == 1 || lr == 1);
            } else if (!ar) {
                ctx = !lr ? 3 : 4 * (lr == 1);
            } else if (!lr) {
                ctx = 4 * (ar == 1);
            } else {
                ctx = 2 * (lr == 1) + 2 * (ar == 1);
            }
        } else {
            if (ai || (!ac && !ar)) ctx = 2;
            else if (ac) ctx = 3 * (fix == 1 || ar == 1);
            else ctx = 4 * (ar == 1);
        }
    } else if (have_l) {
        if (li || (!lc && !lr)) ctx = 2;
        else if (lc) ctx = 3 * (fix == 1 || lr == 1);
        else ctx = 4 * (lr == 1);
    } else {
        ctx = 2;
    }
    bit = bc_bool_e(c, enc, w->pr.p.single_ref[ctx][1], t->ref[0] == 2);
    w->cnt.single_ref[ctx][1][bit]++;
    b->ref[0] = (uint8_t) (1 + bit);
}

/* one block (decode_mode vp9block.c:80-803 + the coefficient call of
 * ff_vp9_decode_block, vp9block.c:1264-1345). Encoder: `t` is the packet's block. */
static inline __attribute__((always_inline)) void walk_block_t(Walk *w, int row, int col, int bl, int bp, const int enc)
{
    static const vp9h_block zero_block;
    BC *c = w->c;
    const Hdr *h = w->h;
    const int bs = bl * 3 + bp;
    const vp9h_block *t = &zero_block;
    if (enc) {
        if (w->bi >= w->in->nblocks) { w->err = 1; return; }
        t = &w->in->blocks[w->bi++];
        if (t->row != row || t->col != col || t->bs != bs) { w->err = 1; return; }
    }
    vp9h_block b;
    memset(&b, 0, sizeof(b));
    b.row = (uint16_t) row; b.col = (uint16_t) col; b.bs = (uint8_t) bs;
    const int row7 = row & 7, max_tx = max_tx_of[bs];
    const int bw4 = vp9t_bwh[1][bs][0], bh4 = vp9t_bwh[1][bs][1];
    const int w4 = MIN(w->cols - col, bw4), h4 = MIN(w->rows - row, bh4);
    const int have_a = row > 0, have_l = col > w->tile_col_start;
    const int intra_frame = h->keyframe || h->intraonly;
    int filter_id = 0, vref = 0;
    w->minx = -(128 + col * 64); w->miny = -(128 + row * 64);
    w->maxx = 128 + (w->cols - col - bw4) * 64; w->maxy = 128 + (w->rows - row - bh4) * 64;

    walk_seg_id_t(w, &b, t, row, col, w4, h4, enc);
    /* skip */
    b.skip = h->seg_enabled && h->seg[b.seg_id].skip;
    if (!b.skip) {
        const int cx = w->l_skip[row7] + w->a_skip[col];
        b.skip = (uint8_t) bc_bool_e(c, enc, w->pr.p.skip[cx], t->skip);
        w->cnt.skip[cx][b.skip]++;
    }
    /* intra / inter */
    if (intra_frame) {
        b.intra = 1;
    } else if (h->seg_enabled && h->seg[b.seg_id].ref_en) {
        b.intra = !h->seg[b.seg_id].ref;
    } else {
        int cx;
        if (have_a && have_l) { cx = w->a_intra[col] + w->l_intra[row7]; cx += cx == 2; }
        else cx = have_a ? 2 * w->a_intra[col] : have_l ? 2 * w->l_intra[row7] : 0;
        const int bit = bc_bool_e(c, enc, w->pr.p.intra[cx], !t->intra);
        w->cnt.intra[cx][bit]++;
        b.intra = !bit;
    }
    /* tx size */
    if ((b.intra || !b.skip) && h->txmode == TX_SEL) {
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
        const PC *pp = &w->pr.p;
        int tx = 0;
        switch (max_tx) {
        case 3:
            tx = bc_bool_e(c, enc, pp->tx32p[cx][0], t->tx > 0);
            if (tx) { tx += bc_bool_e(c, enc, pp->tx32p[cx][1], t->tx > 1); if (tx == 2) tx += bc_bool_e(c, enc, pp->tx32p[cx][2], t->tx > 2); }
            w->cnt.tx32p[cx][tx]++;
            break;
        case 2:
            tx = bc_bool_e(c, enc, pp->tx16p[cx][0], t->tx > 0);
            if (tx) tx += bc_bool_e(c, enc, pp->tx16p[cx][1], t->tx > 1);
            w->cnt.tx16p[cx][tx]++;
            break;
        case 1:
            tx = bc_bool_e(c, enc, pp->tx8p[cx], t->tx > 0);
            w->cnt.tx8p[cx][tx]++;
            break;
        default: tx = 0;
        }
        b.tx = (uint8_t) tx;
    } else {
        b.tx = (uint8_t) MIN(max_tx, h->txmode);
    }

    if (intra_frame) {
        /* intra modes with above / left 4x4 mode contexts (keyframe probabilities) */
        uint8_t *a = w->a_mode + col * 2, *l = w->l_mode + (row7 << 1);
        if (bs > VP9H_BS_8x8) {
            b.mode[0] = a[0] = (uint8_t) bc_tree_e(c, enc, intramode_tree, vp9t_kf_ymode_probs[a[0]][l[0]], t->mode[0]);
            if (bs != VP9H_BS_8x4) {
                b.mode[1] = (uint8_t) bc_tree_e(c, enc, intramode_tree, vp9t_kf_ymode_probs[a[1]][b.mode[0]], t->mode[1]);
                l[0] = a[1] = b.mode[1];
            } else {
                l[0] = a[1] = b.mode[1] = b.mode[0];
            }
            if (bs != VP9H_BS_4x8) {
                b.mode[2] = a[0] = (uint8_t) bc_tree_e(c, enc, intramode_tree, vp9t_kf_ymode_probs[a[0]][l[1]], t->mode[2]);
                if (bs != VP9H_BS_8x4) {
                    b.mode[3] = (uint8_t) bc_tree_e(c, enc, intramode_tree, vp9t_kf_ymode_probs[a[1]][b.mode[2]], t->mode[3]);
                    l[1] = a[1] = b.mode[3];
                } else {
                    l[1] = a[1] = b.mode[3] = b.mode[2];
                }
            } else {
                b.mode[2] = b.mode[0];
                l[1] = a[1] = b.mode[3] = b.mode[1];
            }
        } else {
            b.mode[0] = (uint8_t) bc_tree_e(c, enc, intramode_tree, vp9t_kf_ymode_probs[*a][*l], t->mode[0]);
            b.mode[3] = b.mode[2] = b.mode[1] = b.mode[0];
            fill_ctx(a, b.mode[0], vp9t_bwh[0][bs][0]);
            fill_ctx(l, b.mode[0], vp9t_bwh[0][bs][1]);
        }
        b.uvmode = (uint8_t) bc_tree_e(c, enc, intramode_tree, vp9t_kf_uvmode_probs[b.mode[3]], t->uvmode);
    } else if (b.intra) {
        /* intra block of an inter frame: adaptive probabilities, no neighbour context */
        static const uint8_t size_group[10] = { 3, 3, 3, 3, 2, 2, 2, 1, 1, 1 };
        if (bs > VP9H_BS_8x8) {
            b.mode[0] = (uint8_t) bc_tree_e(c, enc, intramode_tree, w->pr.p.y_mode[0], t->mode[0]);
            w->cnt.y_mode[0][b.mode[0]]++;
            if (bs != VP9H_BS_8x4) {
                b.mode[1] = (uint8_t) bc_tree_e(c, enc, intramode_tree, w->pr.p.y_mode[0], t->mode[1]);
                w->cnt.y_mode[0][b.mode[1]]++;
            } else {
                b.mode[1] = b.mode[0];
            }
            if (bs != VP9H_BS_4x8) {
                b.mode[2] = (uint8_t) bc_tree_e(c, enc, intramode_tree, w->pr.p.y_mode[0], t->mode[2]);
                w->cnt.y_mode[0][b.mode[2]]++;
                if (bs != VP9H_BS_8x4) {
                    b.mode[3] = (uint8_t) bc_tree_e(c, enc, intramode_tree, w->pr.p.y_mode[0], t->mode[3]);
                    w->cnt.y_mode[0][b.mode[3]]++;
                } else {
                    b.mode[3] = b.mode[2];
                }
            } else {
                b.mode[2] = b.mode[0];
                b.mode[3] = b.mode[1];
            }
        } else {
            const int sz = size_group[bs];
            b.mode[0] = (uint8_t) bc_tree_e(c, enc, intramode_tree, w->pr.p.y_mode[sz], t->mode[0]);
            b.mode[1] = b.mode[2] = b.mode[3] = b.mode[0];
            w->cnt.y_mode[sz][b.mode[3]]++;
        }
        b.uvmode = (uint8_t) bc_tree_e(c, enc, intramode_tree, w->pr.p.uv_mode[b.mode[3]], t->uvmode);
        w->cnt.uv_mode[b.mode[3]][b.uvmode]++;
    } else {
        walk_refs_t(w, &b, t, have_a, have_l, col, row7, enc);
        Mv tm[4][2], out[2];
        for (int k = 0; k < 4; k++)
            for (int z = 0; z < 2; z++) { tm[k][z].x = t->mv[k][z][0]; tm[k][z].y = t->mv[k][z][1]; }
        if (bs <= VP9H_BS_8x8) {
            if (h->seg_enabled && h->seg[b.seg_id].skip) {
                b.mode[0] = b.mode[1] = b.mode[2] = b.mode[3] = VP9H_ZEROMV;
            } else {
                static const uint8_t off[10] = { 3, 0, 0, 1, 0, 0, 0, 0, 0, 0 };
                const int cx = inter_mode_ctx[w->a_mode[col + off[bs]]][w->l_mode[row7 + off[bs]]];
                const int want = enc ? choose_mode(w, &b, row, col, -1, t->mode[0], tm[0]) : 0;
                b.mode[0] = (uint8_t) bc_tree_e(c, enc, inter_mode_tree, w->pr.p.mv_mode[cx], want);
                b.mode[1] = b.mode[2] = b.mode[3] = b.mode[0];
                w->cnt.mv_mode[cx][b.mode[0] - 10]++;
            }
        }
        /* interpolation filter */
        if (h->filtermode == FILTER_SWITCHABLE) {
            int cx;
            if (have_a && w->a_mode[col] >= VP9H_NEARESTMV) {
                if (have_l && w->l_mode[row7] >= VP9H_NEARESTMV)
                    cx = w->a_filter[col] == w->l_filter[row7] ? w->l_filter[row7] : 3;
                else
                    cx = w->a_filter[col];
            } else if (have_l && w->l_mode[row7] >= VP9H_NEARESTMV) {
                cx = w->l_filter[row7];
            } else {
                cx = 3;
            }
            filter_id = bc_tree_e(c, enc, filter_tree, w->pr.p.filter[cx], t->filter < 3 ? id_of_filter[t->filter] : 0);
            w->cnt.filter[cx][filter_id]++;
            b.filter = filter_of_id[filter_id];
        } else {
            b.filter = (uint8_t) h->filtermode;
        }
        if (bs > VP9H_BS_8x8) {
            const int cx = inter_mode_ctx[w->a_mode[col]][w->l_mode[row7]];
            for (int k = 0; k < 4; k++) {
                /* 8x4: sub-blocks 1 and 3 copy 0 and 2; 4x8: 2 and 3 copy 0 and 1 */
                const int src = bs == VP9H_BS_8x4 ? (k & 1 ? k - 1 : -1) : bs == VP9H_BS_4x8 ? (k & 2 ? k - 2 : -1) : -1;
                if (src >= 0) {
                    b.mode[k] = b.mode[src];
                    memcpy(b.mv[k], b.mv[src], sizeof(b.mv[k]));
                    continue;
                }
                const int want = enc ? choose_mode(w, &b, row, col, k, t->mode[k], tm[k]) : 0;
                b.mode[k] = (uint8_t) bc_tree_e(c, enc, inter_mode_tree, w->pr.p.mv_mode[cx], want);
                w->cnt.mv_mode[cx][b.mode[k] - 10]++;
                walk_fill_mv_t(w, &b, row, col, b.mode[k], k, out, tm[k], enc);
                for (int z = 0; z < 2; z++) { b.mv[k][z][0] = out[z].x; b.mv[k][z][1] = out[z].y; }
            }
        } else {
            walk_fill_mv_t(w, &b, row, col, b.mode[0], -1, out, tm[0], enc);
            for (int k = 0; k < 4; k++)
                for (int z = 0; z < 2; z++) { b.mv[k][z][0] = out[z].x; b.mv[k][z][1] = out[z].y; }
        }
        vref = b.ref[b.comp ? h->signbias[h->varcompref[0]] : 0];
    }
    b.uvtx = (uint8_t) (b.tx - ((h->ss_h && bw4 * 2 == (1 << b.tx)) || (h->ss_v && bh4 * 2 == (1 << b.tx))));

    /* contexts (SET_CTXS, vp9block.c:718-745) */
    fill_ctx(w->a_skip + col, b.skip, bw4); fill_ctx(w->l_skip + row7, b.skip, bh4);
    fill_ctx(w->a_tx + col, b.tx, bw4); fill_ctx(w->l_tx + row7, b.tx, bh4);
    fill_ctx(w->a_part + col, above_ctx_of[bs], bw4); fill_ctx(w->l_part + row7, left_ctx_of[bs], bh4);
    if (!intra_frame) {
        fill_ctx(w->a_intra + col, b.intra, bw4); fill_ctx(w->l_intra + row7, b.intra, bh4);
        fill_ctx(w->a_comp + col, b.comp, bw4); fill_ctx(w->l_comp + row7, b.comp, bh4);
        fill_ctx(w->a_mode + col, b.mode[3], bw4); fill_ctx(w->l_mode + row7, b.mode[3], bh4);
        if (!b.intra) {
            fill_ctx(w->a_ref + col, vref, bw4); fill_ctx(w->l_ref + row7, vref, bh4);
            if (h->filtermode == FILTER_SWITCHABLE) {
                fill_ctx(w->a_filter + col, filter_id, bw4); fill_ctx(w->l_filter + row7, filter_id, bh4);
            }
        }
        /* MV contexts for the sub-8x8 candidates (vp9block.c:747-770) */
        Mv m3[2] = { { b.mv[3][0][0], b.mv[3][0][1] }, { b.mv[3][1][0], b.mv[3][1][1] } };
        if (bs > VP9H_BS_8x8) {
            for (int z = 0; z < 2; z++) {
                w->l_mv[row7 * 2][z].x = b.mv[1][z][0]; w->l_mv[row7 * 2][z].y = b.mv[1][z][1];
                w->a_mv[col * 2][z].x = b.mv[2][z][0]; w->a_mv[col * 2][z].y = b.mv[2][z][1];
                w->l_mv[row7 * 2 + 1][z] = m3[z];
                w->a_mv[col * 2 + 1][z] = m3[z];
            }
        } else {
            for (int n = 0; n < w4 * 2; n++) { w->a_mv[col * 2 + n][0] = m3[0]; w->a_mv[col * 2 + n][1] = m3[1]; }
            for (int n = 0; n < h4 * 2; n++) { w->l_mv[row7 * 2 + n][0] = m3[0]; w->l_mv[row7 * 2 + n][1] = m3[1]; }
        }
    }
    /* this frame's MV pairs (vp9block.c:773-800) */
    for (int y = 0; y < h4; y++) {
        MvPair *mv = &w->side->mv[(row + y) * w->sb_cols * 8 + col];
        for (int x = 0; x < w4; x++) {
            if (b.intra) {
                mv[x].ref[0] = mv[x].ref[1] = -1;
            } else {
                mv[x].ref[0] = (int8_t) b.ref[0];
                mv[x].ref[1] = b.comp ? (int8_t) b.ref[1] : -1;
                mv[x].mv[0].x = b.mv[3][0][0]; mv[x].mv[0].y = b.mv[3][0][1];
                if (b.comp) { mv[x].mv[1].x = b.mv[3][1][0]; mv[x].mv[1].y = b.mv[3][1][1]; }
            }
        }
    }

    if (!b.skip) {
        const size_t ne0 = w->ne, nc0 = w->nc;
        if (!walk_coeffs_t(w, &b, row, col, enc) && !w->err && bs <= VP9H_BS_8x8 && !b.intra) {
            /* an inter block <= 8x8 without coefficients becomes skip (vp9block.c:1310-1314) */
            b.skip = 1;
            fill_ctx(w->a_skip + col, 1, bw4);
            fill_ctx(w->l_skip + row7, 1, bh4);
            w->ne = ne0; w->nc = nc0;
        }
    } else {
        /* SPLAT_ZERO_YUV (vp9block.c:1313-1345): the whole block, unclipped */
        fill_ctx16(w->a_ynnz + col * 2, 0, 2 * bw4); fill_ctx16(w->l_ynnz + row7 * 2, 0, 2 * bh4);
        const int ux = h->ss_h ? bw4 : 2 * bw4, uy = h->ss_v ? bh4 : 2 * bh4;
        fill_ctx16(w->a_unnz + (col << !h->ss_h), 0, ux); fill_ctx16(w->a_vnnz + (col << !h->ss_h), 0, ux);
        fill_ctx16(w->l_unnz + (row7 << !h->ss_v), 0, uy); fill_ctx16(w->l_vnnz + (row7 << !h->ss_v), 0, uy);
    }
    if (w->err) return;
    w->blocks = grow(w->blocks, &w->cb, w->nb + 1, sizeof(vp9h_block), &w->err);
    if (w->err) return;
    w->blocks[w->nb++] = b;
}

/* decode_sb (vp9.c:1115-1193) */
/* the walkers per direction: the decoder's carries no encoder branches (tools/parse_bench.c) */
static __attribute__((noinline)) void walk_block_dec(Walk *w, int row, int col, int bl, int bp)
{
    walk_block_t(w, row, col, bl, bp, 0);
}
static __attribute__((noinline)) void walk_block_enc(Walk *w, int row, int col, int bl, int bp)
{
    walk_block_t(w, row, col, bl, bp, 1);
}
static void walk_sb_dec(Walk *w, int row, int col, int bl);
static void walk_sb_enc(Walk *w, int row, int col, int bl);
static inline __attribute__((always_inline)) void walk_sb_t(Walk *w, int row, int col, int bl, const int enc)
{
    BC *c = w->c;
    if (w->err) return;
    const int ctx = ((w->a_part[col] >> (3 - bl)) & 1) | (((w->l_part[row & 7] >> (3 - bl)) & 1) << 1);
    const uint8_t *p = (w->h->keyframe || w->h->intraonly) ? vp9t_kf_partition_probs[bl][ctx]
                                                            : w->pr.p.partition[bl][ctx];
    const int hbs = 4 >> bl;
    int bp = 0;
    if (enc) {   /* the packet's next block says which partition this node takes */
        if (w->bi >= w->in->nblocks) { w->err = 1; return; }
        const vp9h_block *nb = &w->in->blocks[w->bi];
        const int nbl = nb->bs == VP9H_BS_4x4 ? 3 : nb->bs / 3;
        bp = (nb->row == row && nb->col == col && nbl == bl) ? nb->bs - 3 * bl : 3;
    }
    if (bl == 3) {
        bp = bc_tree_e(c, enc, partition_tree, p, bp);
        (enc ? walk_block_enc : walk_block_dec)(w, row, col, bl, bp);
    } else if (col + hbs < w->cols) {
        if (row + hbs < w->rows) {
            bp = bc_tree_e(c, enc, partition_tree, p, bp);
            switch (bp) {
            case 0: (enc ? walk_block_enc : walk_block_dec)(w, row, col, bl, bp); break;
            case 1: (enc ? walk_block_enc : walk_block_dec)(w, row, col, bl, bp); (enc ? walk_block_enc : walk_block_dec)(w, row + hbs, col, bl, bp); break;
            case 2: (enc ? walk_block_enc : walk_block_dec)(w, row, col, bl, bp); (enc ? walk_block_enc : walk_block_dec)(w, row, col + hbs, bl, bp); break;
            default:
                (enc ? walk_sb_enc : walk_sb_dec)(w, row, col, bl + 1); (enc ? walk_sb_enc : walk_sb_dec)(w, row, col + hbs, bl + 1);
                (enc ? walk_sb_enc : walk_sb_dec)(w, row + hbs, col, bl + 1); (enc ? walk_sb_enc : walk_sb_dec)(w, row + hbs, col + hbs, bl + 1);
            }
        } else if (bc_bool_e(c, enc, p[1], bp == 3)) {
            bp = 3;
            (enc ? walk_sb_enc : walk_sb_dec)(w, row, col, bl + 1); (enc ? walk_sb_enc : walk_sb_dec)(w, row, col + hbs, bl + 1);
        } else {
            bp = 1;
            (enc ? walk_block_enc : walk_block_dec)(w, row, col, bl, 1);
        }
    } else if (row + hbs < w->rows) {
        if (bc_bool_e(c, enc, p[2], bp == 3)) { bp = 3; (enc ? walk_sb_enc : walk_sb_dec)(w, row, col, bl + 1); (enc ? walk_sb_enc : walk_sb_dec)(w, row + hbs, col, bl + 1); }
        else { bp = 2; (enc ? walk_block_enc : walk_block_dec)(w, row, col, bl, 2); }
    } else {
        bp = 3;
        (enc ? walk_sb_enc : walk_sb_dec)(w, row, col, bl + 1);
    }
    w->cnt.partition[bl][ctx][bp]++;
}
static void walk_sb_dec(Walk *w, int row, int col, int bl) { walk_sb_t(w, row, col, bl, 0); }
static void walk_sb_enc(Walk *w, int row, int col, int bl) { walk_sb_t(w, row, col, bl, 1); }
static void walk_sb(Walk *w, int row, int col, int bl)
{
    if (w->c->enc) walk_sb_enc(w, row, col, bl);
    else walk_sb_dec(w, row, col, bl);
}

/* ------------------------------------------------------------------ headers */
static void set_qmul_lf(Walk *w)
{
    Hdr *h = w->h;
    const int bidx = (h->bpp - 8) >> 1;
    for (int i = 0; i < (h->seg_enabled ? 8 : 1); i++) {
        int qyac = h->qidx, lvl = h->filter_level;
        if (h->seg_enabled && h->seg[i].q_en) qyac = h->seg_abs ? h->seg[i].q : h->qidx + h->seg[i].q;
        qyac = MAX(0, MIN(255, qyac));
        const int qydc = MAX(0, MIN(255, qyac + h->ydc)), quvdc = MAX(0, MIN(255, qyac + h->uvdc)),
                  quvac = MAX(0, MIN(255, qyac + h->uvac));
        h->qmul[i][0][0] = vp9t_dc_q[bidx][qydc];
        h->qmul[i][0][1] = vp9t_ac_q[bidx][qyac];
        h->qmul[i][1][0] = vp9t_dc_q[bidx][quvdc];
        h->qmul[i][1][1] = vp9t_ac_q[bidx][quvac];
        /* LF levels (vp9.c:767-791) */
        const int sh = h->filter_level >= 32;
        if (h->seg_enabled && h->seg[i].lf_en) lvl = h->seg_abs ? h->seg[i].lf : h->filter_level + h->seg[i].lf;
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

/* color config (read_colorspace_details, vp9.c:457-517). Profiles 1 / 3 code the
 * subsampling (4:2:2 / 4:4:0 / 4:4:4; 8-bit 4:2:0 is refused there, 10/12-bit 4:2:0 in
 * profile 3 is accepted, as in the reference) or RGB (4:4:4). The encoder writes BT.709
 * YUV with the packet's subsampling. Returns 0 or -1 (invalid). */
static int walk_color(Bits *b, Hdr *h, int prof)
{
    int bits = 0;
    if (prof >= 2) bits = 1 + bits_rw(b, 1, h->bpp == 12);
    h->bpp = 8 + 2 * bits;
    if (bits_rw(b, 3, 2) == 7) {                                  /* RGB: profiles 1 / 3 only */
        if (!(prof & 1)) return -1;
        h->ss_h = h->ss_v = 0;
        return bits_rw(b, 1, 0) ? -1 : 0;                         /* reserved bit */
    }
    bits_rw(b, 1, 0);                                             /* color range */
    if (prof & 1) {
        h->ss_h = bits_rw(b, 1, h->ss_h);
        h->ss_v = bits_rw(b, 1, h->ss_v);
        if (!bits && h->ss_h && h->ss_v) return -1;               /* YUV 4:2:0 in profile 1 */
        if (bits_rw(b, 1, 0)) return -1;                          /* reserved bit */
    } else {
        h->ss_h = h->ss_v = 1;
    }
    return 0;
}

/* The uncompressed header (decode_frame_header, vp9.c:519-880) into the stream's
 * persistent header, both directions. Returns the bit position of the 16-bit
 * compressed-header size, -1 (invalid), -2 (unsupported) or -3 (show_existing_frame,
 * *existing = the slot). Frame-to-frame state other than the header is not touched. */
static long walk_uncompressed(Walk *w, Bits *b, int *existing)
{
    vp9h_stream *st = w->st;
    Hdr *h = w->h;
    if (bits_rw(b, 2, 2) != 2) return -1;                        /* frame marker */
    int prof = bits_rw(b, 1, h->profile & 1);
    prof |= bits_rw(b, 1, h->profile >> 1) << 1;
    if (prof == 3) prof += bits_rw(b, 1, 0);
    if (prof > 3) return -1;
    h->profile = prof;
    if (bits_rw(b, 1, *existing >= 0)) {                         /* show_existing_frame */
        *existing = bits_rw(b, 3, *existing);
        return -3;
    }
    st->last_keyframe = w->last_keyframe;
    h->keyframe = !bits_rw(b, 1, !h->keyframe);
    const int last_invisible = w->last_invisible;
    h->invisible = !bits_rw(b, 1, !h->invisible);
    h->errorres = bits_rw(b, 1, h->errorres);
    h->use_last_mvs = !h->errorres && !last_invisible;
    int fw, fh;
    if (h->keyframe) {
        if (bits_rw(b, 24, 0x498342) != 0x498342) return -1;     /* sync code */
        if (walk_color(b, h, prof) < 0) return -1;
        h->refreshmask = 0xff;
        fw = bits_rw(b, 16, h->w - 1) + 1;
        fh = bits_rw(b, 16, h->h - 1) + 1;
        if (bits_rw(b, 1, 0)) bits_rw(b, 32, 0);                   /* render size */
    } else {
        h->intraonly = h->invisible ? bits_rw(b, 1, h->intraonly) : 0;
        h->resetctx = h->errorres ? 0 : bits_rw(b, 2, h->resetctx);
        if (h->intraonly) {
            if (bits_rw(b, 24, 0x498342) != 0x498342) return -1;
            if (prof >= 1) {
                if (walk_color(b, h, prof) < 0) return -1;
            } else {
                h->ss_h = h->ss_v = 1;
                h->bpp = 8;
            }
            h->refreshmask = bits_rw(b, 8, h->refreshmask);
            fw = bits_rw(b, 16, h->w - 1) + 1;
            fh = bits_rw(b, 16, h->h - 1) + 1;
            if (bits_rw(b, 1, 0)) bits_rw(b, 32, 0);
        } else {
            h->refreshmask = bits_rw(b, 8, h->refreshmask);
            for (int i = 0; i < 3; i++) {
                h->refidx[i] = bits_rw(b, 3, h->refidx[i]);
                h->signbias[i] = bits_rw(b, 1, h->signbias[i]) && !h->errorres;
            }
            for (int i = 0; i < 3; i++)
                if (!st->slot[h->refidx[i]].valid) return -1;      /* "Not all references are available" */
            /* frame size: from one of the references, or explicit. The encoder takes it
             * from the first reference of the same size. */
            int from = -1;
            if (b->enc)
                for (int i = 0; i < 3 && from < 0; i++)
                    if (st->slot[h->refidx[i]].w == h->w && st->slot[h->refidx[i]].h == h->h) from = i;
            int k = 0;
            for (; k < 3; k++)
                if (bits_rw(b, 1, from == k)) break;
            if (k < 3) {
                fw = st->slot[h->refidx[k]].w;
                fh = st->slot[h->refidx[k]].h;
            } else {
                fw = bits_rw(b, 16, h->w - 1) + 1;
                fh = bits_rw(b, 16, h->h - 1) + 1;
            }
            h->use_last_mvs &= st->cur && st->cur->w == fw && st->cur->h == fh;
            if (bits_rw(b, 1, 0)) bits_rw(b, 32, 0);
            h->hp = bits_rw(b, 1, h->hp);
            const int sw = bits_rw(b, 1, h->filtermode == FILTER_SWITCHABLE);
            h->filtermode = sw ? FILTER_SWITCHABLE : bits_rw(b, 2, h->filtermode);
            h->allowcomp = h->signbias[0] != h->signbias[1] || h->signbias[0] != h->signbias[2];
            if (h->allowcomp) {
                if (h->signbias[0] == h->signbias[1]) { h->fixcompref = 2; h->varcompref[0] = 0; h->varcompref[1] = 1; }
                else if (h->signbias[0] == h->signbias[2]) { h->fixcompref = 1; h->varcompref[0] = 0; h->varcompref[1] = 2; }
                else { h->fixcompref = 0; h->varcompref[0] = 1; h->varcompref[1] = 2; }
            }
            /* the format of an inter frame is its references' (all must match, vp9.c:606-616
             * via update_size's pixel format) */
            h->bpp = st->slot[h->refidx[0]].bpp;
            h->ss_h = st->slot[h->refidx[0]].ss_h;
            h->ss_v = st->slot[h->refidx[0]].ss_v;
            for (int i = 1; i < 3; i++)
                if (st->slot[h->refidx[i]].bpp != h->bpp || st->slot[h->refidx[i]].ss_h != h->ss_h ||
                    st->slot[h->refidx[i]].ss_v != h->ss_v) return -1;
        }
    }
    h->w = fw; h->h = fh;
    h->refreshctx = h->errorres ? 0 : bits_rw(b, 1, h->refreshctx);
    h->parallel = h->errorres ? 1 : bits_rw(b, 1, h->parallel);
    h->ctxid_raw = bits_rw(b, 2, h->ctxid_raw);
    h->ctxid = (h->keyframe || h->intraonly) ? 0 : h->ctxid_raw;  /* libvpx ignores it in intra frames */
    if (h->keyframe || h->errorres || h->intraonly) {
        h->lf_ref[0] = 1; h->lf_ref[1] = 0; h->lf_ref[2] = -1; h->lf_ref[3] = -1;
        h->lf_mode[0] = h->lf_mode[1] = 0;
        memset(h->seg, 0, sizeof(h->seg));
    }
    h->filter_level = bits_rw(b, 6, h->filter_level);
    h->sharpness = bits_rw(b, 3, h->sharpness);
    if ((h->lf_delta_enabled = bits_rw(b, 1, h->lf_delta_enabled))) {
        /* delta update (vp9.c:692-702); the encoder codes the values in effect that differ */
        const vp9h_seg_params *e = b->enc ? w->eseg : NULL;
        const int upd = e && e->lf_delta_update;
        if (bits_rw(b, 1, upd)) {
            for (int i = 0; i < 4; i++)
                if (bits_rw(b, 1, upd && e->lf_ref[i] != h->lf_ref[i])) h->lf_ref[i] = bits_sinv(b, 6, upd ? e->lf_ref[i] : 0);
            for (int i = 0; i < 2; i++)
                if (bits_rw(b, 1, upd && e->lf_mode[i] != h->lf_mode[i])) h->lf_mode[i] = bits_sinv(b, 6, upd ? e->lf_mode[i] : 0);
        }
    }
    h->qidx = bits_rw(b, 8, h->qidx);
    h->ydc = bits_rw(b, 1, h->ydc != 0) ? bits_sinv(b, 4, h->ydc) : 0;
    h->uvdc = bits_rw(b, 1, h->uvdc != 0) ? bits_sinv(b, 4, h->uvdc) : 0;
    h->uvac = bits_rw(b, 1, h->uvac != 0) ? bits_sinv(b, 4, h->uvac) : 0;
    h->lossless = h->qidx == 0 && !h->ydc && !h->uvdc && !h->uvac;
    if ((h->seg_enabled = bits_rw(b, 1, h->seg_enabled))) {
        if ((h->seg_update_map = bits_rw(b, 1, h->seg_update_map))) {
            for (int i = 0; i < 7; i++)
                h->seg_prob[i] = (uint8_t) (bits_rw(b, 1, h->seg_prob[i] != 255) ? bits_rw(b, 8, h->seg_prob[i]) : 255);
            if ((h->seg_temporal = bits_rw(b, 1, h->seg_temporal)))
                for (int i = 0; i < 3; i++)
                    h->seg_pred[i] = (uint8_t) (bits_rw(b, 1, h->seg_pred[i] != 255) ? bits_rw(b, 8, h->seg_pred[i]) : 255);
        }
        if ((h->seg_update_data = bits_rw(b, 1, h->seg_update_data))) {
            if (b->enc && w->eseg)                               /* the features to write */
                for (int i = 0; i < 8; i++) {
                    SegFeat *f = &h->seg[i];
                    memset(f, 0, sizeof(*f));
                    f->q_en = (w->eseg->q_en >> i) & 1;
                    f->q = f->q_en ? w->eseg->q[i] : 0;
                    f->lf_en = (w->eseg->lf_en >> i) & 1;
                    f->lf = f->lf_en ? w->eseg->lf[i] : 0;
                }
            h->seg_abs = bits_rw(b, 1, h->seg_abs);
            for (int i = 0; i < 8; i++) {
                SegFeat *f = &h->seg[i];
                if ((f->q_en = bits_rw(b, 1, f->q_en))) f->q = bits_sinv(b, 8, f->q);
                if ((f->lf_en = bits_rw(b, 1, f->lf_en))) f->lf = bits_sinv(b, 6, f->lf);
                if ((f->ref_en = bits_rw(b, 1, f->ref_en))) f->ref = bits_rw(b, 2, f->ref);
                f->skip = bits_rw(b, 1, f->skip);
            }
        }
    } else {
        h->seg_temporal = h->seg_update_map = 0;
    }
    /* tiling (vp9.c:800-815) */
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

/* the probability contexts a frame starts from (vp9.c:882-897) */
static void reset_contexts(Walk *w)
{
    const Hdr *h = w->h;
    if (h->keyframe || h->errorres || (h->intraonly && h->resetctx == 3))
        for (int i = 0; i < 4; i++) ctx_reset(&w->st->ctx[i]);
    else if (h->intraonly && h->resetctx == 2)
        ctx_reset(&w->st->ctx[h->ctxid_raw]);
}

/* The compressed header (vp9.c:903-1110), both directions: the frame's probabilities
 * start from saved context ctxid_raw, with forward updates. */
static int walk_compressed(Walk *w)
{
    BC *c = w->c;
    Hdr *h = w->h;
    const SavedCtx *ref = &w->st->ctx[h->ctxid_raw];
    PC *p = &w->pr.p;
    *p = ref->p;
    if (bc_bool(c, 128, 0)) return -1;                            /* marker bit */
    if (h->lossless) h->txmode = 0;
    else {
        int m = bc_uint(c, 2, MIN(h->txmode, 3));
        if (m == 3) m += bc_bool(c, 128, h->txmode == TX_SEL);
        h->txmode = m;
        if (m == TX_SEL) {
            for (int i = 0; i < 2; i++) maybe_update(w, &p->tx8p[i]);
            for (int i = 0; i < 2; i++) for (int j = 0; j < 2; j++) maybe_update(w, &p->tx16p[i][j]);
            for (int i = 0; i < 2; i++) for (int j = 0; j < 3; j++) maybe_update(w, &p->tx32p[i][j]);
        }
    }
    for (int t = 0; t < 4; t++) {
        const int upd = bc_bool(c, 128, c->enc && w->prob_updates && (rng_next(w) & 1));
        for (int i = 0; i < 2; i++)
            for (int j = 0; j < 2; j++)
                for (int k = 0; k < 6; k++)
                    for (int l = 0; l < 6; l++) {
                        if (l >= 3 && k == 0) break;          /* dc band: 3 contexts */
                        uint8_t *q = w->pr.coef[t][i][j][k][l];
                        memcpy(q, ref->coef[t][i][j][k][l], 3);
                        if (upd)
                            for (int n = 0; n < 3; n++) maybe_update(w, &q[n]);
                        memcpy(q + 3, vp9t_model_pareto8[q[2]], 8);
                    }
        if (h->txmode == t) break;
    }
    for (int i = 0; i < 3; i++) maybe_update(w, &p->skip[i]);
    if (h->keyframe || h->intraonly) return 0;
    for (int i = 0; i < 7; i++) for (int j = 0; j < 3; j++) maybe_update(w, &p->mv_mode[i][j]);
    if (h->filtermode == FILTER_SWITCHABLE)
        for (int i = 0; i < 4; i++) for (int j = 0; j < 2; j++) maybe_update(w, &p->filter[i][j]);
    for (int i = 0; i < 4; i++) maybe_update(w, &p->intra[i]);
    if (h->allowcomp) {
        int m = bc_bool(c, 128, h->comppred != P_SINGLE);
        if (m) m += bc_bool(c, 128, h->comppred == P_SWITCH);
        h->comppred = m;
        if (m == P_SWITCH)
            for (int i = 0; i < 5; i++) maybe_update(w, &p->comp[i]);
    } else {
        h->comppred = P_SINGLE;
    }
    if (h->comppred != P_COMP)
        for (int i = 0; i < 5; i++) { maybe_update(w, &p->single_ref[i][0]); maybe_update(w, &p->single_ref[i][1]); }
    if (h->comppred != P_SINGLE)
        for (int i = 0; i < 5; i++) maybe_update(w, &p->comp_ref[i]);
    for (int i = 0; i < 4; i++) for (int j = 0; j < 9; j++) maybe_update(w, &p->y_mode[i][j]);
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++)
            for (int k = 0; k < 3; k++) maybe_update(w, &p->partition[3 - i][j][k]);
    for (int i = 0; i < 3; i++) maybe_update_mv(w, &p->mv_joint[i]);
    for (int i = 0; i < 2; i++) {
        MvProbs *m = &p->mv_comp[i];
        maybe_update_mv(w, &m->sign);
        for (int j = 0; j < 10; j++) maybe_update_mv(w, &m->classes[j]);
        maybe_update_mv(w, &m->class0);
        for (int j = 0; j < 10; j++) maybe_update_mv(w, &m->bits[j]);
    }
    for (int i = 0; i < 2; i++) {
        MvProbs *m = &p->mv_comp[i];
        for (int j = 0; j < 2; j++) for (int k = 0; k < 3; k++) maybe_update_mv(w, &m->class0_fp[j][k]);
        for (int j = 0; j < 3; j++) maybe_update_mv(w, &m->fp[j]);
    }
    if (h->hp)
        for (int i = 0; i < 2; i++) { maybe_update_mv(w, &p->mv_comp[i].class0_hp); maybe_update_mv(w, &p->mv_comp[i].hp); }
    return 0;
}

/* ------------------------------------------------------------------ backward adaptation */
/* adapt_prob (vp9prob.c:25-40) */
static void adapt_prob(uint8_t *p, unsigned ct0, unsigned ct1, int max_count, int update_factor)
{
    const unsigned ct = ct0 + ct1;
    if (!ct) return;
    const unsigned uf = (unsigned) update_factor * MIN(ct, (unsigned) max_count) / (unsigned) max_count;
    const unsigned p1 = *p;
    unsigned p2 = (unsigned) ((((uint64_t) ct0 << 8) + (ct >> 1)) / ct);
    p2 = p2 < 1 ? 1 : p2 > 255 ? 255 : p2;
    *p = (uint8_t) (p1 + (((p2 - p1) * uf + 128) >> 8));
}
/* adapt a 10-symbol intra mode tree (vp9prob.c:250-290) */
static void adapt_intra_modes(uint8_t *pp, const unsigned *c)
{
    unsigned sum = c[0] + c[1] + c[3] + c[4] + c[5] + c[6] + c[7] + c[8] + c[9], s2;
    adapt_prob(&pp[0], c[2], sum, 20, 128);                      /* DC */
    sum -= c[9];
    adapt_prob(&pp[1], c[9], sum, 20, 128);                      /* TM */
    sum -= c[0];
    adapt_prob(&pp[2], c[0], sum, 20, 128);                      /* V */
    s2 = c[1] + c[4] + c[5];
    sum -= s2;
    adapt_prob(&pp[3], s2, sum, 20, 128);
    s2 -= c[1];
    adapt_prob(&pp[4], c[1], s2, 20, 128);                       /* H */
    adapt_prob(&pp[5], c[4], c[5], 20, 128);                     /* D135 / D117 */
    sum -= c[3];
    adapt_prob(&pp[6], c[3], sum, 20, 128);                      /* D45 */
    sum -= c[7];
    adapt_prob(&pp[7], c[7], sum, 20, 128);                      /* D63 */
    adapt_prob(&pp[8], c[6], c[8], 20, 128);                     /* D153 / D207 */
}
static void adapt3(uint8_t *pp, const unsigned *c)
{
    adapt_prob(&pp[0], c[0], c[1] + c[2] + c[3], 20, 128);
    adapt_prob(&pp[1], c[1], c[2] + c[3], 20, 128);
    adapt_prob(&pp[2], c[2], c[3], 20, 128);
}

/* ff_vp9_adapt_probs (vp9prob.c:42-290): merge this frame's counts into saved context
 * ctxid, starting from the context's pre-frame probabilities */
static void adapt_probs(Walk *w)
{
    const Hdr *h = w->h;
    SavedCtx *sc = &w->st->ctx[h->ctxid];
    PC *p = &sc->p;
    const Counts *ct = &w->cnt;
    const int uf = (h->keyframe || h->intraonly || !w->last_keyframe) ? 112 : 128;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 2; j++)
            for (int k = 0; k < 2; k++)
                for (int l = 0; l < 6; l++)
                    for (int m = 0; m < 6; m++) {
                        if (l == 0 && m >= 3) break;
                        uint8_t *pp = sc->coef[i][j][k][l][m];
                        const unsigned *e = ct->eob[i][j][k][l][m], *c = ct->coef[i][j][k][l][m];
                        adapt_prob(&pp[0], e[0], e[1], 24, uf);
                        adapt_prob(&pp[1], c[0], c[1] + c[2], 24, uf);
                        adapt_prob(&pp[2], c[1], c[2], 24, uf);
                    }
    if (h->keyframe || h->intraonly) {
        memcpy(p->skip, w->pr.p.skip, sizeof(p->skip));
        memcpy(p->tx32p, w->pr.p.tx32p, sizeof(p->tx32p));
        memcpy(p->tx16p, w->pr.p.tx16p, sizeof(p->tx16p));
        memcpy(p->tx8p, w->pr.p.tx8p, sizeof(p->tx8p));
        return;
    }
    for (int i = 0; i < 3; i++) adapt_prob(&p->skip[i], ct->skip[i][0], ct->skip[i][1], 20, 128);
    for (int i = 0; i < 4; i++) adapt_prob(&p->intra[i], ct->intra[i][0], ct->intra[i][1], 20, 128);
    if (h->comppred == P_SWITCH)
        for (int i = 0; i < 5; i++) adapt_prob(&p->comp[i], ct->comp[i][0], ct->comp[i][1], 20, 128);
    if (h->comppred != P_SINGLE)
        for (int i = 0; i < 5; i++) adapt_prob(&p->comp_ref[i], ct->comp_ref[i][0], ct->comp_ref[i][1], 20, 128);
    if (h->comppred != P_COMP)
        for (int i = 0; i < 5; i++) {
            adapt_prob(&p->single_ref[i][0], ct->single_ref[i][0][0], ct->single_ref[i][0][1], 20, 128);
            adapt_prob(&p->single_ref[i][1], ct->single_ref[i][1][0], ct->single_ref[i][1][1], 20, 128);
        }
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) adapt3(p->partition[i][j], ct->partition[i][j]);
    if (h->txmode == TX_SEL)
        for (int i = 0; i < 2; i++) {
            const unsigned *c16 = ct->tx16p[i], *c32 = ct->tx32p[i];
            adapt_prob(&p->tx8p[i], ct->tx8p[i][0], ct->tx8p[i][1], 20, 128);
            adapt_prob(&p->tx16p[i][0], c16[0], c16[1] + c16[2], 20, 128);
            adapt_prob(&p->tx16p[i][1], c16[1], c16[2], 20, 128);
            adapt3(p->tx32p[i], c32);
        }
    if (h->filtermode == FILTER_SWITCHABLE)
        for (int i = 0; i < 4; i++) {
            const unsigned *c = ct->filter[i];
            adapt_prob(&p->filter[i][0], c[0], c[1] + c[2], 20, 128);
            adapt_prob(&p->filter[i][1], c[1], c[2], 20, 128);
        }
    for (int i = 0; i < 7; i++) {
        const unsigned *c = ct->mv_mode[i];                       /* NEAREST, NEAR, ZERO, NEW */
        adapt_prob(&p->mv_mode[i][0], c[2], c[1] + c[0] + c[3], 20, 128);
        adapt_prob(&p->mv_mode[i][1], c[0], c[1] + c[3], 20, 128);
        adapt_prob(&p->mv_mode[i][2], c[1], c[3], 20, 128);
    }
    adapt3(p->mv_joint, ct->mv_joint);
    for (int i = 0; i < 2; i++) {
        MvProbs *m = &p->mv_comp[i];
        const typeof(ct->mv_comp[0]) *mc = &ct->mv_comp[i];
        adapt_prob(&m->sign, mc->sign[0], mc->sign[1], 20, 128);
        const unsigned *c = mc->classes;
        unsigned sum = c[1] + c[2] + c[3] + c[4] + c[5] + c[6] + c[7] + c[8] + c[9] + c[10];
        adapt_prob(&m->classes[0], c[0], sum, 20, 128);
        sum -= c[1];
        adapt_prob(&m->classes[1], c[1], sum, 20, 128);
        sum -= c[2] + c[3];
        adapt_prob(&m->classes[2], c[2] + c[3], sum, 20, 128);
        adapt_prob(&m->classes[3], c[2], c[3], 20, 128);
        sum -= c[4] + c[5];
        adapt_prob(&m->classes[4], c[4] + c[5], sum, 20, 128);
        adapt_prob(&m->classes[5], c[4], c[5], 20, 128);
        sum -= c[6];
        adapt_prob(&m->classes[6], c[6], sum, 20, 128);
        adapt_prob(&m->classes[7], c[7] + c[8], c[9] + c[10], 20, 128);
        adapt_prob(&m->classes[8], c[7], c[8], 20, 128);
        adapt_prob(&m->classes[9], c[9], c[10], 20, 128);
        adapt_prob(&m->class0, mc->class0[0], mc->class0[1], 20, 128);
        for (int j = 0; j < 10; j++) adapt_prob(&m->bits[j], mc->bits[j][0], mc->bits[j][1], 20, 128);
        for (int j = 0; j < 2; j++) adapt3(m->class0_fp[j], mc->class0_fp[j]);
        adapt3(m->fp, mc->fp);
        if (h->hp) {
            adapt_prob(&m->class0_hp, mc->class0_hp[0], mc->class0_hp[1], 20, 128);
            adapt_prob(&m->hp, mc->hp[0], mc->hp[1], 20, 128);
        }
    }
    for (int i = 0; i < 4; i++) adapt_intra_modes(p->y_mode[i], ct->y_mode[i]);
    for (int i = 0; i < 10; i++) adapt_intra_modes(p->uv_mode[i], ct->uv_mode[i]);
}

/* ------------------------------------------------------------------ frame walk */
static void tile_offsets(int idx, int log2n, int n, int *start, int *end)
{
    const int s0 = MIN((idx * n) >> log2n, n), s1 = MIN(((idx + 1) * n) >> log2n, n);
    *start = s0 * 8; *end = s1 * 8;
}

static int alloc_ctx(Walk *w)
{
    const size_t n = (size_t) w->sb_cols * 8 + 16;
    w->a_part = calloc(n, 1); w->a_skip = calloc(n, 1); w->a_tx = calloc(n, 1);
    w->a_mode = calloc(2 * n, 1); w->a_ynnz = calloc(2 * n, 1); w->a_unnz = calloc(2 * n, 1); w->a_vnnz = calloc(2 * n, 1);
    w->a_segpred = calloc(n, 1); w->a_intra = calloc(n, 1); w->a_comp = calloc(n, 1);
    w->a_ref = calloc(n, 1); w->a_filter = calloc(n, 1);
    w->a_mv = calloc(2 * n, sizeof(*w->a_mv));
    if (!w->a_part || !w->a_skip || !w->a_tx || !w->a_mode || !w->a_ynnz || !w->a_unnz || !w->a_vnnz ||
        !w->a_segpred || !w->a_intra || !w->a_comp || !w->a_ref || !w->a_filter || !w->a_mv)
        return -1;
    if (w->h->keyframe || w->h->intraonly) fill_ctx(w->a_mode, 2 /* DC_PRED */, 2 * n);
    else fill_ctx(w->a_mode, VP9H_NEARESTMV, n);
    return 0;
}
static void free_ctx(Walk *w)
{
    free(w->a_part); free(w->a_skip); free(w->a_tx); free(w->a_mode); free(w->a_ynnz); free(w->a_unnz); free(w->a_vnnz);
    free(w->a_segpred); free(w->a_intra); free(w->a_comp); free(w->a_ref); free(w->a_filter); free(w->a_mv);
}

/* One SB row of one tile: the left contexts restart (vp9.c:1358-1366), then its SBs. The
 * previous frame's MV pairs and the reference segmentation map of this SB row must be final
 * first (a pipelined parse may still be writing them); this row's are published after. */
static int walk_tile_row(Walk *w, BC *coder, int row, int c0, int c1)
{
    const int intra_frame = w->h->keyframe || w->h->intraonly;
    if ((w->mvref && side_wait(w->mvref, row >> 3)) || (w->segref && w->segref != w->mvref && side_wait(w->segref, row >> 3))) {
        w->err = 1;
        return -1;
    }
    w->tile_col_start = c0;
    fill_ctx(w->l_part, 0, sizeof(w->l_part)); fill_ctx(w->l_skip, 0, sizeof(w->l_skip));
    if (intra_frame) fill_ctx(w->l_mode, 2, sizeof(w->l_mode));
    else fill_ctx(w->l_mode, VP9H_NEARESTMV, 8);
    fill_ctx16(w->l_ynnz, 0, sizeof(w->l_ynnz)); fill_ctx16(w->l_unnz, 0, sizeof(w->l_unnz));
    fill_ctx16(w->l_vnnz, 0, sizeof(w->l_vnnz)); fill_ctx(w->l_segpred, 0, sizeof(w->l_segpred));
    w->c = coder;
    for (int col = c0; col < c1; col += 8) {
        /* a tile whose data ran out is invalid (vp9.c:1383-1385) */
        if (!w->c->enc && bd_overrun(&w->c->d) > 10) { w->err = 1; return -1; }
        walk_sb(w, row, col, 0);
        if (w->err) return -1;
    }
    side_publish(w->side, row >> 3);
    return 0;
}

/* Walk every tile (vp9.c:1325-1395): per tile row, SB rows, tile columns, SBs. */
static int walk_tiles(Walk *w, BC *coders)
{
    const int ntc = 1 << w->h->log2_tile_cols, ntr = 1 << w->h->log2_tile_rows;
    for (int tr = 0; tr < ntr; tr++) {
        int r0, r1;
        tile_offsets(tr, w->h->log2_tile_rows, w->sb_rows, &r0, &r1);
        for (int row = r0; row < r1; row += 8)
            for (int tc = 0; tc < ntc; tc++) {
                int c0, c1;
                tile_offsets(tc, w->h->log2_tile_cols, w->sb_cols, &c0, &c1);
                if (walk_tile_row(w, &coders[tr * ntc + tc], row, c0, c1) < 0) return -1;
            }
    }
    return 0;
}

/* ---- tile-column threads (decode_tiles_mt, vp9.c:1441-1520; launched at 1777-1806) ----
 * A tile column decodes independently of the others: its blocks read above / left
 * contexts and MV candidates of its own columns only (have_left and the candidate checks
 * stop at tile_col_start, vp9mvs.c / vp9block.c), and its bool coders are its own. Each
 * column walks all tile rows on a copy of the frame's walk state with its own left
 * contexts, coder, symbol counts and output arrays; the above contexts and the frame's MV /
 * segmentation arrays are shared, written at the column's own positions only. The packet
 * keeps the serial walk's order: per SB row, the tile columns' segments left to right. */
typedef struct TileCol {
    Walk w;
    BC *coders;
    int tc, ntc, ntr;
    size_t *seg;                         /* per SB row of the frame: (nb, ne, nc) at its end */
    int ret;
} TileCol;

static void *tile_col_run(void *arg)
{
    TileCol *t = arg;
    Walk *w = &t->w;
    int c0, c1;
    tile_offsets(t->tc, w->h->log2_tile_cols, w->sb_cols, &c0, &c1);
    for (int tr = 0; tr < t->ntr && !t->ret; tr++) {
        int r0, r1;
        tile_offsets(tr, w->h->log2_tile_rows, w->sb_rows, &r0, &r1);
        for (int row = r0; row < r1; row += 8) {
            if (walk_tile_row(w, &t->coders[tr * t->ntc + t->tc], row, c0, c1) < 0) { t->ret = -1; break; }
            size_t *e = t->seg + 3 * (row >> 3);
            e[0] = w->nb; e[1] = w->ne; e[2] = w->nc;
        }
    }
    return NULL;
}

typedef struct TileWorker { TileCol *cols; int first, step, n; } TileWorker;
static void *tile_worker_run(void *arg)
{
    TileWorker *k = arg;
    for (int i = k->first; i < k->n; i += k->step) tile_col_run(&k->cols[i]);
    return NULL;
}

static int walk_tiles_mt(Walk *w, BC *coders, int nthreads)
{
    const int ntc = 1 << w->h->log2_tile_cols, ntr = 1 << w->h->log2_tile_rows, nsr = w->sb_rows;
    TileCol *cols = calloc((size_t) ntc, sizeof(TileCol));
    size_t *segs = calloc((size_t) ntc * nsr * 3, sizeof(size_t));
    pthread_t th[64];
    TileWorker wk[64];
    int r = cols && segs ? 0 : -1, started = 0;
    nthreads = MIN(MIN(nthreads, ntc), 64);
    for (int tc = 0; tc < ntc && !r; tc++) {
        TileCol *t = &cols[tc];
        t->w = *w;                       /* shared: header, probabilities, above contexts, side buffers */
        memset(&t->w.cnt, 0, sizeof(t->w.cnt));
        t->w.blocks = NULL; t->w.nb = t->w.cb = 0;
        t->w.eobs = NULL; t->w.ne = t->w.ce = 0;
        t->w.coefs = NULL; t->w.nc = t->w.cc = 0;
        t->w.err = 0;
        t->coders = coders; t->tc = tc; t->ntc = ntc; t->ntr = ntr;
        t->seg = segs + (size_t) tc * nsr * 3;
    }
    for (int k = 1; k < nthreads && !r; k++) {
        wk[k] = (TileWorker) { cols, k, nthreads, ntc };
        if (pthread_create(&th[k], NULL, tile_worker_run, &wk[k])) break;
        started = k;
    }
    if (!r)                              /* this thread's share, and that of any thread that did not start */
        for (int k = 0; k < nthreads; k++)
            if (k == 0 || k > started) {
                wk[k] = (TileWorker) { cols, k, nthreads, ntc };
                tile_worker_run(&wk[k]);
            }
    for (int k = 1; k <= started; k++) pthread_join(th[k], NULL);
    for (int tc = 0; tc < ntc && !r; tc++)
        if (cols[tc].ret || cols[tc].w.err) { r = -1; w->err = cols[tc].w.err ? cols[tc].w.err : 1; }
    if (!r) {                            /* concatenate in the serial order: SB rows, then tile columns */
        size_t nb = 0, ne = 0, nc = 0;
        for (int tc = 0; tc < ntc; tc++) { nb += cols[tc].w.nb; ne += cols[tc].w.ne; nc += cols[tc].w.nc; }
        w->blocks = grow(w->blocks, &w->cb, w->nb + nb, sizeof(vp9h_block), &w->err);
        w->eobs = grow(w->eobs, &w->ce, w->ne + ne, sizeof(uint16_t), &w->err);
        w->coefs = grow(w->coefs, &w->cc, w->nc + nc, 1, &w->err);
        if (w->err) r = -1;
        for (int sr = 0; sr < nsr && !r; sr++)
            for (int tc = 0; tc < ntc; tc++) {
                const Walk *t = &cols[tc].w;
                const size_t *e = cols[tc].seg + 3 * sr, *p = sr ? e - 3 : NULL;
                const size_t b0 = p ? p[0] : 0, e0 = p ? p[1] : 0, k0 = p ? p[2] : 0;
                memcpy(w->blocks + w->nb, t->blocks + b0, (e[0] - b0) * sizeof(vp9h_block));
                memcpy(w->eobs + w->ne, t->eobs + e0, (e[1] - e0) * sizeof(uint16_t));
                memcpy(w->coefs + w->nc, t->coefs + k0, e[2] - k0);
                w->nb += e[0] - b0; w->ne += e[1] - e0; w->nc += e[2] - k0;
            }
        /* the columns' symbol counts (backward adaptation reads their sum, vp9prob.c) */
        unsigned *dst = (unsigned *) &w->cnt;
        for (int tc = 0; tc < ntc && !r; tc++) {
            const unsigned *src = (const unsigned *) &cols[tc].w.cnt;
            for (size_t i = 0; i < sizeof(Counts) / sizeof(unsigned); i++) dst[i] += src[i];
        }
    }
    for (int tc = 0; cols && tc < ntc; tc++) {
        free(cols[tc].w.blocks); free(cols[tc].w.eobs); free(cols[tc].w.coefs);
    }
    free(cols);
    free(segs);
    return r;
}

int vp9h_stream_set_threads(vp9h_stream *s, int n)
{
    if (!s || n < 1 || n > 64) return VP9HIP_EINVAL;
    s->tile_threads = n;
    return 0;
}

/* the frame's side buffers and the ones it reads (vp9_decode_frame, vp9.c:1616-1686) */
static int begin_frame(Walk *w, int retain_segmap)
{
    vp9h_stream *st = w->st;
    const Hdr *h = w->h;
    const int inter_src = !h->keyframe && !h->intraonly && !h->errorres;
    if (!retain_segmap || h->keyframe || h->intraonly) {
        side_unref(&st->segref);
        if (inter_src) st->segref = side_ref(st->cur);
    }
    w->mvref = inter_src ? side_ref(st->cur) : NULL;
    w->side = side_new(h->w, h->h);
    if (!w->side) return -1;
    w->side->ntc = 1 << h->log2_tile_cols;
    if (!w->mvref || w->mvref->w != h->w || w->mvref->h != h->h) side_unref(&st->segref);
    /* a counted reference: with a pipelined parse the next frame's begin_frame may drop the
     * stream's reference while this frame's tiles still wait on and read the map */
    w->segref = side_ref(st->segref);
    return 0;
}

/* the reference sizes the packet reports (before this frame refreshes any slot) */
static void capture_refs(Walk *w)
{
    const Hdr *h = w->h;
    for (int i = 0; i < 3; i++) {
        const int s = h->keyframe || h->intraonly ? -1 : h->refidx[i];
        w->ref_w[i] = s >= 0 ? w->st->slot[s].w : h->w;
        w->ref_h[i] = s >= 0 ? w->st->slot[s].h : h->h;
    }
}

/* the slots and CUR_FRAME after a frame (vp9.c:1845-1849): what the next frame's header
 * reads; with a pipelined parse, right after this frame's headers (its side buffers are
 * then written while the next frame's walk reads them, row by row) */
static void end_frame_header(Walk *w, int keep_side)
{
    vp9h_stream *st = w->st;
    const Hdr *h = w->h;
    for (int i = 0; i < 8; i++)
        if (h->refreshmask & (1 << i)) {
            st->slot[i].valid = 1; st->slot[i].w = h->w; st->slot[i].h = h->h; st->slot[i].bpp = h->bpp;
            st->slot[i].ss_h = h->ss_h; st->slot[i].ss_v = h->ss_v;
        }
    side_unref(&st->cur);
    st->cur = keep_side ? side_ref(w->side) : w->side;
    if (!keep_side) w->side = NULL;
}

/* the state after a frame (vp9.c:1738-1751, 1821-1823, 1845-1849) */
static void end_frame(Walk *w)
{
    vp9h_stream *st = w->st;
    const Hdr *h = w->h;
    if (h->refreshctx && !h->parallel) adapt_probs(w);
    for (int i = 0; i < 8; i++)
        if (h->refreshmask & (1 << i)) {
            st->slot[i].valid = 1; st->slot[i].w = h->w; st->slot[i].h = h->h; st->slot[i].bpp = h->bpp;
            st->slot[i].ss_h = h->ss_h; st->slot[i].ss_v = h->ss_v;
        }
    side_unref(&st->cur);
    st->cur = w->side;
    w->side = NULL;
    side_unref(&w->mvref);
}

/* the context save of refresh_frame_context with frame-parallel mode (vp9.c:1738-1752) */
static void save_forward_ctx(Walk *w)
{
    const Hdr *h = w->h;
    if (!h->refreshctx || !h->parallel) return;
    SavedCtx *sc = &w->st->ctx[h->ctxid];
    for (int t = 0; t < 4; t++) {
        for (int i = 0; i < 2; i++)
            for (int j = 0; j < 2; j++)
                for (int k = 0; k < 6; k++)
                    for (int l = 0; l < 6; l++) memcpy(sc->coef[t][i][j][k][l], w->pr.coef[t][i][j][k][l], 3);
        if (h->txmode == t) break;
    }
    sc->p = w->pr.p;
}

static void fill_info(const Walk *w, vp9h_frame_info *info)
{
    const Hdr *h = w->h;
    if (!info) return;
    memset(info, 0, sizeof(*info));
    info->show_existing_frame = 0;
    info->show_frame = !h->invisible;
    info->refresh_mask = h->refreshmask;
    for (int i = 0; i < 3; i++) { info->ref_slot[i] = h->refidx[i]; info->sign_bias[i] = h->signbias[i]; }
    info->error_res = h->errorres;
    info->refresh_ctx = h->refreshctx;
    info->parallel = h->parallel;
    info->ctx_id = h->ctxid_raw;
    info->allow_hp = h->hp;
    info->interp = h->filtermode;
    info->comp_mode = h->comppred;
    info->tx_mode = h->txmode;
}

static void fill_packet(Walk *w, vp9h_frame *out)
{
    const Hdr *h = w->h;
    memset(out, 0, sizeof(*out));
    out->width = h->w; out->height = h->h; out->bpp = (uint8_t) h->bpp;
    out->ss_h = (uint8_t) h->ss_h; out->ss_v = (uint8_t) h->ss_v;
    out->keyframe = (uint8_t) h->keyframe; out->intraonly = (uint8_t) (h->intraonly && !h->keyframe);  /* stale after a keyframe */
    out->lossless = (uint8_t) h->lossless;
    out->filter_level = (uint8_t) h->filter_level; out->sharpness = (uint8_t) h->sharpness;
    out->log2_tile_cols = (uint8_t) h->log2_tile_cols; out->log2_tile_rows = (uint8_t) h->log2_tile_rows;
    memcpy(out->lflvl, h->lflvl, sizeof(out->lflvl));
    for (int i = 0; i < 3; i++) {
        out->ref_w[i] = w->ref_w[i];
        out->ref_h[i] = w->ref_h[i];
    }
    out->nblocks = (uint32_t) w->nb; out->neobs = (uint32_t) w->ne;
    out->ncoefs = w->nc / (h->bpp > 8 ? 4 : 2);
    out->blocks = w->blocks; out->eobs = w->eobs; out->coefs = w->coefs;
    w->blocks = NULL; w->eobs = NULL; w->coefs = NULL;
}

static void walk_free(Walk *w)
{
    free_ctx(w);
    free(w->blocks); free(w->eobs); free(w->coefs);
    side_unref(&w->side);
    side_unref(&w->mvref);
    side_unref(&w->segref);
}

/* ------------------------------------------------------------------ API: decode */
/* A frame between its headers and its tiles. */
struct vp9h_pending {
    Walk *w;
    BC *coders;
    int serial;                          /* the next frame's headers read this frame's adapted probabilities */
    int done;                            /* the tiles' walk completed (else the side is failed) */
};

static void pending_free(vp9h_pending *p)
{
    if (!p) return;
    if (p->w) {
        if (!p->done) side_fail(p->w->side);
        walk_free(p->w);
        free(p->w);
    }
    free(p->coders);
    free(p);
}

/* The uncompressed and compressed headers and the tile layout of one frame (vp9.c:519-1110,
 * 1247-1262): 0 with *pend set, or 0 with *pend NULL for show_existing_frame (info says
 * which slot), or an error. data must outlive the tiles' walk. */
static int decode_headers(vp9h_stream *st, const uint8_t *data, size_t size, vp9h_frame_info *info, vp9h_pending **pend)
{
    *pend = NULL;
    Walk *w = calloc(1, sizeof(Walk));
    if (!w) return VP9HIP_ENOMEM;
    w->st = st;
    w->h = &st->h;
    w->last_keyframe = st->h.keyframe;
    w->last_invisible = st->h.invisible;
    const int retain = st->segref && (!st->h.seg_enabled || !st->h.seg_update_map);
    Bits b;
    memset(&b, 0, sizeof(b));
    b.in = data; b.in_bits = size * 8;
    int existing = -1;
    const long szpos = walk_uncompressed(w, &b, &existing);
    int r = 0;
    if (szpos == -3) {
        if (b.err) r = VP9HIP_EINVALIDDATA;
        else if (!st->slot[existing].valid) r = VP9HIP_EINVALIDDATA;    /* vp9.c:1641-1644 */
        else if (info) {
            memset(info, 0, sizeof(*info));
            info->show_existing_frame = 1;
            info->show_slot = existing;
            info->show_frame = 1;
        }
        free(w);
        return r;
    }
    if (szpos == -2) { free(w); return VP9HIP_ENOSYS; }
    if (szpos < 0 || b.err) { free(w); return VP9HIP_EINVALIDDATA; }
    const Hdr *h = w->h;
    b.bit = (size_t) szpos;
    const size_t csize = (size_t) bits_rw(&b, 16, 0);
    const size_t hbytes = (size_t) ((szpos + 16 + 7) >> 3);
    if (hbytes + csize > size || !csize) { free(w); return VP9HIP_EINVALIDDATA; }
    reset_contexts(w);
    BC ch;
    memset(&ch, 0, sizeof(ch));
    bd_init(&ch.d, data + hbytes, csize);
    w->c = &ch;
    if (walk_compressed(w) < 0) { free(w); return VP9HIP_EINVALIDDATA; }
    capture_refs(w);
    /* tiles */
    const int ntc = 1 << h->log2_tile_cols, ntr = 1 << h->log2_tile_rows, nt = ntc * ntr;
    vp9h_pending *p = calloc(1, sizeof(*p));
    BC *coders = calloc((size_t) nt, sizeof(BC));
    if (p) { p->w = w; p->coders = coders; }
    if (!p || !coders || alloc_ctx(w) < 0 || begin_frame(w, retain) < 0) r = VP9HIP_ENOMEM;
    const uint8_t *q = data + hbytes + csize, *end = data + size;
    for (int i = 0; i < nt && !r; i++) {
        size_t n = (size_t) (end - q);
        if (i + 1 < nt) {
            if (end - q < 4) { r = VP9HIP_EINVALIDDATA; break; }
            n = (size_t) q[0] << 24 | (size_t) q[1] << 16 | (size_t) q[2] << 8 | q[3];
            q += 4;
            if (n > (size_t) (end - q)) { r = VP9HIP_EINVALIDDATA; break; }
        }
        bd_init(&coders[i].d, q, n);
        if (bc_bool(&coders[i], 128, 0)) r = VP9HIP_EINVALIDDATA;   /* marker bit */
        q += n;
    }
    if (!r) save_forward_ctx(w);
    if (r) {
        if (p) pending_free(p);
        else { free(coders); walk_free(w); free(w); }
        return r;
    }
    fill_info(w, info);
    if (info) { info->header_size = (uint32_t) hbytes; info->compressed_header_size = (uint32_t) csize; }
    p->serial = h->refreshctx && !h->parallel;
    *pend = p;
    return 0;
}

/* The tiles of a frame whose headers were read (vp9.c:1325-1395 / 1441-1520): 0 or an error. */
static int decode_tiles(vp9h_pending *p, int threads)
{
    Walk *w = p->w;
    const int ntc = 1 << w->h->log2_tile_cols;
    if ((threads > 1 && ntc > 1 ? walk_tiles_mt(w, p->coders, threads) : walk_tiles(w, p->coders)) < 0) {
        side_fail(w->side);
        return w->err ? VP9HIP_EINVALIDDATA : VP9HIP_ENOMEM;
    }
    return 0;
}

int vp9h_stream_decode(vp9h_stream *st, const uint8_t *data, size_t size, vp9h_frame *out, vp9h_frame_info *info)
{
    if (!st || !data || !out || size < 1) return VP9HIP_EINVAL;
    memset(out, 0, sizeof(*out));
    vp9h_pending *p = NULL;
    int r = decode_headers(st, data, size, info, &p);
    if (r < 0 || !p) return r;
    r = decode_tiles(p, st->tile_threads);
    if (!r) {
        end_frame(p->w);
        fill_packet(p->w, out);
        p->done = 1;
    }
    pending_free(p);
    return r;
}

int vp9h_stream_decode_begin(vp9h_stream *st, const uint8_t *data, size_t size, vp9h_pending **pend,
                             vp9h_frame_info *info, int *serial)
{
    if (!st || !data || !pend || size < 1) return VP9HIP_EINVAL;
    *pend = NULL;
    if (serial) *serial = 0;
    vp9h_pending *p = NULL;
    const int r = decode_headers(st, data, size, info, &p);
    if (r < 0 || !p) return r;
    /* the stream moves on to the next frame's headers: this frame keeps its header as of
     * now, and its side buffers become CUR_FRAME (written row by row by its tiles' walk) */
    p->w->hs = st->h;
    p->w->h = &p->w->hs;
    end_frame_header(p->w, 1);
    if (serial) *serial = p->serial;
    *pend = p;
    return 0;
}

int vp9h_stream_decode_finish(vp9h_pending *p, int threads, vp9h_frame *out)
{
    if (!p || !out || threads < 1 || threads > 64) { pending_free(p); return VP9HIP_EINVAL; }
    memset(out, 0, sizeof(*out));
    int r = decode_tiles(p, threads);
    if (!r) {
        Walk *w = p->w;
        if (p->serial) adapt_probs(w);   /* vp9.c:1821-1823; the next frame's headers wait for it */
        fill_packet(w, out);
        p->done = 1;
    }
    pending_free(p);
    return r;
}

void vp9h_pending_free(vp9h_pending *p) { pending_free(p); }

/* ------------------------------------------------------------------ API: encode */
void vp9h_enc_defaults(vp9h_enc_params *p)
{
    if (!p) return;
    memset(p, 0, sizeof(*p));
    p->base_q_idx = 60;
    p->show_existing_frame = 0;
    p->show_frame = 1;
    p->refresh_mask = -1;                 /* keyframes: all; inter frames: slot 0 */
    p->ref_slot[0] = 0; p->ref_slot[1] = 1; p->ref_slot[2] = 2;
    p->sign_bias[2] = 1;                  /* ALTREF "from the future": compound allowed */
    p->refresh_ctx = 0; p->parallel = 1; p->ctx_id = 0; p->reset_ctx = 3;
    p->allow_hp = 1;
    p->interp = -1;
    p->comp_mode = -1;
    p->tx_mode = -1;
}

static int write_frame(Walk *w, Bits *b, long szpos, BC *ch, BC *coders, int nt, uint8_t **out, size_t *out_size)
{
    const size_t hbytes = (size_t) ((szpos + 16 + 7) >> 3);
    b->bit = (size_t) szpos;
    bits_rw(b, 16, (int) ch->e.pos);
    b->bit = hbytes * 8;
    size_t total = hbytes + ch->e.pos;
    for (int i = 0; i < nt; i++) total += coders[i].e.pos + (i + 1 < nt ? 4 : 0);
    uint8_t *o = malloc(total);
    if (!o || b->err) { free(o); return VP9HIP_ENOMEM; }
    size_t pos = 0;
    memcpy(o, b->buf, hbytes); pos = hbytes;
    memcpy(o + pos, ch->e.buf, ch->e.pos); pos += ch->e.pos;
    for (int i = 0; i < nt; i++) {
        const size_t n = coders[i].e.pos;
        if (i + 1 < nt) { o[pos] = (uint8_t) (n >> 24); o[pos + 1] = (uint8_t) (n >> 16); o[pos + 2] = (uint8_t) (n >> 8); o[pos + 3] = (uint8_t) n; pos += 4; }
        memcpy(o + pos, coders[i].e.buf, n); pos += n;
    }
    (void) w;
    *out = o;
    *out_size = total;
    return 0;
}

int vp9h_stream_encode(vp9h_stream *st, const vp9h_frame *pkt, const vp9h_enc_params *ep,
                       uint8_t **out, size_t *out_size, vp9h_frame *coded)
{
    vp9h_enc_params defp;
    if (!ep) { vp9h_enc_defaults(&defp); ep = &defp; }
    if (!st || !out || !out_size) return VP9HIP_EINVAL;
    if (coded) memset(coded, 0, sizeof(*coded));
    Bits b;
    memset(&b, 0, sizeof(b));
    b.enc = 1;
    Hdr *h = &st->h;
    if (ep->show_existing_frame) {
        /* frame marker, profile, show_existing_frame, the slot (vp9.c:532-545) */
        if (ep->show_slot < 0 || ep->show_slot > 7 || !st->slot[ep->show_slot].valid) return VP9HIP_EINVAL;
        Walk w0;
        memset(&w0, 0, sizeof(w0));
        w0.st = st; w0.h = h;
        int slot = ep->show_slot;
        if (walk_uncompressed(&w0, &b, &slot) != -3 || b.err) { free(b.buf); return VP9HIP_EINVAL; }
        const size_t n = (b.bit + 7) >> 3;        /* 1 byte; 2 in profile 3 (its reserved bit) */
        *out = malloc(n);
        if (!*out) { free(b.buf); return VP9HIP_ENOMEM; }
        memcpy(*out, b.buf, n);
        *out_size = n;
        free(b.buf);
        return 0;
    }
    if (!pkt || ep->base_q_idx < 0 || ep->base_q_idx > 255) return VP9HIP_EINVAL;
    if (pkt->ss_h > 1 || pkt->ss_v > 1 || (pkt->bpp != 8 && pkt->bpp != 10 && pkt->bpp != 12)) return VP9HIP_ENOSYS;
    const int inter = !pkt->keyframe && !pkt->intraonly;
    const int retain = st->segref && (!st->h.seg_enabled || !st->h.seg_update_map);
    const int last_keyframe = h->keyframe, last_invisible = h->invisible;
    /* the frame header this packet needs */
    h->profile = (pkt->bpp > 8 ? 2 : 0) | !(pkt->ss_h && pkt->ss_v);   /* profiles 1 / 3: not 4:2:0 */
    h->keyframe = pkt->keyframe;
    h->intraonly = pkt->intraonly && !pkt->keyframe;
    h->invisible = !ep->show_frame;
    if (h->intraonly) h->invisible = 1;                       /* intra_only is coded in hidden frames only */
    h->errorres = ep->error_res;
    h->w = pkt->width; h->h = pkt->height; h->bpp = pkt->bpp; h->ss_h = pkt->ss_h; h->ss_v = pkt->ss_v;
    h->refreshctx = ep->refresh_ctx; h->parallel = ep->parallel;
    h->ctxid_raw = ep->ctx_id & 3;
    h->resetctx = ep->reset_ctx & 3;
    h->refreshmask = ep->refresh_mask >= 0 ? (ep->refresh_mask & 0xff) : (h->keyframe ? 0xff : inter ? 1 : 0xff);
    h->lf_delta_enabled = 1;         /* libvpx's default ref / mode deltas, as the packet's levels assume */
    h->filter_level = pkt->filter_level; h->sharpness = pkt->sharpness;
    h->qidx = pkt->lossless ? 0 : ep->base_q_idx;
    h->ydc = h->uvdc = h->uvac = 0;
    /* segmentation (vp9.c:707-765): the map's tree / prediction probabilities are coded as 128 */
    h->seg_enabled = !!ep->seg.enabled;
    h->seg_update_map = h->seg_enabled && (ep->seg.update_map || h->keyframe || h->intraonly);
    h->seg_temporal = h->seg_update_map && ep->seg.temporal && inter;
    h->seg_update_data = h->seg_enabled && ep->seg.update_data;
    h->seg_abs = !!ep->seg.abs_delta;
    for (int i = 0; i < 7; i++) h->seg_prob[i] = 128;
    for (int i = 0; i < 3; i++) h->seg_pred[i] = 128;
    h->log2_tile_cols = pkt->log2_tile_cols; h->log2_tile_rows = pkt->log2_tile_rows;
    h->txmode = pkt->lossless ? 0 : ep->tx_mode >= 0 ? ep->tx_mode : TX_SEL;
    if (inter) {
        for (int i = 0; i < 3; i++) {
            h->refidx[i] = ep->ref_slot[i] & 7;
            h->signbias[i] = !!ep->sign_bias[i];
            if (!st->slot[h->refidx[i]].valid || st->slot[h->refidx[i]].bpp != pkt->bpp ||
                st->slot[h->refidx[i]].ss_h != pkt->ss_h || st->slot[h->refidx[i]].ss_v != pkt->ss_v) return VP9HIP_EINVAL;
        }
        h->hp = !!ep->allow_hp;
        /* one filter for every inter block: a fixed filter mode, else switchable */
        int f = -2, any_comp = 0;
        for (uint32_t i = 0; i < pkt->nblocks; i++) {
            const vp9h_block *bk = &pkt->blocks[i];
            if (bk->intra) continue;
            any_comp |= bk->comp;
            f = f == -2 ? bk->filter : f == bk->filter ? f : -1;
        }
        h->filtermode = ep->interp >= 0 ? ep->interp : f >= 0 ? f : f == -2 ? VP9H_FILTER_REGULAR : FILTER_SWITCHABLE;
        if (h->filtermode != FILTER_SWITCHABLE)
            for (uint32_t i = 0; i < pkt->nblocks; i++)
                if (!pkt->blocks[i].intra && pkt->blocks[i].filter != h->filtermode) return VP9HIP_EINVAL;
        if (h->filtermode == FILTER_SWITCHABLE)
            for (uint32_t i = 0; i < pkt->nblocks; i++)
                if (!pkt->blocks[i].intra && pkt->blocks[i].filter > VP9H_FILTER_SHARP) return VP9HIP_EINVAL;
        h->comppred = ep->comp_mode >= 0 ? ep->comp_mode : any_comp ? P_SWITCH : P_SINGLE;
    }
    Walk *w = calloc(1, sizeof(Walk));
    if (!w) return VP9HIP_ENOMEM;
    w->st = st; w->h = h; w->in = pkt;
    w->prob_updates = ep->prob_updates;
    w->eseg = &ep->seg;
    w->keep_modes = ep->keep_modes;
    w->rng = (uint64_t) ep->prob_updates * 0x2545F4914F6CDD1Dull;
    w->last_keyframe = last_keyframe;
    w->last_invisible = last_invisible;
    int existing = -1;
    const long szpos = walk_uncompressed(w, &b, &existing);
    int r = 0;
    if (szpos < 0 || b.err) r = szpos == -2 ? VP9HIP_ENOSYS : VP9HIP_EINVAL;
    else if (h->lossless != !!pkt->lossless) r = VP9HIP_EINVAL;
    else if (inter && h->allowcomp == 0 && h->comppred != P_SINGLE) r = VP9HIP_EINVAL;
    else {
        /* the packet's LF levels must be the ones this header produces */
        for (int s = 0; s < 8 && !r; s++)
            for (int i = 0; i < 4 && !r; i++)
                for (int m = 0; m < 2; m++)
                    if (h->lflvl[s][i][m] != pkt->lflvl[s][i][m]) { r = VP9HIP_EINVAL; break; }
    }
    BC ch;
    memset(&ch, 0, sizeof(ch));
    const int ntc = 1 << h->log2_tile_cols, ntr = 1 << h->log2_tile_rows, nt = ntc * ntr;
    BC *coders = NULL;
    if (!r) {
        reset_contexts(w);
        ch.enc = 1;
        be_init(&ch.e);
        w->c = &ch;
        if (walk_compressed(w) < 0) r = VP9HIP_EBUG;
        be_flush(&ch.e);
        coders = calloc((size_t) nt, sizeof(BC));
        if (!coders || alloc_ctx(w) < 0 || begin_frame(w, retain) < 0) r = VP9HIP_ENOMEM;
    }
    if (!r) {
        save_forward_ctx(w);
        for (int i = 0; i < nt; i++) { coders[i].enc = 1; be_init(&coders[i].e); bc_bool(&coders[i], 128, 0); }
        if (walk_tiles(w, coders) < 0 || w->bi != pkt->nblocks || w->ei != pkt->neobs || w->ci != pkt->ncoefs)
            r = VP9HIP_EINVALIDDATA;
    }
    if (!r) {
        for (int i = 0; i < nt; i++) { be_flush(&coders[i].e); if (coders[i].e.err) r = VP9HIP_EINVALIDDATA; }
        if (ch.e.err || ch.e.pos > 0xffff) r = r ? r : VP9HIP_EINVAL;
    }
    if (!r) r = write_frame(w, &b, szpos, &ch, coders, nt, out, out_size);
    if (!r) {
        capture_refs(w);
        end_frame(w);
        if (coded) fill_packet(w, coded);
    }
    free(b.buf);
    free(ch.e.buf);
    if (coders) for (int i = 0; i < nt; i++) free(coders[i].e.buf);
    free(coders);
    walk_free(w);
    free(w);
    return r;
}

/* ------------------------------------------------------------------ one-frame forms */
int vp9h_encode_frame(const vp9h_frame *pkt, int base_q_idx, uint8_t **out, size_t *out_size)
{
    if (!pkt || !out || !out_size || base_q_idx < 0 || base_q_idx > 255) return VP9HIP_EINVAL;
    if (!pkt->keyframe && !pkt->intraonly) return VP9HIP_ENOSYS;      /* needs reference state */
    vp9h_stream *st;
    int r = vp9h_stream_open(&st);
    if (r) return r;
    vp9h_enc_params ep;
    vp9h_enc_defaults(&ep);
    ep.base_q_idx = base_q_idx;
    ep.show_frame = pkt->keyframe;
    r = vp9h_stream_encode(st, pkt, &ep, out, out_size, NULL);
    vp9h_stream_close(st);
    return r;
}

int vp9h_decode_frame(const uint8_t *data, size_t size, vp9h_frame *out)
{
    if (!data || !out || size < 3) return VP9HIP_EINVAL;
    vp9h_stream *st;
    int r = vp9h_stream_open(&st);
    if (r) return r;
    vp9h_frame_info info;
    r = vp9h_stream_decode(st, data, size, out, &info);
    if (!r && info.show_existing_frame) r = VP9HIP_EINVALIDDATA;    /* no reference state here */
    vp9h_stream_close(st);
    return r;
}

void vp9h_frame_free(vp9h_frame *f)
{
    if (!f) return;
    free((void *) f->blocks); free((void *) f->eobs); free((void *) f->coefs);
    f->blocks = NULL; f->eobs = NULL; f->coefs = NULL;
}

void vp9h_buffer_free(uint8_t *p) { free(p); }

/* ------------------------------------------------------------------ container side */
/* vp9_superframe_split_bsf (bsf/vp9_superframe_split.c:40-95): the frames of a
 * superframe, from the index at its end; one frame otherwise */
/* The frame type from the first header bits (vp9.c:521-545): 0 keyframe, 1 other frame,
 * 2 show_existing_frame; AVERROR_INVALIDDATA for a bad marker / profile. A keyframe's
 * parse depends on no earlier frame (contexts, loop-filter deltas, segmentation and the
 * reference slots are all reset, vp9.c:557-569, 882-892), which lets a decoder parse it
 * on a fresh vp9h_stream in parallel with the frames before it. */
int vp9h_frame_type(const uint8_t *data, size_t size)
{
    if (!data || size < 1) return VP9HIP_EINVALIDDATA;
    const unsigned b = (unsigned) data[0] << 8 | (size > 1 ? data[1] : 0);
    if ((b >> 14) != 2) return VP9HIP_EINVALIDDATA;                 /* frame marker */
    const int prof = (b >> 13 & 1) | (b >> 12 & 1) << 1;
    int pos = 12;                                                    /* next bit (from the top) */
    if (prof == 3 && (b >> --pos & 1)) return VP9HIP_EINVALIDDATA;  /* reserved bit */
    if (b >> --pos & 1) return 2;                                    /* show_existing_frame */
    return (b >> --pos & 1) ? 1 : 0;                                 /* frame_type: 0 = key */
}

/* The reference bookkeeping of a frame from its uncompressed header alone (the start of
 * decode_frame_header, vp9.c:519-611): show_existing_frame / its slot, show_frame,
 * error_res, and refresh_frame_flags with the LAST / GOLDEN / ALTREF slots (refidx) of an
 * inter frame. Everything read here precedes the first field that needs stream state, so
 * it takes no vp9h_stream: what vp9.c knows before ff_thread_finish_setup. */
int vp9h_frame_peek(const uint8_t *data, size_t size, vp9h_frame_info *info)
{
    if (!data || size < 1 || !info) return VP9HIP_EINVAL;
    memset(info, 0, sizeof(*info));
    Bits b;
    memset(&b, 0, sizeof(b));
    b.in = data; b.in_bits = size * 8;
    Hdr h;
    memset(&h, 0, sizeof(h));
    if (bits_rw(&b, 2, 0) != 2) return VP9HIP_EINVALIDDATA;             /* frame marker */
    int prof = bits_rw(&b, 1, 0);
    prof |= bits_rw(&b, 1, 0) << 1;
    if (prof == 3 && bits_rw(&b, 1, 0)) return VP9HIP_EINVALIDDATA;    /* reserved bit */
    if (bits_rw(&b, 1, 0)) {                                            /* show_existing_frame */
        info->show_existing_frame = 1;
        info->show_slot = bits_rw(&b, 3, 0);
        info->show_frame = 1;
        return b.err ? VP9HIP_EINVALIDDATA : 2;
    }
    const int key = !bits_rw(&b, 1, 0);
    info->show_frame = bits_rw(&b, 1, 0);
    info->error_res = bits_rw(&b, 1, 0);
    int type = key ? 0 : 1;
    if (key) {
        info->refresh_mask = 0xff;
    } else {
        const int intraonly = info->show_frame ? 0 : bits_rw(&b, 1, 0);
        if (!info->error_res) bits_rw(&b, 2, 0);                        /* reset_frame_context */
        if (intraonly) {
            if (bits_rw(&b, 24, 0) != 0x498342) return VP9HIP_EINVALIDDATA;
            if (prof >= 1 && walk_color(&b, &h, prof) < 0) return VP9HIP_EINVALIDDATA;
            info->refresh_mask = bits_rw(&b, 8, 0);
            type = 3;
        } else {
            info->refresh_mask = bits_rw(&b, 8, 0);
            for (int i = 0; i < 3; i++) {
                info->ref_slot[i] = bits_rw(&b, 3, 0);
                info->sign_bias[i] = bits_rw(&b, 1, 0) && !info->error_res;
            }
        }
    }
    return b.err ? VP9HIP_EINVALIDDATA : type;
}

int vp9h_superframe_split(const uint8_t *data, size_t size, size_t *offsets, size_t *sizes, int cap)
{
    if (!data || size < 1) return VP9HIP_EINVAL;
    const uint8_t marker = data[size - 1];
    if ((marker & 0xe0) == 0xc0) {
        const int len = 1 + ((marker >> 3) & 3), n = 1 + (marker & 7);
        const size_t idx = 2 + (size_t) n * len;
        if (size >= idx && data[size - idx] == marker) {
            const uint8_t *q = data + size + 1 - idx;
            size_t off = 0;
            for (int i = 0; i < n; i++) {
                size_t fs = 0;
                for (int j = 0; j < len; j++) fs |= (size_t) q[i * len + j] << (8 * j);
                if (!fs || off + fs > size - idx) return VP9HIP_EINVAL;
                if (i < cap) { offsets[i] = off; sizes[i] = fs; }
                off += fs;
            }
            return n;
        }
    }
    if (cap > 0) { offsets[0] = 0; sizes[0] = size; }
    return 1;
}
