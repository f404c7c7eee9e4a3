/*
 * Device work lists built by the host runtime from pass-1 packets and consumed by
 * the gfx950 kernels. Internal to libvp9hip (not part of the C-ABI).
 *
 * HBM layout per frame buffer: three planes, luma padded to 64 x 64 superblocks,
 * chroma to the matching subsampled size; pitch in pixels. Pixels are uint8_t
 * (bpp 8) or uint16_t (bpp 10/12). Nothing outside the 8-aligned frame area is
 * ever read (intra edge rules vp9recon.c:103,192; LF masks vp9block.c:1442; MC
 * clamps to the visible size, videodsp_template.c:27-105), so the padding needs no
 * border extension.
 */
#ifndef VP9HIP_WORK_H
#define VP9HIP_WORK_H
#include <stdint.h>

/* Per-frame descriptor (device array, indexed by SBRec.frame / McUnit.frame). */
typedef struct FrameDesc {
    uint64_t plane[3];        /* device pointers                                      */
    uint64_t ref[3][3];       /* [LAST/GOLDEN/ALTREF][plane] device pointers           */
    int32_t  pitch[2];        /* luma / chroma pitch (pixels)                         */
    int32_t  w8[2], h8[2];    /* 8-aligned plane size (cols*8 >> ss)                  */
    int32_t  refw[3][2], refh[3][2]; /* visible ref plane sizes (MC clamp)           */
    int32_t  sb_cols, sb_rows;
    int32_t  bd;              /* bit depth                                            */
    int32_t  sharp;           /* LF sharpness                                         */
    uint64_t edge;            /* intra frames: per SB (raster) its pre-LF right column,
                                 EDGE_PIX pixels (luma 64, then the chroma planes' rows),
                                 written by its intra workgroup, read by the SB to its
                                 right instead of 128 one-pixel frame rows; 0: none     */
} FrameDesc;
#define EDGE_PIX 192          /* pixels per SB in FrameDesc.edge (64 + 2 x 64 at 4:4:4) */

/* Residual job (k_resid): one tx block with coefficients, 16 bytes. The residual
 * (out + (1 << (bits - 1))) >> bits of itxfm_add (vp9dsp_template.c:1139-1180) depends
 * on the coefficients only, so every tx block of a batch is transformed in parallel;
 * intra residuals go to a scratch buffer (column-major n x n int16) that k_pred adds
 * after prediction, inter residuals are added in place onto the MC prediction. */
typedef struct RJob {
    uint32_t coef;            /* element offset of the scan-order coefficients          */
    uint32_t dst;             /* intra: residual offset / 16 (int16 elements);
                                 inter: pixel offset y * pitch + x in plane of `frame`  */
    uint16_t eob;
    uint16_t frame;
    uint8_t  ptx;             /* plane | tx code << 2 (0..3, 4 = WHT) | inplace << 5 | txtp << 6 */
    uint8_t  nzc, nzr;        /* bounding box of scan[0 .. eob-1] (a zero column transforms to zero) */
    uint8_t  pad;
} RJob;

#define RJ_PLANE(j) ((j).ptx & 3)
#define RJ_INPLACE(j) (((j).ptx >> 5) & 1)
#define RJ_TXTP(j) ((j).ptx >> 6)

/* Intra prediction job (k_pred), 8 bytes, so a whole SB's list fits in LDS. The host
 * resolves check_intra_mode (vp9recon.c:37-221) ahead of time: the final mode after
 * mode_conv and the edge clamps n_px_have (vp9recon.c:103,192) are stored, so the
 * kernel's edge fill is branch-free.
 *   a:  plane (2b) | ts << 2 (2b) | has_residual << 4 | top_right_real << 5 |
 *       have_top << 6 | have_left << 7 | mslot << 8 (4b) | x4 << 12 | y4 << 16 |
 *       ct << 20 (5b: last valid top column) | cl << 25 (5b: last valid left row)
 *   mslot: 0 V, 1 H, 2 DL, 3 DR, 4 VR, 5 HD, 6 VL, 7 HU, 8 TM, 9 DC, 10 LEFT_DC,
 *          11 TOP_DC, 12 DC_128, 13 DC_127, 14 DC_129 */
typedef struct PJob {
    uint32_t a;
    uint32_t roff;            /* residual offset / 16 (absolute in the batch)              */
} PJob;

#define PJ_PLANE(j) ((j).a & 3)
#define PJ_TS(j) (((j).a >> 2) & 3)
#define PJ_RES(j) (((j).a >> 4) & 1)
#define PJ_TRREAL(j) (((j).a >> 5) & 1)
#define PJ_HTOP(j) (((j).a >> 6) & 1)
#define PJ_HLEFT(j) (((j).a >> 7) & 1)
#define PJ_MSLOT(j) (((j).a >> 8) & 15)
#define PJ_X4(j) (((j).a >> 12) & 15)
#define PJ_Y4(j) (((j).a >> 16) & 15)
#define PJ_CT(j) (((j).a >> 20) & 31)
#define PJ_CL(j) (((j).a >> 25) & 31)

/* Intra predictor formula table: for (table slot 0..9, ts, y, x) one word
 *   i0 | i1 << 7 | i2 << 14 | wb << 21 | wc << 23 (2-bit signed: 1 = +1, 3 = -1) | s << 25 | dc << 27
 * pixel = dc ? DC : clip((e[i0] + wb * e[i1] + wc * e[i2] + ((1 << s) >> 1)) >> s) over the
 * job's edge array e (left column bottom-to-top, top-left, top row + top-right). */
#define PTAB_SLOT 1360        /* 16 + 64 + 256 + 1024 entries per slot */
#define PTAB_SIZE (10 * PTAB_SLOT)

/* One superblock of intra work (geometry only; its jobs live in a WGRec). */
typedef struct SBRec {
    uint32_t frame;
    uint16_t sbx, sby;
    uint16_t tile_x0;         /* tile column start, 8x8 units (vp9.c:1244-1250)         */
    uint16_t flags;           /* bit0: load SB interior first (inter frame)             */
} SBRec;

/* One k_pred workgroup: up to PRED_K superblocks of the same wavefront step (any frames)
 * predicted by one wavefront. The host zips the SBs' dependency levels into shared
 * passes: a pass holds up to 64/n independent jobs of one size n, from any of the
 * SBs (each SB's jobs in a pass are of one level, levels in order). */
#define PRED_K 1          /* slots per workgroup (the kernel supports more; 1 measured best) */
typedef struct WGRec {
    uint32_t job0;            /* first PJob (merged, pass order)                        */
    uint32_t pass0;           /* first pass word                                        */
    uint16_t njobs, npass;
    uint32_t sb[PRED_K];      /* SBRec index per slot, 0xffffffff = empty              */
} WGRec;

/* pass word (u32): first job (relative to job0) << 8 | (njobs - 1) << 3 | ts */
#define PASS_FIRST(w) ((w) >> 8)
#define PASS_NJOBS(w) ((((w) >> 3) & 31) + 1)
#define PASS_TS(w) ((w) & 3)
#define MAX_SB_JOBS 768          /* 3 planes x 256 4x4 jobs (4:4:4) */
#define PJ_SLOT(j) ((j).a >> 30)

/* Loop-filter program of one SB: the edge decisions of filter_plane_cols / _rows
 * (vp9lpf.c:31-181), resolved on the host from the SB's VP9Filter levels and masks
 * (vp9dec.h:83-87, vp9block.c:1438-1452). One byte per (band, edge): band = pixel row
 * >> 3 for column edges, pixel column >> 3 for row edges (the decisions are uniform
 * over 8 lines); main edge = width code (1: 4, 2: 8, 3: 16) << 6 | level, 0 = none;
 * inner 4-wide edge = 0x40 | level, 0 = none.
 * A plane dimension of 64 pixels (luma; chroma without subsampling on that axis) has
 * 8 edges 8 pixels apart, each with (main, inner) bytes: 16 bytes per band. A subsampled
 * chroma dimension (32 pixels) has 8 edges 4 pixels apart, main only: 8 bytes per band.
 * U and V share the chroma program (one mask set, vp9lpf.c:189). */
#define LFP_YC 0                 /* luma column edges: band * 16 + edge * 2 + {main, inner} */
#define LFP_YR 128               /* luma row edges:    band * 16 + edge * 2 + {main, inner} */
#define LFP_CC 256               /* chroma column edges: band * LFP_CSTRIDE(ss_h) + ...     */
#define LFP_CSTRIDE(ss) ((ss) ? 8 : 16)
#define LFP_CR(ss_h, ss_v) (LFP_CC + (8 >> (ss_v)) * LFP_CSTRIDE(ss_h))       /* chroma row edges */
#define LF_PROG_OF(ss_h, ss_v) (LFP_CR(ss_h, ss_v) + (8 >> (ss_h)) * LFP_CSTRIDE(ss_v))
#define LF_PROG_BYTES 512        /* LF_PROG_OF(0, 0): 4:2:0 uses the first 320 */
typedef struct LFRec {
    uint32_t frame;
    uint16_t sbx, sby;
    uint8_t  prog[LF_PROG_BYTES];
} LFRec;

/* One fused wavefront launch (k_plf): `npred` intra workgroups (one SB each), `nlf` LF
 * SBs, and per transform code (4x4, 8x8, 16x16, 32x32, WHT) rn[k] residual jobs starting
 * at RJob roff[k] (the residuals of the next intra diagonal). */
typedef struct PlfLaunch {
    uint32_t npred, nlf;
    uint32_t roff[5], rn[5];
} PlfLaunch;

/* One motion-compensated rectangle of one plane (<= 64 x 64) and its references. Per
 * reference, output pixel (i, j) samples the reference at x = ix + ((mx + i dx) >> 4),
 * phase (mx + i dx) & 15 (y likewise): the stepping of do_scaled_8tap / do_scaled_bilin
 * (vp9dsp_template.c:2363-2482). Unscaled references use dx = dy = 16, for which the
 * always-2-D scaled filter equals the 1-D / 2-D / copy selection of the unscaled MC
 * exactly (an identity phase is exact). Reads clamp to the reference's visible size
 * (emulated_edge_mc, videodsp_template.c:27-105). */
typedef struct McRef {
    int32_t  ix, iy;          /* integer reference position of output pixel (0, 0)      */
    uint8_t  mx, my;          /* its 1/16-pel phase                                     */
    uint8_t  dx, dy;          /* phase step per output pixel (16 = unscaled)            */
} McRef;

typedef struct McUnit {
    uint32_t frame;
    uint16_t x, y;            /* plane pixel position                                   */
    uint8_t  w, h;
    uint8_t  plane;
    uint8_t  filter;          /* 0..2 8-tap smooth/regular/sharp, 3 bilinear            */
    uint8_t  nref;            /* 1 or 2 (compound: second ref averaged)                 */
    uint8_t  ref[2];
    uint8_t  pad;
    McRef    r[2];
} McUnit;

/* Kernel selections a context fixes when it opens (vp9hip_open reads the VP9HIP_* switches
 * once; no launcher reads the environment). */
typedef struct KCfg {
    int lfro;                 /* 4:2:0 row LF: 1 k_lfro (default), 0 k_lfrd (VP9HIP_LFRO=0)     */
    int mcq_slices;           /* k_mcq task slices per unit group; 0: from the grid size         */
} KCfg;

/* A level phase's intra SBs inside its k_lfro launch (VP9HIP_PRED_LF_FUSE): the first nblk
 * workgroups are intra workers (LFRI_WAVES waves each, every wave k_predd's loop over the
 * list's tickets), the rest the row-LF tasks. The LF loader waits, before it loads SB (r, c),
 * for the done flags of (r, c) (its pixels) and of (r, c + 1), (r + 1, c - 1 .. c + 1) (they
 * read its pre-LF pixels), and loads the interior with sc1 loads (the workers write whole
 * interiors through). nblk = 0: none. */
typedef struct LfrIntra {
    const uint32_t *list;     /* the phase's level lists back to back: slots                     */
    const uint32_t *sbinfo;   /* per slot: bit 0 has intra jobs, bits 1-3 the producer mask      */
    const WGRec *wgs;
    const SBRec *sbs;
    const PJob *jobs;
    const uint32_t *passes;
    const int16_t *resid;
    const uint32_t *ptab;
    uint32_t *pctr;           /* {ticket, finished waves, timeouts, spin}                        */
    uint32_t *done;           /* slot-indexed done flags                                        */
    int n, nblk, dbg;
} LfrIntra;
#define LFRI_WAVES 4

#endif
