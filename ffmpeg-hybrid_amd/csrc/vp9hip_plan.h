/*
 * Device planner of the pixel path (vp9hip_plan.hip): turns the pass-1 packets resident in
 * HBM into the work records of vp9hip_work.h, on the GPU. Internal to libvp9hip.
 *
 * SB slots: every SB of every batch frame has a fixed slot (frame's slot0 + raster index);
 * its SBRec / WGRec / LFRec live at the slot, its intra jobs and pass words at
 * slot * JCAP, its intra residual scratch at slot * RCAP (16-element units, pl_resid_unit).
 * Residual jobs and MC units are compacted by a count / scan / emit sequence: the count
 * matrix holds, per SB and key (tcode 0..4 x txtp 0..3), one entry at
 *   seg_pre4[seg] + tc * s4 + tp * seg_sz[seg] + slot_pos[slot]
 * (seg = the SB's residual segment: its phase, and its intra diagonal when the phase's
 * residuals run inside the fused launches), so one exclusive scan orders the records by
 * (phase, tcode, segment, txtp, SB) = the launch buckets of the host schedule. MC units
 * have their own count array (entry seg_pre1[seg] + slot_pos[slot]) and scan, in
 * (phase, segment, SB) order.
 */
#ifndef VP9HIP_PLAN_H
#define VP9HIP_PLAN_H
#include <stdint.h>
#include "vp9hip_planlogic.h"

/* One batch frame as the device planner sees it (host-built per stage). */
typedef struct PlanFrame {
    uint32_t blk0, nblk;          /* blocks in the batch block array                      */
    uint32_t eob0, neob;          /* eobs in the batch eob array                          */
    uint32_t coef0, ncoef;        /* coefficient elements in the batch coefficient array  */
    uint32_t slot0;               /* first SB slot                                         */
    uint32_t seg0;                /* first residual segment of the frame's phase           */
    uint32_t s4;                  /* count-matrix stride of one tcode in the phase (4 x SBs) */
    uint32_t key0;                /* first intra-step key of the phase                     */
    int32_t  frame;               /* batch frame index (FrameDesc)                         */
    int32_t  sb_cols, sb_rows;
    int32_t  log2_tc, log2_tr;
    int32_t  tile_lo, tile_hi;    /* tile columns this context reconstructs                */
    int32_t  lossless, filter_level, intra;
    int32_t  by_diag;             /* residual segments by intra diagonal (fused phase)      */
    int32_t  levels;              /* intra SBs by dependency level (inter level schedule)   */
    int32_t  bypp;
    int32_t  pitch[2];
    PlMcGeo  mc;                  /* cols / rows / subsampling / reference scales           */
    uint8_t  lflvl[8][4][2];
} PlanFrame;

/* Status bits (PlanDev.status[0], and per frame in PlanDev.fbad); any bit fails the frame
 * that set it with AVERROR_INVALIDDATA. A frame's records address only its own blocks and SB
 * slots, its residual jobs stay inside its SBs' counted ranges, and its eobs / coefficients
 * are where the batch-wide scans put them as long as every frame's totals match its packet
 * counts (checked: PLS_TOTAL), so a rejected frame leaves the other frames' plans intact.
 * PLS_BOUNDS (a shared buffer's capacity) and PLS_TOTAL cannot be attributed and fail the
 * batch. */
#define PLS_BLOCK      1u         /* a block field out of range                             */
#define PLS_ORDER      2u         /* blocks not in decode order / an SB without blocks      */
#define PLS_EOB        4u         /* eob count or value inconsistent with the packet        */
#define PLS_COEF       8u         /* coefficient count inconsistent                         */
#define PLS_MODE      16u         /* intra mode > 9                                         */
#define PLS_REF       32u         /* reference index / scale invalid                        */
#define PLS_SCHED     64u         /* pass scheduling failed (internal)                      */
#define PLS_BOUNDS   128u         /* a planner index out of its buffer (internal, status[1]) */
#define PLS_TOTAL    256u         /* a frame's eob / coefficient totals disagree with its counts */

/* Device buffers of a device-planned batch (all in the batch arena). */
typedef struct PlanDev {
    const PlanFrame  *frames;
    const vp9h_block *blocks;
    const uint16_t   *eobs;
    uint32_t total_blocks, total_eobs, total_coefs;
    /* geometry (host-built, per stage) */
    const uint32_t *slot_pos;     /* position of the slot in its residual segment          */
    const uint32_t *seg_pre4;     /* per segment: count-matrix base                        */
    const uint32_t *seg_sz;       /* per segment: SBs                                       */
    const uint32_t *seg_pre1;     /* per segment: MC count-array base                       */
    /* intermediates */
    uint32_t *blk_neob, *blk_eob0;   /* per block: eob entries, their exclusive scan       */
    uint32_t *sb_first, *sb_end;     /* per slot: block range (0xffffffff: none)            */
    uint32_t *sb_ncoef, *sb_coef0;   /* per slot (packet order): coefficients, their scan   */
    uint32_t *cnt, *cnt0;            /* residual-job count matrix and its exclusive scan    */
    uint32_t *cntm, *cntm0;          /* MC-unit counts and their exclusive scan              */
    uint32_t *ibits;                 /* per slot: 3 planes x 8 words of intra 4x4 units      */
    uint32_t *sb_info;               /* per slot: has intra | L / T / TL dependency << 1     */
    uint32_t *sb_key, *sb_kpos;      /* per slot: intra-step key and position in its list    */
    uint32_t *key_cnt, *key_off;     /* per key: SBs, exclusive scan (+ total)               */
    uint32_t *status;                /* [0] PLS_* bits                                       */
    uint32_t *fbad;                  /* per frame: the PLS_* bits of that frame              */
    unsigned long long *fbytes;      /* per frame: inter residual pixel bytes, MC bytes     */
    /* products */
    SBRec *sbs; WGRec *wgs; PJob *pjobs; uint32_t *passes; LFRec *lfs; RJob *rjobs; McUnit *mcs;
    uint32_t *dlists;                /* intra step lists (device part of the lists array)    */
    uint32_t *jobw;                  /* per slot: jcap intra job words (k_pjob -> k_plan)     */
    uint32_t *sb_nj;                 /* per slot: intra jobs                                 */
    const uint8_t *nz;               /* [5][4][1025][2] nonzero bounding boxes                */
    uint32_t jcap, rcap;             /* jobs / residual units per SB slot                    */
    uint32_t nslots;
    /* capacities: every planner write is checked against them; a violation sets a bit of
     * status[1] (and PLS_SCHED) instead of writing */
    uint32_t cap_cnt, cap_cntm, cap_rjobs, cap_mcs, cap_dlists, nkeys, nframes;
    unsigned long long *prof;        /* diagnostics (VP9HIP_PLAN_PROF): k_plan cycles per phase, or null */
    int dbg;                         /* diagnostics (VP9HIP_PLAN_DBG): ablation switches, timing only */
    int static_lists;                /* the intra step lists were staged by the host (static plan):  */
                                     /* no step keys; an intra-frame SB without intra jobs fails    */
    const uint32_t *stat_ko;         /* static plan: the step lists' offsets (nkeys + 1), k_psort    */
} PlanDev;

#endif
