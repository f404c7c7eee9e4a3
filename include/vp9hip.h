/*
 * vp9hip.h — C-ABI boundary of the MI355X VP9 hybrid decoder.
 *
 * The host (entropy decode, header parse) produces one "pass-1 frame packet" per
 * frame; the device (gfx950 HIP kernels) runs the whole per-superblock pixel path:
 * inverse transforms, intra prediction, motion compensation and the loop filter.
 *
 * The packet mirrors the reference decoder's 2-pass buffers
 * (/root/reference/libavcodec/vp9.c:335-353, vp9block.c:1352-1362): one VP9Block
 * per coded block (vp9dec.h:89-97), the per-tx-block eobs and the dequantized
 * coefficients in scan order (vp9block.c:805-923), plus the frame-header values the
 * pixel path reads (vp9.c:669-791: LF level / sharpness / lossless / tiling).
 *
 * Entry points replace, one for one, the hooks the reference's hybrid path calls:
 *   vp9hip_open/close      <- ff_vp9_webgpu_init/uninit      (vp9_webgpu.h:370-375; vp9.c:1905-1917, 1281-1292)
 *   vp9hip_submit_frame    <- ff_vp9_webgpu_begin/end_frame  (vp9_webgpu.h:470-480; vp9.c:1319-1324, 1840-1845)
 *                             and FFHWAccel.start_frame/decode_slice/end_frame (hwaccel_internal.h:34-166; vp9.c:1694-1713)
 *   vp9hip_download_frame  <- the end_frame readback         (vp9_webgpu.c:2995-3056)
 *   vp9hip_flush           <- FFHWAccel.flush                (hwaccel_internal.h:165; vp9.c:1865-1883)
 * Errors are FFmpeg-style negative AVERROR codes (VP9HIP_E*).
 * A context is not thread-safe; use one host thread per context.
 */
#ifndef VP9HIP_H
#define VP9HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: vp9h_synth_params / vp9h_enc_params end in a vp9h_seg_params; vp9hip_test_hooks,
 * vp9hip_batch_frame_status and VP9HIP_PIPELINE_SLOTS added. Callers check
 * vp9hip_abi_version() == VP9HIP_ABI_VERSION before passing structs. */
#define VP9HIP_ABI_VERSION 2

/* FFmpeg AVERROR values used by the boundary (libavutil/error.h). */
#define VP9HIP_EINVAL       (-22)          /* AVERROR(EINVAL)   */
#define VP9HIP_ENOMEM       (-12)          /* AVERROR(ENOMEM)   */
#define VP9HIP_ENOSYS       (-38)          /* AVERROR(ENOSYS)   */
#define VP9HIP_EINVALIDDATA (-1094995529)  /* AVERROR_INVALIDDATA */
#define VP9HIP_EEXTERNAL    (-542398533)   /* AVERROR_EXTERNAL (HIP runtime failure) */
#define VP9HIP_EBUG         (-558323010)   /* AVERROR_BUG (internal invariant broken) */
#define VP9HIP_EAGAIN       (-11)          /* AVERROR(EAGAIN)   */
#define VP9HIP_EOF          (-541478725)   /* AVERROR_EOF       */

/* enum BlockSize (vp9shared.h:86-101) */
enum { VP9H_BS_64x64, VP9H_BS_64x32, VP9H_BS_32x64, VP9H_BS_32x32, VP9H_BS_32x16,
       VP9H_BS_16x32, VP9H_BS_16x16, VP9H_BS_16x8, VP9H_BS_8x16, VP9H_BS_8x8,
       VP9H_BS_8x4, VP9H_BS_4x8, VP9H_BS_4x4, VP9H_N_BS };
/* enum TxfmMode (vp9.h:27-35) */
enum { VP9H_TX_4X4, VP9H_TX_8X8, VP9H_TX_16X16, VP9H_TX_32X32 };
/* enum FilterMode (vp9.h:64-71) */
enum { VP9H_FILTER_SMOOTH, VP9H_FILTER_REGULAR, VP9H_FILTER_SHARP, VP9H_FILTER_BILINEAR };
/* intra modes 0..9 (vp9.h:45-62), inter modes (vp9shared.h:43-48) */
enum { VP9H_NEARESTMV = 10, VP9H_NEARMV = 11, VP9H_ZEROMV = 12, VP9H_NEWMV = 13 };

/* One coded block in decode order (VP9Block, vp9dec.h:89-97). 52 bytes. */
typedef struct vp9h_block {
    uint16_t row, col;      /* position in 8x8 units (vp9block.c:1276-1279)            */
    uint8_t  bs;            /* VP9H_BS_*                                               */
    uint8_t  tx, uvtx;      /* luma / chroma transform size (vp9block.c:1291)         */
    uint8_t  skip;          /* final skip flag, after vp9block.c:1310-1314             */
    uint8_t  intra, comp;   /* intra block; compound prediction                       */
    uint8_t  seg_id;        /* segment (selects LF level)                              */
    uint8_t  filter;        /* VP9H_FILTER_* for inter blocks                          */
    uint8_t  mode[4];       /* luma mode per 4x4 sub-block (intra 0..9, inter 10..13)  */
    uint8_t  uvmode;        /* chroma intra mode                                       */
    uint8_t  ref[2];        /* 0=LAST 1=GOLDEN 2=ALTREF                                */
    uint8_t  pad0;
    int16_t  mv[4][2][2];   /* [b_idx][ref][x,y] in 1/8 luma pel                       */
} vp9h_block;

/*
 * One frame of pass-1 output.
 * eobs: for every block with skip == 0, one uint16 per transform block that lies
 *   inside the frame (end_x/end_y clipping of vp9recon.c:243-244), in the reference's
 *   loop order: luma tx blocks row-major, then U, then V (vp9recon.c:269-357).
 *   Blocks with skip == 1 store nothing.
 * coefs: for every tx block with eob > 0, `eob` dequantized coefficients in scan
 *   order (the values decode_coeffs_b_generic stores at coef[scan[i]],
 *   vp9block.c:905-917): int16 for bpp == 8, int32 for bpp > 8.
 */
typedef struct vp9h_frame {
    int32_t  width, height;        /* visible size                                    */
    uint8_t  bpp;                  /* 8, 10, 12                                       */
    uint8_t  ss_h, ss_v;           /* chroma subsampling                              */
    uint8_t  keyframe, intraonly;
    uint8_t  lossless;             /* WHT 4x4 everywhere (vp9.c:704-705)              */
    uint8_t  filter_level;         /* s->s.h.filter.level                             */
    uint8_t  sharpness;            /* s->s.h.filter.sharpness                         */
    uint8_t  log2_tile_cols;
    uint8_t  log2_tile_rows;
    uint8_t  pad0[2];
    uint8_t  lflvl[8][4][2];       /* segmentation.feat[s].lflvl (vp9.c:767-791)       */
    int32_t  ref_w[3], ref_h[3];   /* visible size of LAST/GOLDEN/ALTREF (MC clamp)   */
    uint32_t nblocks;
    uint32_t neobs;
    uint64_t ncoefs;
    const vp9h_block *blocks;
    const uint16_t   *eobs;
    const void       *coefs;
} vp9h_frame;

/* ---- device context ---------------------------------------------------- */
typedef struct vp9hip_ctx vp9hip_ctx;

/* Open a context on HIP device `device`. Returns 0 or a negative error. The context reads
 * its VP9HIP_* environment switches (kernel A/B selections and diagnostics)
 * here, once; nothing later reads the environment. */
int  vp9hip_open(int device, vp9hip_ctx **out);
void vp9hip_close(vp9hip_ctx *ctx);
/* Test hooks, copied by every context opened afterwards (0, 0 = off, the default):
 * reject_batch = k | f << 16 makes frame f of the k-th batch the context stages (k >= 1,
 * restagings count) start with an intra block whose mode the device planner rejects;
 * lfr_spin = n bounds the row loop filter's hand-off waits to n polls (forcing its timeout
 * path). No reference counterpart; never called in production. */
void vp9hip_test_hooks(int reject_batch, uint32_t lfr_spin);

/* Allocate `nbufs` device frame buffers of w x h (padded to 64 internally). */
int  vp9hip_configure(vp9hip_ctx *ctx, int width, int height, int bpp, int ss_h, int ss_v,
                      int nbufs);

/*
 * Queue one frame: `out_buf` receives the reconstruction, ref_buf[0..2] are the
 * device buffers holding LAST/GOLDEN/ALTREF (ignored for intra frames).
 * The packet is copied (staged) before return; execution is asynchronous.
 */
int  vp9hip_submit_frame(vp9hip_ctx *ctx, const vp9h_frame *pkt, int out_buf,
                         const int ref_buf[3]);

/*
 * Batched form for independent (intra-only) frames: stage all packets into device
 * memory once (vp9hip_stage_batch), then run the pixel path over all of them with
 * frames interleaved in each wavefront launch (vp9hip_run_batch). run may be
 * repeated; the inputs stay resident in HBM.
 */
int  vp9hip_stage_batch(vp9hip_ctx *ctx, const vp9h_frame *pkts, int n, const int *out_bufs);
int  vp9hip_run_batch(vp9hip_ctx *ctx);
/*
 * Batch with inter frames: ref_bufs[3*i .. 3*i+2] are the LAST/GOLDEN/ALTREF buffers of
 * frame i (ignored for keyframes). Frames that reference (or overwrite) the output of an
 * earlier frame of the batch run after it; independent chains run concurrently.
 */
int  vp9hip_stage_batch_refs(vp9hip_ctx *ctx, const vp9h_frame *pkts, int n, const int *out_bufs,
                             const int *ref_bufs);

/*
 * Tile-column sharding of ONE stream over several devices (one context per device).
 * Every context stages the same packets. Its reconstruction covers only tile columns
 * [tile_lo, tile_hi), which is MC, residuals and intra; tile columns decode
 * independently (vp9.c:1244-1250, vp9recon.c:46). Its loop filter covers the whole
 * frame. Per phase (vp9hip_batch_phases, the frames of one chain position,
 * vp9hip_phase_frames):
 *   1. vp9hip_run_phase(ctx, ph, VP9HIP_PART_RECON);
 *   2. exchange the pre-LF stripes of that phase's frames (vp9hip_stripe pack, an
 *      all-gather, vp9hip_stripe unpack of the other shards' columns);
 *   3. vp9hip_run_phase(ctx, ph, VP9HIP_PART_LF).
 * Every device then holds the full post-LF frames that later phases reference.
 * The device form of the reference's slice-threaded tile decode: tile-column jobs
 * (decode_tiles_mt, vp9.c:1442-1520), then the loop filter over the whole frame
 * (loopfilter_proc, vp9.c:1522-1551; dispatched at vp9.c:1806).
 */
#define VP9HIP_PART_RECON 0
#define VP9HIP_PART_LF    1
int  vp9hip_stage_batch_tiles(vp9hip_ctx *ctx, const vp9h_frame *pkts, int n, const int *out_bufs,
                              const int *ref_bufs, int tile_lo, int tile_hi);
int  vp9hip_batch_phases(vp9hip_ctx *ctx);
/* Frame groups of the staged batch: independent chains run on that many HIP streams. */
int  vp9hip_batch_groups(vp9hip_ctx *ctx);
/* Batch indices of the frames in `phase` (up to cap written); returns their count. */
int  vp9hip_phase_frames(vp9hip_ctx *ctx, int phase, int *frames, int cap);
int  vp9hip_run_phase(vp9hip_ctx *ctx, int phase, int part);
/*
 * Pack (to_frame = 0) or unpack (1) the pixel columns of tile columns [tile_lo, tile_hi)
 * of batch frame `frame`, all 8-aligned rows, Y then U then V, between its device
 * buffer and contiguous device memory `dev`. The copy is asynchronous on the context's
 * stream. Returns the byte count, which is all it does when dev is NULL.
 */
int64_t vp9hip_stripe(vp9hip_ctx *ctx, int frame, int tile_lo, int tile_hi, void *dev, int to_frame);

/* Batch slots per context. */
#define VP9HIP_MAX_SLOTS 4
/* Batch slots the decoder (vp9hip_decoder_*) and the FFHWAccel adapter rotate: batch k + 3
 * is staged only after batch k's slot is checked, so three batches are in flight, each on
 * one frame-group stream (the context default: the slots' streams fit the 4 hardware
 * queues; bench.py times C3 / C4 / C5 at this depth, C2 at 4). */
#define VP9HIP_PIPELINE_SLOTS 3
/* Select batch slot 0 .. VP9HIP_MAX_SLOTS - 1 (default 0): stage_batch*, run_batch,
 * batch_phases, run_phase and stripe act on the current slot. Each slot holds its own
 * staged batch (arena, plan, launch graph) and runs on HIP streams of its own (slots 2..
 * create theirs at first selection); the frame buffers are the context's. Staged batches
 * that share no frame buffer run concurrently (one batch's device planning and intra
 * wavefront under another's loop filter); a batch that reads or writes a buffer of
 * another slot's batch follows that slot's last run. */
int  vp9hip_set_batch_slot(vp9hip_ctx *ctx, int slot);
/* Wait for the last run of batch slot `slot` only (other slots' work may continue)
 * and check it as vp9hip_sync does (VP9HIP_EBUG: a loop-filter hand-off timed out). */
int  vp9hip_sync_slot(vp9hip_ctx *ctx, int slot);
/* Per-frame outcome of the last stage / run of batch slot `slot` after stage_batch*,
 * run_batch, vp9hip_sync_slot or vp9hip_sync reported AVERROR_INVALIDDATA for it (the device
 * planner or the staging checks rejected frames): status[i] (staging order, up to cap) is 0
 * for a frame that was reconstructed, AVERROR_INVALIDDATA for a rejected frame, and
 * AVERROR(EAGAIN) for a valid frame that was not run (a batch planned on the host's
 * schedule stops before its pixel launches: stage those frames again). Keyframe batches
 * (launch lists fixed at staging) reconstruct the frames the planner did not reject; a
 * rejection that names no frame rejects all. Returns the batch's frame count. No reference
 * counterpart beyond vp9.c failing only the corrupt frame's decode (:1827-1832). */
int  vp9hip_batch_frame_status(vp9hip_ctx *ctx, int slot, int *status, int cap);
/* Make HIP stream `stream` (a hipStream_t; NULL: the null stream) wait for the last run of
 * batch slot `slot`, without a host wait: work enqueued on it afterwards sees that run's
 * frames. The loop-filter hand-off check needs a host wait (vp9hip_sync_slot). */
int  vp9hip_slot_stream_wait(vp9hip_ctx *ctx, int slot, void *stream);
/* 1 while the last run of batch slot `slot` is still executing, 0 once it is done. */
int  vp9hip_slot_busy(vp9hip_ctx *ctx, int slot);
/* Wait for all queued work of every batch slot. VP9HIP_EBUG if a row-pipelined
 * loop-filter launch (k_lfrd / k_lfro) of any slot gave up a bounded wait on another workgroup's
 * progress (frames not trusted). */
int  vp9hip_sync(vp9hip_ctx *ctx);

/* Copy device buffer `buf` into host planes (linesize in bytes). Synchronous. */
int  vp9hip_download_frame(vp9hip_ctx *ctx, int buf, uint8_t *const planes[3],
                           const ptrdiff_t linesize[3]);
/*
 * Zero-copy export of device buffer `buf` (replaces the D2H of vp9hip_download_frame for
 * consumers on the GPU; the hwcontext frame export of SURVEY 8f rank 2,
 * hwaccel_internal.h:146, libavutil/hwcontext.h:26-44): device pointers and byte
 * pitches of the three planes, the visible size, and the current batch slot's main
 * hipStream_t. Each batch slot runs on streams of its own, so a consumer orders its reads
 * after the slot that wrote the frame (vp9hip_slot_stream_wait), or reads after
 * vp9hip_sync / vp9hip_sync_slot. Pointers stay valid until vp9hip_configure /
 * vp9hip_close.
 */
int  vp9hip_frame_device(vp9hip_ctx *ctx, int buf, void *planes[3], ptrdiff_t linesize[3],
                         int *width, int *height, void **stream);
/* Upload host planes into device buffer `buf` (test hook for reference frames). */
int  vp9hip_upload_frame(vp9hip_ctx *ctx, int buf, const uint8_t *const planes[3],
                         const ptrdiff_t linesize[3]);

/* Drop queued work and the staged batches of every slot (FFHWAccel.flush). */
int  vp9hip_flush(vp9hip_ctx *ctx);
/* Fill device buffers [buf0, buf0 + count) with the byte `value`, asynchronously on the
 * context's stream (the bench poisons its frame buffers before the timed steps, so the
 * frames it verifies afterwards were written by those steps). No reference counterpart. */
int  vp9hip_fill_buffers(vp9hip_ctx *ctx, int buf0, int count, int value);

/*
 * Per-kernel timing of the last run (HIP events on the execution stream):
 * names[i] / ms[i] / launches[i] for up to `cap` kernel classes. Returns count.
 */
int  vp9hip_last_timing(vp9hip_ctx *ctx, const char **names, double *ms, int *launches, int cap);

/* Per-launch HIP-event timing on/off (default on). */
int  vp9hip_set_timing(vp9hip_ctx *ctx, int on);
/* Graph replay of a staged batch (default on): run_batch captures the batch's launch
 * sequence into a HIP graph once and replays it. Off: every run_batch enqueues the
 * launches directly (cheaper for a batch that runs once, e.g. the decoder's). */
int  vp9hip_set_graph(vp9hip_ctx *ctx, int on);

/* Algorithmic bytes (B = C + P(1+R) + 2P[LF]) of the staged batch,
 * per kernel class in vp9hip_last_timing order. Returns count. */
int  vp9hip_alg_bytes(vp9hip_ctx *ctx, double *bytes, int cap);

/* Host-only planning statistics of one packet (no device needed), 16 values:
 * SBs with intra work, passes, intra jobs, residual jobs, intra jobs per tx size (4),
 * lane use, max passes per SB, LF records, MC units, intra / LF wavefront steps,
 * intra dependency levels (summed over SBs: the lower bound of the passes), pixel rows
 * the passes loop over (each pass: its largest job size). A 17th value (cap >= 17): intra
 * steps under the dependency-level schedule of inter frames (= the diagonals otherwise);
 * 18-20: pass-packing estimates; 21-23 (cap >= 23): MC predicted-pixel bytes, those x (1 +
 * references), and the 128-byte lines the MC window rows touch, each unit counted alone. */
int  vp9hip_plan_stats(const vp9h_frame *pkt, double *out, int cap);
/* Diagnostics: per SB of one packet (raster order) the pixel rows its intra passes loop
 * over, as staged for the device (the wavefront-tail estimate of tools/wave_tail.py).
 * Returns the SB count, or a negative AVERROR. */
int  vp9hip_plan_sb_costs(const vp9h_frame *pkt, double *out, int cap);

int  vp9hip_abi_version(void);
/* PCI bus id ("0000:75:00.0") and name of HIP device `device` (so a multi-GPU run can show
 * each rank on its own card). VP9HIP_ENOSYS if there is no such device. */
int  vp9hip_device_info(int device, char *pci_bus_id, int len, char *name, int name_len);

/* ---- synthetic pass-1 generator (test / bench input) -------------------- */
/*
 * Generates a pseudo-random but structurally legal frame packet. Defaults follow the
 * stream settings of SURVEY.md §8(d): random partitions (P(split) 0.5 at 64/32, 0.3
 * at 16, 10 % sub-8x8), uniform intra modes, skip 0.2, TX_MODE_SELECT, per tx block
 * eob uniform in [1, min(n,64)] with geometric(0.6) magnitudes and random sign,
 * base_q_idx 60 (no deltas), filter level 36, sharpness 0, LF deltas at the libvpx
 * defaults. inter != 0: LAST-ref inter frame (50 % NEWMV, MVs uniform in +-64 px,
 * 10 % intra blocks). The packet owns heap arrays; release with vp9hip_synth_free.
 */
/* Segmentation and loop-filter deltas of a frame (vp9.c:692-765, vp9block.c:101-141): what
 * vp9h_stream_encode writes into the frame header, and what vp9hip_synth_frame assumes for
 * the packet's segment ids, per-segment dequantization and LF levels. Values are the ones in
 * effect for the frame (the encoder codes the LF deltas that differ from the stream's, and
 * the segment features when update_data). All zero: no segmentation, libvpx's default LF
 * deltas (ref 1, 0, -1, -1; mode 0, 0) unchanged. */
typedef struct vp9h_seg_params {
    int32_t enabled;               /* segmentation_enabled                                  */
    int32_t update_map;            /* code the blocks' segment ids (else the map is kept)   */
    int32_t temporal;              /* inter frames: ids predicted from the previous map     */
    int32_t update_data;           /* code the per-segment features                         */
    int32_t abs_delta;             /* feature values absolute (else deltas to the frame's)  */
    int32_t q_en, lf_en;           /* bit s: segment s has the alternate q / LF feature     */
    int32_t q[8], lf[8];
    int32_t nseg;                  /* synth: segment ids drawn from 0 .. nseg - 1           */
    int32_t lf_delta_update;       /* lf_ref / lf_mode below are in effect (else defaults)  */
    int32_t lf_ref[4], lf_mode[2];
} vp9h_seg_params;

typedef struct vp9h_synth_params {
    int32_t  width, height;
    int32_t  bpp;              /* 8 / 10 / 12                                   */
    int32_t  ss_h, ss_v;       /* 1,1 = 4:2:0                                   */
    int32_t  log2_tile_cols;
    int32_t  inter;            /* 0 = keyframe; 1 = inter frame on LAST         */
    int32_t  compound;         /* inter: allow compound LAST+ALTREF blocks      */
    int32_t  q_idx;            /* base_q_idx (0 + lossless -> WHT)              */
    int32_t  lossless;
    int32_t  filter_level;
    int32_t  sharpness;
    int32_t  bilinear;         /* frame-level bilinear MC filter                */
    int32_t  coef_stress;      /* 1: coefficients uniform over the full range   */
    float    p_zero_eob;       /* chance that a tx block codes eob 0            */
    float    p_skip;           /* default 0.2                                   */
    uint64_t seed;
    vp9h_seg_params seg;       /* segmentation / LF deltas (default: none)      */
} vp9h_synth_params;

/* Fill p with the §8(d) defaults for a w x h bpp stream. */
void vp9hip_synth_defaults(vp9h_synth_params *p, int width, int height, int bpp);
int  vp9hip_synth_frame(vp9h_frame *out, const vp9h_synth_params *p);
void vp9hip_synth_free(vp9h_frame *f);

/* ---- host bitstream side: VP9 frame <-> pass-1 packet ----------
 * vp9h_decode_frame parses one frame's compressed data (uncompressed + compressed
 * header, tiles) into a pass-1 packet: the host entropy decode whose output the device
 * path consumes. It follows decode_frame_header / decode_tiles / decode_sb /
 * ff_vp9_decode_block of the reference (vp9.c:519-1395, vp9block.c:80-1130). The packet
 * owns heap arrays; release them with vp9h_frame_free.
 * vp9h_encode_frame writes a pass-1 packet as a VP9 bitstream (the synthetic stream
 * generator): default probabilities, frame_parallel, tx_mode = TX_MODE_SELECT, libvpx's
 * default LF deltas. Release the buffer with vp9h_buffer_free.
 * These one-frame forms take keyframes and intra-only frames (no reference state);
 * streams with inter frames go through a vp9h_stream below. Profiles 0-3. */
int  vp9h_decode_frame(const uint8_t *data, size_t size, vp9h_frame *out);
int  vp9h_encode_frame(const vp9h_frame *pkt, int base_q_idx, uint8_t **out, size_t *size);
void vp9h_frame_free(vp9h_frame *f);
void vp9h_buffer_free(uint8_t *p);

/*
 * A stream's host parse state (VP9Context's frame-to-frame state: the 4 saved probability
 * contexts prob_ctx, the 8 reference slots' sizes, the last frame's MV pairs and the
 * segmentation-map reference, vp9.c:1616-1686; the persistent header s->s.h). One
 * vp9h_stream either decodes or encodes one stream, frame by frame, in order.
 */
typedef struct vp9h_stream vp9h_stream;
int  vp9h_stream_open(vp9h_stream **out);
void vp9h_stream_close(vp9h_stream *s);

/* Tile-column threads of vp9h_stream_decode (default 1): the tile columns of a frame are
 * entropy-decoded concurrently, as decode_tiles_mt does with slice threads
 * (vp9.c:1441-1520, launched at 1777-1806). The packet is the serial walk's, byte for byte. */
int  vp9h_stream_set_threads(vp9h_stream *s, int n);

/* What the frame header decided beyond the packet (reference slot bookkeeping for the
 * device buffers, vp9.c:1686-1691, 1845-1849). */
typedef struct vp9h_frame_info {
    int32_t show_existing_frame;   /* 1: no packet; output reference slot show_slot        */
    int32_t show_slot;
    int32_t show_frame;            /* 0: decoded into the slots but not output             */
    int32_t refresh_mask;          /* slots that receive this frame                        */
    int32_t ref_slot[3];           /* LAST / GOLDEN / ALTREF slots (inter frames)           */
    int32_t sign_bias[3];
    int32_t error_res, refresh_ctx, parallel, ctx_id;
    int32_t allow_hp, interp, comp_mode, tx_mode;
    uint32_t header_size, compressed_header_size;
} vp9h_frame_info;

/* Parse one frame (one superframe part) of the stream: the packet, or for
 * show_existing_frame only `info` (out is left empty). */
int  vp9h_stream_decode(vp9h_stream *s, const uint8_t *data, size_t size, vp9h_frame *out,
                        vp9h_frame_info *info);

/*
 * The same parse in two steps, so consecutive frames of one stream overlap as the
 * reference's frame threads do (ff_thread_finish_setup once the headers are parsed,
 * vp9.c:1752-1754; the next frame then waits per SB row for this frame's MV pairs and
 * segmentation map, vp9mvs.c:177-178, vp9block.c:116-117):
 *   vp9h_stream_decode_begin parses the headers and advances the stream: the next frame's
 *   begin may follow at once unless *serial is set (refresh_frame_context without
 *   frame_parallel_decoding_mode: the next headers read the probabilities this frame's tiles
 *   adapt, so its finish must complete first). *pending is NULL for show_existing_frame
 *   (info says which slot). data must stay valid until finish.
 *   vp9h_stream_decode_finish walks the tiles on `threads` tile-column threads, waiting for
 *   the rows of the earlier frames' side buffers it reads, and frees the pending frame. The
 *   finishes of one stream may run concurrently on different threads if each frame's finish
 *   starts after the previous frame's finish has started.
 * The packets equal vp9h_stream_decode's byte for byte (tests/c/host_san.cpp). A frame
 * whose tiles fail makes the later frames that read its side buffers fail too. */
typedef struct vp9h_pending vp9h_pending;
int  vp9h_stream_decode_begin(vp9h_stream *s, const uint8_t *data, size_t size, vp9h_pending **pending,
                              vp9h_frame_info *info, int *serial);
int  vp9h_stream_decode_finish(vp9h_pending *pending, int threads, vp9h_frame *out);
void vp9h_pending_free(vp9h_pending *pending);     /* a begun frame that will not be finished */

/* Encoder choices for one frame (vp9h_enc_defaults: the SURVEY 8(d) stream settings). */
typedef struct vp9h_enc_params {
    int32_t base_q_idx;
    int32_t show_existing_frame, show_slot;   /* 1: write a show_existing_frame header only */
    int32_t show_frame;
    int32_t error_res;
    int32_t refresh_mask;          /* -1: keyframes / intra-only all slots, inter slot 0   */
    int32_t ref_slot[3];
    int32_t sign_bias[3];          /* default 0, 0, 1: compound prediction allowed          */
    int32_t refresh_ctx, parallel, ctx_id, reset_ctx;
    int32_t allow_hp;
    int32_t interp;                /* -1: fixed if every inter block shares one filter      */
    int32_t comp_mode;             /* -1: switchable when the packet has compound blocks    */
    int32_t tx_mode;               /* -1: TX_MODE_SELECT                                    */
    int32_t prob_updates;          /* 0: none; else the seed of random forward updates      */
    int32_t keep_modes;            /* 1: code the packet's inter modes, taking the MVs they  */
                                   /*    predict (NEAREST / NEAR / ZERO); 0: keep the MVs    */
    vp9h_seg_params seg;           /* segmentation / LF deltas to code (default: none)      */
} vp9h_enc_params;
void vp9h_enc_defaults(vp9h_enc_params *p);

/*
 * Write one frame. `coded` (optional) receives the packet exactly as written, which is
 * what vp9h_stream_decode returns for the bitstream. It differs from `pkt` only where
 * the syntax cannot say what the packet says:
 *   - an inter mode whose predicted MV is not the packet's MV becomes NEWMV (keep_modes:
 *     the mode stays and the MV becomes the predicted one);
 *   - a low-precision MV difference loses its odd 1/8-pel step (vp9mvs.c:302-318);
 *   - a skipped inter block takes the largest transform size (vp9block.c:213-215);
 *   - an inter block <= 8x8 without coefficients becomes skip (vp9block.c:1310-1314);
 *   - fields the syntax does not carry are zero (intra blocks' MVs / refs / filter,
 *     single-reference blocks' second MV and reference).
 */
int  vp9h_stream_encode(vp9h_stream *s, const vp9h_frame *pkt, const vp9h_enc_params *p,
                        uint8_t **out, size_t *size, vp9h_frame *coded);

/* The frame type from the first header bits: 0 keyframe (its parse needs no earlier
 * frame), 1 other frame, 2 show_existing_frame, or AVERROR_INVALIDDATA. */
int  vp9h_frame_type(const uint8_t *data, size_t size);

/* The slot bookkeeping of a frame from the start of its uncompressed header, without
 * stream state (vp9.c:519-611, what vp9.c knows before ff_thread_finish_setup):
 * show_existing_frame + show_slot, show_frame, error_res, refresh_mask, and ref_slot /
 * sign_bias of inter frames; the other fields are zero. Returns 0 keyframe, 1 inter frame,
 * 2 show_existing_frame, 3 intra-only frame, or AVERROR_INVALIDDATA. */
int  vp9h_frame_peek(const uint8_t *data, size_t size, vp9h_frame_info *info);

/* Split a superframe into its frames (vp9_superframe_split_bsf,
 * bsf/vp9_superframe_split.c:40-95): up to cap (offset, size) pairs; returns the frame
 * count (1 for a plain frame) or a negative error. */
int  vp9h_superframe_split(const uint8_t *data, size_t size, size_t *offsets, size_t *sizes, int cap);

/* ---- IVF container (libavformat/ivfdec.c, ivfenc.c) ------------- */
typedef struct vp9h_ivf_header {
    char     fourcc[5];            /* "VP90" for VP9, NUL-terminated                        */
    int32_t  width, height;
    uint32_t time_base_den, time_base_num;
    uint32_t nb_frames;
    uint32_t header_size;
} vp9h_ivf_header;
/* ivfdec.c probe (:27-34): 98 (AVPROBE_SCORE_MAX - 2) for an IVF header, else 0. */
int  vp9h_ivf_probe(const uint8_t *buf, size_t size);
/* ivfdec.c read_header (:36-77): AVERROR_INVALIDDATA for a zero time base. */
int  vp9h_ivf_read_header(const uint8_t *buf, size_t size, vp9h_ivf_header *h);
/* ivfdec.c read_packet (:79-90): the frame at *pos (32 = the first), advancing *pos.
 * Returns 0, or VP9HIP_EOF at the end; a short last frame sets *truncated. */
int  vp9h_ivf_read_frame(const uint8_t *buf, size_t size, size_t *pos, const uint8_t **data, uint32_t *frame_size,
                         int64_t *pts, int *truncated);
/* ivfenc.c write_header (:54-73) with fourcc VP90, and write_packet's frame header (:75-88). */
int  vp9h_ivf_write_header(uint8_t out[32], int width, int height, uint32_t time_base_den, uint32_t time_base_num,
                           uint32_t nb_frames);
void vp9h_ivf_write_frame_header(uint8_t out[12], uint32_t frame_size, int64_t pts);

/* ---- WebM / Matroska demux of a VP9 track (libavformat/matroskadec.c) -- */
typedef struct vp9h_webm_info {
    char     doctype[16];          /* "webm" / "matroska" (EBML DocType)                     */
    char     codec_id[32];         /* "V_VP9"                                                */
    uint64_t track;                /* TrackNumber of the first VP9 video track               */
    int32_t  width, height;        /* PixelWidth / PixelHeight                               */
    uint64_t timecode_scale;       /* ns per timecode unit (Info TimecodeScale, 1000000)     */
} vp9h_webm_info;
/* Reading position (opaque to callers beyond zero-initialisation by read_header). */
typedef struct vp9h_webm_cursor {
    uint64_t pos, seg_end, cluster_end, track;
    int64_t  cluster_tc, block_pts, block_duration;
    int32_t  cluster_unknown, keyframe;
    int32_t  nlaces, lace_idx;
    uint64_t lace_pos;
    uint32_t lace_size[256];
} vp9h_webm_cursor;
/* matroska_probe (matroskadec.c:1614-1660): 100 for an EBML header with a matroska / webm
 * DocType, 50 for another EBML document, else 0. */
int  vp9h_webm_probe(const uint8_t *buf, size_t size);
/* matroska_read_header (matroskadec.c:3303-3490): EBML header checks, Info, the first
 * VP9 video track; *cur then points at the first Cluster. AVERROR_INVALIDDATA if there
 * is no V_VP9 track or the header is malformed. */
int  vp9h_webm_read_header(const uint8_t *buf, size_t size, vp9h_webm_info *info, vp9h_webm_cursor *cur);
/* matroska_read_packet: the next frame (one lace of a SimpleBlock / Block of the track),
 * pts in timecode units (INT64_MIN: none), keyframe flag (SimpleBlock; -1 unknown).
 * Returns 0, VP9HIP_EOF at the end, or AVERROR_INVALIDDATA. */
int  vp9h_webm_read_frame(const uint8_t *buf, size_t size, vp9h_webm_cursor *cur, const uint8_t **data,
                          uint32_t *frame_size, int64_t *pts, int *keyframe);

/* ---- bitstream decoder: avcodec_send_packet / avcodec_receive_frame for VP9 -------------
 * The decode loop of vp9_decode_frame (vp9.c:1558-1865) over the host parse (vp9h_stream)
 * and the device path (vp9hip_ctx): superframes split, show_existing_frame, hidden frames,
 * reference slots by refresh mask. Frames are reconstructed in batches of up to
 * max_batch frames (decoder delay, like frame threading); send_packet(NULL) drains.
 * The host parse runs on parse_threads threads ahead of the caller.
 * Errors: VP9HIP_EAGAIN from send_packet = read frames first (no free buffer);
 * from receive_frame = send more input; VP9HIP_EOF after a drain. */
typedef struct vp9hip_decoder vp9hip_decoder;
typedef struct vp9hip_decoder_params {
    int32_t device;
    int32_t max_batch;             /* frames per GPU batch (decoder delay), default 16; the  */
                                   /* decoder holds 8 + (VP9HIP_PIPELINE_SLOTS + 1) max_batch */
                                   /* + extra_bufs buffers                                    */
    int32_t extra_bufs;            /* output frames the caller may hold at once, default 4     */
    int32_t max_width, max_height; /* buffer size; 0: the first keyframe's (larger inter      */
                                   /* frames, e.g. reference scaling up, need it set)         */
    int32_t parse_threads;         /* host parse threads (0: parse in the caller's thread);    */
                                   /* a keyframe starts a new parse chain, so keyframe-only   */
                                   /* streams parse frame-parallel, GOPs GOP-parallel         */
} vp9hip_decoder_params;
typedef struct vp9hip_decoded_frame {
    int32_t buf;                   /* device buffer of vp9hip_decoder_context()              */
    int32_t width, height, bpp, ss_h, ss_v;
    int64_t pts;
} vp9hip_decoded_frame;
void vp9hip_decoder_defaults(vp9hip_decoder_params *p);
int  vp9hip_decoder_open(const vp9hip_decoder_params *p, vp9hip_decoder **out);
void vp9hip_decoder_close(vp9hip_decoder *d);
/* The device context holding the frames: vp9hip_download_frame / vp9hip_frame_device. */
vp9hip_ctx *vp9hip_decoder_context(vp9hip_decoder *d);
int  vp9hip_decoder_send_packet(vp9hip_decoder *d, const uint8_t *data, size_t size, int64_t pts);
/* The next output frame; its buffer stays valid until vp9hip_decoder_release. */
int  vp9hip_decoder_receive_frame(vp9hip_decoder *d, vp9hip_decoded_frame *out);
int  vp9hip_decoder_release(vp9hip_decoder *d, int buf);
/* avcodec_flush_buffers: drop queued frames and reference state (seek). */
int  vp9hip_decoder_flush(vp9hip_decoder *d);

#ifdef __cplusplus
}
#endif
#endif /* VP9HIP_H */
