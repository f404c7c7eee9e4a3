/*
 * ORACLE — test infrastructure only. A scalar CPU restatement of the reference
 * libavcodec VP9 pixel path (vp9recon.c, vp9_mc_template.c, vp9lpf.c, the
 * reconstruction half of vp9block.c and vp9dsp_template.c) that consumes the same
 * pass-1 frame packet (include/vp9hip.h) as the HIP path. Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 *
 * Parity status: the reference decoder could not be built or run in this pipeline
 * (SURVEY.md §8c), and the FATE bitstreams are absent, so this restatement is
 * "parity unpinned" against reference outputs; it is pinned by property tests built
 * from the reference's own checkasm generators (tests/checkasm/vp9dsp.c).
 */
#ifndef VP9_ORACLE_H
#define VP9_ORACLE_H
#include <stddef.h>
#include <stdint.h>
#include "../include/vp9hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* A frame: planes of uint8_t (bpp 8) or uint16_t (bpp > 8); stride in PIXELS.
 * Buffers must cover the frame size rounded up to 64 luma pixels. */
typedef struct vp9o_planes {
    void     *data[3];
    ptrdiff_t stride[3];
    int       w, h;        /* visible size */
} vp9o_planes;

/* Reconstruct + loop-filter one frame. refs[i] = LAST/GOLDEN/ALTREF (may be NULL
 * for intra frames). Returns 0 or a negative error. */
int vp9o_decode_frame(const vp9h_frame *f, vp9o_planes *cur, const vp9o_planes *refs);
/* The same frame with the tile columns of each SB row on up to nthreads threads and the
 * loop filter of the previous row overlapped (decode_tiles_mt + loopfilter_proc,
 * vp9.c:1442-1551): the slice-threaded CPU baseline. Output identical. */
int vp9o_decode_frame_tiles(const vp9h_frame *f, vp9o_planes *cur, const vp9o_planes *refs, int nthreads);

/* DSP entry points for unit tests (stride in pixels). */
void vp9o_itxfm_add(int bpp, void *dst, ptrdiff_t stride, void *coef, int eob, int tx, int txtp);
void vp9o_intra_pred(int bpp, void *dst, ptrdiff_t stride, const void *left, const void *top,
                     int tx, int mode);
void vp9o_loop_filter(int bpp, void *dst, ptrdiff_t stride, int kind, int wd1, int wd2, int dir,
                      int E, int I, int H);
/* scaled MC (do_scaled_8tap / do_scaled_bilin, vp9dsp_template.c:2363-2482) */
void vp9o_mc_scaled(int bpp, void *dst, ptrdiff_t ds, const void *src, ptrdiff_t ss, int w, int h,
                    int mx, int my, int dx, int dy, int filter, int avg);
void vp9o_mc(int bpp, void *dst, ptrdiff_t ds, const void *src, ptrdiff_t ss, int w, int h,
             int mx, int my, int filter, int avg);
/* scan table access: returns pointer to the scan for tx (0..3, 4 = lossless) / txtp */
const int16_t *vp9o_scan(int tx, int txtp);

#ifdef __cplusplus
}
#endif
#endif
