/*
 * The FFHWAccel adapter of the hybrid VP9 decoder over libvp9hip (include/vp9hip_hwaccel.h).
 *
 * One context per stream, as avctx->internal->hwaccel_priv_data: the device context, the
 * host entropy decoder state, the frame being decoded, and the device frame pool with the
 * reference slots. The call order is the reference's (vp9.c:1694-1713): start_frame,
 * decode_slice, end_frame per coded frame; show_existing_frame never reaches the
 * hwaccel (vp9.c:1636-1653) and is answered from the slots.
 *
 * Pool: a buffer is free when no reference slot holds it, no handed-out frame references
 * it and it is not the frame being decoded (the AVBufferPool of an AVHWFramesContext).
 */
#include <stdlib.h>
#include <string.h>

#include "../../include/vp9hip_hwaccel.h"

struct vp9hip_hwaccel {
    vp9hip_ctx *gpu;
    vp9h_stream *st;               /* host entropy decoder: contexts, segmentation, MVs   */
    vp9hip_frames_params fp;
    int slot[8];                   /* device buffer of each reference slot (s->s.ref_frames) */
    int *refs;                     /* per pool buffer: handed-out frame references         */
    int cur;                       /* buffer of the frame being decoded, -1 between frames  */
    int64_t pts;
    int have_pkt;
    vp9h_frame pkt;                /* pass-1 packet of the current frame                    */
    vp9h_frame_info info;          /* its header decisions (refidx, refreshrefmask, show)   */
};

static int swfmt(int bpp, int ss_h, int ss_v)
{
    const int chroma = ss_h && ss_v ? 0 : ss_h ? 1 : ss_v ? 2 : 3;
    return (bpp == 8 ? 0 : bpp == 10 ? 4 : 8) + chroma;
}

int vp9hip_hwaccel_frame_params(int width, int height, int bpp, int ss_h, int ss_v, int extra,
                                vp9hip_frames_params *out)
{
    if (!out || width <= 0 || height <= 0 || (bpp != 8 && bpp != 10 && bpp != 12) || ss_h < 0 || ss_h > 1 ||
        ss_v < 0 || ss_v > 1 || extra < 0)
        return VP9HIP_EINVAL;
    memset(out, 0, sizeof(*out));
    out->sw_format = swfmt(bpp, ss_h, ss_v);
    out->width = width;
    out->height = height;
    out->initial_pool_size = 8 + 1 + extra;
    out->bpp = bpp;
    out->ss_h = ss_h;
    out->ss_v = ss_v;
    return 0;
}

int vp9hip_hwaccel_init(int device, const vp9hip_frames_params *fp, vp9hip_hwaccel **out)
{
    if (!fp || !out || fp->initial_pool_size < 9) return VP9HIP_EINVAL;
    *out = NULL;
    vp9hip_hwaccel *h = calloc(1, sizeof(*h));
    if (!h) return VP9HIP_ENOMEM;
    h->fp = *fp;
    h->cur = -1;
    for (int i = 0; i < 8; i++) h->slot[i] = -1;
    h->refs = calloc((size_t) fp->initial_pool_size, sizeof(int));
    int r = h->refs ? 0 : VP9HIP_ENOMEM;
    if (!r) r = vp9hip_open(device, &h->gpu);
    if (!r) r = vp9hip_configure(h->gpu, fp->width, fp->height, fp->bpp, fp->ss_h, fp->ss_v, fp->initial_pool_size);
    if (!r) r = vp9h_stream_open(&h->st);
    if (r < 0) {
        vp9hip_hwaccel_uninit(h);
        return r;
    }
    *out = h;
    return 0;
}

int vp9hip_hwaccel_uninit(vp9hip_hwaccel *h)
{
    if (!h) return 0;
    if (h->have_pkt) vp9h_frame_free(&h->pkt);
    if (h->st) vp9h_stream_close(h->st);
    if (h->gpu) vp9hip_close(h->gpu);
    free(h->refs);
    free(h);
    return 0;
}

static int buf_busy(const vp9hip_hwaccel *h, int b)
{
    if (h->refs[b] || b == h->cur) return 1;
    for (int s = 0; s < 8; s++)
        if (h->slot[s] == b) return 1;
    return 0;
}

int vp9hip_hwaccel_start_frame(vp9hip_hwaccel *h, const uint8_t *buf, uint32_t size, int64_t pts)
{
    if (!h || (!buf && size)) return VP9HIP_EINVAL;
    if (h->have_pkt) {                      /* a frame that never reached end_frame */
        vp9h_frame_free(&h->pkt);
        h->have_pkt = 0;
    }
    h->cur = -1;
    for (int b = 0; b < h->fp.initial_pool_size; b++)
        if (!buf_busy(h, b)) { h->cur = b; break; }
    if (h->cur < 0) return VP9HIP_EAGAIN;  /* every buffer held: the caller must unref frames */
    h->pts = pts;
    return 0;
}

int vp9hip_hwaccel_decode_slice(vp9hip_hwaccel *h, const uint8_t *buf, uint32_t size)
{
    if (!h || !buf || !size || h->cur < 0) return VP9HIP_EINVAL;
    memset(&h->pkt, 0, sizeof(h->pkt));
    memset(&h->info, 0, sizeof(h->info));
    const int r = vp9h_stream_decode(h->st, buf, size, &h->pkt, &h->info);
    if (r < 0) return r;
    if (h->info.show_existing_frame) return VP9HIP_EINVALIDDATA;     /* vp9.c answers these itself */
    h->have_pkt = 1;
    if (h->pkt.width > h->fp.width || h->pkt.height > h->fp.height || h->pkt.bpp != h->fp.bpp ||
        h->pkt.ss_h != h->fp.ss_h || h->pkt.ss_v != h->fp.ss_v)
        return VP9HIP_ENOSYS;                /* a new format: get_format re-inits the hwaccel */
    return 0;
}

static void fill_frame(vp9hip_hwaccel *h, int b, int64_t pts, vp9hip_hwframe *out)
{
    memset(out, 0, sizeof(*out));
    int w = 0, ht = 0;
    vp9hip_frame_device(h->gpu, b, out->data, out->linesize, &w, &ht, &out->stream);
    out->width = w;
    out->height = ht;
    out->sw_format = h->fp.sw_format;
    out->buf = b;
    out->pts = pts;
    h->refs[b]++;
}

int vp9hip_hwaccel_end_frame(vp9hip_hwaccel *h, vp9hip_hwframe *out)
{
    if (!h || h->cur < 0 || !h->have_pkt) return VP9HIP_EINVAL;
    const vp9h_frame *f = &h->pkt;
    const int intra = f->keyframe || f->intraonly;
    int refs[3] = { 0, 0, 0 };
    for (int i = 0; i < 3 && !intra; i++) {  /* s->s.h.refidx -> the slots' device buffers */
        refs[i] = h->slot[h->info.ref_slot[i] & 7];
        if (refs[i] < 0) return VP9HIP_EINVALIDDATA;
    }
    int r = vp9hip_submit_frame(h->gpu, f, h->cur, refs);
    vp9h_frame_free(&h->pkt);
    h->have_pkt = 0;
    if (r < 0) { h->cur = -1; return r; }
    for (int i = 0; i < 8; i++)              /* vp9.c:1705-1711: slots of refreshrefmask */
        if (h->info.refresh_mask & (1 << i)) h->slot[i] = h->cur;
    const int shown = h->info.show_frame != 0;
    if (shown && out) fill_frame(h, h->cur, h->pts, out);
    h->cur = -1;
    return shown;
}

int vp9hip_hwaccel_show_existing(vp9hip_hwaccel *h, int slot, int64_t pts, vp9hip_hwframe *out)
{
    if (!h || !out || slot < 0 || slot > 7) return VP9HIP_EINVAL;
    if (h->slot[slot] < 0) return VP9HIP_EINVALIDDATA;               /* "Requested reference ... not available" */
    fill_frame(h, h->slot[slot], pts, out);
    return 0;
}

void vp9hip_hwaccel_flush(vp9hip_hwaccel *h)
{
    if (!h) return;
    for (int i = 0; i < 8; i++) h->slot[i] = -1;
    if (h->have_pkt) { vp9h_frame_free(&h->pkt); h->have_pkt = 0; }
    h->cur = -1;
    if (h->st) { vp9h_stream_close(h->st); h->st = NULL; vp9h_stream_open(&h->st); }
    vp9hip_flush(h->gpu);
}

int vp9hip_hwaccel_last_header(const vp9hip_hwaccel *h, vp9h_frame_info *info)
{
    if (!h || !info) return VP9HIP_EINVAL;
    *info = h->info;
    return 0;
}

int vp9hip_hwframe_transfer(vp9hip_hwaccel *h, const vp9hip_hwframe *src, uint8_t *const dst[3],
                            const ptrdiff_t dst_linesize[3])
{
    if (!h || !src || src->buf < 0 || src->buf >= h->fp.initial_pool_size || !h->refs[src->buf]) return VP9HIP_EINVAL;
    return vp9hip_download_frame(h->gpu, src->buf, dst, dst_linesize);
}

int vp9hip_hwframe_unref(vp9hip_hwaccel *h, vp9hip_hwframe *f)
{
    if (!h || !f || f->buf < 0 || f->buf >= h->fp.initial_pool_size || h->refs[f->buf] <= 0) return VP9HIP_EINVAL;
    h->refs[f->buf]--;
    memset(f, 0, sizeof(*f));
    f->buf = -1;
    return 0;
}
