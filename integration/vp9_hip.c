/*
 * VP9 HIP hwaccel: libavcodec/vp9_hip.c in an FFmpeg tree (new file).
 *
 * The FFHWAccel (libavcodec/hwaccel_internal.h:34-166) that routes vp9.c's per-frame
 * hwaccel calls (vp9.c:1694-1713) to the adapter compiled into libvp9hip.so
 * (include/vp9hip_hwaccel.h, ffmpeg-hybrid_amd/csrc/vp9hip_hwaccel.cpp). Everything with
 * logic lives in the library, where tests/c/hwaccel_harness.c exercises it on the GPU in
 * vp9.c's call order; this file only maps FFmpeg's objects onto it:
 *   frame_params  -> vp9hip_hwaccel_frame_params: sizes, the frame count FFmpeg's consumer
 *                    may hold (max(0, extra_hw_frames) + frame threads, decode.c:1130-1140,
 *                    the default -1 of options_table.h:397 counting as 0)
 *   init          -> ff_decode_get_hw_frames_ctx (AV_HWDEVICE_TYPE_HIP) + vp9hip_hwaccel_init
 *   start_frame / decode_slice / end_frame -> the adapter's calls of the same names;
 *                    end_frame wraps the device frame it returns in CUR_FRAME's AVFrame
 *                    (buf[0] = a reference whose free is vp9hip_hwframe_unref, data[0..2] the
 *                    device planes, data[3] an AVHIPFrameSource: hwcontext_hip.h)
 *   flush / uninit -> vp9hip_hwaccel_flush / the last reference's release
 * show_existing_frame stays in vp9.c (vp9.c:1636-1653): it outputs a new reference to the
 * slot's AVFrame, whose buffer is already the device frame.
 *
 * Registration: hwaccels.h:80-88, the decoder's hw_configs (vp9.c:1982-2011,
 * HWACCEL_HIP(vp9)), AV_PIX_FMT_HIP in update_size's offer list (vp9.c:168-266), and
 * libavcodec/Makefile: OBJS-$(CONFIG_VP9_HIP_HWACCEL) += vp9_hip.o, -lvp9hip.
 *
 * Not built into a library here (it needs an FFmpeg tree).
 * tests/test_glue_typecheck.py type-checks it (gcc -fsyntax-only -Wall -Werror) against the
 * FFmpeg 8.0 declarations it binds, restated in tests/glue/ffmpeg_decls.h and pinned line by
 * line to the reference headers.
 */
#include "libavutil/hwcontext.h"
#include "libavutil/hwcontext_hip.h"
#include "libavutil/mem.h"
#include "libavutil/pixdesc.h"

#include "avcodec.h"
#include "decode.h"
#include "hwaccel_internal.h"
#include "hwconfig.h"
#include "internal.h"
#include "thread.h"
#include "vp9shared.h"

#include "vp9hip_hwaccel.h"

/* The adapter, shared by the decoder and every frame it handed out: a frame may outlive
 * avcodec_free_context (the adapter's pool holds its pixels), so the adapter is released
 * with the last reference. */
typedef struct VP9HIPShared {
    vp9hip_hwaccel *h;
} VP9HIPShared;

typedef struct VP9HIPContext {       /* hwaccel_priv_data */
    AVBufferRef *shared;             /* -> VP9HIPShared */
} VP9HIPContext;

typedef struct VP9HIPFrame {         /* data[3] of an output AVFrame; the free of its buf[0] */
    AVHIPFrameSource src;            /* first: data[3] is read as an AVHIPFrameSource */
    vp9hip_hwframe hf;
    AVBufferRef *shared;
} VP9HIPFrame;

static void vp9_hip_shared_free(void *opaque, uint8_t *data)
{
    VP9HIPShared *s = (VP9HIPShared *) data;
    vp9hip_hwaccel_uninit(s->h);     /* waits for what was launched, frees the device pool */
    av_free(s);
}

static vp9hip_hwaccel *adapter(AVCodecContext *avctx)
{
    VP9HIPContext *c = avctx->internal->hwaccel_priv_data;
    return ((VP9HIPShared *) c->shared->data)->h;
}

/* the frame count FFmpeg's consumers may hold beyond the decoder's own references: the
 * surfaces decode.c:1130-1140 adds to a frames pool, with extra_hw_frames' default of -1
 * counting as none */
static int vp9_hip_extra(const AVCodecContext *avctx)
{
    return FFMAX(0, avctx->extra_hw_frames) +
           ((avctx->active_thread_type & FF_THREAD_FRAME) ? avctx->thread_count : 0);
}

static int vp9_hip_params(AVCodecContext *avctx, enum AVPixelFormat sw, int w, int h, vp9hip_frames_params *fp)
{
    const AVPixFmtDescriptor *d = av_pix_fmt_desc_get(sw);
    if (!d)
        return AVERROR(EINVAL);
    return vp9hip_hwaccel_frame_params(w, h, d->comp[0].depth, d->log2_chroma_w, d->log2_chroma_h,
                                       vp9_hip_extra(avctx), fp);
}

static int vp9_hip_frame_params(AVCodecContext *avctx, AVBufferRef *hw_frames_ctx)
{
    AVHWFramesContext *fc = (AVHWFramesContext *) hw_frames_ctx->data;
    vp9hip_frames_params fp;
    int ret = vp9_hip_params(avctx, avctx->sw_pix_fmt, avctx->coded_width, avctx->coded_height, &fp);
    if (ret < 0)
        return ret;
    fc->format = AV_PIX_FMT_HIP;
    fc->sw_format = avctx->sw_pix_fmt;
    fc->width = fp.width;
    fc->height = fp.height;
    /* ff_get_buffer's surfaces are placeholders (end_frame replaces buf[0] by the adapter's
     * device frame): a pool of 1-byte host buffers instead of device memory; frames_get_buffer
     * leaves data[0..2] NULL for them (hwcontext_hip.c) */
    fc->pool = av_buffer_pool_init(1, NULL);
    fc->initial_pool_size = 0;
    return fc->pool ? 0 : AVERROR(ENOMEM);
}

static int vp9_hip_init(AVCodecContext *avctx)
{
    VP9HIPContext *c = avctx->internal->hwaccel_priv_data;
    const AVHWFramesContext *fc;
    const AVHIPDeviceContext *dev;
    VP9HIPShared *s;
    vp9hip_frames_params fp;
    int ret = ff_decode_get_hw_frames_ctx(avctx, AV_HWDEVICE_TYPE_HIP);
    if (ret < 0)
        return ret;
    fc = (const AVHWFramesContext *) avctx->hw_frames_ctx->data;
    dev = fc->device_ctx->hwctx;
    if ((ret = vp9_hip_params(avctx, fc->sw_format, fc->width, fc->height, &fp)) < 0)
        return ret;
    if (avctx->thread_count > 0)      /* host entropy-decode threads */
        fp.parse_threads = FFMIN(avctx->thread_count, 64);
    if (!(s = av_mallocz(sizeof(*s))))
        return AVERROR(ENOMEM);
    if ((ret = vp9hip_hwaccel_init(dev->device, &fp, &s->h)) < 0) {
        av_free(s);
        return ret;
    }
    c->shared = av_buffer_create((uint8_t *) s, sizeof(*s), vp9_hip_shared_free, NULL, 0);
    if (!c->shared) {
        vp9hip_hwaccel_uninit(s->h);
        av_free(s);
        return AVERROR(ENOMEM);
    }
    return 0;
}

static int vp9_hip_start_frame(AVCodecContext *avctx, const AVBufferRef *buf_ref, const uint8_t *buf, uint32_t size)
{
    const VP9SharedContext *s = avctx->priv_data;
    return vp9hip_hwaccel_start_frame(adapter(avctx), buf, size, s->frames[CUR_FRAME].tf.f->pts);
}

static int vp9_hip_decode_slice(AVCodecContext *avctx, const uint8_t *buf, uint32_t size)
{
    return vp9hip_hwaccel_decode_slice(adapter(avctx), buf, size);   /* header peek; entropy decode queued */
}

static int vp9_hip_src_sync(void *opaque, void *stream)
{
    VP9HIPFrame *fr = opaque;
    return vp9hip_hwframe_ready(((VP9HIPShared *) fr->shared->data)->h, &fr->hf, stream);
}

static int vp9_hip_src_transfer(void *opaque, uint8_t *const dst[3], const ptrdiff_t ls[3])
{
    VP9HIPFrame *fr = opaque;
    return vp9hip_hwframe_transfer(((VP9HIPShared *) fr->shared->data)->h, &fr->hf, dst, ls);
}

static void vp9_hip_frame_free(void *opaque, uint8_t *data)
{
    VP9HIPFrame *fr = (VP9HIPFrame *) data;
    vp9hip_hwframe_unref(((VP9HIPShared *) fr->shared->data)->h, &fr->hf);   /* thread-safe in the adapter */
    av_buffer_unref(&fr->shared);
    av_free(fr);
}

static int vp9_hip_end_frame(AVCodecContext *avctx)
{
    VP9HIPContext *c = avctx->internal->hwaccel_priv_data;
    VP9SharedContext *s = avctx->priv_data;
    AVFrame *f = s->frames[CUR_FRAME].tf.f;
    VP9HIPFrame *fr = av_mallocz(sizeof(*fr));
    AVBufferRef *ref;
    int ret;
    if (!fr)
        return AVERROR(ENOMEM);
    ret = vp9hip_hwaccel_end_frame(adapter(avctx), &fr->hf);   /* 1 shown, 0 hidden: both referenced */
    if (ret < 0) {
        av_free(fr);
        return ret;
    }
    fr->shared = av_buffer_ref(c->shared);
    ref = fr->shared ? av_buffer_create((uint8_t *) fr, sizeof(*fr), vp9_hip_frame_free, NULL, 0) : NULL;
    if (!ref) {
        vp9hip_hwframe_unref(adapter(avctx), &fr->hf);
        av_buffer_unref(&fr->shared);
        av_free(fr);
        return AVERROR(ENOMEM);
    }
    fr->src.sync = vp9_hip_src_sync;
    fr->src.transfer = vp9_hip_src_transfer;
    fr->src.opaque = fr;
    av_buffer_unref(&f->buf[0]);                               /* the placeholder surface */
    f->buf[0] = ref;
    for (int i = 0; i < 3; i++) {                              /* zero-copy: the device planes */
        f->data[i] = fr->hf.data[i];
        f->linesize[i] = (int) fr->hf.linesize[i];
    }
    f->data[3] = (uint8_t *) &fr->src;
    return 0;
}

static void vp9_hip_flush(AVCodecContext *avctx)
{
    VP9HIPContext *c = avctx->internal->hwaccel_priv_data;
    if (c->shared)
        vp9hip_hwaccel_flush(adapter(avctx));
}

static int vp9_hip_uninit(AVCodecContext *avctx)
{
    VP9HIPContext *c = avctx->internal->hwaccel_priv_data;
    av_buffer_unref(&c->shared);     /* the adapter goes with the last frame that needs it */
    return 0;
}

const FFHWAccel ff_vp9_hip_hwaccel = {
    .p.name         = "vp9_hip",
    .p.type         = AVMEDIA_TYPE_VIDEO,
    .p.id           = AV_CODEC_ID_VP9,
    .p.pix_fmt      = AV_PIX_FMT_HIP,
    .start_frame    = vp9_hip_start_frame,
    .decode_slice   = vp9_hip_decode_slice,
    .end_frame      = vp9_hip_end_frame,
    .frame_params   = vp9_hip_frame_params,
    .init           = vp9_hip_init,
    .uninit         = vp9_hip_uninit,
    .flush          = vp9_hip_flush,
    .priv_data_size = sizeof(VP9HIPContext),
    /* not THREAD_SAFE: frame threads hand the one context along under hwaccel_mutex
     * (pthread_frame.c:163, 675-705); nothing in the per-frame calls waits on the GPU */
    .caps_internal  = HWACCEL_CAP_ASYNC_SAFE,
};
