/*
 * HIP hardware context: libavutil/hwcontext_hip.c in an FFmpeg tree (new file).
 *
 * The HWContextType (libavutil/hwcontext_internal.h:28-98) behind AV_HWDEVICE_TYPE_HIP and
 * AV_PIX_FMT_HIP, the pixel format the vp9_hip hwaccel (integration/vp9_hip.c) outputs.
 * Callbacks, by the slots of hwcontext_internal.h:
 *   device_create (:58)        HIP device ordinal from the device string, a stream of its own
 *   device_uninit (:64)        destroys that stream
 *   frames_init (:70)          checks sw_format, sets up a pool of pitched device frames
 *   frames_get_buffer (:73)    a pool frame: data[0..2] device planes, data[3] = NULL
 *   transfer_get_formats (:74) sw_format both ways
 *   transfer_data_from (:79)   device -> host: a producer-owned frame (data[3] = an
 *                              AVHIPFrameSource) through its producer's transfer, which waits for
 *                              the frame's own batch and checks it (vp9hip_hwframe_transfer);
 *                              a pool frame by hipMemcpy2DAsync on the context's stream
 *   transfer_data_to (:77)     host -> a pool frame
 * Modelled on the shape of hwcontext_cuda.c (a pitched device pool, 2-D copies on the device
 * context's stream); HIP is linked directly (libamdhip64), there is no dynamic loader.
 *
 * Not built into a library here (it needs an FFmpeg tree; INTEGRATION.md lists the
 * registration lines: hwcontext.c tables, pixfmt.h / pixdesc.c entries, Makefile).
 * tests/test_glue_typecheck.py type-checks it (gcc -fsyntax-only -Wall -Werror) against the
 * FFmpeg 8.0 declarations it binds, restated in tests/glue/ffmpeg_decls.h and pinned line by
 * line to the reference headers.
 */
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "buffer.h"
#include "common.h"
#include "hwcontext.h"
#include "hwcontext_internal.h"
#include "hwcontext_hip.h"
#include "mem.h"
#include "pixdesc.h"
#include "pixfmt.h"

#define HIP_PITCH_ALIGN 256          /* 128-B lines, pairs of them: 16-byte loads stay aligned */

/* the software formats the vp9_hip hwaccel produces (profiles 0-3 at 8/10/12 bit) */
static const enum AVPixelFormat hip_sw_formats[] = {
    AV_PIX_FMT_YUV420P, AV_PIX_FMT_YUV422P, AV_PIX_FMT_YUV440P, AV_PIX_FMT_YUV444P,
    AV_PIX_FMT_YUV420P10, AV_PIX_FMT_YUV422P10, AV_PIX_FMT_YUV440P10, AV_PIX_FMT_YUV444P10,
    AV_PIX_FMT_YUV420P12, AV_PIX_FMT_YUV422P12, AV_PIX_FMT_YUV440P12, AV_PIX_FMT_YUV444P12,
};

typedef struct HIPFramesPriv {       /* AVHWFramesContext.hwctx */
    int nplanes;
    ptrdiff_t pitch[3];              /* bytes */
    size_t offset[3], size;          /* plane offsets inside one allocation, its size */
} HIPFramesPriv;

#define HIPCHECK(ctx, x) hip_check((ctx), (x), #x)
static int hip_check(void *log_ctx, hipError_t e, const char *what)
{
    if (e == hipSuccess)
        return 0;
    av_log(log_ctx, AV_LOG_ERROR, "%s failed: %s\n", what, hipGetErrorString(e));
    return AVERROR_EXTERNAL;
}

static int hip_device_create(AVHWDeviceContext *ctx, const char *device, AVDictionary *opts, int flags)
{
    AVHIPDeviceContext *hwctx = ctx->hwctx;
    int n = 0, dev = device ? atoi(device) : 0, ret;
    hipStream_t st = NULL;
    if ((ret = HIPCHECK(ctx, hipGetDeviceCount(&n))) < 0)
        return ret;
    if (dev < 0 || dev >= n) {
        av_log(ctx, AV_LOG_ERROR, "HIP device %d not present (%d devices)\n", dev, n);
        return AVERROR(ENODEV);
    }
    if ((ret = HIPCHECK(ctx, hipSetDevice(dev))) < 0 ||
        (ret = HIPCHECK(ctx, hipStreamCreateWithFlags(&st, hipStreamNonBlocking))) < 0)
        return ret;
    hwctx->device = dev;
    hwctx->stream = st;
    return 0;
}

static void hip_device_uninit(AVHWDeviceContext *ctx)
{
    AVHIPDeviceContext *hwctx = ctx->hwctx;
    if (hwctx->stream) {
        hipSetDevice(hwctx->device);
        hipStreamDestroy((hipStream_t) hwctx->stream);
        hwctx->stream = NULL;
    }
}

static void hip_pool_free(void *opaque, uint8_t *data)
{
    hipFree(data);
}

static AVBufferRef *hip_pool_alloc(void *opaque, size_t size)
{
    AVHWFramesContext *ctx = opaque;
    const AVHIPDeviceContext *dev = ctx->device_ctx->hwctx;
    void *p = NULL;
    AVBufferRef *ref;
    if (hipSetDevice(dev->device) != hipSuccess || hipMalloc(&p, size) != hipSuccess)
        return NULL;
    ref = av_buffer_create(p, size, hip_pool_free, NULL, 0);
    if (!ref)
        hipFree(p);
    return ref;
}

static int hip_frames_init(AVHWFramesContext *ctx)
{
    HIPFramesPriv *priv = ctx->hwctx;
    const AVPixFmtDescriptor *d = av_pix_fmt_desc_get(ctx->sw_format);
    int ok = 0;
    size_t off = 0;
    for (int i = 0; i < FF_ARRAY_ELEMS(hip_sw_formats); i++)
        ok |= hip_sw_formats[i] == ctx->sw_format;
    if (!ok || !d) {
        av_log(ctx, AV_LOG_ERROR, "Pixel format %s is not supported by HIP frames\n",
               av_get_pix_fmt_name(ctx->sw_format));
        return AVERROR(ENOSYS);
    }
    priv->nplanes = 3;
    for (int p = 0; p < 3; p++) {
        const int w = p ? AV_CEIL_RSHIFT(ctx->width, d->log2_chroma_w) : ctx->width;
        const int h = p ? AV_CEIL_RSHIFT(ctx->height, d->log2_chroma_h) : ctx->height;
        const int by = d->comp[0].depth > 8 ? 2 : 1;
        priv->pitch[p] = FFALIGN((ptrdiff_t) w * by, HIP_PITCH_ALIGN);
        priv->offset[p] = off;
        off += (size_t) priv->pitch[p] * h;
    }
    priv->size = off;
    if (!ctx->pool) {
        ffhwframesctx(ctx)->pool_internal = av_buffer_pool_init2(priv->size, ctx, hip_pool_alloc, NULL);
        if (!ffhwframesctx(ctx)->pool_internal)
            return AVERROR(ENOMEM);
    }
    return 0;
}

static int hip_frames_get_buffer(AVHWFramesContext *ctx, AVFrame *frame)
{
    const HIPFramesPriv *priv = ctx->hwctx;
    frame->buf[0] = av_buffer_pool_get(ctx->pool ? ctx->pool : ffhwframesctx(ctx)->pool_internal);
    if (!frame->buf[0])
        return AVERROR(ENOMEM);
    /* a user pool smaller than a frame holds placeholders (the vp9_hip hwaccel's: end_frame
     * replaces buf[0] by its device frame): no plane pointers into it */
    const int real = frame->buf[0]->size >= priv->size;
    for (int p = 0; p < priv->nplanes; p++) {
        frame->data[p] = real ? frame->buf[0]->data + priv->offset[p] : NULL;
        frame->linesize[p] = (int) priv->pitch[p];
    }
    frame->data[3] = NULL;             /* a pool frame: plain device memory */
    frame->format = AV_PIX_FMT_HIP;
    frame->width = ctx->width;
    frame->height = ctx->height;
    return 0;
}

static int hip_transfer_get_formats(AVHWFramesContext *ctx, enum AVHWFrameTransferDirection dir,
                                    enum AVPixelFormat **formats)
{
    enum AVPixelFormat *f = av_malloc_array(2, sizeof(*f));
    if (!f)
        return AVERROR(ENOMEM);
    f[0] = ctx->sw_format;
    f[1] = AV_PIX_FMT_NONE;
    *formats = f;
    return 0;
}

/* 2-D copies of the three planes on the device context's stream, then a wait */
static int hip_copy_planes(AVHWFramesContext *ctx, AVFrame *dst, const AVFrame *src, enum hipMemcpyKind kind)
{
    const AVHIPDeviceContext *dev = ctx->device_ctx->hwctx;
    const AVPixFmtDescriptor *d = av_pix_fmt_desc_get(ctx->sw_format);
    const int by = d->comp[0].depth > 8 ? 2 : 1;
    int ret;
    if ((ret = HIPCHECK(ctx, hipSetDevice(dev->device))) < 0)
        return ret;
    for (int p = 0; p < 3; p++) {
        const int w = p ? AV_CEIL_RSHIFT(dst->width, d->log2_chroma_w) : dst->width;
        const int h = p ? AV_CEIL_RSHIFT(dst->height, d->log2_chroma_h) : dst->height;
        if ((ret = HIPCHECK(ctx, hipMemcpy2DAsync(dst->data[p], dst->linesize[p], src->data[p], src->linesize[p],
                                                  (size_t) w * by, h, kind, (hipStream_t) dev->stream))) < 0)
            return ret;
    }
    return HIPCHECK(ctx, hipStreamSynchronize((hipStream_t) dev->stream));
}

static int hip_transfer_data_from(AVHWFramesContext *ctx, AVFrame *dst, const AVFrame *src)
{
    const AVHIPFrameSource *s = (const AVHIPFrameSource *) src->data[3];
    if (dst->format != ctx->sw_format || dst->width > src->width || dst->height > src->height)
        return AVERROR(EINVAL);
    if (s)                              /* producer-owned: its batch, its checks, its copy */
        return s->transfer(s->opaque, dst->data, (const ptrdiff_t[3]) { dst->linesize[0], dst->linesize[1],
                                                                         dst->linesize[2] });
    return hip_copy_planes(ctx, dst, src, hipMemcpyDeviceToHost);
}

static int hip_transfer_data_to(AVHWFramesContext *ctx, AVFrame *dst, const AVFrame *src)
{
    if (dst->data[3])                   /* a producer's frame is read-only */
        return AVERROR(EINVAL);
    if (src->format != ctx->sw_format || src->width > dst->width || src->height > dst->height)
        return AVERROR(EINVAL);
    return hip_copy_planes(ctx, dst, src, hipMemcpyHostToDevice);
}

int av_hip_frame_sync(const AVFrame *frame, void *stream)
{
    const AVHIPFrameSource *s;
    if (!frame || frame->format != AV_PIX_FMT_HIP)
        return AVERROR(EINVAL);
    s = (const AVHIPFrameSource *) frame->data[3];
    return s ? s->sync(s->opaque, stream) : 0;   /* pool frames: ordered by their writer */
}

const HWContextType ff_hwcontext_type_hip = {
    .type                 = AV_HWDEVICE_TYPE_HIP,
    .name                 = "HIP",
    .device_hwctx_size    = sizeof(AVHIPDeviceContext),
    .frames_hwctx_size    = sizeof(HIPFramesPriv),
    .device_create        = hip_device_create,
    .device_uninit        = hip_device_uninit,
    .frames_init          = hip_frames_init,
    .frames_get_buffer    = hip_frames_get_buffer,
    .transfer_get_formats = hip_transfer_get_formats,
    .transfer_data_to     = hip_transfer_data_to,
    .transfer_data_from   = hip_transfer_data_from,
    .pix_fmts             = (const enum AVPixelFormat[]) { AV_PIX_FMT_HIP, AV_PIX_FMT_NONE },
};
