/*
 * TEST INFRASTRUCTURE: the FFmpeg 8.0 declarations integration/vp9_hip.c and
 * integration/hwcontext_hip.c bind, restated so the glue can be type-checked without an
 * FFmpeg build tree (tests/test_glue_typecheck.py: gcc -fsyntax-only through the shim
 * headers under tests/glue/inc/). FFmpeg's own headers cannot be compiled here: they need
 * the configure-generated config.h / avconfig.h.
 *
 * Every restated line ends with a marker the test checks against /root/reference when it is
 * present:
 *   / *@ FILE * /            the line (comments and white space normalised; for a function,
 *                           its declaration up to the parameter list's closing parenthesis)
 *                           appears in FILE;
 *   / *@ FILE in NAME * /    ... inside the body of struct / union / enum NAME of FILE.
 * Members the glue does not touch are left out of the partial structs (AVCodecContext,
 * AVFrame, ...); FFHWAccel and HWContextType, whose slots the glue fills, are complete.
 * The section at the end is not FFmpeg's yet: the registration lines INTEGRATION.md adds.
 */
#ifndef VP9HIP_TEST_FFMPEG_DECLS_H
#define VP9HIP_TEST_FFMPEG_DECLS_H

#include <errno.h>
#include <stddef.h>
#include <stdint.h>

/* ---- libavutil/attributes.h, macros.h, common.h, error.h, log.h ---- */
#define av_builtin_constant_p __builtin_constant_p                                     /*@ libavutil/attributes.h */
#define FFMAX(a,b) ((a) > (b) ? (a) : (b))                                            /*@ libavutil/macros.h */
#define FFMIN(a,b) ((a) > (b) ? (b) : (a))                                            /*@ libavutil/macros.h */
#define FF_ARRAY_ELEMS(a) (sizeof(a) / sizeof((a)[0]))                                /*@ libavutil/macros.h */
#define MKTAG(a,b,c,d) ((a) | ((b) << 8) | ((c) << 16) | ((unsigned)(d) << 24))        /*@ libavutil/macros.h */
#define FFALIGN(x, a) (((x)+(a)-1)&~((a)-1))                                          /*@ libavutil/macros.h */
#define AV_CEIL_RSHIFT(a,b) (!av_builtin_constant_p(b) ? -((-(a)) >> (b)) : ((a) + (1<<(b)) - 1) >> (b)) /*@ libavutil/common.h */
#define AVERROR(e) (-(e))                                                             /*@ libavutil/error.h */
#define FFERRTAG(a, b, c, d) (-(int)MKTAG(a, b, c, d))                                /*@ libavutil/error.h */
#define AVERROR_EXTERNAL FFERRTAG( 'E','X','T',' ')                                   /*@ libavutil/error.h */
#define AV_LOG_ERROR 16                                                               /*@ libavutil/log.h */
void av_log(void *avcl, int level, const char *fmt, ...);                             /*@ libavutil/log.h */

/* ---- libavutil/avutil.h, dict.h, mem.h ---- */
enum AVMediaType {                                                                    /*@ libavutil/avutil.h */
    AVMEDIA_TYPE_VIDEO,                                                               /*@ libavutil/avutil.h in AVMediaType */
};
typedef struct AVDictionary AVDictionary;                                             /*@ libavutil/dict.h */
typedef struct AVClass AVClass;
void *av_mallocz(size_t size);                                                        /*@ libavutil/mem.h */
void *av_malloc_array(size_t nmemb, size_t size);                                     /*@ libavutil/mem.h */
void av_free(void *ptr);                                                              /*@ libavutil/mem.h */

/* ---- libavutil/buffer.h ---- */
typedef struct AVBuffer AVBuffer;                                                     /*@ libavutil/buffer.h */
typedef struct AVBufferRef {                                                          /*@ libavutil/buffer.h */
    AVBuffer *buffer;                                                                 /*@ libavutil/buffer.h in AVBufferRef */
    uint8_t *data;                                                                    /*@ libavutil/buffer.h in AVBufferRef */
    size_t size;                                                                      /*@ libavutil/buffer.h in AVBufferRef */
} AVBufferRef;                                                                        /*@ libavutil/buffer.h */
AVBufferRef *av_buffer_create(uint8_t *data, size_t size, void (*free)(void *opaque, uint8_t *data), void *opaque, int flags); /*@ libavutil/buffer.h */
AVBufferRef *av_buffer_ref(const AVBufferRef *buf);                                   /*@ libavutil/buffer.h */
void av_buffer_unref(AVBufferRef **buf);                                              /*@ libavutil/buffer.h */
typedef struct AVBufferPool AVBufferPool;                                             /*@ libavutil/buffer.h */
AVBufferPool *av_buffer_pool_init(size_t size, AVBufferRef* (*alloc)(size_t size));   /*@ libavutil/buffer.h */
AVBufferPool *av_buffer_pool_init2(size_t size, void *opaque, AVBufferRef* (*alloc)(void *opaque, size_t size), void (*pool_free)(void *opaque)); /*@ libavutil/buffer.h */
AVBufferRef *av_buffer_pool_get(AVBufferPool *pool);                                  /*@ libavutil/buffer.h */

/* ---- libavutil/pixfmt.h, pixdesc.h ---- */
enum AVPixelFormat {                                                                  /*@ libavutil/pixfmt.h */
    AV_PIX_FMT_NONE = -1,                                                             /*@ libavutil/pixfmt.h in AVPixelFormat */
    AV_PIX_FMT_YUV420P,                                                               /*@ libavutil/pixfmt.h in AVPixelFormat */
    AV_PIX_FMT_YUV422P,                                                               /*@ libavutil/pixfmt.h in AVPixelFormat */
    AV_PIX_FMT_YUV444P,                                                               /*@ libavutil/pixfmt.h in AVPixelFormat */
    AV_PIX_FMT_YUV440P,                                                               /*@ libavutil/pixfmt.h in AVPixelFormat */
    AV_PIX_FMT_YUV420P10LE,                                                           /*@ libavutil/pixfmt.h in AVPixelFormat */
    AV_PIX_FMT_YUV422P10LE,                                                           /*@ libavutil/pixfmt.h in AVPixelFormat */
    AV_PIX_FMT_YUV444P10LE,                                                           /*@ libavutil/pixfmt.h in AVPixelFormat */
    AV_PIX_FMT_YUV440P10LE,                                                           /*@ libavutil/pixfmt.h in AVPixelFormat */
    AV_PIX_FMT_YUV420P12LE,                                                           /*@ libavutil/pixfmt.h in AVPixelFormat */
    AV_PIX_FMT_YUV422P12LE,                                                           /*@ libavutil/pixfmt.h in AVPixelFormat */
    AV_PIX_FMT_YUV444P12LE,                                                           /*@ libavutil/pixfmt.h in AVPixelFormat */
    AV_PIX_FMT_YUV440P12LE,                                                           /*@ libavutil/pixfmt.h in AVPixelFormat */
    AV_PIX_FMT_NB                                                                     /*@ libavutil/pixfmt.h in AVPixelFormat */
};
#define AV_PIX_FMT_NE(be, le) AV_PIX_FMT_##le                                         /*@ libavutil/pixfmt.h */
#define AV_PIX_FMT_YUV420P10 AV_PIX_FMT_NE(YUV420P10BE, YUV420P10LE)                  /*@ libavutil/pixfmt.h */
#define AV_PIX_FMT_YUV422P10 AV_PIX_FMT_NE(YUV422P10BE, YUV422P10LE)                  /*@ libavutil/pixfmt.h */
#define AV_PIX_FMT_YUV440P10 AV_PIX_FMT_NE(YUV440P10BE, YUV440P10LE)                  /*@ libavutil/pixfmt.h */
#define AV_PIX_FMT_YUV444P10 AV_PIX_FMT_NE(YUV444P10BE, YUV444P10LE)                  /*@ libavutil/pixfmt.h */
#define AV_PIX_FMT_YUV420P12 AV_PIX_FMT_NE(YUV420P12BE, YUV420P12LE)                  /*@ libavutil/pixfmt.h */
#define AV_PIX_FMT_YUV422P12 AV_PIX_FMT_NE(YUV422P12BE, YUV422P12LE)                  /*@ libavutil/pixfmt.h */
#define AV_PIX_FMT_YUV440P12 AV_PIX_FMT_NE(YUV440P12BE, YUV440P12LE)                  /*@ libavutil/pixfmt.h */
#define AV_PIX_FMT_YUV444P12 AV_PIX_FMT_NE(YUV444P12BE, YUV444P12LE)                  /*@ libavutil/pixfmt.h */
typedef struct AVComponentDescriptor {                                                /*@ libavutil/pixdesc.h */
    int plane;                                                                        /*@ libavutil/pixdesc.h in AVComponentDescriptor */
    int step;                                                                         /*@ libavutil/pixdesc.h in AVComponentDescriptor */
    int offset;                                                                       /*@ libavutil/pixdesc.h in AVComponentDescriptor */
    int shift;                                                                        /*@ libavutil/pixdesc.h in AVComponentDescriptor */
    int depth;                                                                        /*@ libavutil/pixdesc.h in AVComponentDescriptor */
} AVComponentDescriptor;                                                              /*@ libavutil/pixdesc.h */
typedef struct AVPixFmtDescriptor {                                                   /*@ libavutil/pixdesc.h */
    const char *name;                                                                 /*@ libavutil/pixdesc.h in AVPixFmtDescriptor */
    uint8_t nb_components;                                                            /*@ libavutil/pixdesc.h in AVPixFmtDescriptor */
    uint8_t log2_chroma_w;                                                            /*@ libavutil/pixdesc.h in AVPixFmtDescriptor */
    uint8_t log2_chroma_h;                                                            /*@ libavutil/pixdesc.h in AVPixFmtDescriptor */
    uint64_t flags;                                                                   /*@ libavutil/pixdesc.h in AVPixFmtDescriptor */
    AVComponentDescriptor comp[4];                                                    /*@ libavutil/pixdesc.h in AVPixFmtDescriptor */
    const char *alias;                                                                /*@ libavutil/pixdesc.h in AVPixFmtDescriptor */
} AVPixFmtDescriptor;                                                                 /*@ libavutil/pixdesc.h */
const AVPixFmtDescriptor *av_pix_fmt_desc_get(enum AVPixelFormat pix_fmt);           /*@ libavutil/pixdesc.h */
const char *av_get_pix_fmt_name(enum AVPixelFormat pix_fmt);                          /*@ libavutil/pixdesc.h */

/* ---- libavutil/frame.h (partial AVFrame) ---- */
#define AV_NUM_DATA_POINTERS 8                                                        /*@ libavutil/frame.h */
typedef struct AVFrame {                                                              /*@ libavutil/frame.h */
    uint8_t *data[AV_NUM_DATA_POINTERS];                                              /*@ libavutil/frame.h in AVFrame */
    int linesize[AV_NUM_DATA_POINTERS];                                               /*@ libavutil/frame.h in AVFrame */
    int width, height;                                                                /*@ libavutil/frame.h in AVFrame */
    int format;                                                                       /*@ libavutil/frame.h in AVFrame */
    int64_t pts;                                                                      /*@ libavutil/frame.h in AVFrame */
    AVBufferRef *buf[AV_NUM_DATA_POINTERS];                                           /*@ libavutil/frame.h in AVFrame */
} AVFrame;                                                                            /*@ libavutil/frame.h */

/* ---- libavutil/hwcontext.h (partial contexts) ---- */
enum AVHWDeviceType {                                                                 /*@ libavutil/hwcontext.h */
    AV_HWDEVICE_TYPE_NONE,                                                            /*@ libavutil/hwcontext.h in AVHWDeviceType */
    AV_HWDEVICE_TYPE_CUDA,                                                            /*@ libavutil/hwcontext.h in AVHWDeviceType */
};
typedef struct AVHWDeviceContext {                                                    /*@ libavutil/hwcontext.h */
    const AVClass *av_class;                                                          /*@ libavutil/hwcontext.h in AVHWDeviceContext */
    enum AVHWDeviceType type;                                                         /*@ libavutil/hwcontext.h in AVHWDeviceContext */
    void *hwctx;                                                                      /*@ libavutil/hwcontext.h in AVHWDeviceContext */
} AVHWDeviceContext;                                                                  /*@ libavutil/hwcontext.h */
typedef struct AVHWFramesContext {                                                    /*@ libavutil/hwcontext.h */
    const AVClass *av_class;                                                          /*@ libavutil/hwcontext.h in AVHWFramesContext */
    AVBufferRef *device_ref;                                                          /*@ libavutil/hwcontext.h in AVHWFramesContext */
    AVHWDeviceContext *device_ctx;                                                    /*@ libavutil/hwcontext.h in AVHWFramesContext */
    void *hwctx;                                                                      /*@ libavutil/hwcontext.h in AVHWFramesContext */
    AVBufferPool *pool;                                                               /*@ libavutil/hwcontext.h in AVHWFramesContext */
    int initial_pool_size;                                                            /*@ libavutil/hwcontext.h in AVHWFramesContext */
    enum AVPixelFormat format;                                                        /*@ libavutil/hwcontext.h in AVHWFramesContext */
    enum AVPixelFormat sw_format;                                                     /*@ libavutil/hwcontext.h in AVHWFramesContext */
    int width, height;                                                                /*@ libavutil/hwcontext.h in AVHWFramesContext */
} AVHWFramesContext;                                                                  /*@ libavutil/hwcontext.h */
enum AVHWFrameTransferDirection {                                                     /*@ libavutil/hwcontext.h */
    AV_HWFRAME_TRANSFER_DIRECTION_FROM,                                               /*@ libavutil/hwcontext.h in AVHWFrameTransferDirection */
    AV_HWFRAME_TRANSFER_DIRECTION_TO,                                                 /*@ libavutil/hwcontext.h in AVHWFrameTransferDirection */
};
typedef struct AVHWFramesConstraints AVHWFramesConstraints;

/* ---- libavutil/hwcontext_internal.h (complete HWContextType) ---- */
typedef struct HWContextType {                                                        /*@ libavutil/hwcontext_internal.h */
    enum AVHWDeviceType type;                                                         /*@ libavutil/hwcontext_internal.h in HWContextType */
    const char *name;                                                                 /*@ libavutil/hwcontext_internal.h in HWContextType */
    const enum AVPixelFormat *pix_fmts;                                               /*@ libavutil/hwcontext_internal.h in HWContextType */
    size_t device_hwctx_size;                                                         /*@ libavutil/hwcontext_internal.h in HWContextType */
    size_t device_hwconfig_size;                                                      /*@ libavutil/hwcontext_internal.h in HWContextType */
    size_t frames_hwctx_size;                                                         /*@ libavutil/hwcontext_internal.h in HWContextType */
    int (*device_create)(AVHWDeviceContext *ctx, const char *device, AVDictionary *opts, int flags); /*@ libavutil/hwcontext_internal.h in HWContextType */
    int (*device_derive)(AVHWDeviceContext *dst_ctx, AVHWDeviceContext *src_ctx, AVDictionary *opts, int flags); /*@ libavutil/hwcontext_internal.h in HWContextType */
    int (*device_init)(AVHWDeviceContext *ctx);                                       /*@ libavutil/hwcontext_internal.h in HWContextType */
    void (*device_uninit)(AVHWDeviceContext *ctx);                                    /*@ libavutil/hwcontext_internal.h in HWContextType */
    int (*frames_get_constraints)(AVHWDeviceContext *ctx, const void *hwconfig, AVHWFramesConstraints *constraints); /*@ libavutil/hwcontext_internal.h in HWContextType */
    int (*frames_init)(AVHWFramesContext *ctx);                                       /*@ libavutil/hwcontext_internal.h in HWContextType */
    void (*frames_uninit)(AVHWFramesContext *ctx);                                    /*@ libavutil/hwcontext_internal.h in HWContextType */
    int (*frames_get_buffer)(AVHWFramesContext *ctx, AVFrame *frame);                 /*@ libavutil/hwcontext_internal.h in HWContextType */
    int (*transfer_get_formats)(AVHWFramesContext *ctx, enum AVHWFrameTransferDirection dir, enum AVPixelFormat **formats); /*@ libavutil/hwcontext_internal.h in HWContextType */
    int (*transfer_data_to)(AVHWFramesContext *ctx, AVFrame *dst, const AVFrame *src); /*@ libavutil/hwcontext_internal.h in HWContextType */
    int (*transfer_data_from)(AVHWFramesContext *ctx, AVFrame *dst, const AVFrame *src); /*@ libavutil/hwcontext_internal.h in HWContextType */
    int (*map_to)(AVHWFramesContext *ctx, AVFrame *dst, const AVFrame *src, int flags); /*@ libavutil/hwcontext_internal.h in HWContextType */
    int (*map_from)(AVHWFramesContext *ctx, AVFrame *dst, const AVFrame *src, int flags); /*@ libavutil/hwcontext_internal.h in HWContextType */
    int (*frames_derive_to)(AVHWFramesContext *dst_ctx, AVHWFramesContext *src_ctx, int flags); /*@ libavutil/hwcontext_internal.h in HWContextType */
    int (*frames_derive_from)(AVHWFramesContext *dst_ctx, AVHWFramesContext *src_ctx, int flags); /*@ libavutil/hwcontext_internal.h in HWContextType */
} HWContextType;                                                                      /*@ libavutil/hwcontext_internal.h */
typedef struct FFHWFramesContext {                                                    /*@ libavutil/hwcontext_internal.h */
    AVHWFramesContext p;                                                              /*@ libavutil/hwcontext_internal.h in FFHWFramesContext */
    const HWContextType *hw_type;                                                     /*@ libavutil/hwcontext_internal.h in FFHWFramesContext */
    AVBufferPool *pool_internal;                                                      /*@ libavutil/hwcontext_internal.h in FFHWFramesContext */
    AVBufferRef *source_frames;                                                       /*@ libavutil/hwcontext_internal.h in FFHWFramesContext */
    int source_allocation_map_flags;                                                  /*@ libavutil/hwcontext_internal.h in FFHWFramesContext */
} FFHWFramesContext;                                                                  /*@ libavutil/hwcontext_internal.h */
static inline FFHWFramesContext *ffhwframesctx(AVHWFramesContext *ctx)                /*@ libavutil/hwcontext_internal.h */
{
    return (FFHWFramesContext*)ctx;                                                   /*@ libavutil/hwcontext_internal.h */
}

/* ---- libavutil/refstruct.h ---- */
typedef union {                                                                       /*@ libavutil/refstruct.h */
    void *nc;                                                                         /*@ libavutil/refstruct.h */
    const void *c;                                                                    /*@ libavutil/refstruct.h */
} AVRefStructOpaque;                                                                  /*@ libavutil/refstruct.h */

/* ---- libavcodec/codec_id.h, avcodec.h, internal.h, decode.h (partial contexts) ---- */
enum AVCodecID {                                                                      /*@ libavcodec/codec_id.h */
    AV_CODEC_ID_NONE,                                                                 /*@ libavcodec/codec_id.h in AVCodecID */
    AV_CODEC_ID_VP9,                                                                  /*@ libavcodec/codec_id.h in AVCodecID */
};
typedef struct AVCodecContext {                                                       /*@ libavcodec/avcodec.h */
    void *priv_data;                                                                  /*@ libavcodec/avcodec.h in AVCodecContext */
    struct AVCodecInternal *internal;                                                 /*@ libavcodec/avcodec.h in AVCodecContext */
    int coded_width, coded_height;                                                    /*@ libavcodec/avcodec.h in AVCodecContext */
    enum AVPixelFormat sw_pix_fmt;                                                    /*@ libavcodec/avcodec.h in AVCodecContext */
    AVBufferRef *hw_frames_ctx;                                                       /*@ libavcodec/avcodec.h in AVCodecContext */
    int extra_hw_frames;                                                              /*@ libavcodec/avcodec.h in AVCodecContext */
    int thread_count;                                                                 /*@ libavcodec/avcodec.h in AVCodecContext */
    int active_thread_type;                                                           /*@ libavcodec/avcodec.h in AVCodecContext */
} AVCodecContext;                                                                     /*@ libavcodec/avcodec.h */
#define FF_THREAD_FRAME 1                                                             /*@ libavcodec/avcodec.h */
typedef struct AVHWAccel {                                                            /*@ libavcodec/avcodec.h */
    const char *name;                                                                 /*@ libavcodec/avcodec.h in AVHWAccel */
    enum AVMediaType type;                                                            /*@ libavcodec/avcodec.h in AVHWAccel */
    enum AVCodecID id;                                                                /*@ libavcodec/avcodec.h in AVHWAccel */
    enum AVPixelFormat pix_fmt;                                                       /*@ libavcodec/avcodec.h in AVHWAccel */
    int capabilities;                                                                 /*@ libavcodec/avcodec.h in AVHWAccel */
} AVHWAccel;                                                                          /*@ libavcodec/avcodec.h */
typedef struct AVCodecInternal {                                                      /*@ libavcodec/internal.h */
    void *hwaccel_priv_data;                                                          /*@ libavcodec/internal.h in AVCodecInternal */
} AVCodecInternal;                                                                    /*@ libavcodec/internal.h */
int ff_decode_get_hw_frames_ctx(AVCodecContext *avctx, enum AVHWDeviceType dev_type); /*@ libavcodec/decode.h */

/* ---- libavcodec/hwaccel_internal.h (complete FFHWAccel) ---- */
#define HWACCEL_CAP_ASYNC_SAFE (1 << 0)                                               /*@ libavcodec/hwaccel_internal.h */
#define HWACCEL_CAP_THREAD_SAFE (1 << 1)                                              /*@ libavcodec/hwaccel_internal.h */
typedef struct FFHWAccel {                                                            /*@ libavcodec/hwaccel_internal.h */
    AVHWAccel p;                                                                      /*@ libavcodec/hwaccel_internal.h in FFHWAccel */
    int (*alloc_frame)(AVCodecContext *avctx, AVFrame *frame);                        /*@ libavcodec/hwaccel_internal.h in FFHWAccel */
    int (*start_frame)(AVCodecContext *avctx, const AVBufferRef *buf_ref, const uint8_t *buf, uint32_t buf_size); /*@ libavcodec/hwaccel_internal.h in FFHWAccel */
    int (*decode_params)(AVCodecContext *avctx, int type, const uint8_t *buf, uint32_t buf_size); /*@ libavcodec/hwaccel_internal.h in FFHWAccel */
    int (*decode_slice)(AVCodecContext *avctx, const uint8_t *buf, uint32_t buf_size); /*@ libavcodec/hwaccel_internal.h in FFHWAccel */
    int (*end_frame)(AVCodecContext *avctx);                                          /*@ libavcodec/hwaccel_internal.h in FFHWAccel */
    int frame_priv_data_size;                                                         /*@ libavcodec/hwaccel_internal.h in FFHWAccel */
    int priv_data_size;                                                               /*@ libavcodec/hwaccel_internal.h in FFHWAccel */
    int caps_internal;                                                                /*@ libavcodec/hwaccel_internal.h in FFHWAccel */
    int (*init)(AVCodecContext *avctx);                                               /*@ libavcodec/hwaccel_internal.h in FFHWAccel */
    int (*uninit)(AVCodecContext *avctx);                                             /*@ libavcodec/hwaccel_internal.h in FFHWAccel */
    int (*frame_params)(AVCodecContext *avctx, AVBufferRef *hw_frames_ctx);           /*@ libavcodec/hwaccel_internal.h in FFHWAccel */
    int (*update_thread_context)(AVCodecContext *dst, const AVCodecContext *src);     /*@ libavcodec/hwaccel_internal.h in FFHWAccel */
    void (*free_frame_priv)(AVRefStructOpaque hwctx, void *data);                     /*@ libavcodec/hwaccel_internal.h in FFHWAccel */
    void (*flush)(AVCodecContext *avctx);                                             /*@ libavcodec/hwaccel_internal.h in FFHWAccel */
} FFHWAccel;                                                                          /*@ libavcodec/hwaccel_internal.h */

/* ---- libavcodec/progressframe.h, vp9shared.h (partial VP9 contexts) ---- */
typedef struct ProgressFrame {                                                        /*@ libavcodec/progressframe.h */
    struct AVFrame *f;                                                                /*@ libavcodec/progressframe.h in ProgressFrame */
    struct ProgressInternal *progress;                                                /*@ libavcodec/progressframe.h in ProgressFrame */
} ProgressFrame;                                                                      /*@ libavcodec/progressframe.h */
typedef struct VP9Frame {                                                             /*@ libavcodec/vp9shared.h */
    ProgressFrame tf;                                                                 /*@ libavcodec/vp9shared.h in VP9Frame */
    void *hwaccel_picture_private;                                                    /*@ libavcodec/vp9shared.h in VP9Frame */
} VP9Frame;                                                                           /*@ libavcodec/vp9shared.h */
typedef struct VP9SharedContext {                                                     /*@ libavcodec/vp9shared.h */
#define CUR_FRAME 0                                                                   /*@ libavcodec/vp9shared.h in VP9SharedContext */
    VP9Frame frames[4];                                                               /*@ libavcodec/vp9shared.h in VP9SharedContext */
    VP9Frame ref_frames[8];                                                           /*@ libavcodec/vp9shared.h in VP9SharedContext */
} VP9SharedContext;                                                                   /*@ libavcodec/vp9shared.h */

/* ---- the registration INTEGRATION.md adds (not in FFmpeg 8.0) ---- */
#define AV_HWDEVICE_TYPE_HIP ((enum AVHWDeviceType) (AV_HWDEVICE_TYPE_CUDA + 100))
#define AV_PIX_FMT_HIP ((enum AVPixelFormat) (AV_PIX_FMT_NB + 100))

#endif
