/*
 * The HIP hardware context: libavutil/hwcontext_hip.h in an FFmpeg tree (new file).
 *
 * AV_HWDEVICE_TYPE_HIP / AV_PIX_FMT_HIP beside AV_HWDEVICE_TYPE_CUDA / AV_PIX_FMT_CUDA
 * (libavutil/hwcontext.h:26-44, pixfmt.h). An AV_PIX_FMT_HIP frame holds device pointers in
 * data[0..2] (one per plane, pitched) and, in data[3], either NULL (a frame of the frames
 * pool: plain device memory) or an AVHIPFrameSource (a frame a producer such as the vp9_hip
 * hwaccel still owns: its pixels are final only after the producer says so).
 *
 * Not compiled in this repository (it needs an FFmpeg tree); see INTEGRATION.md.
 */
#ifndef AVUTIL_HWCONTEXT_HIP_H
#define AVUTIL_HWCONTEXT_HIP_H

#include <stddef.h>
#include <stdint.h>

/* AVHWDeviceContext.hwctx */
typedef struct AVHIPDeviceContext {
    int device;              /* HIP device ordinal */
    void *stream;            /* hipStream_t the context's copies run on (created at device_create) */
} AVHIPDeviceContext;

/* data[3] of a producer-owned AV_PIX_FMT_HIP frame. The hwcontext never touches the planes
 * of such a frame before `sync` (device consumers) or instead of `transfer` (host copies):
 *   sync(opaque, stream):      order `stream` after the frame's producing work (no host wait);
 *                              0 or a negative AVERROR (the frame failed on the device)
 *   transfer(opaque, dst, ls): wait for the frame, check it, copy its visible planes to host
 *                              memory; 0 or a negative AVERROR */
typedef struct AVHIPFrameSource {
    int (*sync)(void *opaque, void *stream);
    int (*transfer)(void *opaque, uint8_t *const dst[3], const ptrdiff_t dst_linesize[3]);
    void *opaque;
} AVHIPFrameSource;

/* Order `stream` (a hipStream_t) after a HIP frame's producer: what a device consumer (a
 * filter, an encoder, a torch tensor view) calls before reading data[0..2]. */
int av_hip_frame_sync(const struct AVFrame *frame, void *stream);

#endif /* AVUTIL_HWCONTEXT_HIP_H */
