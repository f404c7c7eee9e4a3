/*
 * vp9hip_hwaccel.h — the FFHWAccel callbacks of a hybrid VP9 hwaccel over libvp9hip, and the
 * HIP hwcontext pieces its frames need. Plain C ABI, no FFmpeg types: the FFmpeg-side file
 * (libavcodec/vp9_hip.c) forwards each FFHWAccel / HWContextType callback
 * to one of these functions in a few lines.
 *
 * Reference interfaces each entry point stands behind:
 *   FFHWAccel (libavcodec/hwaccel_internal.h:34-166) as vp9_decode_frame calls it
 *   (libavcodec/vp9.c:1694-1713: start_frame, decode_slice, end_frame once per frame, then
 *   the reference slots are replaced by refreshrefmask, vp9.c:1705-1711);
 *   show_existing_frame is answered by vp9.c itself from s->s.ref_frames (vp9.c:1636-1653);
 *   FFHWAccel.frame_params (hwaccel_internal.h:146) fills an AVHWFramesContext;
 *   HWContextType.frames_get_buffer / transfer_data_from (libavutil/hwcontext_internal.h:73-80)
 *   for a device type next to AV_HWDEVICE_TYPE_CUDA (libavutil/hwcontext.h:26-44) whose frames
 *   carry device pointers in data[] (as AV_PIX_FMT_CUDA frames do, pixfmt.h:260).
 *
 * The adapter owns the host entropy decoder state (vp9h_stream: probability contexts,
 * segmentation, the previous frame's MVs), so decode_slice turns the frame's bytes into the
 * pass-1 packet the device path reconstructs, and the reference slots (refidx /
 * refreshrefmask, vp9shared.h:112,120) map to device frame buffers.
 */
#ifndef VP9HIP_HWACCEL_H
#define VP9HIP_HWACCEL_H
#include <stddef.h>
#include <stdint.h>

#include "vp9hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* The pixel format of a device frame's data (sw_format of the frames context):
 * AV_PIX_FMT_YUV420P / YUV422P / YUV440P / YUV444P at 8 bits, the P10 / P12 forms above. */
enum {
    VP9HIP_SWFMT_YUV420P, VP9HIP_SWFMT_YUV422P, VP9HIP_SWFMT_YUV440P, VP9HIP_SWFMT_YUV444P,
    VP9HIP_SWFMT_YUV420P10, VP9HIP_SWFMT_YUV422P10, VP9HIP_SWFMT_YUV440P10, VP9HIP_SWFMT_YUV444P10,
    VP9HIP_SWFMT_YUV420P12, VP9HIP_SWFMT_YUV422P12, VP9HIP_SWFMT_YUV440P12, VP9HIP_SWFMT_YUV444P12,
};

/* FFHWAccel.frame_params: what the AVHWFramesContext of the stream's frames gets
 * (format = the HIP hw pix_fmt, sw_format, width, height, initial_pool_size). */
/* async_depth = the largest power of two <= extra / 2 (the consumer's frame delay: FFmpeg
 * passes its frame threads and extra_hw_frames as `extra`), at most
 * VP9HIP_HWACCEL_ASYNC_DEPTH: a consumer that reads a frame `extra` frames after the decoder
 * finds its batch launched and parsed. Measured C3 (realistic density, lag 16, extra 18):
 * depth 8 1,210 fps, 4 1,100, 9 830, 16 910 (profiles/r03i). */
#define VP9HIP_HWACCEL_ASYNC_DEPTH 16
/* Filled batches that may wait for their entropy decode before the oldest is launched
 * anyway: the parse look-ahead is (1 + VP9HIP_HWACCEL_AHEAD) x async_depth frames, so that
 * several GOP chains (whose frames parse one after another) parse at once. */
#define VP9HIP_HWACCEL_AHEAD 4
typedef struct vp9hip_frames_params {
    int32_t sw_format;             /* VP9HIP_SWFMT_*                                         */
    int32_t width, height;         /* coded size                                             */
    int32_t initial_pool_size;     /* 8 reference slots + the frame being decoded +          */
                                   /* (1 + VP9HIP_HWACCEL_AHEAD) x async_depth + extra       */
    int32_t bpp, ss_h, ss_v;
    /* set by frame_params, adjustable before init (the FFmpeg glue maps its options here): */
    int32_t async_depth;           /* frames per device launch (see above);                  */
                                   /* 1 = each frame launched by its end_frame               */
    int32_t parse_threads;         /* host entropy-decode threads (0: in decode_slice)       */
} vp9hip_frames_params;
int vp9hip_hwaccel_frame_params(int width, int height, int bpp, int ss_h, int ss_v, int extra,
                                vp9hip_frames_params *out);

/* A device frame (the AVFrame of a HIP frames context): data[] are device pointers with
 * byte pitches, valid until vp9hip_hwframe_unref; consumers order their reads after the
 * frame's batch with vp9hip_hwframe_ready (GPU) or vp9hip_hwframe_sync (host). `stream` is
 * the context's stream at hand-out, informational. */
typedef struct vp9hip_hwframe {
    void     *data[3];
    ptrdiff_t linesize[3];
    int32_t   width, height;
    int32_t   sw_format;
    int32_t   buf;                 /* pool buffer (the AVBufferRef of the frame)             */
    int64_t   pts;
    void     *stream;
} vp9hip_hwframe;

typedef struct vp9hip_hwaccel vp9hip_hwaccel;    /* hwaccel_priv_data (VP9HIPContext) */

/* FFHWAccel.init: open the device, size its frame pool from frame_params. */
int  vp9hip_hwaccel_init(int device, const vp9hip_frames_params *fp, vp9hip_hwaccel **out);
/* FFHWAccel.uninit */
int  vp9hip_hwaccel_uninit(vp9hip_hwaccel *h);
/* FFHWAccel.start_frame(avctx, buf_ref, buf, size): the whole frame's bytes (one frame of
 * a split superframe, not show_existing_frame). */
int  vp9hip_hwaccel_start_frame(vp9hip_hwaccel *h, const uint8_t *buf, uint32_t size, int64_t pts);
/* FFHWAccel.decode_slice(avctx, buf, size): the header's slot bookkeeping (vp9h_frame_peek)
 * now; the host entropy decode of the frame (all its tiles) into the pass-1 packet
 * (vp9h_stream_decode) queued on the parse threads. */
int  vp9hip_hwaccel_decode_slice(vp9hip_hwaccel *h, const uint8_t *buf, uint32_t size);
/* FFHWAccel.end_frame: queue the frame's reconstruction on the device (its LAST / GOLDEN /
 * ALTREF are the device buffers of slots refidx[]) and replace the slots of
 * refreshrefmask. Asynchronous (HWACCEL_CAP_ASYNC_SAFE): frames are launched in batches
 * of async_depth, and nothing here waits for the GPU. *out (may be NULL) is the frame,
 * shown or hidden: the device frame behind vp9.c's AVFrame of this VP9Frame, referenced
 * until vp9hip_hwframe_unref (the AVBufferRef's free callback). Its pixels are complete
 * after vp9hip_hwframe_sync / vp9hip_hwframe_ready. Returns 1 if shown, 0 if hidden, or an
 * error (also one of an earlier frame's batch launched by this call). */
int  vp9hip_hwaccel_end_frame(vp9hip_hwaccel *h, vp9hip_hwframe *out);
/* vp9.c:1636-1653 show_existing_frame: the frame of reference slot `slot`, referenced. */
int  vp9hip_hwaccel_show_existing(vp9hip_hwaccel *h, int slot, int64_t pts, vp9hip_hwframe *out);
/* FFHWAccel.flush: launch what is queued (frames handed out stay valid), drop the
 * reference slots; the next frame must be a keyframe. */
void vp9hip_hwaccel_flush(vp9hip_hwaccel *h);
/* The header fields the adapter read in the last decode_slice (vp9h_frame_peek:
 * s->s.h.refidx / refreshrefmask / show_frame, vp9shared.h:112,120). */
int  vp9hip_hwaccel_last_header(const vp9hip_hwaccel *h, vp9h_frame_info *info);

/* Host wait for a frame's pixels (launching its batch if it is still being filled), with
 * its batch's checks: VP9HIP_EBUG if the loop filter's row hand-off gave up, or the error
 * of the frame's entropy decode. The hwcontext's frame sync. */
int  vp9hip_hwframe_sync(vp9hip_hwaccel *h, const vp9hip_hwframe *f);
/* Order HIP stream `stream` (a hipStream_t) after a frame's pixels without a host wait
 * (launching its batch if needed): a GPU consumer's wait. The batch's hand-off check runs
 * at the next host wait on it. */
int  vp9hip_hwframe_ready(vp9hip_hwaccel *h, const vp9hip_hwframe *f, void *stream);
/* HWContextType.transfer_data_from: device frame -> host planes (visible size); syncs. */
int  vp9hip_hwframe_transfer(vp9hip_hwaccel *h, const vp9hip_hwframe *src, uint8_t *const dst[3],
                             const ptrdiff_t dst_linesize[3]);
/* av_frame_ref of a device frame (av_buffer_ref of its AVBufferRef): *dst is another
 * reference to src's pool buffer. */
int  vp9hip_hwframe_ref(vp9hip_hwaccel *h, const vp9hip_hwframe *src, vp9hip_hwframe *dst);
/* av_frame_unref of a device frame: its pool buffer is free once no reference and no slot
 * holds it. */
int  vp9hip_hwframe_unref(vp9hip_hwaccel *h, vp9hip_hwframe *f);

#ifdef __cplusplus
}
#endif
#endif
