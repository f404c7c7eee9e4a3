/*
 * FFHWAccel call-order harness for libvp9hip (tests/test_hwaccel_harness.py runs it on the GPU;
 * bench.py times it as the `hwaccel_path` field).
 *
 * Plays the part of libavcodec's VP9 decoder around the hwaccel, in the reference order:
 *   get_format -> FFHWAccel.frame_params + init           (decode.c:1153-1200, hwaccel_internal.h:146)
 *   per packet: the superframe split BSF                  (vp9.c:1977, vp9_superframe_split.c:40-95)
 *   per frame: show_existing_frame answered from the slots (vp9.c:1636-1653)
 *              else start_frame, decode_slice, end_frame  (vp9.c:1694-1713)
 *   output frames: av_hwframe_transfer_data + av_frame_unref (hwcontext_internal.h:79)
 *   avcodec_flush_buffers -> FFHWAccel.flush, then the stream again from its first packet
 *   avcodec_free_context -> FFHWAccel.uninit
 * Frame ownership follows FFmpeg's: every decoded frame (shown or hidden) is an AVFrame whose
 * buffer reference comes from end_frame; vp9.c keeps it as s->s.frames[CUR_FRAME] until the
 * next frame and as a reference in s->s.ref_frames[] for each slot of its refresh mask
 * (vp9.c:1686-1691, 1845-1849); an output frame is one more reference (av_frame_ref), which
 * the consumer drops after reading it. Every drop is vp9hip_hwframe_unref (the
 * AVBufferRef's free callback).
 *
 * The consumer reads output frames LAG frames behind the decoder (FFmpeg's frame-threading
 * delay; 0 = each frame as soon as end_frame returns it). MODE: "download" transfers each
 * output frame to host planes (appended to OUT unless OUT is "-"); "device" only waits for
 * its pixels on the GPU (vp9hip_hwframe_sync), as a consumer of device frames does;
 * "thread" downloads on a consumer thread of its own, as a user thread of FFmpeg does while
 * the decoder keeps calling the hwaccel (at most max(LAG, 1) frames queued to it; a full pool
 * makes start_frame answer EAGAIN until the consumer releases frames).
 * Prints "frames N seconds S" (wall time of the decode loop, init / uninit excluded).
 *
 * EXTRA (default 2 + LAG) is the frame count the FFmpeg glue hands frame_params
 * (integration/vp9_hip.c: max(0, extra_hw_frames) + frame threads); -1 plays a glue that passes
 * FFmpeg's default extra_hw_frames (-1, options_table.h:397) through unclamped.
 *
 * usage: hwaccel_harness IN.ivf OUT.yuv|- BPP SS_H SS_V [PASSES [LAG [MODE [ASYNC_DEPTH [EXTRA]]]]]
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "../../include/vp9hip_hwaccel.h"

/* The first header bits (vp9.c decode_frame_header:497-515): frame marker, profile,
 * show_existing_frame, frame_to_show_map_idx. Returns the slot, or -1 if not a
 * show_existing_frame header. */
static int getbit(const uint8_t *d, size_t n, size_t *bit)
{
    const size_t b = (*bit)++;
    return b < 8 * n ? (d[b >> 3] >> (7 - (b & 7))) & 1 : 0;
}

static int show_existing_slot(const uint8_t *d, size_t n)
{
    size_t bit = 0;
    const int marker = getbit(d, n, &bit) << 1;
    if ((marker | getbit(d, n, &bit)) != 2) return -1;
    int prof = getbit(d, n, &bit);
    prof |= getbit(d, n, &bit) << 1;
    if (prof == 3) getbit(d, n, &bit);                     /* reserved zero */
    if (!getbit(d, n, &bit)) return -1;                    /* show_existing_frame */
    int s = 0;
    for (int i = 0; i < 3; i++) s = (s << 1) | getbit(d, n, &bit);
    return s;
}

typedef struct Consumer {
    vp9hip_hwaccel *h;
    int bpp, ssh, ssv, download, lag;
    FILE *out;
    vp9hip_hwframe q[512];             /* output frames not read yet (av_frame_ref'd) */
    int head, n;
    int frames_out;
    /* frames whose read failed (transfer / sync: the frame's own decode error, as
     * av_hwframe_transfer_data reports it for that frame); the decode goes on */
    int nfailed, failed_idx[1024], failed_err[1024];
    /* MODE "thread": the queue is shared with the consumer thread */
    int threaded, busy, stop, err;
    pthread_t th;
    pthread_mutex_t mu;
    pthread_cond_t cv;
} Consumer;

static int consume_one(Consumer *c)
{
    vp9hip_hwframe *f = &c->q[c->head];      /* MODE thread: only the consumer moves head */
    int r;
    if (c->download) {
        const int by = c->bpp > 8 ? 2 : 1, w = f->width, ht = f->height;
        const int cw = (w + c->ssh) >> c->ssh, chh = (ht + c->ssv) >> c->ssv;
        uint8_t *pl[3];
        ptrdiff_t ls[3] = { (ptrdiff_t) w * by, (ptrdiff_t) cw * by, (ptrdiff_t) cw * by };
        pl[0] = malloc((size_t) ls[0] * ht);
        pl[1] = malloc((size_t) ls[1] * chh);
        pl[2] = malloc((size_t) ls[2] * chh);
        r = vp9hip_hwframe_transfer(c->h, f, pl, ls);               /* transfer_data_from */
        if (r < 0 && c->out) {           /* a failed frame keeps its place in the output: zeros */
            memset(pl[0], 0, (size_t) ls[0] * ht);
            memset(pl[1], 0, (size_t) ls[1] * chh);
            memset(pl[2], 0, (size_t) ls[2] * chh);
        }
        if ((r >= 0 || r == VP9HIP_EINVALIDDATA || r == VP9HIP_EBUG) && c->out) {
            fwrite(pl[0], 1, (size_t) ls[0] * ht, c->out);
            fwrite(pl[1], 1, (size_t) ls[1] * chh, c->out);
            fwrite(pl[2], 1, (size_t) ls[2] * chh, c->out);
        }
        free(pl[0]); free(pl[1]); free(pl[2]);
    } else {
        r = vp9hip_hwframe_sync(c->h, f);                            /* the frame's pixels are final */
    }
    const int u = vp9hip_hwframe_unref(c->h, f);                     /* av_frame_unref */
    if (r == VP9HIP_EINVALIDDATA || r == VP9HIP_EBUG) {               /* this frame's error */
        if (c->nfailed < 1024) {
            c->failed_idx[c->nfailed] = c->frames_out;
            c->failed_err[c->nfailed] = r;
        }
        c->nfailed++;
        r = 0;
    }
    if (c->threaded) pthread_mutex_lock(&c->mu);
    c->head = (c->head + 1) % 512;
    c->n--;
    c->frames_out++;
    if (c->threaded) pthread_mutex_unlock(&c->mu);
    return r < 0 ? r : u;
}

/* the consumer thread: reads queued frames in order until stopped with an empty queue */
static void *consumer_main(void *arg)
{
    Consumer *c = arg;
    pthread_mutex_lock(&c->mu);
    for (;;) {
        while (!c->n && !c->stop) pthread_cond_wait(&c->cv, &c->mu);
        if (!c->n) break;
        c->busy = 1;
        pthread_mutex_unlock(&c->mu);
        const int r = consume_one(c);  /* the queue head is the consumer's: n > 0 */
        pthread_mutex_lock(&c->mu);
        c->busy = 0;
        if (r < 0 && !c->err) c->err = r;
        pthread_cond_broadcast(&c->cv);
    }
    pthread_mutex_unlock(&c->mu);
    return NULL;
}

/* av_frame_ref of an output frame into the consumer's queue; reads the frames more than
 * LAG behind */
static int output(Consumer *c, const vp9hip_hwframe *f)
{
    if (c->threaded) {
        const int cap = c->lag > 0 ? c->lag : 1;
        int r = 0;
        pthread_mutex_lock(&c->mu);
        while (c->n >= cap && !c->err) pthread_cond_wait(&c->cv, &c->mu);
        if (c->err) r = c->err;
        else if ((r = vp9hip_hwframe_ref(c->h, f, &c->q[(c->head + c->n) % 512])) >= 0) c->n++;
        pthread_cond_broadcast(&c->cv);
        pthread_mutex_unlock(&c->mu);
        return r;
    }
    if (c->n == 512) return -1;
    vp9hip_hwframe *d = &c->q[(c->head + c->n) % 512];
    int r = vp9hip_hwframe_ref(c->h, f, d);
    if (r < 0) return r;
    c->n++;
    while (c->n > c->lag && r >= 0) r = consume_one(c);
    return r;
}

static int drain(Consumer *c)
{
    if (c->threaded) {                 /* wait until the consumer thread has read everything */
        pthread_mutex_lock(&c->mu);
        while ((c->n || c->busy) && !c->err) pthread_cond_wait(&c->cv, &c->mu);
        const int r = c->err;
        pthread_mutex_unlock(&c->mu);
        return r;
    }
    int r = 0;
    while (c->n && r >= 0) r = consume_one(c);
    return r;
}

int main(int argc, char **argv)
{
    if (argc < 6) {
        fprintf(stderr, "usage: %s IN.ivf OUT.yuv|- BPP SS_H SS_V [PASSES [LAG [MODE [ASYNC_DEPTH [EXTRA [REJECT,SPIN]]]]]]\n", argv[0]);
        return 2;
    }
    const int bpp = atoi(argv[3]), ssh = atoi(argv[4]), ssv = atoi(argv[5]), passes = argc > 6 ? atoi(argv[6]) : 2;
    const int lag = argc > 7 ? atoi(argv[7]) : 0;
    const int download = argc > 8 ? strcmp(argv[8], "device") != 0 : 1;
    const int threaded = argc > 8 && !strcmp(argv[8], "thread");
    const int depth = argc > 9 ? atoi(argv[9]) : 0;
    const int extra = argc > 10 ? atoi(argv[10]) : 2 + lag;
    if (argc > 11) {                     /* test hooks: reject a frame of the k-th batch, row-LF spin bound */
        char *e = NULL;
        const int reject = (int) strtol(argv[11], &e, 0);
        vp9hip_test_hooks(reject, e && *e == ',' ? (uint32_t) strtoul(e + 1, NULL, 0) : 0u);
    }
    FILE *fi = fopen(argv[1], "rb");
    if (!fi) { perror(argv[1]); return 2; }
    fseek(fi, 0, SEEK_END);
    const long n = ftell(fi);
    fseek(fi, 0, SEEK_SET);
    uint8_t *buf = malloc((size_t) n);
    if (fread(buf, 1, (size_t) n, fi) != (size_t) n) { fclose(fi); return 2; }
    fclose(fi);
    FILE *out = NULL;
    if (strcmp(argv[2], "-") && !(out = fopen(argv[2], "wb"))) { perror(argv[2]); return 2; }

    vp9h_ivf_header ih;
    int r = vp9h_ivf_read_header(buf, (size_t) n, &ih);
    if (r < 0) { fprintf(stderr, "ivf header: %d\n", r); return 1; }
    /* get_format: frame_params (+ the options the glue maps onto it) then init */
    vp9hip_frames_params fp;
    vp9hip_hwaccel *h = NULL;
    if ((r = vp9hip_hwaccel_frame_params(ih.width, ih.height, bpp, ssh, ssv, extra, &fp)) < 0) {
        fprintf(stderr, "frame_params: %d\n", r);
        return 1;
    }
    if (depth > 0) {
        fp.initial_pool_size += (1 + VP9HIP_HWACCEL_AHEAD) * (depth - fp.async_depth);
        fp.async_depth = depth;
    }
    if ((r = vp9hip_hwaccel_init(0, &fp, &h)) < 0) {
        fprintf(stderr, "init: %d\n", r);
        return 1;
    }
    static Consumer c;
    c.h = h; c.bpp = bpp; c.ssh = ssh; c.ssv = ssv; c.download = download; c.lag = lag; c.out = out;
    c.threaded = threaded;
    if (threaded) {
        pthread_mutex_init(&c.mu, NULL);
        pthread_cond_init(&c.cv, NULL);
        pthread_create(&c.th, NULL, consumer_main, &c);
    }
    vp9hip_hwframe slots[8], cur;                  /* s->s.ref_frames[], s->s.frames[CUR_FRAME] */
    int have_slot[8] = { 0 }, have_cur = 0;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int pass = 0; pass < passes && r >= 0; pass++) {
        if (pass) {                                                 /* avcodec_flush_buffers */
            if ((r = drain(&c)) < 0) break;
            vp9hip_hwaccel_flush(h);
            for (int s = 0; s < 8; s++)
                if (have_slot[s]) { vp9hip_hwframe_unref(h, &slots[s]); have_slot[s] = 0; }
            if (have_cur) { vp9hip_hwframe_unref(h, &cur); have_cur = 0; }
        }
        size_t pos = ih.header_size;
        const uint8_t *pkt;
        uint32_t psz;
        int64_t pts;
        int trunc;
        while (r >= 0 && vp9h_ivf_read_frame(buf, (size_t) n, &pos, &pkt, &psz, &pts, &trunc) == 0) {
            size_t offs[8], sizes[8];
            const int nf = vp9h_superframe_split(pkt, psz, offs, sizes, 8);
            if (nf < 0) { r = nf; break; }
            for (int k = 0; k < nf && r >= 0; k++) {
                const uint8_t *d = pkt + offs[k];
                const int ex = show_existing_slot(d, sizes[k]);
                if (ex >= 0) {
                    vp9hip_hwframe f;
                    r = vp9hip_hwaccel_show_existing(h, ex, pts, &f);
                    if (r >= 0) {
                        r = output(&c, &f);
                        vp9hip_hwframe_unref(h, &f);
                    }
                    continue;
                }
                if (have_cur) { vp9hip_hwframe_unref(h, &cur); have_cur = 0; }   /* vp9_frame_unref(CUR_FRAME) */
                /* a full pool (the consumer thread still holds frames): wait for releases */
                for (int tries = 0; (r = vp9hip_hwaccel_start_frame(h, d, (uint32_t) sizes[k], pts)) == VP9HIP_EAGAIN &&
                                    threaded && tries < 200000; tries++)
                    usleep(50);
                if (r < 0) break;
                if ((r = vp9hip_hwaccel_decode_slice(h, d, (uint32_t) sizes[k])) < 0) break;
                if ((r = vp9hip_hwaccel_end_frame(h, &cur)) < 0) break;
                have_cur = 1;
                const int shown = r;
                vp9h_frame_info info;
                vp9hip_hwaccel_last_header(h, &info);
                for (int s = 0; s < 8 && r >= 0; s++)                 /* s->s.ref_frames[] by refreshrefmask */
                    if (info.refresh_mask & (1 << s)) {
                        if (have_slot[s]) vp9hip_hwframe_unref(h, &slots[s]);
                        r = vp9hip_hwframe_ref(h, &cur, &slots[s]);
                        have_slot[s] = r >= 0;
                    }
                if (r >= 0 && shown) r = output(&c, &cur);
            }
        }
    }
    if (r >= 0) r = drain(&c);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (threaded) {
        pthread_mutex_lock(&c.mu);
        c.stop = 1;
        pthread_cond_broadcast(&c.cv);
        pthread_mutex_unlock(&c.mu);
        pthread_join(c.th, NULL);
        if (r >= 0 && c.err < 0) r = c.err;
    }
    for (int s = 0; s < 8; s++)
        if (have_slot[s]) vp9hip_hwframe_unref(h, &slots[s]);
    if (have_cur) vp9hip_hwframe_unref(h, &cur);
    vp9hip_hwaccel_uninit(h);
    if (out) fclose(out);
    free(buf);
    if (r < 0) { fprintf(stderr, "decode: %d after %d frames\n", r, c.frames_out); return 1; }
    printf("frames %d seconds %.6f\n", c.frames_out, (double) (t1.tv_sec - t0.tv_sec) + 1e-9 * (double) (t1.tv_nsec - t0.tv_nsec));
    if (c.nfailed) {                     /* rc 3: every other frame was read; these failed */
        fprintf(stderr, "failed frames:");
        for (int i = 0; i < c.nfailed && i < 1024; i++) fprintf(stderr, " %d:%d", c.failed_idx[i], c.failed_err[i]);
        fprintf(stderr, "\n");
        return 3;
    }
    return 0;
}
