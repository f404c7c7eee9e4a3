/*
 * FFHWAccel call-order harness for libvp9hip (tests/test_hwaccel_harness.py runs it on the GPU).
 *
 * Plays the part of libavcodec's VP9 decoder around the hwaccel, in the reference order:
 *   get_format -> FFHWAccel.frame_params + init           (decode.c:1153-1200, hwaccel_internal.h:146)
 *   per packet: the superframe split BSF                  (vp9.c:1977, vp9_superframe_split.c:40-95)
 *   per frame: show_existing_frame answered from the slots (vp9.c:1636-1653)
 *              else start_frame, decode_slice, end_frame  (vp9.c:1694-1713)
 *   shown frames: av_hwframe_transfer_data + av_frame_unref (hwcontext_internal.h:79)
 *   avcodec_flush_buffers -> FFHWAccel.flush, then the stream again from its first packet
 *   avcodec_free_context -> FFHWAccel.uninit
 * Output: the visible planes of every output frame, in output order, appended to OUT.
 *
 * usage: hwaccel_harness IN.ivf OUT.yuv BPP SS_H SS_V [PASSES]
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

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

static int emit(vp9hip_hwaccel *h, vp9hip_hwframe *f, int bpp, int ssh, int ssv, FILE *out)
{
    const int by = bpp > 8 ? 2 : 1, w = f->width, ht = f->height;
    const int cw = (w + ssh) >> ssh, chh = (ht + ssv) >> ssv;
    uint8_t *pl[3];
    ptrdiff_t ls[3] = { (ptrdiff_t) w * by, (ptrdiff_t) cw * by, (ptrdiff_t) cw * by };
    pl[0] = malloc((size_t) ls[0] * ht);
    pl[1] = malloc((size_t) ls[1] * chh);
    pl[2] = malloc((size_t) ls[2] * chh);
    int r = vp9hip_hwframe_transfer(h, f, pl, ls);                 /* transfer_data_from */
    if (r >= 0) {
        fwrite(pl[0], 1, (size_t) ls[0] * ht, out);
        fwrite(pl[1], 1, (size_t) ls[1] * chh, out);
        fwrite(pl[2], 1, (size_t) ls[2] * chh, out);
        r = vp9hip_hwframe_unref(h, f);                              /* av_frame_unref */
    }
    free(pl[0]); free(pl[1]); free(pl[2]);
    return r;
}

int main(int argc, char **argv)
{
    if (argc < 6) { fprintf(stderr, "usage: %s IN.ivf OUT.yuv BPP SS_H SS_V [PASSES]\n", argv[0]); return 2; }
    const int bpp = atoi(argv[3]), ssh = atoi(argv[4]), ssv = atoi(argv[5]), passes = argc > 6 ? atoi(argv[6]) : 2;
    FILE *fi = fopen(argv[1], "rb");
    if (!fi) { perror(argv[1]); return 2; }
    fseek(fi, 0, SEEK_END);
    const long n = ftell(fi);
    fseek(fi, 0, SEEK_SET);
    uint8_t *buf = malloc((size_t) n);
    if (fread(buf, 1, (size_t) n, fi) != (size_t) n) { fclose(fi); return 2; }
    fclose(fi);
    FILE *out = fopen(argv[2], "wb");
    if (!out) { perror(argv[2]); return 2; }

    vp9h_ivf_header ih;
    int r = vp9h_ivf_read_header(buf, (size_t) n, &ih);
    if (r < 0) { fprintf(stderr, "ivf header: %d\n", r); return 1; }
    /* get_format: frame_params then init */
    vp9hip_frames_params fp;
    vp9hip_hwaccel *h = NULL;
    if ((r = vp9hip_hwaccel_frame_params(ih.width, ih.height, bpp, ssh, ssv, 2, &fp)) < 0 ||
        (r = vp9hip_hwaccel_init(0, &fp, &h)) < 0) {
        fprintf(stderr, "init: %d\n", r);
        return 1;
    }
    int frames_out = 0;
    for (int pass = 0; pass < passes && r >= 0; pass++) {
        if (pass) vp9hip_hwaccel_flush(h);                         /* avcodec_flush_buffers */
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
                vp9hip_hwframe f;
                const int ex = show_existing_slot(d, sizes[k]);
                if (ex >= 0) {
                    r = vp9hip_hwaccel_show_existing(h, ex, pts, &f);
                    if (r >= 0) { r = emit(h, &f, bpp, ssh, ssv, out); frames_out++; }
                    continue;
                }
                if ((r = vp9hip_hwaccel_start_frame(h, d, (uint32_t) sizes[k], pts)) < 0) break;
                if ((r = vp9hip_hwaccel_decode_slice(h, d, (uint32_t) sizes[k])) < 0) break;
                if ((r = vp9hip_hwaccel_end_frame(h, &f)) < 0) break;
                if (r == 1) { r = emit(h, &f, bpp, ssh, ssv, out); frames_out++; }
            }
        }
    }
    vp9hip_hwaccel_uninit(h);
    fclose(out);
    free(buf);
    if (r < 0) { fprintf(stderr, "decode: %d after %d frames\n", r, frames_out); return 1; }
    printf("frames %d\n", frames_out);
    return 0;
}
