/*
 * IVF container: the file format the reference's VP9 conformance
 * vectors ship in (tests/fate/vpx.mak: vp90-2-*.webm / *.ivf) and the one its synthetic
 * stream generator writes.
 *   probe / read_header / read_packet   libavformat/ivfdec.c:27-90
 *   write_header / write_packet         libavformat/ivfenc.c:54-88 (frame count patched at
 *                                       the trailer, 90-104)
 * Layout: a 32-byte little-endian file header ("DKIF", version 0, header size 32, fourcc,
 * width, height, time base den / num, frame count, unused), then per frame a 12-byte
 * header (size, pts) and the frame's bytes.
 */
#include <string.h>

#include "../../../include/vp9hip.h"

static uint32_t rl16(const uint8_t *p) { return (uint32_t) p[0] | (uint32_t) p[1] << 8; }
static uint32_t rl32(const uint8_t *p) { return rl16(p) | rl16(p + 2) << 16; }
static void wl16(uint8_t *p, uint32_t v) { p[0] = (uint8_t) v; p[1] = (uint8_t) (v >> 8); }
static void wl32(uint8_t *p, uint32_t v) { wl16(p, v); wl16(p + 2, v >> 16); }

/* ivfdec.c probe: "DKIF", version 0, header size 32 -> AVPROBE_SCORE_MAX - 2 */
int vp9h_ivf_probe(const uint8_t *buf, size_t size)
{
    if (!buf || size < 8) return 0;
    return (!memcmp(buf, "DKIF", 4) && !rl16(buf + 4) && rl16(buf + 6) == 32) ? 98 : 0;
}

/* ivfdec.c read_header: a zero time base numerator / denominator is invalid data */
int vp9h_ivf_read_header(const uint8_t *buf, size_t size, vp9h_ivf_header *h)
{
    if (!buf || !h) return VP9HIP_EINVAL;
    if (size < 32) return VP9HIP_EINVALIDDATA;
    memcpy(h->fourcc, buf + 8, 4);
    h->fourcc[4] = 0;
    h->width = (int32_t) rl16(buf + 12);
    h->height = (int32_t) rl16(buf + 14);
    h->time_base_den = rl32(buf + 16);
    h->time_base_num = rl32(buf + 20);
    h->nb_frames = rl32(buf + 24);
    h->header_size = rl16(buf + 6);
    if (!h->time_base_den || !h->time_base_num) return VP9HIP_EINVALIDDATA;   /* "Invalid frame rate" */
    return 0;
}

/* ivfdec.c read_packet: 32-bit size, 64-bit pts, then the data (the demuxer reads the
 * frame data from offset 32 on, whatever header size the file states). A short final
 * frame returns what is there with *truncated = 1, as av_get_packet does. */
int vp9h_ivf_read_frame(const uint8_t *buf, size_t size, size_t *pos, const uint8_t **data, uint32_t *frame_size,
                        int64_t *pts, int *truncated)
{
    if (!buf || !pos || !data || !frame_size || !pts) return VP9HIP_EINVAL;
    if (*pos < 32) *pos = 32;
    if (*pos >= size) return VP9HIP_EOF;
    if (size - *pos < 12) return VP9HIP_EOF;                /* avio_rl32 / rl64 past the end */
    const uint8_t *p = buf + *pos;
    uint32_t n = rl32(p);
    *pts = (int64_t) ((uint64_t) rl32(p + 4) | (uint64_t) rl32(p + 8) << 32);
    const size_t avail = size - *pos - 12;
    if (truncated) *truncated = n > avail;
    if (n > avail) n = (uint32_t) avail;
    *data = p + 12;
    *frame_size = n;
    *pos += 12 + (size_t) n;
    return 0;                       /* an empty frame is an empty packet (a decoder drain) */
}

/* ivfenc.c write_header (VP9: fourcc "VP90"); nb_frames is what write_trailer patches in */
int vp9h_ivf_write_header(uint8_t out[32], int width, int height, uint32_t time_base_den, uint32_t time_base_num,
                          uint32_t nb_frames)
{
    if (!out || width <= 0 || height <= 0 || width > 65535 || height > 65535) return VP9HIP_EINVAL;
    memcpy(out, "DKIF", 4);
    wl16(out + 4, 0);
    wl16(out + 6, 32);
    memcpy(out + 8, "VP90", 4);
    wl16(out + 12, (uint32_t) width);
    wl16(out + 14, (uint32_t) height);
    wl32(out + 16, time_base_den);
    wl32(out + 20, time_base_num);
    wl32(out + 24, nb_frames);
    wl32(out + 28, 0);
    return 0;
}

/* ivfenc.c write_packet: the 12-byte frame header */
void vp9h_ivf_write_frame_header(uint8_t out[12], uint32_t frame_size, int64_t pts)
{
    wl32(out, frame_size);
    wl32(out + 4, (uint32_t) (uint64_t) pts);
    wl32(out + 8, (uint32_t) ((uint64_t) pts >> 32));
}
