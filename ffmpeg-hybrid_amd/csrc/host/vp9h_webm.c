/*
 * WebM / Matroska demuxing of a VP9 video track: the container of the
 * reference's VP9 conformance vectors (tests/fate/vpx.mak:98-104 read *.webm).
 *
 * Restates what libavformat/matroskadec.c does for one VP9 track, over a buffer:
 *   - EBML numbers: the first byte's leading zeros give the length (1..8), the marker bit is
 *     dropped for sizes and kept for IDs; an all-ones size is "unknown length"
 *     (ebml_read_num / ebml_read_length, matroskadec.c:913-985);
 *   - probe: the EBML header ID and a "matroska" / "webm" DocType inside the header
 *     (matroska_probe, matroskadec.c:1614-1660);
 *   - header: EBML header checks (EBMLReadVersion <= 1, EBMLMaxIDLength <= 4,
 *     EBMLMaxSizeLength <= 8, DocTypeReadVersion <= 3), then the Segment's Info
 *     (TimecodeScale, default 1000000 ns) and Tracks (the first video TrackEntry with
 *     CodecID V_VP9: TrackNumber, PixelWidth / PixelHeight), up to the first Cluster
 *     (matroska_read_header, matroskadec.c:3303-3490);
 *   - clusters of known or unknown size (an unknown-size element ends at the first ID of
 *     its parent's level), Cluster Timecode, SimpleBlock and BlockGroup / Block (+
 *     BlockDuration); blocks of other tracks are skipped (matroska_parse_cluster /
 *     matroska_parse_block, matroskadec.c:4093-4300);
 *   - lacing: none, Xiph, fixed-size, EBML (matroska_parse_laces, matroskadec.c:3491-3580);
 *     every lace is one packet; a laced block's later laces get pts + i * duration / laces
 *     when the block has a duration, else no pts;
 *   - pts = cluster timecode + the block's signed 16-bit relative timecode, in
 *     TimecodeScale units.
 * Void, CRC-32, SeekHead, Cues, Tags, Chapters, Attachments are skipped.
 */
#include <stdint.h>
#include <string.h>

#include "../../../include/vp9hip.h"

#define ID_EBML           0x1A45DFA3u
#define ID_EBMLREADVER    0x42F7u
#define ID_EBMLMAXIDLEN   0x42F2u
#define ID_EBMLMAXSIZELEN 0x42F3u
#define ID_DOCTYPE        0x4282u
#define ID_DOCTYPEREADVER 0x4285u
#define ID_SEGMENT        0x18538067u
#define ID_INFO           0x1549A966u
#define ID_TIMECODESCALE  0x2AD7B1u
#define ID_TRACKS         0x1654AE6Bu
#define ID_TRACKENTRY     0xAEu
#define ID_TRACKNUMBER    0xD7u
#define ID_TRACKTYPE      0x83u
#define ID_CODECID        0x86u
#define ID_VIDEO          0xE0u
#define ID_PIXELWIDTH     0xB0u
#define ID_PIXELHEIGHT    0xBAu
#define ID_CLUSTER        0x1F43B675u
#define ID_CLUSTERTC      0xE7u
#define ID_SIMPLEBLOCK    0xA3u
#define ID_BLOCKGROUP     0xA0u
#define ID_BLOCK          0xA1u
#define ID_BLOCKDURATION  0x9Bu
#define ID_CUES           0x1C53BB6Bu
#define ID_TAGS           0x1254C367u
#define ID_CHAPTERS       0x1043A770u
#define ID_ATTACHMENTS    0x1941A469u
#define ID_SEEKHEAD       0x114D9B74u

#define UNKNOWN UINT64_MAX

/* ebml_read_num: length from the first byte's leading zeros; keep_marker for IDs */
static int rd_num(const uint8_t *b, size_t size, uint64_t pos, int max_len, int keep_marker, uint64_t *out)
{
    if (pos >= size) return VP9HIP_EOF;
    const uint8_t first = b[pos];
    if (!first) return VP9HIP_EINVALIDDATA;
    int len = 1;
    while (!(first & (0x80 >> (len - 1)))) len++;
    if (len > max_len) return VP9HIP_EINVALIDDATA;
    if (pos + (uint64_t) len > size) return VP9HIP_EINVALIDDATA;
    uint64_t v = keep_marker ? first : (uint64_t) (first & ((0x80 >> (len - 1)) - 1));
    for (int i = 1; i < len; i++) v = v << 8 | b[pos + i];
    *out = v;
    return len;
}

/* an element header: ID (1..4 bytes, marker kept) and size (unknown length -> UNKNOWN) */
typedef struct { uint32_t id; uint64_t size, data; } Elem;
static int rd_elem(const uint8_t *b, size_t size, uint64_t pos, Elem *e)
{
    uint64_t id, len;
    int n = rd_num(b, size, pos, 4, 1, &id);
    if (n < 0) return n;
    int m = rd_num(b, size, pos + n, 8, 0, &len);
    if (m < 0) return m == VP9HIP_EOF ? VP9HIP_EINVALIDDATA : m;
    if (len + 1 == 1ull << (7 * m)) len = UNKNOWN;          /* ebml_read_length */
    e->id = (uint32_t) id;
    e->size = len;
    e->data = pos + n + m;
    if (len != UNKNOWN && (e->data > size || len > size - e->data)) return VP9HIP_EINVALIDDATA;
    return 0;
}

static uint64_t rd_uint(const uint8_t *b, const Elem *e)
{
    uint64_t v = 0;
    for (uint64_t i = 0; i < e->size && i < 8; i++) v = v << 8 | b[e->data + i];
    return v;
}

/* level-1 elements of a Segment: where an unknown-size Cluster ends */
static int is_level1(uint32_t id)
{
    return id == ID_CLUSTER || id == ID_CUES || id == ID_TAGS || id == ID_CHAPTERS || id == ID_ATTACHMENTS ||
           id == ID_SEEKHEAD || id == ID_INFO || id == ID_TRACKS;
}

int vp9h_webm_probe(const uint8_t *buf, size_t size)
{
    if (!buf || size < 5) return 0;
    if (!(buf[0] == 0x1A && buf[1] == 0x45 && buf[2] == 0xDF && buf[3] == 0xA3)) return 0;   /* EBML_ID_HEADER */
    uint64_t len;
    int m = rd_num(buf, size, 4, 8, 0, &len);
    if (m < 0) return 0;
    uint64_t end;
    if (len + 1 == 1ull << (7 * m)) end = size;             /* unknown-length header: the whole buffer */
    else if (4 + m + len > size) return 0;                  /* the probe data must hold the header */
    else end = 4 + m + len;
    static const char *docs[] = { "matroska", "webm" };
    for (int d = 0; d < 2; d++) {
        const size_t L = strlen(docs[d]);
        for (uint64_t i = 4 + m; i + L <= end; i++)
            if (!memcmp(buf + i, docs[d], L)) return 100;   /* AVPROBE_SCORE_MAX */
    }
    return 50;                                              /* EBML, unknown doctype */
}

static int parse_ebml_header(const uint8_t *b, size_t size, const Elem *h, vp9h_webm_info *info)
{
    uint64_t p = h->data, end = h->size == UNKNOWN ? size : h->data + h->size;
    while (p < end) {
        Elem e;
        int r = rd_elem(b, size, p, &e);
        if (r < 0) return r;
        if (e.size == UNKNOWN || e.data + e.size > end) return VP9HIP_EINVALIDDATA;
        const uint64_t v = rd_uint(b, &e);
        switch (e.id) {
        case ID_EBMLREADVER:    if (v > 1) return VP9HIP_EINVALIDDATA; break;
        case ID_EBMLMAXIDLEN:   if (v > 4) return VP9HIP_EINVALIDDATA; break;
        case ID_EBMLMAXSIZELEN: if (v > 8) return VP9HIP_EINVALIDDATA; break;
        case ID_DOCTYPEREADVER: if (v > 3) return VP9HIP_EINVALIDDATA; break;
        case ID_DOCTYPE: {
            const size_t n = e.size < sizeof(info->doctype) - 1 ? (size_t) e.size : sizeof(info->doctype) - 1;
            memcpy(info->doctype, b + e.data, n);
            info->doctype[n] = 0;
            break;
        }
        default: break;
        }
        p = e.data + e.size;
    }
    return 0;
}

static int parse_tracks(const uint8_t *b, size_t size, const Elem *t, vp9h_webm_info *info)
{
    uint64_t p = t->data, end = t->size == UNKNOWN ? size : t->data + t->size;
    while (p < end) {
        Elem te;
        int r = rd_elem(b, size, p, &te);
        if (r < 0) return r;
        if (te.size == UNKNOWN) return VP9HIP_EINVALIDDATA;
        if (te.id == ID_TRACKENTRY && !info->track) {
            uint64_t num = 0, type = 0, w = 0, h = 0;
            char codec[32] = { 0 };
            for (uint64_t q = te.data; q < te.data + te.size;) {
                Elem c;
                if ((r = rd_elem(b, size, q, &c)) < 0) return r;
                if (c.size == UNKNOWN) return VP9HIP_EINVALIDDATA;
                if (c.id == ID_TRACKNUMBER) num = rd_uint(b, &c);
                else if (c.id == ID_TRACKTYPE) type = rd_uint(b, &c);
                else if (c.id == ID_CODECID) {
                    const size_t n = c.size < sizeof(codec) - 1 ? (size_t) c.size : sizeof(codec) - 1;
                    memcpy(codec, b + c.data, n);
                } else if (c.id == ID_VIDEO)
                    for (uint64_t v = c.data; v < c.data + c.size;) {
                        Elem d;
                        if ((r = rd_elem(b, size, v, &d)) < 0) return r;
                        if (d.size == UNKNOWN) return VP9HIP_EINVALIDDATA;
                        if (d.id == ID_PIXELWIDTH) w = rd_uint(b, &d);
                        else if (d.id == ID_PIXELHEIGHT) h = rd_uint(b, &d);
                        v = d.data + d.size;
                    }
                q = c.data + c.size;
            }
            if (type == 1 && !strcmp(codec, "V_VP9") && num) {
                info->track = num;
                info->width = (int32_t) w;
                info->height = (int32_t) h;
                memcpy(info->codec_id, codec, sizeof(info->codec_id) - 1);
            }
        }
        p = te.data + te.size;
    }
    return 0;
}

int vp9h_webm_read_header(const uint8_t *buf, size_t size, vp9h_webm_info *info, vp9h_webm_cursor *cur)
{
    if (!buf || !info || !cur) return VP9HIP_EINVAL;
    memset(info, 0, sizeof(*info));
    memset(cur, 0, sizeof(*cur));
    info->timecode_scale = 1000000;
    Elem h;
    int r = rd_elem(buf, size, 0, &h);
    if (r < 0) return VP9HIP_EINVALIDDATA;
    if (h.id != ID_EBML) return VP9HIP_EINVALIDDATA;
    if ((r = parse_ebml_header(buf, size, &h, info)) < 0) return r;
    if (h.size == UNKNOWN) return VP9HIP_EINVALIDDATA;
    uint64_t p = h.data + h.size;
    Elem seg;
    for (;;) {                                               /* the Segment (skip anything before it) */
        if ((r = rd_elem(buf, size, p, &seg)) < 0) return r == VP9HIP_EOF ? VP9HIP_EINVALIDDATA : r;
        if (seg.id == ID_SEGMENT) break;
        if (seg.size == UNKNOWN) return VP9HIP_EINVALIDDATA;
        p = seg.data + seg.size;
    }
    const uint64_t seg_end = seg.size == UNKNOWN ? size : seg.data + seg.size;
    p = seg.data;
    while (p < seg_end) {
        Elem e;
        if ((r = rd_elem(buf, size, p, &e)) < 0) return r == VP9HIP_EOF ? VP9HIP_EINVALIDDATA : r;
        if (e.id == ID_CLUSTER) break;                       /* the first cluster: frames start here */
        if (e.size == UNKNOWN) return VP9HIP_EINVALIDDATA;
        if (e.id == ID_INFO)
            for (uint64_t q = e.data; q < e.data + e.size;) {
                Elem c;
                if ((r = rd_elem(buf, size, q, &c)) < 0) return r;
                if (c.size == UNKNOWN) return VP9HIP_EINVALIDDATA;
                if (c.id == ID_TIMECODESCALE) info->timecode_scale = rd_uint(buf, &c);
                q = c.data + c.size;
            }
        else if (e.id == ID_TRACKS && (r = parse_tracks(buf, size, &e, info)) < 0)
            return r;
        p = e.data + e.size;
    }
    if (!info->track) return VP9HIP_EINVALIDDATA;            /* no VP9 video track */
    if (!info->timecode_scale) info->timecode_scale = 1000000;
    cur->pos = p;
    cur->seg_end = seg_end;
    cur->cluster_end = 0;
    cur->track = info->track;
    return 0;
}

/* Xiph / fixed / EBML lacing (matroska_parse_laces): lace sizes, data start */
static int parse_laces(const uint8_t *b, size_t size, uint64_t p, uint64_t end, int type, vp9h_webm_cursor *c)
{
    if (!type) {
        c->nlaces = 1;
        c->lace_size[0] = (uint32_t) (end - p);
        c->lace_pos = p;
        return 0;
    }
    if (p >= end) return VP9HIP_EINVALIDDATA;
    const int n = b[p] + 1;
    p++;
    uint64_t left = end - p, total = 0;
    c->nlaces = n;
    if (type == 1) {                                         /* Xiph: 255-runs per lace but the last */
        for (int i = 0; i < n - 1; i++) {
            uint32_t s = 0;
            uint8_t t;
            do {
                if (p >= end || left <= total) return VP9HIP_EINVALIDDATA;
                t = b[p++];
                left--;
                s += t;
                total += t;
            } while (t == 0xff);
            c->lace_size[i] = s;
        }
        if (left < total) return VP9HIP_EINVALIDDATA;
        c->lace_size[n - 1] = (uint32_t) (left - total);
    } else if (type == 2) {                                  /* fixed size */
        if (left % (uint64_t) n) return VP9HIP_EINVALIDDATA;
        for (int i = 0; i < n; i++) c->lace_size[i] = (uint32_t) (left / (uint64_t) n);
    } else {                                                 /* EBML: first size, then signed deltas */
        uint64_t v;
        int k = rd_num(b, end, p, 8, 0, &v);
        if (k < 0) return VP9HIP_EINVALIDDATA;
        if (v > 0x7fffffff) return VP9HIP_EINVALIDDATA;
        p += (uint64_t) k;
        c->lace_size[0] = (uint32_t) v;
        total = v;
        for (int i = 1; i < n - 1; i++) {
            k = rd_num(b, end, p, 8, 0, &v);
            if (k < 0) return VP9HIP_EINVALIDDATA;
            p += (uint64_t) k;
            const int64_t d = (int64_t) v - (int64_t) ((1ull << (7 * k - 1)) - 1);   /* matroska_ebmlnum_sint */
            const int64_t s = (int64_t) c->lace_size[i - 1] + d;
            if (s < 0 || s > 0x7fffffff) return VP9HIP_EINVALIDDATA;
            c->lace_size[i] = (uint32_t) s;
            total += (uint64_t) s;
        }
        left = end - p;
        if (left < total) return VP9HIP_EINVALIDDATA;
        c->lace_size[n - 1] = (uint32_t) (left - total);
    }
    c->lace_pos = p;
    return 0;
}

/* a Block / SimpleBlock body of our track -> its laces in the cursor; 1 = ours, 0 = skipped */
static int parse_block(const uint8_t *b, size_t size, uint64_t p, uint64_t end, int simple, int64_t duration,
                       vp9h_webm_cursor *c)
{
    uint64_t track;
    int k = rd_num(b, end, p, 8, 0, &track);
    if (k < 0) return VP9HIP_EINVALIDDATA;
    p += (uint64_t) k;
    if (p + 3 > end) return VP9HIP_EINVALIDDATA;
    if (track != c->track) return 0;
    const int16_t rel = (int16_t) (b[p] << 8 | b[p + 1]);
    const uint8_t flags = b[p + 2];
    p += 3;
    int r = parse_laces(b, size, p, end, (flags & 0x06) >> 1, c);
    if (r < 0) return r;
    c->lace_idx = 0;
    c->block_pts = c->cluster_tc + rel;
    c->block_duration = duration;
    c->keyframe = simple ? (flags & 0x80) != 0 : -1;
    return 1;
}

int vp9h_webm_read_frame(const uint8_t *buf, size_t size, vp9h_webm_cursor *c, const uint8_t **data,
                         uint32_t *frame_size, int64_t *pts, int *keyframe)
{
    if (!buf || !c || !data || !frame_size) return VP9HIP_EINVAL;
    for (;;) {
        if (c->lace_idx < c->nlaces) {                       /* the next lace of the current block */
            const int i = c->lace_idx++;
            if (c->lace_pos + c->lace_size[i] > size) return VP9HIP_EINVALIDDATA;
            *data = buf + c->lace_pos;
            *frame_size = c->lace_size[i];
            c->lace_pos += c->lace_size[i];
            if (pts)
                *pts = !i ? c->block_pts
                     : c->block_duration > 0 ? c->block_pts + c->block_duration * i / c->nlaces : INT64_MIN;
            if (keyframe) *keyframe = i ? 0 : c->keyframe;
            return 0;
        }
        c->nlaces = c->lace_idx = 0;
        const uint64_t lim = c->cluster_end ? c->cluster_end : c->seg_end;
        if (c->pos >= (c->cluster_end ? c->cluster_end : c->seg_end) || c->pos >= size) {
            if (c->cluster_end) { c->cluster_end = 0; continue; }     /* leave the cluster */
            return VP9HIP_EOF;
        }
        Elem e;
        int r = rd_elem(buf, size, c->pos, &e);
        if (r == VP9HIP_EOF) return VP9HIP_EOF;
        if (r < 0) return r;
        if (c->cluster_end) {                                 /* inside a cluster */
            if (c->cluster_unknown && is_level1(e.id)) { c->cluster_end = 0; continue; }
            if (e.size == UNKNOWN) return VP9HIP_EINVALIDDATA;
            const uint64_t end = e.data + e.size;
            if (end > lim) return VP9HIP_EINVALIDDATA;
            c->pos = end;
            if (e.id == ID_CLUSTERTC) c->cluster_tc = (int64_t) rd_uint(buf, &e);
            else if (e.id == ID_SIMPLEBLOCK) {
                if ((r = parse_block(buf, size, e.data, end, 1, 0, c)) < 0) return r;
            } else if (e.id == ID_BLOCKGROUP) {
                uint64_t bp = 0, bend = 0;
                int64_t dur = 0;
                for (uint64_t q = e.data; q < end;) {
                    Elem g;
                    if ((r = rd_elem(buf, size, q, &g)) < 0) return r;
                    if (g.size == UNKNOWN || g.data + g.size > end) return VP9HIP_EINVALIDDATA;
                    if (g.id == ID_BLOCK) { bp = g.data; bend = g.data + g.size; }
                    else if (g.id == ID_BLOCKDURATION) dur = (int64_t) rd_uint(buf, &g);
                    q = g.data + g.size;
                }
                if (bend && (r = parse_block(buf, size, bp, bend, 0, dur, c)) < 0) return r;
            }
            continue;
        }
        /* segment level */
        if (e.id == ID_CLUSTER) {
            c->cluster_unknown = e.size == UNKNOWN;
            c->cluster_end = c->cluster_unknown ? c->seg_end : e.data + e.size;
            if (c->cluster_end > size) c->cluster_end = size;
            c->cluster_tc = 0;
            c->pos = e.data;
            continue;
        }
        if (e.size == UNKNOWN) return VP9HIP_EINVALIDDATA;
        c->pos = e.data + e.size;
    }
}
