// VP9 bitstream decoder over the C-ABI: the avcodec_send_packet / avcodec_receive_frame
// loop of libavcodec/vp9.c for AV_CODEC_ID_VP9, with the host parse (vp9h_stream) in
// front of the device pixel path (vp9hip_ctx).
//
// What it restates of the reference decode loop (vp9.c:1558-1865, vp9_decode_frame):
//   - superframes split into frames first (the vp9_superframe_split BSF the decoder
//     declares, vp9.c:1977; bsf/vp9_superframe_split.c:40-95);
//   - show_existing_frame outputs a reference slot without decoding (vp9.c:1636-1653);
//   - every decoded frame goes to the slots of its refresh mask (vp9.c:1686-1691,
//     1845-1849); hidden frames (show_frame = 0) are decoded but not output;
//   - inter frames read their LAST / GOLDEN / ALTREF slots (s->s.h.refidx).
// Frames are parsed on the host as packets arrive and reconstructed on the GPU in
// batches of up to max_batch frames (vp9hip_stage_batch_refs: reference chains in
// order, independent chains concurrently); the parse of the next batch overlaps the
// GPU work of the previous one. receive_frame hands out frames whose batch has been
// submitted, in output order. Like libavcodec's frame threading, this adds decoder delay
// (up to max_batch frames); flushing (send_packet with data = NULL) drains it.
#include <cstring>
#include <deque>
#include <vector>

#include "../../include/vp9hip.h"

namespace {
struct Pending { vp9h_frame pkt; int out; int refs[3]; };   // refs: -1 for keyframes / intra-only
struct Out { int buf; int64_t pts; bool submitted; };
}

struct vp9hip_decoder {
    vp9hip_decoder_params p;
    vp9hip_ctx *ctx = nullptr;
    vp9h_stream *st = nullptr;
    bool configured = false, draining = false;
    int cw = 0, ch = 0, cbpp = 0, css_h = 0, css_v = 0, nbufs = 0;
    int slot[8];
    std::vector<int> pins, busy, bw, bh;   // per device buffer
    std::vector<Pending> batch;
    std::deque<Out> outq;
    int64_t decoded = 0;
};

static int slot_refs(const vp9hip_decoder *d, int b)
{
    int n = 0;
    for (int s = 0; s < 8; s++) n += d->slot[s] == b;
    return n;
}

static int free_buffers(const vp9hip_decoder *d)
{
    int n = 0;
    for (int b = 0; b < d->nbufs; b++) n += !d->pins[b] && !d->busy[b] && !slot_refs(d, b);
    return n;
}

static int alloc_buffer(vp9hip_decoder *d)
{
    for (int b = 0; b < d->nbufs; b++)
        if (!d->pins[b] && !d->busy[b] && !slot_refs(d, b)) return b;
    return -1;
}

// Stage + launch the pending frames as one batch.
static int submit(vp9hip_decoder *d)
{
    if (d->batch.empty()) return 0;
    const int n = (int) d->batch.size();
    std::vector<vp9h_frame> pk(n);
    std::vector<int> outs(n), refs(3 * n);
    for (int i = 0; i < n; i++) {
        pk[i] = d->batch[i].pkt;
        outs[i] = d->batch[i].out;
        for (int r = 0; r < 3; r++) refs[3 * i + r] = d->batch[i].refs[r] >= 0 ? d->batch[i].refs[r] : 0;
    }
    int ret = vp9hip_stage_batch_refs(d->ctx, pk.data(), n, outs.data(), refs.data());
    if (ret >= 0) ret = vp9hip_run_batch(d->ctx);
    for (auto &f : d->batch) {
        vp9h_frame_free(&f.pkt);
        d->busy[f.out]--;
        for (int r = 0; r < 3; r++)
            if (f.refs[r] >= 0) d->busy[f.refs[r]]--;
    }
    d->batch.clear();
    for (auto &o : d->outq) o.submitted = true;
    return ret < 0 ? ret : 0;
}

static int configure(vp9hip_decoder *d, const vp9h_frame &f)
{
    const int w = d->p.max_width > 0 ? d->p.max_width : f.width;
    const int h = d->p.max_height > 0 ? d->p.max_height : f.height;
    if (f.width > w || f.height > h) return VP9HIP_ENOSYS;
    const int nb = 8 + d->p.max_batch + (d->p.extra_bufs > 0 ? d->p.extra_bufs : 4);
    int r = vp9hip_configure(d->ctx, w, h, f.bpp, f.ss_h, f.ss_v, nb);
    if (r < 0) return r;
    d->configured = true;
    d->cw = w; d->ch = h; d->cbpp = f.bpp; d->css_h = f.ss_h; d->css_v = f.ss_v;
    d->nbufs = nb;
    d->pins.assign(nb, 0); d->busy.assign(nb, 0); d->bw.assign(nb, 0); d->bh.assign(nb, 0);
    for (int s = 0; s < 8; s++) d->slot[s] = -1;
    return 0;
}

extern "C" void vp9hip_decoder_defaults(vp9hip_decoder_params *p)
{
    memset(p, 0, sizeof(*p));
    p->max_batch = 16;
    p->extra_bufs = 4;
}

extern "C" int vp9hip_decoder_open(const vp9hip_decoder_params *params, vp9hip_decoder **out)
{
    if (!out) return VP9HIP_EINVAL;
    *out = nullptr;
    vp9hip_decoder *d = new vp9hip_decoder();
    if (params) d->p = *params; else vp9hip_decoder_defaults(&d->p);
    if (d->p.max_batch <= 0) d->p.max_batch = 1;
    if (d->p.max_batch > 256) d->p.max_batch = 256;
    for (int s = 0; s < 8; s++) d->slot[s] = -1;
    int r = vp9hip_open(d->p.device, &d->ctx);
    if (r >= 0) r = vp9h_stream_open(&d->st);
    if (r < 0) { vp9hip_decoder_close(d); return r; }
    *out = d;
    return 0;
}

extern "C" void vp9hip_decoder_close(vp9hip_decoder *d)
{
    if (!d) return;
    for (auto &f : d->batch) vp9h_frame_free(&f.pkt);
    if (d->st) vp9h_stream_close(d->st);
    if (d->ctx) vp9hip_close(d->ctx);
    delete d;
}

extern "C" vp9hip_ctx *vp9hip_decoder_context(vp9hip_decoder *d) { return d ? d->ctx : nullptr; }

extern "C" int vp9hip_decoder_send_packet(vp9hip_decoder *d, const uint8_t *data, size_t size, int64_t pts)
{
    if (!d) return VP9HIP_EINVAL;
    if (!data || !size) {                      // flush: drain the decoder delay
        d->draining = true;
        return submit(d);
    }
    if (d->draining) return VP9HIP_EOF;
    size_t offs[8], sizes[8];
    const int nf = vp9h_superframe_split(data, size, offs, sizes, 8);
    if (nf < 0) return nf;
    // every frame of the packet may need a buffer: ask for output to be read first
    // (avcodec_send_packet's EAGAIN) instead of parsing what cannot be placed
    if (d->configured && free_buffers(d) < nf) {
        int r = submit(d);
        if (r < 0) return r;
        if (free_buffers(d) < nf) return VP9HIP_EAGAIN;
    }
    for (int k = 0; k < nf; k++) {
        vp9h_frame f;
        vp9h_frame_info info;
        memset(&f, 0, sizeof(f));
        int r = vp9h_stream_decode(d->st, data + offs[k], sizes[k], &f, &info);
        if (r < 0) return r;
        if (info.show_existing_frame) {
            const int b = d->configured ? d->slot[info.show_slot & 7] : -1;
            if (b < 0) return VP9HIP_EINVALIDDATA;
            d->pins[b]++;
            d->outq.push_back({ b, pts, d->batch.empty() });
            continue;
        }
        const bool intra = f.keyframe || f.intraonly;
        if (!d->configured || f.bpp != d->cbpp || f.ss_h != d->css_h || f.ss_v != d->css_v ||
            f.width > d->cw || f.height > d->ch) {
            // a new format or size: only at a keyframe with nothing outstanding
            bool idle = d->batch.empty();
            for (int b = 0; b < d->nbufs && idle; b++) idle = !d->pins[b];
            if (!intra || !idle) { vp9h_frame_free(&f); return d->configured ? VP9HIP_ENOSYS : VP9HIP_EINVALIDDATA; }
            r = configure(d, f);
            if (r < 0) { vp9h_frame_free(&f); return r; }
        }
        Pending q;
        q.pkt = f;
        q.out = alloc_buffer(d);
        if (q.out < 0) { vp9h_frame_free(&f); return VP9HIP_EBUG; }
        for (int i = 0; i < 3; i++) {
            q.refs[i] = intra ? -1 : d->slot[info.ref_slot[i] & 7];
            if (!intra && q.refs[i] < 0) { vp9h_frame_free(&f); return VP9HIP_EINVALIDDATA; }
        }
        d->busy[q.out]++;
        for (int i = 0; i < 3; i++)
            if (q.refs[i] >= 0) d->busy[q.refs[i]]++;
        d->bw[q.out] = f.width; d->bh[q.out] = f.height;
        for (int s = 0; s < 8; s++)
            if (info.refresh_mask & (1 << s)) d->slot[s] = q.out;
        d->batch.push_back(q);
        d->decoded++;
        if (info.show_frame) {
            d->pins[q.out]++;
            d->outq.push_back({ q.out, pts, false });
        }
        if ((int) d->batch.size() >= d->p.max_batch) {
            r = submit(d);
            if (r < 0) return r;
        }
    }
    return 0;
}

extern "C" int vp9hip_decoder_receive_frame(vp9hip_decoder *d, vp9hip_decoded_frame *out)
{
    if (!d || !out) return VP9HIP_EINVAL;
    if (!d->outq.empty() && !d->outq.front().submitted && d->draining) {
        int r = submit(d);
        if (r < 0) return r;
    }
    if (d->outq.empty()) return d->draining ? VP9HIP_EOF : VP9HIP_EAGAIN;
    if (!d->outq.front().submitted) return VP9HIP_EAGAIN;
    const Out o = d->outq.front();
    d->outq.pop_front();
    memset(out, 0, sizeof(*out));
    out->buf = o.buf;
    out->width = d->bw[o.buf];
    out->height = d->bh[o.buf];
    out->bpp = d->cbpp;
    out->ss_h = d->css_h;
    out->ss_v = d->css_v;
    out->pts = o.pts;
    return 0;                      // the buffer stays pinned until vp9hip_decoder_release
}

extern "C" int vp9hip_decoder_release(vp9hip_decoder *d, int buf)
{
    if (!d || buf < 0 || buf >= d->nbufs || d->pins[buf] <= 0) return VP9HIP_EINVAL;
    d->pins[buf]--;
    return 0;
}

// avcodec_flush_buffers (vp9.c:1865-1883): drop the decoder delay and the reference
// state; frames already handed out stay valid until released.
extern "C" int vp9hip_decoder_flush(vp9hip_decoder *d)
{
    if (!d) return VP9HIP_EINVAL;
    for (auto &f : d->batch) {
        vp9h_frame_free(&f.pkt);
        d->busy[f.out]--;
        for (int r = 0; r < 3; r++)
            if (f.refs[r] >= 0) d->busy[f.refs[r]]--;
    }
    d->batch.clear();
    for (auto &o : d->outq) d->pins[o.buf]--;
    d->outq.clear();
    for (int s = 0; s < 8; s++) d->slot[s] = -1;
    vp9h_stream_close(d->st);
    d->st = nullptr;
    d->draining = false;
    int r = vp9h_stream_open(&d->st);
    if (r < 0) return r;
    return d->ctx ? vp9hip_flush(d->ctx) : 0;
}
