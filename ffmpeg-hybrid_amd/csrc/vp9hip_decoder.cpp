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
//
// Pipeline:
//   1. host parse on a pool of threads. Frames of one parse chain parse in order on one
//      vp9h_stream; a keyframe starts a new chain on a fresh vp9h_stream, because its
//      parse depends on no earlier frame (vp9h_frame_type). All-keyframe streams thus
//      parse frame-parallel, GOP streams GOP-parallel (the reference's frame threads get
//      the same freedom from ff_thread_finish_setup after the header, vp9.c:1736);
//   2. in decode order, on the caller's thread: reference slots, device buffers, and
//      batches of up to max_batch frames staged and launched on the GPU
//      (vp9hip_stage_batch_refs: reference chains in order, independent chains
//      concurrently; the batch planning itself runs on host threads);
//   3. receive_frame hands out frames whose batch has been launched, in output order.
// Like libavcodec's frame threading this adds decoder delay (up to max_batch frames plus
// the frames in parse); flushing (send_packet with data = NULL) drains it.
// Errors are per frame (vp9hip_pipeline.h): a packet whose parse fails is reported by the
// send_packet / receive_frame call that consumes it and updates no reference slot (vp9.c
// fails that decode, :1827-1832, and refreshes no slot); a frame the device rejects, or
// one predicted from a failed frame, fails when it is received.
#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <memory>
#include <utility>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/vp9hip.h"
#include "vp9hip_parse.h"
#include "vp9hip_pipeline.h"

using vp9hip::Chain;
using vp9hip::LFrame;
using vp9hip::ParseJob;
using vp9hip::ParsePool;

namespace {
struct Pending { vp9h_frame pkt; LFrame f; };   // f.refs: -1 for keyframes / intra-only
struct Out { int buf; int64_t pts; bool submitted; uint64_t id; };
// Batches are numbered as launched (1, 2, ...) and rotate over VP9HIP_PIPELINE_SLOTS batch
// slots (vp9hip::Ledger), so batches k + 1 and k + 2 are staged and planned while batch k's
// pixel kernels run. A frame's batch is the one that wrote its buffer (Ledger::seq_of). A
// batch is checked (vp9hip_sync_slot: its slot's work is drained, the planner's verdicts and
// k_lfr's hand-off timeout words are read) before its slot is staged again, which resets
// them, or before one of its frames is handed out, whichever comes first.
const int STALL = 1;                   // consume: no free device buffer until frames are released
}

struct vp9hip_decoder {
    vp9hip_decoder_params p;
    vp9hip_ctx *ctx = nullptr;
    bool configured = false, draining = false;
    bool stalled = false;                  // send_packet answered EAGAIN: receive must block
    int cw = 0, ch = 0, cbpp = 0, css_h = 0, css_v = 0, nbufs = 0;
    int slot[8];
    std::vector<int> pins, busy, bw, bh;   // per device buffer
    vp9hip::Ledger led;                    // batches in flight, per-frame outcomes
    std::vector<Pending> batch;
    std::deque<Out> outq;
    // parse pipeline
    std::deque<std::unique_ptr<ParseJob>> inflight;   // decode order
    std::shared_ptr<Chain> chain;                     // the chain of the next non-key frame
    std::unique_ptr<ParsePool> pool;
    int max_inflight = 0;
};

static int slot_refs(const vp9hip_decoder *d, int b)
{
    int n = 0;
    for (int s = 0; s < 8; s++) n += d->slot[s] == b;
    return n;
}

static int alloc_buffer(vp9hip_decoder *d)
{
    for (int b = 0; b < d->nbufs; b++)
        if (!d->pins[b] && !d->busy[b] && !slot_refs(d, b)) return b;
    return -1;
}

// ---- parse (vp9hip_parse.h) ----
static void enqueue_parse(vp9hip_decoder *d, std::unique_ptr<ParseJob> j)
{
    ParseJob *raw = j.get();
    d->inflight.push_back(std::move(j));
    d->pool->enqueue(raw);
}

static bool front_done(vp9hip_decoder *d, bool block)
{
    if (d->inflight.empty()) return false;
    if (block) d->pool->wait(d->inflight.front().get());
    return d->pool->done(d->inflight.front().get());
}

static void wait_all_parsed(vp9hip_decoder *d)
{
    for (auto &j : d->inflight) d->pool->wait(j.get());
}

// ---- device side ----
// Stage + launch the pending frames as one batch in the next pipeline slot (frames the
// device rejects fail alone, Ledger::launch). 0, or a failure of the device context.
static int submit(vp9hip_decoder *d)
{
    if (d->batch.empty()) return 0;
    const int n = (int) d->batch.size();
    std::vector<const vp9h_frame *> pk(n);
    std::vector<LFrame> fr(n);
    for (int i = 0; i < n; i++) {
        pk[i] = &d->batch[i].pkt;
        fr[i] = d->batch[i].f;
    }
    const int ret = d->led.launch(d->ctx, pk, fr);
    for (auto &p : d->batch) {
        vp9h_frame_free(&p.pkt);
        d->busy[p.f.out]--;
        for (int r = 0; r < 3; r++)
            if (p.f.refs[r] >= 0) d->busy[p.f.refs[r]]--;
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
    // 8 reference slots, the batch being filled, the launched batches' frames still to be
    // received (VP9HIP_PIPELINE_SLOTS in flight), and the frames the caller holds
    const int nb = 8 + (VP9HIP_PIPELINE_SLOTS + 1) * d->p.max_batch + (d->p.extra_bufs > 0 ? d->p.extra_bufs : 4);
    int r = vp9hip_configure(d->ctx, w, h, f.bpp, f.ss_h, f.ss_v, nb);
    if (r < 0) return r;
    d->configured = true;
    d->cw = w; d->ch = h; d->cbpp = f.bpp; d->css_h = f.ss_h; d->css_v = f.ss_v;
    d->nbufs = nb;
    d->pins.assign(nb, 0); d->busy.assign(nb, 0); d->bw.assign(nb, 0); d->bh.assign(nb, 0);
    d->led.reset_buffers(nb);
    for (int s = 0; s < 8; s++) d->slot[s] = -1;
    return 0;
}

// One parsed frame, in decode order: slots, buffer, batch. 0, STALL (no free buffer;
// the job stays queued) or an error.
static int consume_one(vp9hip_decoder *d, ParseJob &j)
{
    if (j.ret < 0) return j.ret;
    vp9h_frame &f = j.pkt;
    const vp9h_frame_info &info = j.info;
    if (info.show_existing_frame) {
        const int b = d->configured ? d->slot[info.show_slot & 7] : -1;
        if (b < 0) return VP9HIP_EINVALIDDATA;
        d->pins[b]++;
        d->outq.push_back({ b, j.pts, d->batch.empty(), d->led.holder(b) });
        return 0;
    }
    const bool intra = f.keyframe || f.intraonly;
    if (!d->configured || f.bpp != d->cbpp || f.ss_h != d->css_h || f.ss_v != d->css_v ||
        f.width > d->cw || f.height > d->ch) {
        // a new format or size: only at an intra frame with nothing outstanding
        int r = submit(d);
        if (r < 0) return r;
        bool idle = true;
        for (int b = 0; b < d->nbufs && idle; b++) idle = !d->pins[b];
        if (!intra) return d->configured ? VP9HIP_ENOSYS : VP9HIP_EINVALIDDATA;
        if (!idle) return STALL;          // frames of the old format are still out: receive / release them
        r = configure(d, f);
        if (r < 0) return r;
    }
    int out = alloc_buffer(d);
    if (out < 0) {                        // the batch's busy buffers come back when it is launched
        int r = submit(d);
        if (r < 0) return r;
        out = alloc_buffer(d);
        if (out < 0) return STALL;
    }
    int refs[3];
    for (int i = 0; i < 3; i++) {
        refs[i] = intra ? -1 : d->slot[info.ref_slot[i] & 7];
        if (!intra && refs[i] < 0) return VP9HIP_EINVALIDDATA;
    }
    Pending q;
    q.pkt = f;
    q.f = d->led.frame(out, refs);
    memset(&f, 0, sizeof(f));            // the batch owns the packet now
    d->busy[out]++;
    for (int i = 0; i < 3; i++)
        if (refs[i] >= 0) d->busy[refs[i]]++;
    d->bw[out] = q.pkt.width; d->bh[out] = q.pkt.height;
    for (int s = 0; s < 8; s++)
        if (info.refresh_mask & (1 << s)) d->slot[s] = out;
    d->batch.push_back(q);
    if (info.show_frame) {
        d->pins[out]++;
        d->outq.push_back({ out, j.pts, false, q.f.id });
    }
    if ((int) d->batch.size() >= d->p.max_batch) return submit(d);
    return 0;
}

// Consume parsed frames in decode order; block: wait for their parse. Returns 0 when the
// parsed front is consumed (or nothing is ready), STALL, or an error.
static int consume(vp9hip_decoder *d, bool block, size_t keep = 0)
{
    while (d->inflight.size() > keep && front_done(d, block)) {
        int r = consume_one(d, *d->inflight.front());
        if (r == STALL) return STALL;
        d->inflight.pop_front();
        if (r < 0) return r;
    }
    return 0;
}

// ---- C-ABI ----
extern "C" void vp9hip_decoder_defaults(vp9hip_decoder_params *p)
{
    memset(p, 0, sizeof(*p));
    p->max_batch = 16;
    p->extra_bufs = 4;
    p->parse_threads = (int) std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
}

extern "C" int vp9hip_decoder_open(const vp9hip_decoder_params *params, vp9hip_decoder **out)
{
    if (!out) return VP9HIP_EINVAL;
    *out = nullptr;
    vp9hip_decoder *d = new vp9hip_decoder();
    if (params) d->p = *params; else vp9hip_decoder_defaults(&d->p);
    if (d->p.max_batch <= 0) d->p.max_batch = 1;
    if (d->p.max_batch > 256) d->p.max_batch = 256;
    if (d->p.parse_threads < 0) d->p.parse_threads = 0;
    if (d->p.parse_threads > 64) d->p.parse_threads = 64;
    // parse lookahead: enough frames that the pool keeps parsing while the caller's thread
    // waits on the device (the batches in flight)
    d->max_inflight = 4 * d->p.parse_threads + VP9HIP_PIPELINE_SLOTS * d->p.max_batch + 1;
    for (int s = 0; s < 8; s++) d->slot[s] = -1;
    int r = vp9hip_open(d->p.device, &d->ctx);
    if (r < 0) { vp9hip_decoder_close(d); return r; }
    vp9hip_set_timing(d->ctx, 0);             // every batch runs once: plain launches, no events
    vp9hip_set_graph(d->ctx, 0);
    d->pool.reset(new ParsePool(d->p.parse_threads));
    *out = d;
    return 0;
}

static void drop_inflight(vp9hip_decoder *d)
{
    wait_all_parsed(d);
    d->inflight.clear();
}

extern "C" void vp9hip_decoder_close(vp9hip_decoder *d)
{
    if (!d) return;
    if (d->pool) drop_inflight(d);
    d->pool.reset();
    for (auto &f : d->batch) vp9h_frame_free(&f.pkt);
    d->chain.reset();
    if (d->ctx) vp9hip_close(d->ctx);
    delete d;
}

extern "C" vp9hip_ctx *vp9hip_decoder_context(vp9hip_decoder *d) { return d ? d->ctx : nullptr; }

extern "C" int vp9hip_decoder_send_packet(vp9hip_decoder *d, const uint8_t *data, size_t size, int64_t pts)
{
    if (!d) return VP9HIP_EINVAL;
    if (!data || !size) {                      // flush: drain the decoder delay (receive_frame does it)
        d->draining = true;
        int r = consume(d, false);
        return r < 0 ? r : 0;
    }
    if (d->draining) return VP9HIP_EOF;
    size_t offs[8], sizes[8];
    const int nf = vp9h_superframe_split(data, size, offs, sizes, 8);
    if (nf < 0) return nf;
    // bound the frames in flight: consume parsed ones first; a stall (no free device
    // buffer) asks the caller to receive frames (avcodec_send_packet's EAGAIN). An earlier
    // frame's error found here is returned after this packet is queued: the packet is taken
    int err = 0;
    if (d->inflight.size() + nf > (size_t) d->max_inflight) {
        int r = consume(d, true, d->max_inflight > nf ? d->max_inflight - nf : 0);
        if (r == STALL) { d->stalled = true; return VP9HIP_EAGAIN; }
        if (r < 0) err = r;
    }
    d->stalled = false;
    for (int k = 0; k < nf; k++) {
        const int type = vp9h_frame_type(data + offs[k], sizes[k]);
        if (type < 0) return err < 0 ? err : type;
        std::unique_ptr<ParseJob> j(new ParseJob());
        j->data.assign(data + offs[k], data + offs[k] + sizes[k]);
        j->pts = pts;
        if (type == 0 || !d->chain) {          // a keyframe parses on a fresh stream
            int r = 0;
            std::shared_ptr<Chain> c = ParsePool::new_chain(&r);
            if (!c) return err < 0 ? err : r;
            d->chain = c;
        }
        j->chain = d->chain;
        enqueue_parse(d, std::move(j));
    }
    if (err < 0) return err;
    int r = consume(d, false);
    return r < 0 ? r : 0;
}

extern "C" int vp9hip_decoder_receive_frame(vp9hip_decoder *d, vp9hip_decoded_frame *out)
{
    if (!d || !out) return VP9HIP_EINVAL;
    int r = 0;
    if (d->outq.empty() || !d->outq.front().submitted) {   // nothing to hand out yet: make progress
        r = consume(d, d->draining);
        if (r < 0) return r;
    }
    if (d->draining) {                         // everything parsed that can be placed: launch it
        r = submit(d);
        if (r < 0) return r;
    }
    if (d->outq.empty())
        return d->draining && d->inflight.empty() && d->batch.empty() ? VP9HIP_EOF : VP9HIP_EAGAIN;
    if (!d->outq.front().submitted) return VP9HIP_EAGAIN;
    const Out o = d->outq.front();
    if (!d->led.error(o.id)) {                 // its batch may still run: drain and check it
        const uint64_t b = d->led.seq_of(o.buf);
        const int s = d->led.unchecked(b);
        if (s >= 0) {
            // the newest batch still running: EAGAIN (frame-threading delay), so the caller
            // sends the next packets while it runs; an older batch, a drain or a stalled
            // send_packet wait for it (and for the batches before it: checks run in order)
            if (!d->draining && !d->stalled && b == d->led.last() && vp9hip_slot_busy(d->ctx, s) == 1)
                return VP9HIP_EAGAIN;
            if ((r = d->led.check_through(d->ctx, b)) < 0) return r;
        }
    }
    d->outq.pop_front();
    if (const int e = d->led.error(o.id)) {    // rejected on the device, or read a failed frame
        d->pins[o.buf]--;
        return e;
    }
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
    drop_inflight(d);
    d->chain.reset();
    for (auto &p : d->batch) {
        vp9h_frame_free(&p.pkt);
        d->busy[p.f.out]--;
        for (int r = 0; r < 3; r++)
            if (p.f.refs[r] >= 0) d->busy[p.f.refs[r]]--;
    }
    d->batch.clear();
    for (auto &o : d->outq) d->pins[o.buf]--;
    d->outq.clear();
    for (int s = 0; s < 8; s++) d->slot[s] = -1;
    d->draining = false;
    d->stalled = false;
    d->led.reset();                            // vp9hip_flush drops the batches in flight
    return d->ctx ? vp9hip_flush(d->ctx) : 0;
}
