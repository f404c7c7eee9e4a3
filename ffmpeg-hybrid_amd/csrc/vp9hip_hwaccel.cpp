// The FFHWAccel adapter of the hybrid VP9 decoder over libvp9hip (include/vp9hip_hwaccel.h).
//
// One context per stream, as avctx->internal->hwaccel_priv_data: the device context, the
// host parse pool, the frames in flight, and the device frame pool with the reference
// slots. The call order is the reference's (vp9.c:1694-1713): start_frame, decode_slice,
// end_frame per coded frame; show_existing_frame never reaches the hwaccel
// (vp9.c:1636-1653) and is answered from the slots.
//
// Asynchronous, as an HWACCEL_CAP_ASYNC_SAFE hwaccel is (hwaccel_internal.h:31-32, the cap
// vulkan_vp9.c:369 sets; frame threading gates on it at pthread_frame.c:687): nothing
// waits on the GPU or on the entropy decode inside the per-frame calls.
//   - decode_slice reads the slot bookkeeping from the start of the uncompressed header
//     (vp9h_frame_peek, what vp9.c knows before ff_thread_finish_setup) and queues the
//     entropy decode on the parse pool (vp9hip_parse.h): keyframes start new chains, so
//     they parse in parallel; a lone chain's tile columns parse on the idle threads.
//   - end_frame maps refidx to device buffers, replaces the slots of refreshrefmask and
//     appends the frame to the batch being filled. A batch of `async_depth` frames is staged
//     into the next of VP9HIP_PIPELINE_SLOTS batch slots and launched
//     (vp9hip_stage_batch_refs / run_batch: dependent frames chained, independent chains
//     concurrent) once its parses are done, checked at each later end_frame, so the pool
//     parses the next batches meanwhile; with more than max_full filled batches waiting the
//     oldest launches anyway.
//   - A frame handed out is a device frame whose pixels are complete once
//     vp9hip_hwframe_sync (host) or vp9hip_hwframe_ready (a consumer's HIP stream) says so;
//     both launch the batch holding it if it is still being filled. transfer syncs.
// Errors of asynchronous work surface on the call that waits for the frame, and they are
// the frame's own (vp9hip_pipeline.h), as vp9.c fails only the corrupt frame's decode
// (:1827-1832): a frame whose entropy decode fails fails with that error, a frame the device
// planner rejects with AVERROR_INVALIDDATA, and so does every frame predicted from a failed
// one (its slots were mapped to the failed frame's buffer at end_frame, before the outcome
// was known); the other frames of the same batch decode. A batch whose row-pipelined loop
// filter gave up a hand-off (k_lfr timeout words, read by vp9hip_sync_slot) fails its frames
// with VP9HIP_EBUG.
//
// Pool: a buffer is free when no reference slot holds it, no frame reference (the
// AVBufferRef of an AVFrame, vp9hip_hwframe_unref) holds it, it is not the frame being
// decoded, and it is not in the batch being filled.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <utility>
#include <vector>

#include "../../include/vp9hip_hwaccel.h"
#include "vp9hip_parse.h"
#include "vp9hip_pipeline.h"

using vp9hip::Chain;
using vp9hip::LFrame;
using vp9hip::ParseJob;
using vp9hip::ParsePool;

namespace {
struct Pend { std::unique_ptr<ParseJob> job; LFrame f; };

// VP9HIP_HWACCEL_TRACE=1: host wall time of the adapter's steps, printed at uninit
enum { T_SLICE, T_END, T_PARSE_WAIT, T_RUN, T_SYNC_WAIT, T_N };
const char *const tname[T_N] = { "decode_slice", "end_frame (excl. launches)", "submit: wait for parses",
                                  "submit: check the slot's previous batch, stage, run_batch",
                                  "hwframe_sync: wait for the frame's batch" };
struct Trace {
    bool on = false;
    double ms[T_N] = {};
    long batches = 0, frames = 0;
    std::chrono::steady_clock::time_point t0;
    void start() { if (on) t0 = std::chrono::steady_clock::now(); }
    void stop(int k)
    {
        if (!on) return;
        const auto t = std::chrono::steady_clock::now();
        ms[k] += std::chrono::duration<double, std::milli>(t - t0).count();
        t0 = t;
    }
};
}

struct vp9hip_hwaccel {
    vp9hip_ctx *gpu = nullptr;
    vp9hip_frames_params fp;
    std::unique_ptr<ParsePool> pool;
    std::shared_ptr<Chain> chain;           // the parse chain of the next non-key frame
    int slot[8];                            // device buffer of each reference slot (s->s.ref_frames)
    std::vector<int> refs;                  // per pool buffer: frame references handed out
    // Every entry point holds mu: FFmpeg calls the per-frame callbacks from its decoding
    // thread(s) while the user's thread transfers and unrefs output frames
    // (av_hwframe_transfer_data, av_frame_unref run the hwcontext / buffer callbacks there).
    mutable std::mutex mu;
    std::vector<int> pend;                  // per pool buffer: in the batch being filled
    std::vector<int> inref;                 // per pool buffer: read by frames of that batch
    vp9hip::Ledger led;                     // batches in flight, per-frame outcomes
    int cur = -1;                           // buffer of the frame being decoded
    int64_t pts = 0;
    std::unique_ptr<ParseJob> job;          // decode_slice -> end_frame
    int intra = 0;
    vp9h_frame_info info;                   // the peeked header of the current frame
    std::vector<Pend> batch;                // the batch being filled
    std::deque<std::vector<Pend>> full;     // filled batches waiting for their parses (decode order)
    size_t max_full = 1;                    // filled batches that may wait for their parses
    Trace tr;
};

static int swfmt(int bpp, int ss_h, int ss_v)
{
    const int chroma = ss_h && ss_v ? 0 : ss_h ? 1 : ss_v ? 2 : 3;
    return (bpp == 8 ? 0 : bpp == 10 ? 4 : 8) + chroma;
}

extern "C" int vp9hip_hwaccel_frame_params(int width, int height, int bpp, int ss_h, int ss_v, int extra,
                                           vp9hip_frames_params *out)
{
    if (!out || width <= 0 || height <= 0 || (bpp != 8 && bpp != 10 && bpp != 12) || ss_h < 0 || ss_h > 1 ||
        ss_v < 0 || ss_v > 1)
        return VP9HIP_EINVAL;
    // FFmpeg's extra_hw_frames defaults to -1 (options_table.h:397; decode.c:1135 adds it
    // only when > 0): a negative count asks for no extra frames
    if (extra < 0) extra = 0;
    memset(out, 0, sizeof(*out));
    out->sw_format = swfmt(bpp, ss_h, ss_v);
    out->width = width;
    out->height = height;
    // batches of half the consumer's frame delay, rounded down to a power of two
    // (include/vp9hip_hwaccel.h)
    int d = 1;
    while (2 * d <= extra / 2 && 2 * d <= VP9HIP_HWACCEL_ASYNC_DEPTH) d *= 2;
    out->async_depth = d;
    // 8 reference slots, the frame being decoded, the frames of the batch being filled and
    // of the filled batches waiting for their parses (each also handed out until the
    // consumer has waited for it) and the caller's extra
    out->initial_pool_size = 8 + 1 + (1 + VP9HIP_HWACCEL_AHEAD) * out->async_depth + extra;
    out->bpp = bpp;
    out->ss_h = ss_h;
    out->ss_v = ss_v;
    out->parse_threads = (int) std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    return 0;
}

extern "C" int vp9hip_hwaccel_uninit(vp9hip_hwaccel *h);

extern "C" int vp9hip_hwaccel_init(int device, const vp9hip_frames_params *fp, vp9hip_hwaccel **out)
{
    if (!fp || !out || fp->initial_pool_size < 9 || fp->async_depth < 1 || fp->async_depth > 256 ||
        fp->parse_threads < 0 || fp->parse_threads > 64)
        return VP9HIP_EINVAL;
    *out = nullptr;
    vp9hip_hwaccel *h = new (std::nothrow) vp9hip_hwaccel();
    if (!h) return VP9HIP_ENOMEM;
    h->fp = *fp;
    for (int i = 0; i < 8; i++) h->slot[i] = -1;
    const size_t n = (size_t) fp->initial_pool_size;
    h->refs.assign(n, 0);
    h->pend.assign(n, 0);
    h->inref.assign(n, 0);
    h->led.reset_buffers((int) n);
    int r = vp9hip_open(device, &h->gpu);
    if (!r) r = vp9hip_configure(h->gpu, fp->width, fp->height, fp->bpp, fp->ss_h, fp->ss_v, fp->initial_pool_size);
    if (r < 0) {
        vp9hip_hwaccel_uninit(h);
        return r;
    }
    vp9hip_set_timing(h->gpu, 0);              // every batch runs once: plain launches, no events
    vp9hip_set_graph(h->gpu, 0);
    h->tr.on = getenv("VP9HIP_HWACCEL_TRACE") && atoi(getenv("VP9HIP_HWACCEL_TRACE"));
    // the look-ahead the pool affords beyond the batch being filled
    h->max_full = (size_t) std::max(1, (fp->initial_pool_size - 9) / fp->async_depth - 1);
    h->pool.reset(new ParsePool(fp->parse_threads));
    *out = h;
    return 0;
}

// Stage + launch one batch in the next pipeline slot. Its packets are parsed by now or
// soon: wait for them (in decode order). A frame whose parse failed fails alone (with the
// frames that read it); the others launch (Ledger::launch). 0, or a failure of the device
// context.
static int submit_list(vp9hip_hwaccel *h, std::vector<Pend> &batch)
{
    if (batch.empty()) return 0;
    const int n = (int) batch.size();
    Trace &tr = h->tr;
    tr.start();
    std::vector<const vp9h_frame *> pk(n, nullptr);
    std::vector<LFrame> fr(n);
    for (int i = 0; i < n; i++) {
        Pend &p = batch[i];
        h->pool->wait(p.job.get());
        const vp9h_frame &f = p.job->pkt;
        int e = p.job->ret;
        if (!e && (f.width > h->fp.width || f.height > h->fp.height || f.bpp != h->fp.bpp ||
                   f.ss_h != h->fp.ss_h || f.ss_v != h->fp.ss_v))
            e = VP9HIP_ENOSYS;               // a new format: get_format re-inits the hwaccel
        fr[i] = p.f;
        if (e) h->led.fail(p.f, e);
        else pk[i] = &f;
    }
    tr.stop(T_PARSE_WAIT);
    const int ret = h->led.launch(h->gpu, pk, fr);   // checks the slot's last batch, stages, runs
    tr.stop(T_RUN);
    tr.batches++;
    tr.frames += n;
    for (auto &p : batch) {
        h->pend[p.f.out] = 0;
        for (int r = 0; r < 3; r++)
            if (p.f.refs[r] >= 0) h->inref[p.f.refs[r]]--;
    }
    batch.clear();                           // the jobs free their packets
    return ret < 0 ? ret : 0;
}

// Launch every queued batch in decode order (the filled ones, then, with partial, the one
// being filled); the first error, after all were handled.
static int submit(vp9hip_hwaccel *h, bool partial = true)
{
    int err = 0;
    while (!h->full.empty()) {
        const int r = submit_list(h, h->full.front());
        h->full.pop_front();
        if (r < 0 && !err) err = r;
    }
    if (partial) {
        const int r = submit_list(h, h->batch);
        if (r < 0 && !err) err = r;
    }
    return err;
}

// The filled batches whose parses are done launch now, without waiting; more than
// max_full filled batches waiting launch the oldest anyway (bounds the frames in flight).
// The parse pool meanwhile works on the frames the caller keeps handing over.
static int pump(vp9hip_hwaccel *h)
{
    int err = 0;
    while (!h->full.empty()) {
        bool ready = h->full.size() > h->max_full;
        if (!ready) {
            ready = true;
            for (auto &p : h->full.front())
                if (!h->pool->done(p.job.get())) { ready = false; break; }
        }
        if (!ready) break;
        const int r = submit_list(h, h->full.front());
        h->full.pop_front();
        if (r < 0 && !err) err = r;
    }
    return err;
}

static int nrefs(const vp9hip_hwaccel *h, int b) { return h->refs[b]; }

// drop the frame decode_slice queued for parsing (the pool may be working on it)
static void drop_job(vp9hip_hwaccel *h)
{
    if (h->job) h->pool->wait(h->job.get());
    h->job.reset();
}

static bool buf_busy(const vp9hip_hwaccel *h, int b)
{
    // a buffer a batched frame reads is not rewritten by a later frame of the same batch
    if (nrefs(h, b) || h->pend[b] || h->inref[b] || b == h->cur) return true;
    for (int s = 0; s < 8; s++)
        if (h->slot[s] == b) return true;
    return false;
}

static int find_free(const vp9hip_hwaccel *h)
{
    for (int b = 0; b < h->fp.initial_pool_size; b++)
        if (!buf_busy(h, b)) return b;
    return -1;
}

extern "C" int vp9hip_hwaccel_start_frame(vp9hip_hwaccel *h, const uint8_t *buf, uint32_t size, int64_t pts)
{
    if (!h || (!buf && size)) return VP9HIP_EINVAL;
    std::lock_guard<std::mutex> g(h->mu);
    drop_job(h);                             // a frame that never reached end_frame
    h->cur = -1;
    // a full pool: launch the oldest filled batches first (waiting for their parses), then
    // the one being filled; their unreferenced hidden frames free up once launched
    int b = find_free(h), err = 0;
    while (b < 0 && !h->full.empty()) {
        const int r = submit_list(h, h->full.front());
        h->full.pop_front();
        if (r < 0 && !err) err = r;
        b = find_free(h);
    }
    if (b < 0 && !h->batch.empty()) {
        const int r = submit_list(h, h->batch);
        if (r < 0 && !err) err = r;
        b = find_free(h);
    }
    if (err < 0) return err;
    if (b < 0) return VP9HIP_EAGAIN;         // every buffer held: the caller must unref frames
    h->cur = b;
    h->pts = pts;
    return 0;
}

extern "C" int vp9hip_hwaccel_decode_slice(vp9hip_hwaccel *h, const uint8_t *buf, uint32_t size)
{
    if (!h || !buf || !size) return VP9HIP_EINVAL;
    std::lock_guard<std::mutex> g(h->mu);
    if (h->cur < 0) return VP9HIP_EINVAL;
    h->tr.start();
    vp9h_frame_info info;
    const int type = vp9h_frame_peek(buf, size, &info);
    if (type < 0) return type;
    if (type == 2) return VP9HIP_EINVALIDDATA;           // show_existing_frame: vp9.c answers it itself
    std::unique_ptr<ParseJob> j(new (std::nothrow) ParseJob());
    if (!j) return VP9HIP_ENOMEM;
    if (type == 0) {                                     // a keyframe parses on a fresh stream
        int r = 0;
        h->chain = ParsePool::new_chain(&r);
        if (!h->chain) return r;
    } else if (!h->chain) {
        return VP9HIP_EINVALIDDATA;                      // no keyframe yet since init / flush
    }
    j->data.assign(buf, buf + size);
    j->pts = h->pts;
    j->chain = h->chain;
    h->pool->enqueue(j.get());
    h->job = std::move(j);
    h->info = info;
    h->intra = type == 0 || type == 3;
    h->tr.stop(T_SLICE);
    return 0;
}

static void fill_frame(vp9hip_hwaccel *h, int b, int64_t pts, vp9hip_hwframe *out)
{
    memset(out, 0, sizeof(*out));
    int w = 0, ht = 0;
    vp9hip_frame_device(h->gpu, b, out->data, out->linesize, &w, &ht, &out->stream);
    out->width = w;
    out->height = ht;
    out->sw_format = h->fp.sw_format;
    out->buf = b;
    out->pts = pts;
    h->refs[b]++;
}

extern "C" int vp9hip_hwaccel_end_frame(vp9hip_hwaccel *h, vp9hip_hwframe *out)
{
    if (!h) return VP9HIP_EINVAL;
    std::lock_guard<std::mutex> g(h->mu);
    if (h->cur < 0 || !h->job) return VP9HIP_EINVAL;
    h->tr.start();
    int refs[3];
    for (int i = 0; i < 3; i++) {            // s->s.h.refidx -> the slots' device buffers
        refs[i] = h->intra ? -1 : h->slot[h->info.ref_slot[i] & 7];
        if (!h->intra && refs[i] < 0) { drop_job(h); h->cur = -1; return VP9HIP_EINVALIDDATA; }
    }
    Pend p;
    p.f = h->led.frame(h->cur, refs);
    p.job = std::move(h->job);
    for (int i = 0; i < 8; i++)              // vp9.c:1705-1711: slots of refreshrefmask
        if (h->info.refresh_mask & (1 << i)) h->slot[i] = h->cur;
    h->pend[p.f.out] = 1;
    for (int i = 0; i < 3; i++)
        if (refs[i] >= 0) h->inref[refs[i]]++;
    h->batch.push_back(std::move(p));
    if (out) fill_frame(h, h->cur, h->pts, out);          // shown or hidden: vp9.c's AVFrame of the frame
    const int shown = h->info.show_frame != 0;
    h->cur = -1;
    if ((int) h->batch.size() >= h->fp.async_depth) {
        h->full.push_back(std::move(h->batch));
        h->batch.clear();
    }
    h->tr.stop(T_END);
    const int r = pump(h);
    if (r < 0) return r;
    return shown;
}

extern "C" int vp9hip_hwaccel_show_existing(vp9hip_hwaccel *h, int slot, int64_t pts, vp9hip_hwframe *out)
{
    if (!h || !out || slot < 0 || slot > 7) return VP9HIP_EINVAL;
    std::lock_guard<std::mutex> g(h->mu);
    if (h->slot[slot] < 0) return VP9HIP_EINVALIDDATA;   // "Requested reference ... not available"
    fill_frame(h, h->slot[slot], pts, out);
    return 0;
}

// Launch the frame's batch if it has not been launched yet (and the filled batches before
// it; the batch being filled only when the frame is in it, so batches stay whole); 0 or
// the frame's error known so far.
static int launch_for(vp9hip_hwaccel *h, int b)
{
    int err = 0;
    while (h->pend[b] && !h->full.empty()) {
        const int r = submit_list(h, h->full.front());
        h->full.pop_front();
        if (r < 0 && !err) err = r;
    }
    if (h->pend[b]) {
        const int r = submit_list(h, h->batch);
        if (r < 0 && !err) err = r;
    }
    if (err < 0) return err;
    return h->led.error(h->led.holder(b));
}

static int hwframe_sync_l(vp9hip_hwaccel *h, const vp9hip_hwframe *f)
{
    if (f->buf < 0 || f->buf >= h->fp.initial_pool_size || !nrefs(h, f->buf)) return VP9HIP_EINVAL;
    int r = launch_for(h, f->buf);
    if (r < 0) return r;
    const uint64_t b = h->led.seq_of(f->buf);
    if (!b) return 0;                                    // written before any batch (never decoded)
    h->tr.start();
    // the frame's batch and every batch before it (an older batch of its slot was drained
    // and checked before the slot was reused)
    if (h->led.unchecked(b) >= 0 && (r = h->led.check_through(h->gpu, b)) < 0) return r;
    h->tr.stop(T_SYNC_WAIT);
    return h->led.error(h->led.holder(f->buf));
}

extern "C" int vp9hip_hwframe_sync(vp9hip_hwaccel *h, const vp9hip_hwframe *f)
{
    if (!h || !f) return VP9HIP_EINVAL;
    std::lock_guard<std::mutex> g(h->mu);
    return hwframe_sync_l(h, f);
}

extern "C" int vp9hip_hwframe_ready(vp9hip_hwaccel *h, const vp9hip_hwframe *f, void *stream)
{
    if (!h || !f) return VP9HIP_EINVAL;
    std::lock_guard<std::mutex> g(h->mu);
    if (f->buf < 0 || f->buf >= h->fp.initial_pool_size || !nrefs(h, f->buf)) return VP9HIP_EINVAL;
    int r = launch_for(h, f->buf);
    if (r < 0) return r;
    const uint64_t b = h->led.seq_of(f->buf);
    if (!b) return 0;
    // the slot's last run is this batch or a later one (which follows it on the slot's
    // stream): ordering the consumer's stream after it orders it after the frame
    return vp9hip_slot_stream_wait(h->gpu, vp9hip::Ledger::slot_of(b), stream);
}

extern "C" int vp9hip_hwaccel_uninit(vp9hip_hwaccel *h)
{
    if (!h) return 0;
    if (h->tr.on) {
        fprintf(stderr, "vp9hip hwaccel trace: %ld batches, %ld frames; host ms:", h->tr.batches, h->tr.frames);
        for (int k = 0; k < T_N; k++) fprintf(stderr, " [%s] %.1f", tname[k], h->tr.ms[k]);
        fprintf(stderr, "\n");
    }
    {
        std::lock_guard<std::mutex> g(h->mu);
        if (h->pool) drop_job(h);
        if (h->gpu) {
            submit(h);                       // frames handed out may still be read by the caller
            vp9hip_sync(h->gpu);
        }
    }
    h->batch.clear();
    h->full.clear();
    h->pool.reset();
    h->chain.reset();
    if (h->gpu) vp9hip_close(h->gpu);
    delete h;
    return 0;
}

extern "C" void vp9hip_hwaccel_flush(vp9hip_hwaccel *h)
{
    if (!h) return;
    std::lock_guard<std::mutex> g(h->mu);
    drop_job(h);
    h->cur = -1;
    // frames already handed out stay valid: their batch runs, then the slots are dropped
    if (submit(h) >= 0) h->led.check_through(h->gpu, ~0ull);
    h->batch.clear();
    h->full.clear();
    for (int i = 0; i < 8; i++) h->slot[i] = -1;
    h->chain.reset();                        // the next frame must be a keyframe
    vp9hip_sync(h->gpu);
}

extern "C" int vp9hip_hwaccel_last_header(const vp9hip_hwaccel *h, vp9h_frame_info *info)
{
    if (!h || !info) return VP9HIP_EINVAL;
    std::lock_guard<std::mutex> g(h->mu);
    *info = h->info;
    return 0;
}

extern "C" int vp9hip_hwframe_transfer(vp9hip_hwaccel *h, const vp9hip_hwframe *src, uint8_t *const dst[3],
                                       const ptrdiff_t dst_linesize[3])
{
    if (!h || !src || !dst || !dst_linesize) return VP9HIP_EINVAL;
    std::lock_guard<std::mutex> g(h->mu);
    const int r = hwframe_sync_l(h, src);
    if (r < 0) return r;
    return vp9hip_download_frame(h->gpu, src->buf, dst, dst_linesize);
}

extern "C" int vp9hip_hwframe_unref(vp9hip_hwaccel *h, vp9hip_hwframe *f)
{
    if (!h || !f) return VP9HIP_EINVAL;
    {
        std::lock_guard<std::mutex> g(h->mu);
        if (f->buf < 0 || f->buf >= h->fp.initial_pool_size || h->refs[f->buf] <= 0) return VP9HIP_EINVAL;
        h->refs[f->buf]--;
    }
    memset(f, 0, sizeof(*f));
    f->buf = -1;
    return 0;
}

extern "C" int vp9hip_hwframe_ref(vp9hip_hwaccel *h, const vp9hip_hwframe *src, vp9hip_hwframe *dst)
{
    if (!h || !src || !dst) return VP9HIP_EINVAL;
    std::lock_guard<std::mutex> g(h->mu);
    if (src->buf < 0 || src->buf >= h->fp.initial_pool_size || h->refs[src->buf] <= 0) return VP9HIP_EINVAL;
    *dst = *src;
    h->refs[src->buf]++;
    return 0;
}
