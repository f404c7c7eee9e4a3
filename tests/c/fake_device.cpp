// TEST INFRASTRUCTURE: a CPU stand-in for the device half of libvp9hip's C ABI
// (include/vp9hip.h: open / configure / batch slots / stage / run / sync / download /
// frame_device), so the FFHWAccel adapter (csrc/vp9hip_hwaccel.cpp), the host parse and the
// call-order harness (tests/c/hwaccel_harness.c) can run without a GPU: under ASan / UBSan /
// TSan (make -C ffmpeg-hybrid_amd/csrc sanitize, tools/sanitize.sh) and in the CPU test suite
// (tests/test_sanitize.py). Frames are reconstructed by the oracle (oracle/vp9_oracle.c), the
// checker, on one worker thread that runs the launched batches in order, asynchronously to
// the caller, like a device queue; sync / sync_slot / download wait for it. Never part of the
// product: the library build does not compile this file.
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/vp9hip.h"
#include "../../oracle/vp9_oracle.h"

namespace {
struct Pkt {                                   // a deep copy of a staged vp9h_frame
    vp9h_frame f;
    std::vector<vp9h_block> blocks;
    std::vector<uint16_t> eobs;
    std::vector<uint8_t> coefs;
};
struct Batch {
    std::vector<Pkt> pk;
    std::vector<int> out, refs;
    std::vector<std::pair<int, int>> refwh;     // visible sizes of the references, as staged
    uint64_t seq = 0;
    int slot = 0;
};
}

struct vp9hip_ctx {
    int w = 0, h = 0, bpp = 8, ssh = 1, ssv = 1, bypp = 1;
    int pw[2] = { 0, 0 }, ph[2] = { 0, 0 };         // padded plane sizes (luma, chroma), pixels
    std::vector<std::vector<uint8_t>> bufs;
    std::vector<std::pair<int, int>> wh;
    int slot = 0;
    Batch staged[VP9HIP_MAX_SLOTS];
    bool have[VP9HIP_MAX_SLOTS] = {};
    uint64_t slot_last[VP9HIP_MAX_SLOTS] = {};     // sequence of each slot's last launch
    int serr[VP9HIP_MAX_SLOTS] = {};               // per slot: error of its last run
    std::vector<int> fstat[VP9HIP_MAX_SLOTS];      // per slot: per-frame outcome of its last run
    // the worker ("device queue")
    std::mutex mu;
    std::condition_variable cv, cv_done;
    std::deque<Batch> q;
    uint64_t launched = 0, finished = 0;
    bool stop = false;
    std::thread worker;
};

static void planes_of(vp9hip_ctx *c, int b, vp9o_planes *p, std::pair<int, int> wh)
{
    uint8_t *base = c->bufs[(size_t) b].data();
    p->data[0] = base;
    p->data[1] = base + (size_t) c->pw[0] * c->ph[0] * c->bypp;
    p->data[2] = (uint8_t *) p->data[1] + (size_t) c->pw[1] * c->ph[1] * c->bypp;
    p->stride[0] = c->pw[0];
    p->stride[1] = p->stride[2] = c->pw[1];
    p->w = wh.first;
    p->h = wh.second;
}

static void run_worker(vp9hip_ctx *c)
{
    std::unique_lock<std::mutex> lk(c->mu);
    for (;;) {
        c->cv.wait(lk, [&] { return c->stop || !c->q.empty(); });
        if (c->q.empty()) return;
        Batch b = std::move(c->q.front());
        c->q.pop_front();
        lk.unlock();
        int e = 0;
        std::vector<int> fst(b.pk.size(), 0);
        for (size_t i = 0; i < b.pk.size(); i++) {
            const vp9h_frame &f = b.pk[i].f;
            const int o = b.out[i];
            vp9o_planes cur, refs[3];
            planes_of(c, o, &cur, std::make_pair((int) f.width, (int) f.height));
            const bool intra = f.keyframe || f.intraonly;
            for (int r = 0; r < 3; r++) planes_of(c, b.refs[3 * i + r], &refs[r], b.refwh[3 * i + r]);
            // FAKE_NO_RECON=1: no reconstruction (host-side timing of the adapter only)
            static const bool norecon = getenv("FAKE_NO_RECON") && atoi(getenv("FAKE_NO_RECON"));
            const int fe = norecon ? 0 : vp9o_decode_frame(&f, &cur, intra ? nullptr : refs);
            if (fe) { fst[i] = VP9HIP_EINVALIDDATA; e = VP9HIP_EINVALIDDATA; }   // that frame only
        }
        lk.lock();
        c->serr[b.slot] = e;
        c->fstat[b.slot] = fst;
        c->finished = b.seq;
        c->cv_done.notify_all();
    }
}

static void wait_seq(vp9hip_ctx *c, uint64_t seq)
{
    std::unique_lock<std::mutex> lk(c->mu);
    c->cv_done.wait(lk, [&] { return c->finished >= seq; });
}

extern "C" {
void vp9hip_test_hooks(int, uint32_t) {}
int vp9hip_open(int device, vp9hip_ctx **out)
{
    if (!out || device != 0) return VP9HIP_EINVAL;
    vp9hip_ctx *c = new vp9hip_ctx;
    c->worker = std::thread(run_worker, c);
    *out = c;
    return 0;
}

void vp9hip_close(vp9hip_ctx *c)
{
    if (!c) return;
    {
        std::lock_guard<std::mutex> lk(c->mu);
        c->stop = true;
    }
    c->cv.notify_all();
    c->worker.join();
    delete c;
}

int vp9hip_configure(vp9hip_ctx *c, int width, int height, int bpp, int ss_h, int ss_v, int nbufs)
{
    if (!c || width <= 0 || height <= 0 || nbufs <= 0) return VP9HIP_EINVAL;
    wait_seq(c, c->launched);
    c->w = width; c->h = height; c->bpp = bpp; c->ssh = ss_h; c->ssv = ss_v; c->bypp = bpp > 8 ? 2 : 1;
    c->pw[0] = (width + 63) & ~63; c->ph[0] = (height + 63) & ~63;
    c->pw[1] = c->pw[0] >> ss_h; c->ph[1] = c->ph[0] >> ss_v;
    const size_t bytes = ((size_t) c->pw[0] * c->ph[0] + 2 * (size_t) c->pw[1] * c->ph[1]) * c->bypp;
    c->bufs.assign((size_t) nbufs, std::vector<uint8_t>(bytes, 0));
    c->wh.assign((size_t) nbufs, std::make_pair(width, height));
    return 0;
}

int vp9hip_set_timing(vp9hip_ctx *c, int) { return c ? 0 : VP9HIP_EINVAL; }
int vp9hip_set_graph(vp9hip_ctx *c, int) { return c ? 0 : VP9HIP_EINVAL; }

int vp9hip_set_batch_slot(vp9hip_ctx *c, int slot)
{
    if (!c || slot < 0 || slot >= VP9HIP_MAX_SLOTS) return VP9HIP_EINVAL;
    c->slot = slot;
    return 0;
}

int vp9hip_stage_batch_refs(vp9hip_ctx *c, const vp9h_frame *pkts, int n, const int *out_bufs, const int *ref_bufs)
{
    if (!c || !pkts || n <= 0 || !out_bufs || c->bufs.empty()) return VP9HIP_EINVAL;
    wait_seq(c, c->slot_last[c->slot]);            // the slot's previous batch may still read its copies
    Batch &b = c->staged[c->slot];
    b.pk.assign((size_t) n, Pkt());
    b.out.assign(out_bufs, out_bufs + n);
    b.refs.assign((size_t) 3 * n, 0);
    b.refwh.assign((size_t) 3 * n, std::make_pair(0, 0));
    for (int i = 0; i < n; i++) {
        const vp9h_frame &f = pkts[i];
        if (out_bufs[i] < 0 || out_bufs[i] >= (int) c->bufs.size()) return VP9HIP_EINVAL;
        if (f.width > c->w || f.height > c->h || f.bpp != c->bpp) return VP9HIP_EINVAL;
        Pkt &p = b.pk[(size_t) i];
        p.f = f;
        p.blocks.assign(f.blocks, f.blocks + f.nblocks);
        p.eobs.assign(f.eobs, f.eobs + f.neobs);
        const size_t cb = (size_t) f.ncoefs * (f.bpp > 8 ? 4 : 2);
        p.coefs.assign((const uint8_t *) f.coefs, (const uint8_t *) f.coefs + cb);
        p.f.blocks = p.blocks.data();
        p.f.eobs = p.eobs.data();
        p.f.coefs = p.coefs.data();
        c->wh[(size_t) out_bufs[i]] = std::make_pair((int) f.width, (int) f.height);
        for (int r = 0; r < 3; r++) {
            const int rb = ref_bufs ? ref_bufs[3 * i + r] : 0;
            if (rb < 0 || rb >= (int) c->bufs.size()) return VP9HIP_EINVAL;
            b.refs[(size_t) 3 * i + r] = rb;
            b.refwh[(size_t) 3 * i + r] = c->wh[(size_t) rb];   // before this batch's own outputs
        }
    }
    c->have[c->slot] = true;
    return 0;
}

int vp9hip_run_batch(vp9hip_ctx *c)
{
    if (!c || !c->have[c->slot]) return VP9HIP_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    Batch b = c->staged[c->slot];                  // the slot keeps its staging for reruns
    for (Pkt &p : b.pk) {                          // the copy's arrays are its own
        p.f.blocks = p.blocks.data();
        p.f.eobs = p.eobs.data();
        p.f.coefs = p.coefs.data();
    }
    b.seq = ++c->launched;
    b.slot = c->slot;
    c->serr[c->slot] = 0;
    c->fstat[c->slot].assign(b.pk.size(), 0);
    c->slot_last[c->slot] = b.seq;
    c->q.push_back(std::move(b));
    c->cv.notify_one();
    return 0;
}

int vp9hip_sync_slot(vp9hip_ctx *c, int slot)
{
    if (!c || slot < 0 || slot >= VP9HIP_MAX_SLOTS) return VP9HIP_EINVAL;
    wait_seq(c, c->slot_last[slot]);
    std::lock_guard<std::mutex> lk(c->mu);
    return c->serr[slot];
}

int vp9hip_batch_frame_status(vp9hip_ctx *c, int slot, int *status, int cap)
{
    if (!c || slot < 0 || slot >= VP9HIP_MAX_SLOTS || cap < 0 || (cap > 0 && !status)) return VP9HIP_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    const int n = (int) c->fstat[slot].size();
    for (int i = 0; i < n && i < cap; i++) status[i] = c->fstat[slot][i];
    return n;
}

int vp9hip_sync(vp9hip_ctx *c)
{
    if (!c) return VP9HIP_EINVAL;
    wait_seq(c, c->launched);
    std::lock_guard<std::mutex> lk(c->mu);
    for (int k = 0; k < VP9HIP_MAX_SLOTS; k++)
        if (c->serr[k]) return c->serr[k];
    return 0;
}

int vp9hip_slot_stream_wait(vp9hip_ctx *c, int slot, void *)
{
    // no streams on the CPU: the consumer's "stream" is the host, so wait here
    return vp9hip_sync_slot(c, slot);
}

int vp9hip_frame_device(vp9hip_ctx *c, int buf, void *planes[3], ptrdiff_t linesize[3], int *width, int *height,
                        void **stream)
{
    if (!c || buf < 0 || buf >= (int) c->bufs.size() || !planes || !linesize) return VP9HIP_EINVAL;
    vp9o_planes p;
    planes_of(c, buf, &p, c->wh[(size_t) buf]);
    for (int i = 0; i < 3; i++) {
        planes[i] = p.data[i];
        linesize[i] = p.stride[i] * c->bypp;
    }
    if (width) *width = p.w;
    if (height) *height = p.h;
    if (stream) *stream = nullptr;
    return 0;
}

int vp9hip_download_frame(vp9hip_ctx *c, int buf, uint8_t *const planes[3], const ptrdiff_t linesize[3])
{
    if (!c || buf < 0 || buf >= (int) c->bufs.size() || !planes) return VP9HIP_EINVAL;
    wait_seq(c, c->launched);
    vp9o_planes p;
    planes_of(c, buf, &p, c->wh[(size_t) buf]);
    for (int i = 0; i < 3; i++) {
        const int pw = i ? (p.w + c->ssh) >> c->ssh : p.w, ph = i ? (p.h + c->ssv) >> c->ssv : p.h;
        for (int y = 0; y < ph; y++)
            memcpy(planes[i] + (ptrdiff_t) y * linesize[i], (const uint8_t *) p.data[i] + (size_t) y * p.stride[i] * c->bypp,
                   (size_t) pw * c->bypp);
    }
    return 0;
}
}
