// Batches in flight and the outcome of every frame, for the two decode front ends over one
// device context: the bitstream decoder (vp9hip_decoder.cpp) and the FFHWAccel adapter
// (vp9hip_hwaccel.cpp). Internal to libvp9hip.
//
// Batches launch in decode order, round-robin over VP9HIP_PIPELINE_SLOTS batch slots: batch
// b runs in slot (b - 1) % NS, and slot s is staged again only after its previous batch was
// checked (vp9hip_sync_slot), so NS batches are in flight. Checks run in launch order, so a
// frame's producers (the frames whose output it reads, always earlier in decode order) have
// their final outcome when it is checked.
//
// Errors are per frame, as in the reference, where vp9_decode_frame fails only the corrupt
// frame's packet (AVERROR_INVALIDDATA, /root/reference/libavcodec/vp9.c:1827-1832,
// vp9recon.c:661-668) and the frames around it decode. A frame fails when
//   - its entropy decode failed (the front end reports it: fail());
//   - the device planner or the staging checks rejected its packet
//     (vp9hip_batch_frame_status; the other frames of the batch are reconstructed, or
//     staged again without it when the batch stopped before its pixel launches);
//   - its batch failed as a whole (VP9HIP_EBUG: a loop-filter hand-off gave up);
//   - a frame it reads failed (AVERROR_INVALIDDATA): the front ends map reference slots to
//     buffers before the decode outcome is known (the adapter is asynchronous), so a frame
//     predicted from a failed one has no valid reference.
#ifndef VP9HIP_PIPELINE_H
#define VP9HIP_PIPELINE_H

#include <cstdint>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/vp9hip.h"

namespace vp9hip {

// One frame given to the device in decode order: its output buffer, the buffers it reads
// (-1: none), its id (from 1) and the ids of the frames whose output it reads (0: none).
struct LFrame {
    int out = -1;
    int refs[3] = { -1, -1, -1 };
    uint64_t id = 0;
    uint64_t src[3] = { 0, 0, 0 };
};

class Ledger {
public:
    static constexpr int NS = VP9HIP_PIPELINE_SLOTS;
    static_assert(NS >= 1 && NS <= VP9HIP_MAX_SLOTS, "pipeline slots are batch slots");

    Ledger() { reset(); }

    void reset_buffers(int nbufs)
    {
        buf_id.assign(nbufs, 0);
        buf_seq.assign(nbufs, 0);
    }

    // A new frame in decode order writing `out` and reading `refs` (null or -1: intra).
    LFrame frame(int out, const int *refs)
    {
        LFrame f;
        f.out = out;
        f.id = next_id++;
        for (int r = 0; r < 3; r++) {
            f.refs[r] = refs ? refs[r] : -1;
            f.src[r] = f.refs[r] >= 0 ? buf_id[f.refs[r]] : 0;
        }
        buf_id[out] = f.id;
        return f;
    }

    uint64_t holder(int buf) const { return buf_id[buf]; }          // the frame `buf` holds
    uint64_t seq_of(int buf) const { return buf_seq[buf]; }         // the batch that wrote it (0: none)
    uint64_t last() const { return launched; }
    static int slot_of(uint64_t seq) { return (int) ((seq - 1) % NS); }

    int error(uint64_t id) const
    {
        const auto it = bad.find(id);
        return it == bad.end() ? 0 : it->second;
    }
    void fail(const LFrame &f, int e)
    {
        if (f.id) bad.emplace(f.id, e);      // the first error of a frame stays
    }

    // Slot of batch `seq` if it is launched and not yet checked, else -1.
    int unchecked(uint64_t seq) const
    {
        if (!seq) return -1;
        const int s = slot_of(seq);
        return seq_[s] == seq && !checked_[s] ? s : -1;
    }

    // Check every launched batch up to batch `seq` (all when seq = ~0), oldest first. 0, or
    // a failure of the device context itself (the batch stays unchecked).
    int check_through(vp9hip_ctx *ctx, uint64_t seq)
    {
        for (;;) {
            int s = -1;
            for (int k = 0; k < NS; k++)
                if (!checked_[k] && seq_[k] <= seq && (s < 0 || seq_[k] < seq_[s])) s = k;
            if (s < 0) return 0;
            if (const int r = check(ctx, s)) return r;
        }
    }

    // Stage and run one batch in the next slot: pk[i] / fr[i] in decode order; a frame with
    // pk[i] == null, or one already failed, is not staged. Frames the planner or the staging
    // checks reject fail, the rest are staged again until the batch runs. Returns 0, or a
    // failure of the device context (every frame not launched then fails with it).
    int launch(vp9hip_ctx *ctx, const std::vector<const vp9h_frame *> &pk, const std::vector<LFrame> &fr)
    {
        const int s = (int) (launched % NS);
        if (const int r = check_through(ctx, seq_[s])) {         // before the staging resets its words
            for (const LFrame &f : fr) fail(f, r);
            return r;
        }
        std::vector<int> keep;
        for (size_t i = 0; i < fr.size(); i++) {
            if (!pk[i] || error(fr[i].id)) continue;
            if (reads_failed(fr[i])) { fail(fr[i], VP9HIP_EINVALIDDATA); continue; }
            keep.push_back((int) i);
        }
        int r = 0;
        while (!keep.empty()) {
            const int n = (int) keep.size();
            std::vector<vp9h_frame> p(n);
            std::vector<int> outs(n), refs(3 * n);
            for (int k = 0; k < n; k++) {
                const LFrame &f = fr[keep[k]];
                p[k] = *pk[keep[k]];
                outs[k] = f.out;
                for (int j = 0; j < 3; j++) refs[3 * k + j] = f.refs[j] >= 0 ? f.refs[j] : 0;
            }
            r = vp9hip_set_batch_slot(ctx, s);
            if (r >= 0) r = vp9hip_stage_batch_refs(ctx, p.data(), n, outs.data(), refs.data());   // copies the packets
            if (r >= 0) r = vp9hip_run_batch(ctx);
            if (r != VP9HIP_EINVALIDDATA) break;
            // rejected frames fail; the valid ones (and not their dependents) go again
            std::vector<int> st(n, VP9HIP_EINVALIDDATA);
            if (vp9hip_batch_frame_status(ctx, s, st.data(), n) != n) st.assign(n, VP9HIP_EINVALIDDATA);
            std::vector<int> next;
            bool named = false;
            for (int k = 0; k < n; k++) {
                const LFrame &f = fr[keep[k]];
                if (st[k] == VP9HIP_EINVALIDDATA) { fail(f, st[k]); named = true; }
                else if (reads_failed(f)) fail(f, VP9HIP_EINVALIDDATA);
                else next.push_back(keep[k]);
            }
            if (!named) {                    // no frame named: the whole batch fails
                for (int i : next) fail(fr[i], VP9HIP_EINVALIDDATA);
                next.clear();
            }
            keep.swap(next);
            r = 0;
        }
        if (r < 0) {
            for (int i : keep) fail(fr[i], r);
            return r;
        }
        if (keep.empty()) return 0;           // nothing left to run
        launched++;
        seq_[s] = launched;
        checked_[s] = false;
        frames_[s].clear();
        for (int i : keep) {
            frames_[s].push_back(fr[i]);
            buf_seq[fr[i].out] = launched;
        }
        return 0;
    }

    // Forget the batches in flight (vp9hip_flush dropped them) and every outcome.
    void reset()
    {
        for (int s = 0; s < NS; s++) { checked_[s] = true; frames_[s].clear(); }
        bad.clear();
    }

private:
    bool reads_failed(const LFrame &f) const
    {
        for (int r = 0; r < 3; r++)
            if (f.src[r] && bad.count(f.src[r])) return true;
        return false;
    }

    // Wait for slot s's batch and record its frames' outcomes.
    int check(vp9hip_ctx *ctx, int s)
    {
        const int r = vp9hip_sync_slot(ctx, s);
        if (r < 0 && r != VP9HIP_EBUG && r != VP9HIP_EINVALIDDATA) return r;
        std::vector<LFrame> &F = frames_[s];
        const int n = (int) F.size();
        std::vector<int> st(n, 0);
        if (r == VP9HIP_EBUG) st.assign(n, VP9HIP_EBUG);
        else if (r == VP9HIP_EINVALIDDATA && vp9hip_batch_frame_status(ctx, s, st.data(), n) != n)
            st.assign(n, VP9HIP_EINVALIDDATA);
        for (int i = 0; i < n; i++) {
            int e = st[i] < 0 ? st[i] : 0;
            if (e == VP9HIP_EAGAIN) e = VP9HIP_EINVALIDDATA;    // not run (cannot happen after a launch)
            if (!e && reads_failed(F[i])) e = VP9HIP_EINVALIDDATA;
            if (e) fail(F[i], e);
        }
        checked_[s] = true;
        F.clear();
        prune();
        return 0;
    }

    // Outcomes nothing can ask for any more: ids no buffer holds and no frame in flight reads.
    void prune()
    {
        if (bad.size() < 64) return;
        std::unordered_set<uint64_t> live(buf_id.begin(), buf_id.end());
        for (int s = 0; s < NS; s++)
            for (const LFrame &f : frames_[s]) {
                live.insert(f.id);
                for (uint64_t x : f.src) live.insert(x);
            }
        for (auto it = bad.begin(); it != bad.end();) it = live.count(it->first) ? std::next(it) : bad.erase(it);
    }

    uint64_t next_id = 1, launched = 0;
    uint64_t seq_[NS] = {};
    bool checked_[NS];
    std::vector<LFrame> frames_[NS];
    std::unordered_map<uint64_t, int> bad;
    std::vector<uint64_t> buf_id, buf_seq;   // per buffer: the frame it holds, the batch that wrote it
};

} // namespace vp9hip

#endif
