// Host parse pool shared by the decoder loop (vp9hip_decoder.cpp) and the FFHWAccel
// adapter (vp9hip_hwaccel.cpp): the entropy decode of frames into pass-1 packets on a pool
// of threads, ahead of the thread that stages them for the GPU.
//
// Frames of one parse chain parse on one vp9h_stream. A keyframe starts a new chain on a
// fresh vp9h_stream, because its parse depends on no earlier frame (vp9h_frame_type);
// keyframe-only streams therefore parse frame-parallel and GOP streams GOP-parallel.
// Inside a chain the frames are pipelined as the reference's frame threads pipeline them
// (ff_thread_finish_setup after the headers, vp9.c:1752-1754): a frame's headers
// (vp9h_stream_decode_begin) parse in chain order, and its tiles (vp9h_stream_decode_finish)
// are a task of their own that any worker may run while the chain goes on to the next
// frame's headers; the tiles wait per SB row for the previous frame's MV pairs and
// segmentation map (vp9mvs.c:177-178, vp9block.c:116-117). A frame whose tiles adapt the
// probabilities the next headers read (refresh_frame_context without frame_parallel) holds
// its chain until its tiles are done. Tile tasks start in the order their headers parsed
// (one FIFO), so a waiting tile task always waits on one that runs: no deadlock on any
// number of workers. A frame's tiles also use tile-column threads
// (vp9h_stream_decode_finish's `threads`: decode_tiles_mt, vp9.c:1441-1520), the idle
// workers' share.
#pragma once

#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/vp9hip.h"

namespace vp9hip {

struct ParseJob;

struct Chain {                         // one parse state: its frames' headers parse in order
    vp9h_stream *st = nullptr;
    std::deque<ParseJob *> q;          // queued, headers not parsed
    bool scheduled = false;            // on the run queue or having headers parsed by a worker
    ParseJob *held = nullptr;          // a frame whose tiles the next headers wait for
    ~Chain() { if (st) vp9h_stream_close(st); }
};

struct ParseJob {
    std::vector<uint8_t> data;
    int64_t pts = 0;
    std::shared_ptr<Chain> chain;
    vp9h_frame pkt;
    vp9h_frame_info info;
    int ret = 0;
    bool done = false;
    vp9h_pending *pend = nullptr;      // headers parsed, tiles to do
    ParseJob() { memset(&pkt, 0, sizeof(pkt)); memset(&info, 0, sizeof(info)); }
    ~ParseJob() { vp9h_pending_free(pend); vp9h_frame_free(&pkt); }     // a consumer that takes pkt zeroes it
};

class ParsePool {
public:
    explicit ParsePool(int threads) : nthreads_(threads)
    {
        workers_.reserve((size_t) threads);
        for (int t = 0; t < threads; t++) workers_.emplace_back([this] { run(); });
    }
    ~ParsePool()
    {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_work_.notify_all();
        for (auto &t : workers_) t.join();
    }
    int threads() const { return nthreads_; }

    // A chain on a fresh stream (a keyframe's), or nullptr with *err set.
    static std::shared_ptr<Chain> new_chain(int *err)
    {
        std::shared_ptr<Chain> c = std::make_shared<Chain>();
        *err = vp9h_stream_open(&c->st);
        return *err < 0 ? nullptr : c;
    }

    // Queue j (j->chain set) behind the earlier frames of its chain; without workers it
    // parses now, on the caller's thread.
    void enqueue(ParseJob *j)
    {
        if (!nthreads_) {
            j->ret = vp9h_stream_decode(j->chain->st, j->data.data(), j->data.size(), &j->pkt, &j->info);
            j->done = true;
            return;
        }
        std::lock_guard<std::mutex> lk(mu_);
        Chain *c = j->chain.get();
        c->q.push_back(j);
        schedule(j->chain);
        cv_work_.notify_one();
    }
    bool done(ParseJob *j)
    {
        if (!nthreads_) return j->done;
        std::lock_guard<std::mutex> lk(mu_);
        return j->done;
    }
    void wait(ParseJob *j)
    {
        if (!nthreads_) return;
        std::unique_lock<std::mutex> lk(mu_);
        cv_done_.wait(lk, [&] { return j->done; });
    }

private:
    // (mu_ held) a chain with queued headers, not held by a frame's tiles, goes on the run queue
    void schedule(const std::shared_ptr<Chain> &c)
    {
        if (!c->scheduled && !c->held && !c->q.empty()) {
            c->scheduled = true;
            runq_.push_back(c);
        }
    }
    void finish_job(ParseJob *j, int ret)            // (mu_ held)
    {
        j->ret = ret;
        j->done = true;
        cv_done_.notify_all();
        Chain *c = j->chain.get();
        if (c->held == j) {
            c->held = nullptr;
            schedule(j->chain);
            cv_work_.notify_one();
        }
    }
    void run()
    {
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            cv_work_.wait(lk, [&] { return stop_ || !tiles_.empty() || !runq_.empty(); });
            if (stop_) return;
            if (!tiles_.empty()) {                          // tiles first, in header order
                ParseJob *j = tiles_.front();
                tiles_.pop_front();
                active_++;
                const int share = std::max(1, std::min(16, nthreads_ / std::max<int>(1, active_ + (int) tiles_.size())));
                vp9h_pending *p = j->pend;
                j->pend = nullptr;
                lk.unlock();
                const int r = vp9h_stream_decode_finish(p, share, &j->pkt);
                lk.lock();
                active_--;
                finish_job(j, r);
                continue;
            }
            std::shared_ptr<Chain> c = runq_.front();
            runq_.pop_front();
            while (!c->q.empty() && !c->held) {            // the chain's headers, in order
                ParseJob *j = c->q.front();
                c->q.pop_front();
                lk.unlock();
                vp9h_pending *p = nullptr;
                int serial = 0;
                const int r = vp9h_stream_decode_begin(c->st, j->data.data(), j->data.size(), &p, &j->info, &serial);
                lk.lock();
                if (r < 0 || !p) {                          // an error, or show_existing_frame
                    finish_job(j, r);
                    continue;
                }
                j->pend = p;
                if (serial) c->held = j;
                tiles_.push_back(j);
                cv_work_.notify_one();
            }
            c->scheduled = false;
            schedule(c);                                    // frames queued meanwhile
            if (c->scheduled) cv_work_.notify_one();
        }
    }

    const int nthreads_;
    std::vector<std::thread> workers_;
    std::mutex mu_;
    std::condition_variable cv_work_, cv_done_;
    std::deque<std::shared_ptr<Chain>> runq_;
    std::deque<ParseJob *> tiles_;                          // frames whose headers parsed, in that order
    int active_ = 0;                                        // tile tasks being run
    bool stop_ = false;
};

} // namespace vp9hip
