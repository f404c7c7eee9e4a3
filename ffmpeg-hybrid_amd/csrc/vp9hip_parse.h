// Host parse pool shared by the decoder loop (vp9hip_decoder.cpp) and the FFHWAccel
// adapter (vp9hip_hwaccel.cpp): the entropy decode of frames into pass-1 packets on a pool
// of threads, ahead of the thread that stages them for the GPU.
//
// Frames of one parse chain parse in order on one vp9h_stream. A keyframe starts a new
// chain on a fresh vp9h_stream, because its parse depends on no earlier frame
// (vp9h_frame_type); keyframe-only streams therefore parse frame-parallel and GOP streams
// GOP-parallel, the freedom the reference's frame threads get from ff_thread_finish_setup
// after the header (vp9.c:1736). A chain that parses alone gets the idle threads' share
// for its frames' tile columns (vp9h_stream_set_threads: decode_tiles_mt, vp9.c:1441-1520).
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

struct Chain {                         // one parse state: its frames parse in order
    vp9h_stream *st = nullptr;
    std::deque<ParseJob *> q;          // queued, not started
    bool scheduled = false;            // on the run queue or being run by a worker
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
    ParseJob() { memset(&pkt, 0, sizeof(pkt)); memset(&info, 0, sizeof(info)); }
    ~ParseJob() { vp9h_frame_free(&pkt); }     // a consumer that takes pkt zeroes it
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
            parse(j, 1);
            j->done = true;
            return;
        }
        std::lock_guard<std::mutex> lk(mu_);
        Chain *c = j->chain.get();
        c->q.push_back(j);
        if (!c->scheduled) {
            c->scheduled = true;
            runq_.push_back(j->chain);
            cv_work_.notify_one();
        }
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
    static void parse(ParseJob *j, int tile_threads)
    {
        vp9h_stream_set_threads(j->chain->st, std::max(1, std::min(tile_threads, 16)));
        j->ret = vp9h_stream_decode(j->chain->st, j->data.data(), j->data.size(), &j->pkt, &j->info);
    }
    void run()
    {
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            cv_work_.wait(lk, [&] { return stop_ || !runq_.empty(); });
            if (stop_) return;
            std::shared_ptr<Chain> c = runq_.front();
            runq_.pop_front();
            active_++;
            while (!c->q.empty()) {                       // the chain's frames, in order
                ParseJob *j = c->q.front();
                c->q.pop_front();
                const int share = nthreads_ / std::max<int>(1, active_ + (int) runq_.size());
                lk.unlock();
                parse(j, share);
                lk.lock();
                j->done = true;
                cv_done_.notify_all();
            }
            active_--;
            c->scheduled = false;
        }
    }

    const int nthreads_;
    std::vector<std::thread> workers_;
    std::mutex mu_;
    std::condition_variable cv_work_, cv_done_;
    std::deque<std::shared_ptr<Chain>> runq_;
    int active_ = 0;                                      // chains being parsed by a worker
    bool stop_ = false;
};

} // namespace vp9hip
