// Host entropy-decode throughput of one GOP chain (measurement, not a test): a synthetic
// key + P stream encoded with vp9h_stream_encode, then parsed back
//   serial      vp9h_stream_decode frame after frame (1 tile thread)
//   tiles       the same on T tile-column threads (vp9h_stream_set_threads)
//   pipelined   the parse pool (csrc/vp9hip_parse.h): headers in order, each frame's tiles
//               a task of its own waiting per SB row for the previous frame (frame threads)
// and every packet compared with the serial parse. usage: parse_bench W H BPP LOG2TC N THREADS
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

#include "../../include/vp9hip.h"
#include "../../ffmpeg-hybrid_amd/csrc/vp9hip_parse.h"

typedef std::vector<uint8_t> Bytes;

static std::vector<Bytes> make_stream(int w, int h, int bpp, int log2tc, int n)
{
    std::vector<Bytes> out;
    vp9h_stream *enc = nullptr;
    if (vp9h_stream_open(&enc) < 0) return out;
    for (int i = 0; i < n; i++) {
        vp9h_synth_params sp;
        vp9hip_synth_defaults(&sp, w, h, bpp);
        sp.log2_tile_cols = log2tc;
        sp.inter = i > 0;
        sp.seed = 0x70a5e + (uint64_t) i;
        vp9h_frame f;
        memset(&f, 0, sizeof(f));
        if (vp9hip_synth_frame(&f, &sp) < 0) break;
        vp9h_enc_params ep;
        vp9h_enc_defaults(&ep);
        if (i) {
            const int prev = (i - 1) % 8;
            ep.ref_slot[0] = prev; ep.ref_slot[1] = 0; ep.ref_slot[2] = prev;
            ep.refresh_mask = 1 << (i % 8);
        }
        uint8_t *buf = nullptr;
        size_t sz = 0;
        const int r = vp9h_stream_encode(enc, &f, &ep, &buf, &sz, nullptr);
        vp9hip_synth_free(&f);
        if (r < 0) break;
        out.push_back(Bytes(buf, buf + sz));
        vp9h_buffer_free(buf);
    }
    vp9h_stream_close(enc);
    return out;
}

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

static bool same(const vp9h_frame &a, const vp9h_frame &b)
{
    return a.nblocks == b.nblocks && a.neobs == b.neobs && a.ncoefs == b.ncoefs &&
           !memcmp(a.blocks, b.blocks, a.nblocks * sizeof(vp9h_block)) && !memcmp(a.eobs, b.eobs, a.neobs * 2) &&
           !memcmp(a.coefs, b.coefs, a.ncoefs * (a.bpp > 8 ? 4 : 2));
}

int main(int argc, char **argv)
{
    if (argc < 7) { fprintf(stderr, "usage: parse_bench W H BPP LOG2TC N THREADS\n"); return 2; }
    const int w = atoi(argv[1]), h = atoi(argv[2]), bpp = atoi(argv[3]), l2 = atoi(argv[4]), n = atoi(argv[5]),
              nt = atoi(argv[6]);
    const std::vector<Bytes> s = make_stream(w, h, bpp, l2, n);
    if ((int) s.size() != n) { fprintf(stderr, "encode failed\n"); return 1; }
    std::vector<vp9h_frame> ref(n);
    int bad = 0;
    for (int mode = 0; mode < 3; mode++) {
        const double t0 = now();
        std::vector<vp9h_frame> got(n);
        if (mode < 2) {
            vp9h_stream *st = nullptr;
            vp9h_stream_open(&st);
            vp9h_stream_set_threads(st, mode ? nt : 1);
            for (int i = 0; i < n; i++) {
                vp9h_frame_info info;
                memset(&got[i], 0, sizeof(got[i]));
                if (vp9h_stream_decode(st, s[i].data(), s[i].size(), &got[i], &info) < 0) bad++;
            }
            vp9h_stream_close(st);
        } else {
            vp9hip::ParsePool pool(nt);
            int err = 0;
            std::shared_ptr<vp9hip::Chain> ch = vp9hip::ParsePool::new_chain(&err);
            std::vector<std::unique_ptr<vp9hip::ParseJob>> jobs;
            for (int i = 0; i < n; i++) {
                jobs.emplace_back(new vp9hip::ParseJob);
                jobs.back()->data = s[i];
                jobs.back()->chain = ch;
                pool.enqueue(jobs.back().get());
            }
            for (int i = 0; i < n; i++) {
                pool.wait(jobs[i].get());
                if (jobs[i]->ret < 0) bad++;
                got[i] = jobs[i]->pkt;
                memset(&jobs[i]->pkt, 0, sizeof(jobs[i]->pkt));
            }
        }
        const double dt = now() - t0;
        for (int i = 0; i < n; i++) {
            if (mode == 0) ref[i] = got[i];
            else { if (!same(ref[i], got[i])) bad++; vp9h_frame_free(&got[i]); }
        }
        printf("%-9s %dx%d@%d tiles %d, %d frames, %d threads: %.1f frames/s\n", mode == 0 ? "serial" : mode == 1 ? "tiles" : "pipelined",
               w, h, bpp, 1 << l2, n, mode ? nt : 1, n / dt);
    }
    for (auto &f : ref) vp9h_frame_free(&f);
    printf("mismatches %d\n", bad);
    return bad ? 1 : 0;
}
