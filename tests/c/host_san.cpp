// TEST INFRASTRUCTURE: the host side of libvp9hip (bitstream walker, tile-column threads,
// parse pool, IVF / WebM demuxers) driven for the sanitizer builds (make -C
// ffmpeg-hybrid_amd/csrc sanitize: ASan + UBSan, and TSan; tools/sanitize.sh runs them and
// keeps the logs under profiles/). Built from the same host sources as the library, without
// HIP. Exit status 0 = every check passed; the sanitizers report on stderr.
//
//   host_san [N_MUTATIONS] [FILE.ivf|FILE.webm ...]
//
// 1. streams (key + inter frames, 1-8 tile columns, backward adaptation on and off, 8/10-bit,
//    4:2:0 / 4:4:4) encoded by vp9h_stream_encode and parsed back: serially, with 2 / 3 / 8
//    tile-column threads (vp9h_stream_set_threads), frame-pipelined (vp9h_stream_decode_begin /
//    _finish: every frame's tiles on a thread of its own, started in order, waiting per SB row
//    for the previous frame's side buffers) and through the parse pool (csrc/vp9hip_parse.h,
//    4 workers, several chains at once, pipelined the same way): every packet equal byte for byte;
// 2. the same streams with bit flips and truncations: every frame parses or fails with an
//    error, nothing else;
// 3. each FILE demuxed (vp9h_ivf_* / vp9h_webm_*) and parsed, then N_MUTATIONS mutated copies
//    of it demuxed and parsed the same way.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <thread>
#include <vector>

#include "../../ffmpeg-hybrid_amd/csrc/vp9hip_parse.h"

typedef std::vector<uint8_t> Bytes;

static int fails = 0;
#define CHECK(c, ...) do { if (!(c)) { fails++; fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
    fprintf(stderr, __VA_ARGS__); fprintf(stderr, "\n"); } } while (0)

static uint64_t rng_state = 0x5a17c0de;
static uint32_t rnd()
{
    rng_state = rng_state * 6364136223846793005ull + 1442695040888963407ull;
    return (uint32_t) (rng_state >> 33);
}

struct Cfg { int w, h, bpp, ssh, ssv, log2tc, n, adapt; };

// key + n - 1 inter frames: frame i > 0 refreshes slot i % 8, LAST = ALTREF = the previous
// frame's slot, GOLDEN = slot 0 (tests/test_stream.py encode_stream)
static std::vector<Bytes> make_stream(const Cfg &c, uint64_t seed)
{
    std::vector<Bytes> out;
    vp9h_stream *enc = nullptr;
    if (vp9h_stream_open(&enc) < 0) return out;
    for (int i = 0; i < c.n; i++) {
        vp9h_synth_params sp;
        vp9hip_synth_defaults(&sp, c.w, c.h, c.bpp);
        sp.ss_h = c.ssh; sp.ss_v = c.ssv;
        sp.log2_tile_cols = c.log2tc;
        sp.inter = i > 0;
        sp.compound = i > 1;
        sp.seed = seed + (uint64_t) i;
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
        if (c.adapt) { ep.refresh_ctx = 1; ep.parallel = 0; }
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

// segmentation stream (the advisor's round-4 use-after-free): key with a coded map, an inter
// frame with its own map, two keeping it, then a hidden intra-only frame (its headers drop
// the kept map while the previous frame's tiles may still walk, frame-pipelined), an inter
// frame on it, an error-resilient frame, one updating the map. Without the counted segref
// reference ASan reports the use-after-free here (3 of 3 runs).
static std::vector<Bytes> make_seg_stream(int w, int h, int log2tc, uint64_t seed)
{
    std::vector<Bytes> out;
    vp9h_stream *enc = nullptr;
    if (vp9h_stream_open(&enc) < 0) return out;
    vp9h_seg_params sg;
    memset(&sg, 0, sizeof(sg));
    sg.enabled = 1; sg.update_map = 1; sg.update_data = 1; sg.nseg = 4;
    sg.q_en = 0x6; sg.q[1] = 8; sg.q[2] = -12;
    sg.lf_en = 0xb; sg.lf[0] = 3; sg.lf[2] = -5; sg.lf[3] = 10;
    sg.lf_delta_update = 1; sg.lf_ref[0] = 2; sg.lf_ref[2] = -2; sg.lf_ref[3] = -1; sg.lf_mode[0] = 1; sg.lf_mode[1] = -1;
    struct F { int inter, intraonly, update_map, temporal, q_en, errres, refresh, ref; };
    // (a frame keeps the map only after a frame that did not update it: frame 3 reads frame
    // 1's map through its own reference while frame 4's headers drop the stream's)
    static const F fs[] = { { 0, 0, 1, 0, 0x6, 0, 0xff, 0 }, { 1, 0, 1, 1, 0x6, 0, 2, 0 }, { 1, 0, 0, 0, 0, 0, 4, 1 },
                            { 1, 0, 0, 0, 0, 0, 8, 2 }, { 0, 1, 1, 0, 0x6, 0, 16, 0 }, { 1, 0, 0, 0, 0, 0, 32, 4 },
                            { 1, 0, 1, 0, 0x6, 1, 64, 5 }, { 1, 0, 1, 1, 0x6, 0, 128, 6 } };
    for (size_t i = 0; i < sizeof(fs) / sizeof(fs[0]); i++) {
        vp9h_synth_params sp;
        vp9hip_synth_defaults(&sp, w, h, 8);
        sp.log2_tile_cols = log2tc;
        sp.inter = fs[i].inter;
        sp.seed = seed + i;
        sp.seg = sg;
        sp.seg.update_map = fs[i].update_map; sp.seg.temporal = fs[i].temporal; sp.seg.q_en = fs[i].q_en;
        vp9h_frame f;
        memset(&f, 0, sizeof(f));
        if (vp9hip_synth_frame(&f, &sp) < 0) break;
        if (fs[i].intraonly) { f.keyframe = 0; f.intraonly = 1; }
        vp9h_enc_params ep;
        vp9h_enc_defaults(&ep);
        ep.seg = sp.seg;
        ep.refresh_mask = fs[i].refresh;
        ep.error_res = fs[i].errres;
        if (fs[i].intraonly) ep.show_frame = 0;
        for (int k = 0; k < 3; k++) ep.ref_slot[k] = fs[i].ref;
        uint8_t *buf = nullptr;
        size_t sz = 0;
        const int r = vp9h_stream_encode(enc, &f, &ep, &buf, &sz, nullptr);
        vp9hip_synth_free(&f);
        if (r < 0) { fprintf(stderr, "seg stream frame %zu: encode %d\n", i, r); break; }
        out.push_back(Bytes(buf, buf + sz));
        vp9h_buffer_free(buf);
    }
    vp9h_stream_close(enc);
    return out;
}

static bool same_packet(const vp9h_frame &a, const vp9h_frame &b)
{
    if (a.width != b.width || a.height != b.height || a.bpp != b.bpp || a.nblocks != b.nblocks || a.neobs != b.neobs ||
        a.ncoefs != b.ncoefs || a.keyframe != b.keyframe || a.filter_level != b.filter_level)
        return false;
    if (memcmp(a.lflvl, b.lflvl, sizeof(a.lflvl)) || memcmp(a.ref_w, b.ref_w, sizeof(a.ref_w)))
        return false;
    if (a.nblocks && memcmp(a.blocks, b.blocks, a.nblocks * sizeof(vp9h_block))) return false;
    if (a.neobs && memcmp(a.eobs, b.eobs, a.neobs * 2)) return false;
    return !a.ncoefs || !memcmp(a.coefs, b.coefs, a.ncoefs * (a.bpp > 8 ? 4 : 2));
}

// parse a stream on one vp9h_stream with `threads` tile threads; packets into out (owned)
static int parse_stream(const std::vector<Bytes> &s, int threads, std::vector<vp9h_frame> *out)
{
    vp9h_stream *st = nullptr;
    int r = vp9h_stream_open(&st);
    if (r < 0) return r;
    vp9h_stream_set_threads(st, threads);
    int err = 0;
    for (const Bytes &d : s) {
        vp9h_frame f;
        vp9h_frame_info info;
        memset(&f, 0, sizeof(f));
        r = vp9h_stream_decode(st, d.data(), d.size(), &f, &info);
        if (r < 0 && !err) err = r;
        if (out) out->push_back(f);
        else vp9h_frame_free(&f);
    }
    vp9h_stream_close(st);
    return err;
}

// frame-pipelined parse: each frame's headers on this thread in order, its tiles on a thread
// of its own (tthreads tile-column threads each); a frame whose tiles adapt the next
// headers' probabilities is finished before the next begin
static int parse_pipelined(const std::vector<Bytes> &s, int tthreads, std::vector<vp9h_frame> *out)
{
    vp9h_stream *st = nullptr;
    int r = vp9h_stream_open(&st);
    if (r < 0) return r;
    out->assign(s.size(), vp9h_frame());
    for (auto &f : *out) memset(&f, 0, sizeof(f));
    std::vector<int> rets(s.size(), 0);
    std::vector<std::thread> th;
    for (size_t i = 0; i < s.size(); i++) {
        vp9h_pending *p = nullptr;
        vp9h_frame_info info;
        int serial = 0;
        r = vp9h_stream_decode_begin(st, s[i].data(), s[i].size(), &p, &info, &serial);
        if (r < 0 || !p) { rets[i] = r; continue; }
        if (serial) rets[i] = vp9h_stream_decode_finish(p, tthreads, &(*out)[i]);
        else th.emplace_back([p, tthreads, out, &rets, i] { rets[i] = vp9h_stream_decode_finish(p, tthreads, &(*out)[i]); });
    }
    for (auto &t : th) t.join();
    vp9h_stream_close(st);
    int err = 0;
    for (int e : rets) if (e < 0 && !err) err = e;
    return err;
}

static void free_all(std::vector<vp9h_frame> &v)
{
    for (auto &f : v) vp9h_frame_free(&f);
    v.clear();
}

static void check_streams(int nmut)
{
    static const Cfg cfgs[] = {
        // (w, h, bpp, ss_h, ss_v, log2 tile columns: at least 4 SBs per column, frames, adaptation)
        { 352, 288, 8, 1, 1, 0, 5, 0 },  { 704, 288, 8, 1, 1, 1, 4, 1 }, { 1056, 200, 8, 1, 1, 2, 3, 0 },
        { 520, 140, 10, 1, 1, 1, 4, 1 }, { 264, 136, 8, 0, 0, 0, 3, 0 }, { 2112, 96, 8, 1, 1, 3, 2, 1 },
    };
    std::vector<std::vector<Bytes>> streams;
    for (const Cfg &c : cfgs) {
        std::vector<Bytes> s = make_stream(c, 1000u + (uint64_t) streams.size() * 37u);
        CHECK((int) s.size() == c.n, "encode %dx%d: %zu of %d frames", c.w, c.h, s.size(), c.n);
        std::vector<vp9h_frame> ser;
        CHECK(parse_stream(s, 1, &ser) == 0, "serial parse %dx%d", c.w, c.h);
        for (int t : { 2, 3, 8 }) {
            std::vector<vp9h_frame> thr;
            CHECK(parse_stream(s, t, &thr) == 0, "threaded parse (%d)", t);
            for (size_t i = 0; i < ser.size() && i < thr.size(); i++)
                CHECK(same_packet(ser[i], thr[i]), "%dx%d tiles %d frame %zu: %d threads != serial", c.w, c.h,
                      1 << c.log2tc, i, t);
            free_all(thr);
        }
        for (int t : { 1, 3 }) {
            std::vector<vp9h_frame> pip;
            CHECK(parse_pipelined(s, t, &pip) == 0, "pipelined parse (%d tile threads)", t);
            for (size_t i = 0; i < ser.size() && i < pip.size(); i++)
                CHECK(same_packet(ser[i], pip[i]), "%dx%d adapt %d frame %zu: pipelined (%d) != serial", c.w, c.h, c.adapt,
                      i, t);
            free_all(pip);
        }
        free_all(ser);
        streams.push_back(std::move(s));
    }
    // segmentation streams: a kept map read by a frame whose successor's headers drop it
    for (int tc = 0; tc < 2; tc++) {
        std::vector<Bytes> s = make_seg_stream(tc ? 704 : 352, 288, tc, 5000u + (uint64_t) tc * 17u);
        CHECK(s.size() == 8, "seg stream: %zu of 8 frames", s.size());
        std::vector<vp9h_frame> ser;
        CHECK(parse_stream(s, 1, &ser) == 0, "seg stream serial parse");
        for (int rep = 0; rep < 8; rep++)
            for (int t : { 1, 2 }) {
                std::vector<vp9h_frame> pip;
                CHECK(parse_pipelined(s, t, &pip) == 0, "seg stream pipelined parse (%d)", t);
                for (size_t i = 0; i < ser.size() && i < pip.size(); i++)
                    CHECK(same_packet(ser[i], pip[i]), "seg stream frame %zu: pipelined (%d) != serial", i, t);
                free_all(pip);
            }
        free_all(ser);
        streams.push_back(std::move(s));
    }
    // the parse pool: every stream as its own chain, all queued at once on 4 workers
    {
        vp9hip::ParsePool pool(4);
        std::vector<std::unique_ptr<vp9hip::ParseJob>> jobs;
        for (auto &s : streams) {
            int err = 0;
            std::shared_ptr<vp9hip::Chain> ch = vp9hip::ParsePool::new_chain(&err);
            CHECK(ch != nullptr, "new_chain");
            if (!ch) continue;
            for (const Bytes &d : s) {
                std::unique_ptr<vp9hip::ParseJob> j(new vp9hip::ParseJob());
                j->data = d;
                j->chain = ch;
                pool.enqueue(j.get());
                jobs.push_back(std::move(j));
            }
        }
        size_t k = 0;
        for (auto &s : streams) {
            std::vector<vp9h_frame> ser;
            parse_stream(s, 1, &ser);
            for (size_t i = 0; i < s.size(); i++, k++) {
                pool.wait(jobs[k].get());
                CHECK(jobs[k]->ret == 0 && same_packet(jobs[k]->pkt, ser[i]), "pool frame %zu", i);
            }
            free_all(ser);
        }
    }
    // corrupted copies: parse or fail, nothing else
    for (int m = 0; m < nmut && !streams.empty(); m++) {
        const std::vector<Bytes> &s = streams[(size_t) m % streams.size()];
        if (s.empty()) continue;
        std::vector<Bytes> bad = s;
        Bytes &d = bad[rnd() % bad.size()];
        if (rnd() & 1) {
            for (int k = 0, nf = 1 + (int) (rnd() % 8); k < nf && !d.empty(); k++) d[rnd() % d.size()] ^= (uint8_t) (1u << (rnd() % 8));
        } else if (!d.empty()) {
            d.resize(rnd() % d.size());
        }
        parse_stream(bad, (m % 3) + 1, nullptr);
    }
}

// demux a container, then parse its frames (superframes split)
static int demux_parse(const Bytes &b, int threads)
{
    std::vector<Bytes> frames;
    if (vp9h_ivf_probe(b.data(), b.size())) {
        vp9h_ivf_header h;
        if (vp9h_ivf_read_header(b.data(), b.size(), &h) < 0) return -1;
        size_t pos = h.header_size;
        const uint8_t *d;
        uint32_t sz;
        int64_t pts;
        int trunc;
        while (vp9h_ivf_read_frame(b.data(), b.size(), &pos, &d, &sz, &pts, &trunc) == 0) frames.push_back(Bytes(d, d + sz));
    } else if (vp9h_webm_probe(b.data(), b.size())) {
        vp9h_webm_info info;
        vp9h_webm_cursor cur;
        if (vp9h_webm_read_header(b.data(), b.size(), &info, &cur) < 0) return -1;
        const uint8_t *d;
        uint32_t sz;
        int64_t pts;
        int key;
        for (int k = 0; k < 100000 && vp9h_webm_read_frame(b.data(), b.size(), &cur, &d, &sz, &pts, &key) == 0; k++)
            frames.push_back(Bytes(d, d + sz));
    } else {
        return -1;
    }
    std::vector<Bytes> split;
    for (const Bytes &f : frames) {
        size_t off[8], szs[8];
        const int n = vp9h_superframe_split(f.data(), f.size(), off, szs, 8);
        for (int i = 0; i < n; i++) split.push_back(Bytes(f.begin() + (ptrdiff_t) off[i], f.begin() + (ptrdiff_t) (off[i] + szs[i])));
    }
    return parse_stream(split, threads, nullptr);
}

int main(int argc, char **argv)
{
    const int nmut = argc > 1 ? atoi(argv[1]) : 40;
    check_streams(nmut);
    for (int a = 2; a < argc; a++) {
        FILE *f = fopen(argv[a], "rb");
        if (!f) { CHECK(false, "open %s", argv[a]); continue; }
        Bytes b;
        uint8_t tmp[65536];
        for (size_t n; (n = fread(tmp, 1, sizeof(tmp), f)) > 0;) b.insert(b.end(), tmp, tmp + n);
        fclose(f);
        CHECK(demux_parse(b, 1) == 0, "%s: demux + parse", argv[a]);
        CHECK(demux_parse(b, 4) == 0, "%s: demux + parse, 4 tile threads", argv[a]);
        for (int m = 0; m < nmut; m++) {
            Bytes x = b;
            const int kind = (int) (rnd() % 3);
            if (kind == 0) for (int k = 0; k < 4; k++) x[rnd() % x.size()] ^= (uint8_t) (1u << (rnd() % 8));
            else if (kind == 1) x.resize(rnd() % x.size());
            else x[rnd() % x.size()] = (uint8_t) rnd();
            demux_parse(x, 1 + m % 2);
        }
    }
    printf("host_san: %s (%d failures)\n", fails ? "FAILED" : "ok", fails);
    return fails ? 1 : 0;
}
