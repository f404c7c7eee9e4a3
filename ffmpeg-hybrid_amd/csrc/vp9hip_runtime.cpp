// Host runtime of the MI355X VP9 hybrid decoder: implements the C-ABI of
// include/vp9hip.h on top of the gfx950 kernels in vp9hip_kernels.hip.
//
// From each pass-1 frame packet it builds, on the host:
//   * residual jobs: every coded tx block of the batch, bucketed by tx size and type,
//     for the dependency-free inverse-transform kernel k_resid;
//   * per-superblock intra prediction job lists, topologically levelled by the
//     intra dependencies of check_intra_mode (vp9recon.c:37-221) and packed into
//     passes of independent jobs, so one SB is predicted by one wavefront in LDS;
//   * the loop-filter level/mask record of every SB (VP9Filter, restating
//     vp9block.c:1142-1262 and 1438-1452);
//   * motion-compensation rectangles restating inter_pred's sub-8x8 MV rules
//     (vp9_mc_template.c:30-464);
//   * launch schedules: the intra SB wavefront (t = x_in_tile + y) and the LF SB
//     wavefront (t = x + 2y) that reproduces the reference's SB-raster LF order
//     (vp9.c:1419-1429).
// Everything is uploaded into one HBM arena per staged batch; run launches only.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <array>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#pragma clang diagnostic ignored "-Wunused-result"
#pragma clang diagnostic ignored "-Wunused-value"

#include "../../include/vp9hip.h"
#include "vp9_tables.h"
#include "vp9hip_work.h"
#include "vp9hip_planlogic.h"
#include "vp9hip_plan.h"

extern "C" {
int vp9hip_launch_resid_multi(int hb, hipStream_t st, const uint32_t *off, const uint32_t *n, const RJob *jobs,
                              const FrameDesc *frames, const void *coefs, int16_t *resid);
int vp9hip_launch_resid(int hb, hipStream_t st, int tcode, int n, const RJob *jobs, const FrameDesc *frames,
                        const void *coefs, int16_t *resid);
int vp9hip_launch_resid_dev(int hb, hipStream_t st, int tcode, int ub, const RJob *jobs, const uint32_t *rng,
                            const FrameDesc *frames, const void *coefs, int16_t *resid);
int vp9hip_launch_pred(int fmt, hipStream_t st, int nwg, const uint32_t *list, const WGRec *wgs, const SBRec *sbs,
                       const PJob *jobs, const uint32_t *passes, const FrameDesc *frames, const int16_t *resid,
                       const uint32_t *ptab, int dbg);
int vp9hip_launch_lf(int fmt, hipStream_t st, int nsb, const uint32_t *list, const LFRec *recs,
                     const FrameDesc *frames, int dbg);
int vp9hip_launch_predd(int fmt, hipStream_t st, int n, int wgcap, const uint32_t *list, const uint32_t *sbinfo, const WGRec *wgs,
                        const SBRec *sbs, const PJob *jobs, const uint32_t *passes, const FrameDesc *frames,
                        const int16_t *resid, const uint32_t *ptab, uint32_t *ctr, uint32_t *done, int dbg);
int vp9hip_launch_mc(int hb, hipStream_t st, int n, const McUnit *units, const FrameDesc *frames, const KCfg *k);
size_t vp9hip_plan_scan_bytes(size_t n);
int vp9hip_plan_enqueue(hipStream_t st, const PlanDev *D, int ss, int nframes, int max_blk, int max_sb, uint32_t nb,
                        uint32_t nslots, uint32_t ncnt, int nk, const uint32_t *gidx, int ng, uint32_t *summary,
                        void *scan_tmp, size_t scan_bytes, int any_levels, int flags, int guard);
int vp9hip_launch_lfr(int fmt, hipStream_t st, int ntasks, const uint32_t *tasks, const LFRec *recs,
                      const FrameDesc *frames, uint32_t *ctr, const KCfg *k, const LfrIntra *li);
int vp9hip_launch_plf(int fmt, hipStream_t st, const PlfLaunch *pl, const uint32_t *plist, const uint32_t *llist,
                      const WGRec *wgs, const SBRec *sbs, const PJob *jobs, const uint32_t *passes, const LFRec *recs,
                      const RJob *rjobs, const FrameDesc *frames, const void *coefs, int16_t *resid, const uint32_t *ptab,
                      int dbg);
}

namespace {

// K_PLAN: the device planner (k_pblk, scans, k_psb, k_plan, k_plevel, k_pkeys, k_plists) of a run
enum { K_MC, K_RESID, K_PRED, K_LF, K_PLF, K_LFR, K_PLAN, K_N };
const char *const kname[K_N] = { "k_mc", "k_resid", "k_pred", "k_lf", "k_plf", "k_lfr", "k_plan" };


// step: wavefront diagonal of a K_PRED (x_in_tile + y) or K_LF (x + 2y) launch; K_PLF
// (intra diagonal `step` + LF diagonal step - PLF_LAG in one launch): off / n the intra
// workgroups, off2 / n2 the LF SBs; K_LFR (row-pipelined loop filter of a phase): off / n
// its task table, arg its counter block (uint32 index into the arena's counter words)
struct Launch { int kind; uint32_t off; uint32_t n; int arg; int grp; int ph; int part; int step;
                uint32_t off2 = 0, n2 = 0;
                uint32_t roff[5] = { 0, 0, 0, 0, 0 }, rn[5] = { 0, 0, 0, 0, 0 };   // K_PLF residual jobs by tx code
                int devr = 0;   // K_RESID of a static plan: off = the summary index of its job range, n = a bound
                int flow = -1;  // K_PRED of a level phase as one k_predd launch: its counter block;
                                // K_LFR with the phase's intra SBs inside (off2 / n2 their list)
};
#define PLF_LAG 3   // see the schedule in stage()
// Residuals run inside the fused launches (one intra diagonal ahead) for phases of fewer
// frames than this; wide phases (keyframe batches) keep their separate k_resid launches:
// measured C2 +6.5 % fused, C3 -2 %, C4 -8 %
#define RES_FUSE_MAX_FRAMES 8
// The loop filter of phases of fewer frames than this runs as one row-pipelined k_lfr launch
// (its tail after the fused diagonals); wide phases keep diagonal launches: measured C2
// +8-10 %, C3 -6 % with k_lfr everywhere (its long-lived workgroups crowd the other groups'
// intra wavefronts)
#define LFR_MAX_FRAMES 8
enum { PART_RECON, PART_LF };           // a phase's reconstruction launches, then its loop filter
#define MAX_GROUPS 8                    // independent frame groups = concurrent launch chains
#define MAX_SLOTS VP9HIP_MAX_SLOTS      // batch slots per context (include/vp9hip.h)

struct Staged {
    // host images (kept for rebuilds / inspection)
    std::vector<FrameDesc> frames;
    std::vector<SBRec> sbs;
    std::vector<PJob> pjobs;            // merged per workgroup, pass order (device)
    std::vector<uint32_t> passes;       // pass words (device)
    std::vector<WGRec> wgs;             // k_pred workgroups (device)
    // per-SB intra jobs before pass packing (host), in decode order, with the SB-local
    // indices of the jobs whose pixels each one reads (jdep0[k] .. jdep0[k + 1])
    struct SBHost { uint32_t job0, njobs, nlev; };
    std::vector<SBHost> sbh;
    std::vector<PJob> sbjobs;
    std::vector<uint32_t> jdep0;        // per job, plus one end marker per SB
    std::vector<uint16_t> jdeps;
    // residual jobs by (phase, tx code, txtp); a phase = (stream group, chain position)
    std::vector<std::array<std::array<std::vector<RJob>, 4>, 5>> rbucket;
    int ngroups = 1;
    std::vector<RJob> rjobs;            // concatenated buckets
    uint64_t resid16 = 0;               // residual scratch size, 16-element units
    std::vector<LFRec> lfs;
    std::vector<McUnit> mcs;
    std::vector<uint32_t> lists;        // concatenated SB index lists of all launches
    std::vector<Launch> launches;
    int nphases = 0;
    std::vector<int> frame_phase;       // phase of each batch frame
    std::vector<int> frame_log2;        // log2 tile columns of each batch frame
    int tile_lo = 0, tile_hi = 64;      // tile columns this context reconstructs (sharded batches)
    std::vector<uint8_t> coefs;         // concatenated coefficient streams (bytes)
    double alg_bytes[K_N] = {};
    // record counts of the arena (the host images above are not kept for these)
    uint32_t n_sbs = 0, n_pjobs = 0, n_passes = 0, n_wgs = 0, n_rjobs = 0, n_lfs = 0, n_mcs = 0;
    uint32_t n_ctr = 0;                 // k_lfr counter words (zero between launches)
    std::vector<uint32_t> lfr_ctr;      // counter block offset of every k_lfr / k_predd launch
    uint32_t pdone = 0;                 // k_predd: slot-indexed intra done flags (counter words)
    uint8_t *pinned = nullptr;          // pinned host image of the arena (one DMA per stage)
    size_t pinned_cap = 0;
    // device arena
    uint8_t *arena = nullptr;
    size_t arena_cap = 0;
    size_t o_frames = 0, o_sbs = 0, o_pjobs = 0, o_passes = 0, o_wgs = 0, o_rjobs = 0, o_lfs = 0, o_mcs = 0, o_lists = 0,
           o_coefs = 0, o_ctr = 0;
    int16_t *resid = nullptr;           // intra residual scratch (column-major n x n blocks)
    size_t resid_cap = 0;               // bytes
    uint8_t *edge = nullptr;            // intra frames' SB right columns (FrameDesc.edge)
    size_t edge_cap = 0;                // bytes
    bool ready = false;
    hipGraphExec_t graph = nullptr;     // captured launch sequence of this batch (timing off)
    std::vector<Launch> graph_launches; // the launch list the graph was captured from

    // ---- device-planned batch (the default; VP9HIP_HOST_PLAN=1 plans on the host): stage
    // uploads the packets and the batch geometry, every run plans on the device
    bool dev = false, planned = false, fuse = false;
    struct DevPhase {
        std::vector<int> frames;
        int group = 0, nseg = 1, nkey = 0, np = 0, nlf = 0;
        bool fused = false, levels = false, lfr = false;
        uint32_t key0 = 0;
        std::vector<uint32_t> seg_sz;                         // SBs per residual segment
        std::vector<std::pair<uint32_t, uint32_t>> lf;        // per LF diagonal: host list (offset, count)
        std::vector<double> pred_bytes, lf_bytes;             // per intra diagonal (intra frames) / LF diagonal
        uint32_t lfr_off = 0, lfr_n = 0;                      // k_lfr task table in the host lists
        int lfr_ctr = 0;
        int pred_ctr = -1;                                    // k_predd counter block (level phases)
        bool all_lf = false;                                  // every frame of the phase is loop-filtered
        double lfr_bytes = 0;
        int g_res = 0, g_mc = 0;                              // summary gather slots
    };
    std::vector<DevPhase> dph;
    std::vector<double> frame_res_bytes;                      // per frame: coefficient bytes
    std::vector<int> frame_fused;                             // per frame: residuals inside k_plf
    double alg_base[K_N] = {};                                // header-derived algorithmic bytes
    uint32_t cap_mcs = 0;
    uint32_t nslots = 0, nblk = 0, neob = 0, ncoef = 0, ncnt = 0, nkey = 0, host_lists = 0, n_gidx = 0;
    int max_blk = 0, max_sb = 0, jcap = 0, rcap = 0, nframes = 0;
    bool any_levels = false;
    int plan_flags = 0;                 // device planner kernels: 1 any filtered frame, 2 any inter frame
    size_t o_pf = 0, o_blocks = 0, o_eobs = 0, o_slotpos = 0, o_segpre = 0, o_segsz = 0, o_segpre1 = 0, o_cntm = 0, o_cntm0 = 0, o_gidx = 0, o_bneob = 0,
           o_beob0 = 0, o_sbfirst = 0, o_sbncoef = 0, o_sbcoef0 = 0, o_cnt = 0, o_cnt0 = 0, o_ibits = 0,
           o_sbinfo = 0, o_sbkey = 0, o_sbkpos = 0, o_expko = 0, o_keycnt = 0, o_keyoff = 0, o_status = 0, o_fbytes = 0, o_fbad = 0,
           o_summary = 0, o_scan = 0, zero_bytes = 0, o_jobw = 0, o_sbnj = 0;
    size_t scan_bytes = 0, summary_words = 0;
    uint32_t *summary_h = nullptr;                            // pinned readback of the summary
    size_t summary_cap = 0;
    hipEvent_t done_ev = nullptr;       // recorded on the main stream after this batch's last run
    hipEvent_t up_ev = nullptr;         // recorded after the staging upload: the pinned image is
                                        // rewritten by the next staging only once it completed
    // ---- static plan (keyframe batches): the launch list is built at staging from the batch
    // geometry (every SB of an intra frame has intra work, so the step lists' sizes and
    // offsets are known); only the residual job ranges come from the planner, read by the
    // kernels from the summary in HBM. A run enqueues the planner and, ordered after it by
    // an event, the pixel launches: no host wait. The summary is read (status, the key
    // offsets checked against the staged ones, byte totals) when the host next waits.
    bool stat = false;
    hipEvent_t plan_ev = nullptr;
    bool summary_pending = false;
    int status = 0;                     // sticky until the slot is restaged: the planner rejected
                                        // frames of the batch (AVERROR_INVALIDDATA; k_pguard
                                        // neutralised them) or the batch failed (VP9HIP_EBUG)
    // Per frame (staging order), the outcome of the last stage / run when it failed with
    // AVERROR_INVALIDDATA (vp9hip_batch_frame_status): 0 reconstructed, AVERROR_INVALIDDATA
    // rejected, AVERROR(EAGAIN) valid but not run (the batch stopped before its pixel work).
    std::vector<int> fstat;
    std::vector<uint32_t> exp_ko;       // key offsets the launch list was built with
    std::vector<uint32_t> stat_lists;   // the intra step lists (uploaded with the batch)
    std::vector<int> wr, rd;            // frame buffers the batch writes / reads (sorted)
    uint32_t dep_mask = 0;              // bit k: it touches a buffer of slot k's batch
    double alg_stat[K_N] = {};          // algorithmic bytes after the launch-list moves
};

} // namespace

// Host copies of a download (pinned staging chunk -> the caller's planes) split over a few
// worker threads plus the caller: one thread's memcpy (~8-10 GB/s) was the download path's
// bound at 8K (99.5 MB per 10-bit frame). Rows of a part are copied one by one when the
// strides differ.
struct CopyPool {
    struct Part { uint8_t *dst; ptrdiff_t dstride; const uint8_t *src; size_t sstride, row; int rows; };
    std::vector<std::thread> th;
    std::mutex m;
    std::condition_variable cv, done_cv;
    std::vector<Part> parts;
    size_t next = 0, pending = 0;
    bool quit = false;
    static void copy(const Part &q)
    {
        if ((size_t) q.dstride == q.row && q.sstride == q.row) { memcpy(q.dst, q.src, q.row * (size_t) q.rows); return; }
        for (int y = 0; y < q.rows; y++) memcpy(q.dst + (ptrdiff_t) y * q.dstride, q.src + (size_t) y * q.sstride, q.row);
    }
    bool take(Part &q)
    {
        std::lock_guard<std::mutex> l(m);
        if (next >= parts.size()) return false;
        q = parts[next++];
        return true;
    }
    void finish()
    {
        std::lock_guard<std::mutex> l(m);
        if (--pending == 0) done_cv.notify_all();
    }
    explicit CopyPool(int n)
    {
        for (int i = 0; i < n; i++)
            th.emplace_back([this] {
                for (;;) {
                    Part q;
                    {
                        std::unique_lock<std::mutex> l(m);
                        cv.wait(l, [&] { return quit || next < parts.size(); });
                        if (quit) return;
                        q = parts[next++];
                    }
                    copy(q);
                    finish();
                }
            });
    }
    ~CopyPool()
    {
        { std::lock_guard<std::mutex> l(m); quit = true; }
        cv.notify_all();
        for (auto &t : th) t.join();
    }
    // copy `rows` rows split into parts of the pool's size, the caller taking parts too
    void run(uint8_t *dst, ptrdiff_t dstride, const uint8_t *src, size_t sstride, size_t row, int rows)
    {
        const int np = (int) th.size() + 1, per = (rows + np - 1) / np;
        {
            std::lock_guard<std::mutex> l(m);
            parts.clear();
            for (int y = 0; y < rows; y += per)
                parts.push_back({ dst + (ptrdiff_t) y * dstride, dstride, src + (size_t) y * sstride, sstride, row, std::min(per, rows - y) });
            next = 0;
            pending = parts.size();
        }
        cv.notify_all();
        Part q;
        while (take(q)) { copy(q); finish(); }
        std::unique_lock<std::mutex> l(m);
        done_cv.wait(l, [&] { return pending == 0; });
    }
};

struct vp9hip_ctx {
    int dev = 0;
    hipStream_t st = nullptr;           // main stream: uploads, downloads, group 0
    hipStream_t xst[MAX_GROUPS - 1] = {};   // groups 1.. of a batch (joined back into st)
    hipEvent_t fork_ev = nullptr, join_ev[MAX_GROUPS] = {};
    // frame-group streams per batch slot, VP9HIP_STREAMS overrides (1..8). 1: with 3 or 4
    // batches in flight (the decoder, the FFHWAccel adapter and the bench rotate 3 slots;
    // VP9HIP_PIPELINE_SLOTS) the slots' streams then fit the 4 hardware queues (profiles/r05z:
    // C3 11,205 vs 10,821 fps at 2 groups x 2 slots, C2 at 4 slots 17.6k vs 13.8k). 2 groups
    // were best with two slots in flight (r02k).
    int max_groups = 1;
    bool fuse_plf = true;               // VP9HIP_PLF=0: no fused intra + LF launches
    bool level_sched = true;            // VP9HIP_LEVELS=0: inter frames' intra SBs by diagonal
    int lf_rows = 1;                    // VP9HIP_LFROW: 0 LF as diagonal launches only, 1 k_lfr for
                                        // narrow phases (LFR_MAX_FRAMES), 2 k_lfr for every phase
    int w = 0, h = 0, bpp = 8, ss_h = 1, ss_v = 1, hb = 0, bypp = 1;
    int cols = 0, rows = 0, sb_cols = 0, sb_rows = 0;
    int pitch[2] = { 0, 0 };
    size_t plane_off[3] = { 0, 0, 0 }, buf_bytes = 0;
    std::vector<uint8_t *> bufs;
    std::vector<std::pair<int, int>> buf_wh;   // visible size of the frame each buffer holds
    uint32_t *ptab = nullptr;           // intra predictor formula table (device)
    uint8_t *nz = nullptr;              // nonzero bounding boxes per (tcode, txtp, eob) (device, planner)
    bool host_plan = false;             // VP9HIP_HOST_PLAN=1: plan batches on host threads (A/B, tests)
    hipEvent_t pev[2] = {};             // device planner timing (timing runs)
    unsigned long long *plan_prof = nullptr;   // VP9HIP_PLAN_PROF: k_plan phase cycles (device)
    bool plan_timed = false;
    int dbg = 0;                        // VP9HIP_DEBUG: ablation switches for profiling only
    bool use_graph = true;              // VP9HIP_GRAPH=0 disables graph replay
    // the other VP9HIP_* switches, read once by vp9hip_open (read_config): the staging and
    // launch paths never read the environment
    KCfg kcfg = { 1, 0 };               // kernel selections (VP9HIP_LFRO, VP9HIP_MCQ_SLICES)
    int host_threads = 16;              // VP9HIP_HOST_THREADS: host planning / staging threads
    uint32_t lfr_spin = 0;              // row-LF hand-off spin bound, 0 = 2^22 polls (test hook)
    int test_reject = 0;                // k | f << 16: frame f of the k-th batch staged is made invalid (test hook)
    bool static_plan = true;            // VP9HIP_STATIC=0: keyframe batches planned like the others
    bool edge = true;                   // VP9HIP_EDGE=0: no SB edge columns (4:2:0 tile loader)
    bool resid_multi = true;            // VP9HIP_RESID_MULTI=0: one residual launch per tx size
    bool stage_trace = false;           // VP9HIP_STAGE_TRACE=1: host time of staging / planning
    bool plan_prof_on = false;          // VP9HIP_PLAN_PROF=1: k_plan phase cycles
    int plan_dbg = 0;                   // VP9HIP_PLAN_DBG: planner ablations (timing only)
    bool plan_only = false;             // VP9HIP_PLAN_ONLY=1: run the planner alone (diagnostics)
    bool plan_reuse = false;            // VP9HIP_PLAN_REUSE=1: a static-plan batch's reruns skip the planner
                                        // (its records are unchanged): the pixel launches alone (diagnostics)
    bool pred_df = true;                // VP9HIP_PRED_DF=0: a level phase's intra SBs as one k_pred launch per level
    int pred_df_wgs = 1024;             // VP9HIP_PRED_DF_WGS: k_predd grid cap (workgroups)
    int pred_df_max = 1024;             // VP9HIP_PRED_DF_MAX: phases of more intra SBs keep level launches
    bool pred_lf_fuse = true;           // VP9HIP_PRED_LF_FUSE=0: a phase's k_predd work as its own launch, not
                                        // as intra workers inside the phase's k_lfro launch
    int dl_threads = 3;                 // VP9HIP_DL_THREADS: download copy threads besides the caller
    Staged stg;                         // the current batch slot
    Staged sl[MAX_SLOTS];               // the other slots (sl[slot] is a moved-out placeholder;
                                        // vp9hip_set_batch_slot swaps a slot in and out)
    int slot = 0;
    int nstaged = 0;                    // batches staged (the test_reject hook)
    hipStream_t pst = nullptr;          // device planner stream: a slot's planning overlaps the
                                        // other slot's pixel kernels (VP9HIP_SLOT_STREAMS=0 only)
    // Per-slot streams (default): each batch slot has its own main and group streams, swapped
    // into st / xst with the slot, and plans on its main stream ahead of its pixel work. Two
    // staged batches that share no frame buffer then run concurrently (the second batch's
    // intra wavefront under the first one's loop-filter tail); a batch that reads or writes a
    // buffer of another slot's batch waits for it (dep_mask, found at staging). Slots 0 and 1
    // get their streams at open, slots 2.. at their first use.
    bool slot_streams = true;
    int pix_prio = 0;
    hipStream_t sst[MAX_SLOTS] = {}, sxst[MAX_SLOTS][MAX_GROUPS - 1] = {};   // per slot: main, groups
    // downloads (vp9hip_download_frame): a stream of their own (the slot streams may hold
    // newer batches) and a pinned staging ring of DL_RING chunks, host copies overlapped
    // with the next chunk's D2H
    hipStream_t dst_dl = nullptr;
    uint8_t *dl_pin = nullptr;
    hipEvent_t dl_ev[4] = {};
    std::unique_ptr<CopyPool> dl_pool;  // host copies out of the ring (created at the first download)
    hipEvent_t fill_ev = nullptr;       // after vp9hip_fill_buffers' memsets
    // timing of the last run
    bool timing = true;
    std::vector<hipEvent_t> ev;
    bool timed_run = false;             // the last run recorded per-launch events
    double kms[K_N] = {};
    int kcount[K_N] = {};
};

#define HIPCHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "vp9hip: %s failed: %s\n", #x, hipGetErrorString(e_)); return VP9HIP_EEXTERNAL; } } while (0)

// The planner's stream: the slot's main stream with per-slot streams, else its own.
static hipStream_t plan_stream(const vp9hip_ctx *c) { return c->slot_streams ? c->st : c->pst; }
// Slot k's staged batch (the current one lives in c->stg).
static Staged &slot_ref(vp9hip_ctx *c, int k) { return k == c->slot ? c->stg : c->sl[k]; }
// Wait for everything any slot queued.
static hipError_t sync_all(vp9hip_ctx *c)
{
    hipError_t e = hipStreamSynchronize(c->st);
    for (int k = 0; k < MAX_SLOTS && e == hipSuccess; k++)
        if (c->sst[k] && c->sst[k] != c->st) e = hipStreamSynchronize(c->sst[k]);
    if (e == hipSuccess && c->pst) e = hipStreamSynchronize(c->pst);
    return e;
}
// The streams of slot k (per-slot streams): created at the context's stream priority.
static bool slot_streams_make(vp9hip_ctx *c, int k)
{
    if (c->sst[k]) return true;
    bool ok = hipStreamCreateWithPriority(&c->sst[k], hipStreamNonBlocking, c->pix_prio) == hipSuccess;
    for (int i = 0; ok && i < c->max_groups - 1; i++)
        ok = hipStreamCreateWithPriority(&c->sxst[k][i], hipStreamNonBlocking, c->pix_prio) == hipSuccess;
    if (!ok) {                          // all or nothing: a later selection retries
        for (int i = 0; i < MAX_GROUPS - 1; i++)
            if (c->sxst[k][i]) { hipStreamDestroy(c->sxst[k][i]); c->sxst[k][i] = nullptr; }
        if (c->sst[k]) hipStreamDestroy(c->sst[k]);
        c->sst[k] = nullptr;
    }
    return ok;
}

// Test hooks (vp9hip_test_hooks): process-wide values a context copies when it opens.
static std::atomic<int> g_test_reject{0};
static std::atomic<uint32_t> g_test_lfr_spin{0};

extern "C" void vp9hip_test_hooks(int reject_batch, uint32_t lfr_spin)
{
    g_test_reject = reject_batch;
    g_test_lfr_spin = lfr_spin;
}

// Every VP9HIP_* switch of a context, read here once: A/B and diagnostic switches of the
// pixel path (DESIGN.md §5 names the measurements each default rests on).
static void read_config(vp9hip_ctx *c)
{
    auto num = [](const char *name, int def) { const char *e = getenv(name); return e ? atoi(e) : def; };
    c->dbg = num("VP9HIP_DEBUG", 0);
    c->use_graph = num("VP9HIP_GRAPH", 1) != 0;
    c->max_groups = std::max(1, std::min(MAX_GROUPS, num("VP9HIP_STREAMS", c->max_groups)));
    c->fuse_plf = num("VP9HIP_PLF", 1) != 0;
    c->lf_rows = num("VP9HIP_LFROW", c->lf_rows);
    c->level_sched = num("VP9HIP_LEVELS", 1) != 0;
    c->host_plan = num("VP9HIP_HOST_PLAN", 0) != 0;
    c->slot_streams = num("VP9HIP_SLOT_STREAMS", 1) != 0;
    c->kcfg.lfro = num("VP9HIP_LFRO", 1) != 0;
    c->kcfg.mcq_slices = std::max(0, std::min(16, num("VP9HIP_MCQ_SLICES", 0)));
    c->host_threads = std::max(1, std::min(64, num("VP9HIP_HOST_THREADS",
                                                   (int) std::min(16u, std::max(1u, std::thread::hardware_concurrency())))));
    c->static_plan = num("VP9HIP_STATIC", 1) != 0;
    c->edge = num("VP9HIP_EDGE", 1) != 0;
    c->resid_multi = num("VP9HIP_RESID_MULTI", 1) != 0;
    c->stage_trace = num("VP9HIP_STAGE_TRACE", 0) != 0;
    c->plan_prof_on = num("VP9HIP_PLAN_PROF", 0) != 0;
    c->plan_dbg = num("VP9HIP_PLAN_DBG", 0);
    c->plan_only = num("VP9HIP_PLAN_ONLY", 0) != 0;
    c->plan_reuse = num("VP9HIP_PLAN_REUSE", 0) != 0;
    c->pred_df = num("VP9HIP_PRED_DF", 1) != 0;
    c->pred_lf_fuse = num("VP9HIP_PRED_LF_FUSE", 1) != 0;
    c->pred_df_wgs = std::max(1, num("VP9HIP_PRED_DF_WGS", 1024));
    c->pred_df_max = std::max(0, num("VP9HIP_PRED_DF_MAX", 1024));
    c->dl_threads = std::max(0, std::min(15, num("VP9HIP_DL_THREADS", 3)));
    c->test_reject = g_test_reject;
    c->lfr_spin = g_test_lfr_spin;
}

extern "C" int vp9hip_open(int device, vp9hip_ctx **out)
{
    if (!out) return VP9HIP_EINVAL;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return VP9HIP_ENOSYS;
    vp9hip_ctx *c = new vp9hip_ctx;
    c->dev = device;
    read_config(c);
    // streams in the order their work is busiest: the frame groups' streams, then the
    // planner's, so that (with the default 4 hardware queues, GPU_MAX_HW_QUEUES) each lands
    // on a queue of its own
    // Stream priorities (hipDeviceGetStreamPriorityRange): with per-slot streams every
    // stream of the context is created at the highest priority (measured at C3: 9,320 vs
    // 8,530 frames/s at default priority, r03f/ab5); with one planner stream the pixel
    // streams at the highest priority starve the planner (6,520), so all stay default.
    int prio_lo = 0, prio_hi = 0;
    const int prio = c->slot_streams ? 2 : 0;   // 2: the pixel streams highest
    hipSetDevice(device);
    if (prio) hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
    const int pix_prio = prio == 2 ? prio_hi : prio == 3 ? prio_lo : 0;
    c->pix_prio = pix_prio;
    const int plan_prio = prio == 1 || prio == 3 ? prio_lo : 0;
    bool ok = hipStreamCreateWithPriority(&c->st, hipStreamNonBlocking, pix_prio) == hipSuccess &&
              hipEventCreateWithFlags(&c->fork_ev, hipEventDisableTiming) == hipSuccess;
    for (int i = 0; ok && i < c->max_groups - 1; i++)
        ok = hipStreamCreateWithPriority(&c->xst[i], hipStreamNonBlocking, pix_prio) == hipSuccess;
    if (c->slot_streams) {             // slot 1's set (slots 2.. at their first selection)
        c->sst[0] = c->st;
        for (int i = 0; i < MAX_GROUPS - 1; i++) c->sxst[0][i] = c->xst[i];
        ok = ok && slot_streams_make(c, 1);
    } else {
        ok = ok && hipStreamCreateWithPriority(&c->pst, hipStreamNonBlocking, plan_prio) == hipSuccess;
    }
    for (int i = 0; ok && i < MAX_GROUPS - 1; i++)
        ok = hipEventCreateWithFlags(&c->join_ev[i], hipEventDisableTiming) == hipSuccess;
    if (!ok) {
        delete c;
        return VP9HIP_EEXTERNAL;
    }
    *out = c;
    return 0;
}

static void free_bufs(vp9hip_ctx *c)
{
    for (auto *b : c->bufs) hipFree(b);
    c->bufs.clear();
    c->buf_wh.clear();
}

// Forget the staged batches of every slot (their FrameDescs, graphs and launch lists name
// frame buffers): a later run_batch of any slot needs a new stage. The caller has
// synchronised the main and planner streams.
static void drop_slots(vp9hip_ctx *c)
{
    for (int k = 0; k < MAX_SLOTS; k++) {
        Staged *g = &slot_ref(c, k);
        g->ready = false;
        g->planned = false;
        if (g->graph) hipGraphExecDestroy(g->graph);
        g->graph = nullptr;
        g->graph_launches.clear();
        g->summary_pending = false;
    }
}

extern "C" void vp9hip_close(vp9hip_ctx *c)
{
    if (!c) return;
    hipSetDevice(c->dev);
    sync_all(c);
    free_bufs(c);
    for (int k = 0; k < MAX_SLOTS; k++) {
        Staged *g = &slot_ref(c, k);
        if (g->arena) hipFree(g->arena);
        if (g->resid) hipFree(g->resid);
        if (g->edge) hipFree(g->edge);
        if (g->pinned) hipHostFree(g->pinned);
        if (g->graph) hipGraphExecDestroy(g->graph);
        if (g->summary_h) hipHostFree(g->summary_h);
        if (g->done_ev) hipEventDestroy(g->done_ev);
        if (g->up_ev) hipEventDestroy(g->up_ev);
        if (g->plan_ev) hipEventDestroy(g->plan_ev);
    }
    if (c->ptab) hipFree(c->ptab);
    if (c->nz) hipFree(c->nz);
    if (c->dl_pin) hipHostFree(c->dl_pin);
    if (c->dst_dl) hipStreamDestroy(c->dst_dl);
    for (auto e : c->dl_ev) if (e) hipEventDestroy(e);
    if (c->fill_ev) hipEventDestroy(c->fill_ev);
    if (c->plan_prof) hipFree(c->plan_prof);
    if (c->pst) hipStreamDestroy(c->pst);
    for (auto e : c->pev) if (e) hipEventDestroy(e);
    for (auto e : c->ev) hipEventDestroy(e);
    if (c->slot_streams) {             // every slot's streams (c->st / xst are one slot's)
        for (int k = 0; k < MAX_SLOTS; k++) {
            if (c->sst[k]) hipStreamDestroy(c->sst[k]);
            for (int i = 0; i < MAX_GROUPS - 1; i++)
                if (c->sxst[k][i]) hipStreamDestroy(c->sxst[k][i]);
        }
    } else {
        hipStreamDestroy(c->st);
        for (int i = 0; i < MAX_GROUPS - 1; i++)
            if (c->xst[i]) hipStreamDestroy(c->xst[i]);
    }
    for (int i = 0; i < MAX_GROUPS - 1; i++)
        if (c->join_ev[i]) hipEventDestroy(c->join_ev[i]);
    if (c->fork_ev) hipEventDestroy(c->fork_ev);
    delete c;
}

// --------------------------------------------------------------------------
// Intra predictor formula table (vp9dsp_template.c:28-1106 restated per pixel). Edge
// array e: e[0..n) left column bottom-to-top, e[n] top-left, e[n+1 ..] top row with the
// 4x4 top-right. Kinds: copy, avg2 (a+b+1)>>1, avg3 (a+2b+c+2)>>2, avg31 (a+3b+2)>>2,
// tm clip(a+b-c), dc.
enum { PF_COPY, PF_AVG2, PF_AVG3, PF_AVG31, PF_TM, PF_DC };
// Formula word: byte offsets (2 * index) of the three edge samples a, b, c in bits 0-23,
// then wb (2 bits), wc (2-bit two's complement, 3 = -1), shift s, rounding (1 << s) >> 1:
// pixel = (a + rnd + wb * b + wc * c) >> s. DC predictors copy edge index 2n + 7, where
// the kernel stores the job's DC value.
static uint32_t pf_enc(int kind, int i0 = 0, int i1 = 0, int i2 = 0)
{
    static const int wb[6] = { 0, 1, 2, 3, 1, 0 }, wc[6] = { 0, 0, 1, 0, 3, 0 }, sh[6] = { 0, 1, 2, 2, 0, 0 };
    return (uint32_t) (2 * i0) | (uint32_t) (2 * i1) << 8 | (uint32_t) (2 * i2) << 16 | (uint32_t) wb[kind] << 24 |
           (uint32_t) wc[kind] << 26 | (uint32_t) sh[kind] << 28 | (uint32_t) ((1 << sh[kind]) >> 1) << 30;
}
static uint32_t pix_formula(int slot, int n, int x, int y)
{
    const int T = n + 1, h = n >> 1;        // T[k] = e[T + k]; HU left top-to-bottom L[i] = e[n - 1 - i]
    switch (slot) {
    case 0: return pf_enc(PF_COPY, T + x);                                       // VERT
    case 1: return pf_enc(PF_COPY, n - 1 - y);                                   // HOR
    case 8: return pf_enc(PF_TM, T + x, n - 1 - y, n);                           // TM_VP8
    case 2: {                                                                    // DIAG_DOWN_LEFT
        const int k = x + y;
        if (n == 4) return k < 6 ? pf_enc(PF_AVG3, T + k, T + k + 1, T + k + 2) : pf_enc(PF_COPY, T + 7);
        if (k < n - 2) return pf_enc(PF_AVG3, T + k, T + k + 1, T + k + 2);
        if (k == n - 2) return pf_enc(PF_AVG31, T + n - 2, T + n - 1);
        return pf_enc(PF_COPY, T + n - 1);
    }
    case 3: { const int j = n - 1 - y + x; return pf_enc(PF_AVG3, j, j + 1, j + 2); }   // DIAG_DOWN_RIGHT
    case 4: {                                                                    // VERT_RIGHT
        const int m = h - 1 - (y >> 1) + x;
        if (!(y & 1)) {
            if (m <= h - 2) return pf_enc(PF_AVG3, 2 * m + 2, 2 * m + 3, 2 * m + 4);
            return pf_enc(PF_AVG2, n + m - h + 1, n + m - h + 2);
        }
        if (m <= h - 2) return pf_enc(PF_AVG3, 2 * m + 1, 2 * m + 2, 2 * m + 3);
        return pf_enc(PF_AVG3, n + m - h, n + m - h + 1, n + m - h + 2);
    }
    case 5: {                                                                    // HOR_DOWN
        const int m = 2 * n - 2 - 2 * y + x;
        if (m >= 2 * n) { const int i = m - 2 * n; return pf_enc(PF_AVG3, n + i, n + i + 1, n + i + 2); }
        const int i = m >> 1;
        return (m & 1) ? pf_enc(PF_AVG3, i, i + 1, i + 2) : pf_enc(PF_AVG2, i, i + 1);
    }
    case 6: {                                                                    // VERT_LEFT
        const int k = (y >> 1) + x;
        if (n == 4) return (y & 1) ? pf_enc(PF_AVG3, T + k, T + k + 1, T + k + 2) : pf_enc(PF_AVG2, T + k, T + k + 1);
        if (x >= n - (y >> 1) - 1) return pf_enc(PF_COPY, T + n - 1);
        if (!(y & 1)) return pf_enc(PF_AVG2, T + k, T + k + 1);
        return k < n - 2 ? pf_enc(PF_AVG3, T + k, T + k + 1, T + k + 2) : pf_enc(PF_AVG31, T + n - 2, T + n - 1);
    }
    case 7: {                                                                    // HOR_UP
        auto L = [n](int i) { return n - 1 - i; };
        if (y >= h && x >= 2 * n - 2 - 2 * y) return pf_enc(PF_COPY, L(n - 1));
        const int m = 2 * y + x, i = m >> 1;
        if (!(m & 1)) return pf_enc(PF_AVG2, L(i), L(i + 1));
        return i < n - 2 ? pf_enc(PF_AVG3, L(i), L(i + 1), L(i + 2)) : pf_enc(PF_AVG31, L(n - 2), L(n - 1));
    }
    default: return pf_enc(PF_COPY, 2 * n + 7);                                  // DC family
    }
}
static int upload_ptab(vp9hip_ctx *c)
{
    if (c->ptab) return 0;
    std::vector<uint32_t> t(PTAB_SIZE);
    for (int slot = 0; slot < 10; slot++)
        for (int ts = 0, off = 0; ts < 4; off += 16 << (2 * ts), ts++) {
            const int n = 4 << ts;
            for (int y = 0; y < n; y++)
                for (int x = 0; x < n; x++) t[slot * PTAB_SLOT + off + y * n + x] = pix_formula(slot, n, x, y);
        }
    if (hipMalloc(&c->ptab, t.size() * 4) != hipSuccess) return VP9HIP_ENOMEM;
    return hipMemcpy(c->ptab, t.data(), t.size() * 4, hipMemcpyHostToDevice) == hipSuccess ? 0 : VP9HIP_EEXTERNAL;
}

static int upload_nz(vp9hip_ctx *c);

extern "C" int vp9hip_configure(vp9hip_ctx *c, int width, int height, int bpp, int ss_h, int ss_v, int nbufs)
{
    if (!c || width <= 0 || height <= 0 || nbufs <= 0 || width > 16384 || height > 16384) return VP9HIP_EINVAL;
    if (bpp != 8 && bpp != 10 && bpp != 12) return VP9HIP_EINVAL;
    if (ss_h < 0 || ss_h > 1 || ss_v < 0 || ss_v > 1) return VP9HIP_EINVAL;   // 4:2:0 / 4:2:2 / 4:4:0 / 4:4:4
    hipSetDevice(c->dev);
    sync_all(c);
    drop_slots(c);                      // every slot's records point at the buffers freed here
    free_bufs(c);
    c->w = width; c->h = height; c->bpp = bpp; c->ss_h = ss_h; c->ss_v = ss_v;
    c->hb = bpp > 8; c->bypp = c->hb ? 2 : 1;
    c->cols = (width + 7) >> 3; c->rows = (height + 7) >> 3;
    c->sb_cols = (width + 63) >> 6; c->sb_rows = (height + 63) >> 6;
    c->pitch[0] = c->sb_cols * 64;
    c->pitch[1] = c->sb_cols * 64 >> ss_h;
    size_t hy = (size_t) c->sb_rows * 64, hc = hy >> ss_v;
    c->plane_off[0] = 0;
    c->plane_off[1] = (size_t) c->pitch[0] * hy * c->bypp;
    c->plane_off[2] = c->plane_off[1] + (size_t) c->pitch[1] * hc * c->bypp;
    c->buf_bytes = c->plane_off[2] + (size_t) c->pitch[1] * hc * c->bypp;
    for (int i = 0; i < nbufs; i++) {
        uint8_t *b = nullptr;
        if (hipMalloc(&b, c->buf_bytes) != hipSuccess) { free_bufs(c); return VP9HIP_ENOMEM; }
        hipMemsetAsync(b, 0, c->buf_bytes, c->st);
        c->bufs.push_back(b);
        c->buf_wh.push_back({ width, height });
    }
    int r = upload_ptab(c);
    if (!r) r = upload_nz(c);
    if (r) return r;
    return hipStreamSynchronize(c->st) == hipSuccess ? 0 : VP9HIP_EEXTERNAL;
}

// Bounding box (columns, rows) of the coefficient positions scan[0 .. eob-1] for every
// (tx, txtp, eob): the kernels transform only columns that can hold a nonzero value.
static uint8_t g_nz[5][4][1025][2];
static void init_nz()
{
    static bool done = false;
    if (done) return;
    static const int16_t *const scans[5][4] = {
        { vp9t_scan_default_4x4, vp9t_scan_col_4x4, vp9t_scan_row_4x4, vp9t_scan_default_4x4 },
        { vp9t_scan_default_8x8, vp9t_scan_col_8x8, vp9t_scan_row_8x8, vp9t_scan_default_8x8 },
        { vp9t_scan_default_16x16, vp9t_scan_col_16x16, vp9t_scan_row_16x16, vp9t_scan_default_16x16 },
        { vp9t_scan_default_32x32, vp9t_scan_default_32x32, vp9t_scan_default_32x32, vp9t_scan_default_32x32 },
        { vp9t_scan_default_4x4, vp9t_scan_default_4x4, vp9t_scan_default_4x4, vp9t_scan_default_4x4 },
    };
    for (int tx = 0; tx < 5; tx++)
        for (int tp = 0; tp < 4; tp++) {
            const int n = 4 << (tx & 3);
            int mc = 0, mr = 0;
            g_nz[tx][tp][0][0] = g_nz[tx][tp][0][1] = 0;
            for (int i = 0; i < n * n; i++) {
                const int rc = scans[tx][tp][i];
                mc = std::max(mc, rc % n + 1);
                mr = std::max(mr, rc / n + 1);
                g_nz[tx][tp][i + 1][0] = (uint8_t) mc;
                g_nz[tx][tp][i + 1][1] = (uint8_t) mr;
            }
        }
    done = true;
}

static int upload_nz(vp9hip_ctx *c)
{
    if (c->nz) return 0;
    init_nz();
    if (hipMalloc(&c->nz, sizeof(g_nz)) != hipSuccess) return VP9HIP_ENOMEM;
    return hipMemcpy(c->nz, g_nz, sizeof(g_nz), hipMemcpyHostToDevice) == hipSuccess ? 0 : VP9HIP_EEXTERNAL;
}

// --------------------------------------------------------------------------
// Per-frame work building
namespace {

struct FrameBuild {
    const vp9h_frame *f;
    int frame_idx;
    int cols, rows, sb_cols, sb_rows;
    int ss_h, ss_v, coef_size;
    int pitch[2];
    int phase;                   // (stream group, chain position) of this frame
    int tile_lo = 0, tile_hi = 64;   // tile columns to reconstruct (default: all)
    PlMcGeo mc;                  // size, subsampling, reference scale factors (vp9.c:845-880), 0 = unscaled
    int refw[3][2], refh[3][2];  // visible reference plane sizes
    uint64_t coef_base;          // element offset of this frame's coefficients in the batch stream
    bool by_diag = false;        // residual buckets per intra diagonal of the SB (fused schedule)
    bool levels = false;         // inter frame: SB steps by intra dependency level, not diagonal
};

struct PendingJob { PJob j; int level, ts; uint32_t d0, nd; };   // deps: pdeps[d0 .. d0 + nd)

} // namespace

#define SCALE_INVALID 0xFFFF

// Host LF program of one SB from its levels and masks (pl_lf_item per item).
static void lf_program(const uint8_t *lvl, const uint8_t (*msk)[2][8][4], int ss_h, int ss_v, bool col0, bool row0,
                       uint8_t *prog)
{
    memset(prog, 0, LF_PROG_BYTES);
    for (int i = 0; i < pl_lf_items(ss_h, ss_v); i++)
        pl_lf_item(i, ss_h, ss_v, col0, row0, [&](int pos) { return (int) lvl[pos]; },
                   [&](int cls, int d, int y, int k) { return (unsigned) msk[cls][d][y][k]; },
                   [&](int off, uint8_t v) { prog[off] = v; });
}

// Build jobs/levels/LF/MC for one frame. Appends to stg. Returns 0 or error.
static int build_frame(vp9hip_ctx *c, Staged &s, FrameBuild &fb, std::vector<std::vector<uint32_t>> &pred_steps,
                       std::vector<std::vector<uint32_t>> &lf_steps)
{
    const vp9h_frame *f = fb.f;
    const int ss_h = fb.ss_h, ss_v = fb.ss_v, cols = fb.cols, rows = fb.rows;
    const int lossless = f->lossless;
    const bool intra_frame = f->keyframe || f->intraonly;
    const uint16_t *eob = f->eobs;
    const uint16_t *eob_end = f->eobs + f->neobs;
    uint64_t coef = 0;                      // running element index within the frame's coefficients
    uint32_t bi = 0;
    const int log2 = f->log2_tile_cols;

    std::vector<PendingJob> pj;
    pj.reserve(1024);
    // level schedule (inter frames): the SB level of the intra job that produced each 4x4
    // unit of the frame (per plane), -1 for inter-predicted units. An SB's level is 1 + the
    // highest level among the units of OTHER SBs its intra jobs read (left, top, top-left:
    // above-right reads stay inside the block's columns, vp9recon.c:71-97 / 103-121), 0
    // when they read only inter pixels, which MC and the residual launches finish before
    // the first intra launch.
    const bool levels = fb.levels && !intra_frame;
    thread_local std::vector<int16_t> umap[3];
    int uw[3] = { 0, 0, 0 };
    if (levels)
        for (int p = 0; p < 3; p++) {
            const int u = (64 >> (p ? ss_h : 0)) >> 2, v = (64 >> (p ? ss_v : 0)) >> 2;
            uw[p] = fb.sb_cols * u;
            umap[p].assign((size_t) uw[p] * fb.sb_rows * v, -1);
        }
    int8_t lmap[3][16 * 16];
    int16_t jmap[3][16 * 16];              // SB-local job index that writes each 4x4 unit
    std::vector<uint16_t> pdeps;

    while (bi < f->nblocks) {
        const vp9h_block *b0 = &f->blocks[bi];
        const int sbx = b0->col >> 3, sby = b0->row >> 3;
        // tile column of this SB (vp9.c:1244-1250)
        int tile_x0 = 0, tile_sb0 = 0, tile = 0;
        for (int ti = 0; ti < (1 << log2); ti++) {
            int s0 = std::min((ti * fb.sb_cols) >> log2, fb.sb_cols), s1 = std::min(((ti + 1) * fb.sb_cols) >> log2, fb.sb_cols);
            if (sbx >= s0 && sbx < s1) { tile_x0 = s0 << 3; tile_sb0 = s0; tile = ti; }
        }
        // sharded batches reconstruct their own tile columns only; every SB keeps its LF
        // record (the loop filter runs over the whole frame on every shard)
        const bool mine = tile >= fb.tile_lo && tile < fb.tile_hi;
        // residual bucket: per intra diagonal of the SB (fused schedule) or the phase
        const int rbi = fb.by_diag ? (sbx - tile_sb0) + sby : fb.phase;
        if ((int) s.rbucket.size() <= rbi) s.rbucket.resize(rbi + 1);
        LFRec lf;
        memset(&lf, 0, sizeof(lf));
        lf.frame = fb.frame_idx; lf.sbx = sbx; lf.sby = sby;
        uint8_t lf_level[64], lf_mask[2][2][8][4];           // VP9Filter of the SB (vp9dec.h:83-87)
        memset(lf_level, 0, sizeof(lf_level));
        memset(lf_mask, 0, sizeof(lf_mask));
        pj.clear();
        int sb_lvl = 0;                 // levels: 1 + highest level of the other SBs read
        memset(lmap, -1, sizeof(lmap));
        memset(jmap, -1, sizeof(jmap));
        pdeps.clear();

        for (; bi < f->nblocks; bi++) {
            const vp9h_block *b = &f->blocks[bi];
            if ((b->col >> 3) != sbx || (b->row >> 3) != sby) break;
            if (b->bs >= VP9H_N_BS || b->tx > 3 || b->uvtx > 3) return VP9HIP_EINVALIDDATA;
            const int bw8 = pl_bwh(1, b->bs, 0), bh8 = pl_bwh(1, b->bs, 1);

            for (int p = 0; p < 3; p++) {
                const int sh = p ? ss_h : 0, sv = p ? ss_v : 0;
                const PlTxGrid g = pl_txgrid(*b, p, cols, rows, ss_h, ss_v);
                const int txs = g.txs, step = g.step, bx = g.bx, by = g.by;
                const int sbsz = 64 >> sh, sbszv = 64 >> sv;
                const int ux_sb = (bx - sbx * sbsz) >> 2, uy_sb = (by - sby * sbszv) >> 2;
                const int units = sbsz >> 2, unitsv = sbszv >> 2;   // 4x4 units of this plane's SB (16 luma)
                for (int y = 0; y < g.ey; y += step)
                    for (int x = 0; x < g.ex; x += step) {
                        int e = 0;
                        if (!b->skip) {
                            if (eob >= eob_end) return VP9HIP_EINVALIDDATA;
                            e = *eob++;
                        }
                        int mode = 0xff, txtp = 0;
                        if (b->intra) {
                            mode = p ? b->uvmode : b->mode[b->bs > VP9H_BS_8x8 && b->tx == 0 ? y * 2 + x : 0];
                            if (mode > 9) return VP9HIP_EINVALIDDATA;
                            txtp = p || txs == 3 ? 0 : pl_intra_txfm_type(mode);
                        }
                        const int tcode = lossless ? 4 : txs;
                        if (e > (16 << (2 * txs))) return VP9HIP_EINVALIDDATA;
                        const int ux0 = ux_sb + x, uy0 = uy_sb + y, n4 = step;
                        uint32_t roff = 0;
                        if (e && mine) {
                            RJob r;
                            memset(&r, 0, sizeof(r));
                            r.coef = (uint32_t) (fb.coef_base + coef);
                            r.eob = (uint16_t) e;
                            r.frame = (uint16_t) fb.frame_idx;
                            r.ptx = (uint8_t) (p | tcode << 2 | (b->intra ? 0 : 1) << 5 | txtp << 6);
                            r.nzc = g_nz[tcode][txtp][e][0];
                            r.nzr = g_nz[tcode][txtp][e][1];
                            if (b->intra) {
                                roff = (uint32_t) s.resid16;
                                r.dst = roff;
                                s.resid16 += (uint64_t) 1 << (2 * txs);
                            } else {
                                r.dst = (uint32_t) ((size_t) (by + y * 4) * fb.pitch[p ? 1 : 0] + bx + x * 4);
                            }
                            s.rbucket[rbi][tcode][txtp].push_back(r);
                        }
                        coef += e;
                        if (!b->intra || !mine) continue;
                        // intra: prediction job with check_intra_mode resolved (vp9recon.c:37-221),
                        // ordered after the jobs that produce the pixels its mode reads
                        PendingJob q;
                        const PlIntra pi = pl_intra_job(p, txs, mode, e, bx + x * 4, by + y * 4, x, g.pw4,
                                                        p ? tile_x0 * 8 >> ss_h : tile_x0 * 8,
                                                        p ? cols * 8 >> ss_h : cols * 8, p ? rows * 8 >> ss_v : rows * 8,
                                                        ux0, uy0);
                        q.j.a = pi.a;
                        q.j.roff = roff;
                        q.ts = txs;
                        // level = 1 + the levels of the tx blocks whose pixels this job's
                        // (substituted) mode reads: the edges[] needs of vp9recon.c:71-97.
                        // Pixels a mode does not read impose no order (the kernel may load
                        // them into its edge buffer; no formula of that mode uses them).
                        int lvl = -1;
                        int8_t *lm = lmap[p];
                        int16_t *jm = jmap[p];
                        q.d0 = (uint32_t) pdeps.size();
                        pl_local_reads(ux0, uy0, n4, pi.nd, pi.trx, units, unitsv, [&](int unit) {
                            lvl = std::max<int>(lvl, lm[unit]);
                            const int j = jm[unit];
                            if (j < 0) return;
                            for (size_t k = q.d0; k < pdeps.size(); k++) if (pdeps[k] == j) return;
                            pdeps.push_back((uint16_t) j);
                        });
                        if (levels) {       // reads of other SBs' units (frame unit coordinates)
                            const int16_t *um = umap[p].data();
                            pl_cross_reads(ux0, uy0, sbx * units + ux0, sby * unitsv + uy0, n4, pi.nd, pi.trx,
                                           [&](int ux, int uy) {
                                if (ux < 0 || uy < 0 || ux >= uw[p]) return;
                                const int16_t l = um[(size_t) uy * uw[p] + ux];
                                if (l >= 0) sb_lvl = std::max(sb_lvl, l + 1);
                            });
                        }
                        q.nd = (uint32_t) pdeps.size() - q.d0;
                        lvl += 1;
                        for (int v = uy0; v < uy0 + n4 && v < unitsv; v++)
                            for (int u = ux0; u < ux0 + n4 && u < units; u++) {
                                lm[v * 16 + u] = (int8_t) lvl;
                                jm[v * 16 + u] = (int16_t) pj.size();
                            }
                        q.level = lvl;
                        pj.push_back(q);
                    }
            }

            // inter prediction units (vp9_mc_template.c:30-464)
            if (!b->intra && mine) {
                const int r0 = b->ref[0], r1 = b->comp ? b->ref[1] : r0;
                if (b->ref[0] > 2 || (b->comp && b->ref[1] > 2)) return VP9HIP_EINVALIDDATA;
                if (fb.mc.scale[r0][0] == SCALE_INVALID || fb.mc.scale[r1][0] == SCALE_INVALID) return VP9HIP_EINVALIDDATA;
                pl_mc_block(*b, fb.mc, (uint32_t) fb.frame_idx, [&](const McUnit &m) { s.mcs.push_back(m); });
            }

            // LF level + masks (vp9block.c:1438-1452)
            if (const int lvl = pl_lf_level(*b, f->lflvl, f->filter_level)) {
                const int col7 = b->col & 7, row7 = b->row & 7;
                for (int yy = 0; yy < bh8; yy++)
                    for (int xx = 0; xx < bw8; xx++) lf_level[(row7 + yy) * 8 + col7 + xx] = (uint8_t) lvl;
                pl_lf_block_masks(*b, cols, rows, ss_h, ss_v,
                                  [&](int cls, int d, int y, int k, unsigned v) { lf_mask[cls][d][y][k] |= (uint8_t) v; });
            }
        }

        // intra jobs of the SB, in decode order with their producer lists; pass packing
        // (list scheduling) happens in merge_mixed
        if (pj.size() > MAX_SB_JOBS) return VP9HIP_EINVALIDDATA;
        if (!pj.empty()) {
            SBRec sr;
            memset(&sr, 0, sizeof(sr));
            sr.frame = fb.frame_idx; sr.sbx = sbx; sr.sby = sby;
            sr.tile_x0 = (uint16_t) tile_x0;
            sr.flags = intra_frame ? 0 : 1;
            Staged::SBHost h;
            h.job0 = (uint32_t) s.sbjobs.size();
            h.njobs = (uint32_t) pj.size();
            h.nlev = 0;
            // each job's producers were appended to pdeps right after the previous job's,
            // so the SB's lists go over in one block
            const uint32_t jd = (uint32_t) s.jdeps.size();
            s.jdeps.insert(s.jdeps.end(), pdeps.begin(), pdeps.end());
            const size_t j0 = s.sbjobs.size();
            s.sbjobs.resize(j0 + pj.size());
            for (size_t k = 0; k < pj.size(); k++) {
                s.sbjobs[j0 + k] = pj[k].j;
                s.jdep0.push_back(jd + pj[k].d0);
                h.nlev = std::max<uint32_t>(h.nlev, (uint32_t) pj[k].level + 1);
            }
            s.jdep0.push_back(jd + (uint32_t) pdeps.size());
            s.sbh.push_back(h);
            uint32_t sbi = (uint32_t) s.sbs.size();
            s.sbs.push_back(sr);
            int d = levels ? sb_lvl : (sbx - tile_sb0) + sby;
            if (levels)                                  // this SB's intra units carry its level
                for (const PendingJob &q : pj) {
                    const int p = PJ_PLANE(q.j), n4 = 1 << q.ts;
                    const int units = (64 >> (p ? ss_h : 0)) >> 2, unitsv = (64 >> (p ? ss_v : 0)) >> 2;
                    const int fx = sbx * units + PJ_X4(q.j), fy = sby * unitsv + PJ_Y4(q.j);
                    for (int v = 0; v < n4; v++)
                        for (int u = 0; u < n4; u++)
                            if (PJ_X4(q.j) + u < units && PJ_Y4(q.j) + v < unitsv)
                                umap[p][(size_t) (fy + v) * uw[p] + fx + u] = (int16_t) sb_lvl;
                }
            if ((int) pred_steps.size() <= d) pred_steps.resize(d + 1);
            pred_steps[d].push_back(sbi);
        }
        if (f->filter_level) {
            uint32_t li = (uint32_t) s.lfs.size();
            lf_program(lf_level, lf_mask, ss_h, ss_v, sbx == 0, sby == 0, lf.prog);
            s.lfs.push_back(lf);
            int d = sbx + 2 * sby;
            if ((int) lf_steps.size() <= d) lf_steps.resize(d + 1);
            lf_steps[d].push_back(li);
        }
    }
    if (eob != eob_end) return VP9HIP_EINVALIDDATA;
    if (coef != f->ncoefs) return VP9HIP_EINVALIDDATA;
    return 0;
}

// Pass packing of one SB's intra jobs by list scheduling: every pass takes ready jobs
// (all producers in earlier passes), highest remaining critical path first, up to 64
// lanes (n lanes per n x n job, any sizes mixed). Jobs in a pass are ordered 32x32,
// 16x16, 8x8, 4x4 so every job's lane group is aligned to its size. Pass word:
// first << 14 | c4 << 9 | c8 << 5 | c16 << 2 | c32 (job counts per size).
static int merge_mixed(Staged &s, uint32_t sbi)
{
    WGRec wg;
    memset(&wg, 0xff, sizeof(wg));
    wg.job0 = (uint32_t) s.pjobs.size();
    wg.pass0 = (uint32_t) s.passes.size();
    wg.sb[0] = sbi;
    const Staged::SBHost &h = s.sbh[sbi];
    const int N = (int) h.njobs;
    const PJob *jobs = s.sbjobs.data() + h.job0;
    // the SB's jobs are consecutive, so their producer lists are too: job k's list is
    // jdep0[job0 + k + sbi] .. (one end marker per earlier SB shifts the index by sbi)
    const uint32_t *d0 = s.jdep0.data() + h.job0 + sbi;
    // scratch reused across SBs of this thread (no allocations per SB or pass):
    // successor lists in CSR form, in-degrees, heights (longest path to a sink)
    thread_local std::vector<int> indeg, height, soff, ready, next, take, fresh;
    thread_local std::vector<uint16_t> succ;
    indeg.assign(N, 0); height.assign(N, 1); soff.assign(N + 1, 0);
    const uint32_t e0 = d0[0], e1 = d0[N];
    for (uint32_t e = e0; e < e1; e++) soff[s.jdeps[e] + 1]++;
    for (int k = 0; k < N; k++) soff[k + 1] += soff[k];
    succ.resize(e1 - e0);
    {
        thread_local std::vector<int> fill;
        fill.assign(soff.begin(), soff.end() - 1);
        for (int k = 0; k < N; k++) {
            indeg[k] = (int) (d0[k + 1] - d0[k]);
            for (uint32_t e = d0[k]; e < d0[k + 1]; e++) succ[fill[s.jdeps[e]]++] = (uint16_t) k;
        }
    }
    for (int k = N - 1; k >= 0; k--)                      // producers precede consumers
        for (int e = soff[k]; e < soff[k + 1]; e++) height[k] = std::max(height[k], height[succ[e]] + 1);
    // ready list kept in priority order: highest remaining critical path first, then
    // decode order; each pass merges its newly ready jobs into the leftovers
    auto before = [&](int a, int b) { return height[a] != height[b] ? height[a] > height[b] : a < b; };
    ready.clear();
    for (int k = 0; k < N; k++) if (!indeg[k]) ready.push_back(k);
    std::sort(ready.begin(), ready.end(), before);
    int done = 0;
    while (done < N) {
        if (ready.empty()) return VP9HIP_EBUG;
        int lanes = 0, cnt[4] = { 0, 0, 0, 0 };
        take.clear();
        next.clear();
        for (int k : ready) {
            const int n = 4 << PJ_TS(jobs[k]);
            if (lanes + n <= 64) { take.push_back(k); lanes += n; }
            else next.push_back(k);
        }
        // lane groups by size, largest first (stable: decode order within a size)
        const uint32_t first = (uint32_t) (s.pjobs.size() - wg.job0);
        for (int ts = 3; ts >= 0; ts--)
            for (int k : take)
                if ((int) PJ_TS(jobs[k]) == ts) { s.pjobs.push_back(jobs[k]); cnt[ts]++; }
        s.passes.push_back(first << 14 | (uint32_t) cnt[0] << 9 | (uint32_t) cnt[1] << 5 | (uint32_t) cnt[2] << 2 |
                           (uint32_t) cnt[3]);
        fresh.clear();
        for (int k : take)
            for (int e = soff[k]; e < soff[k + 1]; e++)
                if (--indeg[succ[e]] == 0) fresh.push_back(succ[e]);
        std::sort(fresh.begin(), fresh.end(), before);
        done += (int) take.size();
        ready.resize(next.size() + fresh.size());
        std::merge(next.begin(), next.end(), fresh.begin(), fresh.end(), ready.begin(), before);
    }
    const size_t nj = s.pjobs.size() - wg.job0, np = s.passes.size() - wg.pass0;
    if (nj > MAX_SB_JOBS || np > MAX_SB_JOBS) return VP9HIP_EINVALIDDATA;
    wg.njobs = (uint16_t) nj;
    wg.npass = (uint16_t) np;
    s.wgs.push_back(wg);
    return 0;
}

// The work plan of one frame, built on its own (host threads in parallel): the Staged
// images with frame-local indices, the intra diagonals' workgroups and LF diagonals' SBs.
struct FramePlan {
    Staged s;
    std::vector<std::vector<uint32_t>> wsteps, lsteps;
    int err = 0;
};

static int plan_frame(FrameBuild fb, FramePlan &fp)
{
    fp.s.rbucket.resize(1);
    fb.phase = 0;                                // non-fused: one bucket set (index 0)
    std::vector<std::vector<uint32_t>> ps;
    int r = build_frame(nullptr, fp.s, fb, ps, fp.lsteps);
    if (r < 0) return r;
    fp.wsteps.resize(ps.size());
    for (size_t d = 0; d < ps.size(); d++)
        for (uint32_t sbi : ps[d]) {
            fp.wsteps[d].push_back((uint32_t) fp.s.wgs.size());
            r = merge_mixed(fp.s, sbi);
            if (r) return r;
        }
    return 0;
}

// Pixel bytes of SB (sbx, sby) of frame f (all planes, visible area): its share of the
// frame's algorithmic bytes P.
static double sb_bytes(const vp9hip_ctx *c, const vp9h_frame &f, int sbx, int sby)
{
    const int w = std::min(64, f.width - sbx * 64), h = std::min(64, f.height - sby * 64);
    return (double) w * h * c->bypp * (1.0 + 2.0 / ((1 << c->ss_h) * (1 << c->ss_v)));
}

// ==========================================================================
// Device-planned batches (the default). stage_dev: the batch geometry on the host (SB slots,
// residual segments, intra-step keys, LF diagonal lists, k_lfr task tables: O(SBs), no
// per-block work) and one upload of the packets; plan_dev (every run): the device planner
// (vp9hip_plan.hip), a readback of its summary (record counts, status) and the launch list.
struct DevIn {
    const vp9h_frame *pkts;
    int n, G, maxpos, NP, csz;
    const std::vector<FrameBuild> *fbs;
    const std::vector<char> *res_fused, *lvl_ph;
    bool fuse, lfr_any;
};

// row-LF counter blocks of a staged batch, zeroed; word 3 of each block is the spin bound of
// a hand-off wait (0 = default; vp9hip_test_hooks sets a small one to force the timeout path)
static void init_lfr_ctr(const vp9hip_ctx *c, const Staged &s, uint32_t *ctr)
{
    memset(ctr, 0, (size_t) s.n_ctr * 4);
    for (uint32_t o : s.lfr_ctr) ctr[o + 3] = c->lfr_spin;
}

// Keyframe batches (every phase wide, not fused, no k_lfr, intra frames only): the launch
// list plan_dev would build, from the geometry. Intra frames have intra work in every SB
// (PLS_ORDER rejects an SB without blocks), so step key k holds every SB of its phase's
// frames on intra diagonal k - key0, and the step lists' offsets are the prefix sums of
// those counts (k_pkeys). Residual launches take their job ranges from the summary.
static void build_static_plan(vp9hip_ctx *c, const DevIn &in, const std::vector<uint32_t> &slot0)
{
    Staged &s = c->stg;
    const bool off = !c->static_plan;
    s.stat = false;
    s.launches.clear();
    s.exp_ko.clear();
    if (off || !in.fuse) return;
    const std::vector<FrameBuild> &fbs = *in.fbs;
    for (const Staged::DevPhase &P : s.dph) {
        if (P.frames.empty()) continue;
        if (P.fused || P.levels || P.lfr) return;
        for (int i : P.frames)
            if (!(in.pkts[i].keyframe || in.pkts[i].intraonly)) return;
    }
    std::vector<uint32_t> kc(s.nkey, 0);
    for (const Staged::DevPhase &P : s.dph)
        for (int i : P.frames) {
            const FrameBuild &fb = fbs[i];
            for (int y = 0; y < fb.sb_rows; y++)
                for (int x = 0; x < fb.sb_cols; x++) {
                    int ts0;
                    pl_tile_of(x, fb.sb_cols, fb.f->log2_tile_cols, &ts0);
                    const uint32_t k = P.key0 + (uint32_t) ((x - ts0) + y);
                    if (k < s.nkey) kc[k]++;
                }
        }
    s.exp_ko.assign(s.nkey + 1, 0);
    for (uint32_t k = 0; k < s.nkey; k++) s.exp_ko[k + 1] = s.exp_ko[k] + kc[k];
    // the step lists themselves (k_plists' output): key k's SBs, frames in phase order,
    // raster order inside a frame
    s.stat_lists.assign(s.exp_ko[s.nkey], 0);
    std::vector<uint32_t> fill(s.exp_ko.begin(), s.exp_ko.end() - 1);
    for (const Staged::DevPhase &P : s.dph)
        for (int i : P.frames) {
            const FrameBuild &fb = fbs[i];
            for (int y = 0; y < fb.sb_rows; y++)
                for (int x = 0; x < fb.sb_cols; x++) {
                    int ts0;
                    pl_tile_of(x, fb.sb_cols, fb.f->log2_tile_cols, &ts0);
                    const uint32_t k = P.key0 + (uint32_t) ((x - ts0) + y);
                    if (k < s.nkey) s.stat_lists[fill[k]++] = slot0[i] + (uint32_t) (y * fb.sb_cols + x);
                }
        }
    for (int k = 0; k < K_N; k++) s.alg_stat[k] = s.alg_base[k];
    const uint32_t H = s.host_lists;
    const int nph = (int) s.dph.size();
    for (int g = 0; g < s.ngroups; g++)
        for (int ph = 0; ph < nph; ph++) {
            const Staged::DevPhase &P = s.dph[ph];
            if (P.frames.empty() || P.group != g) continue;
            // per transform code, the tx blocks of the phase's coded blocks: a bound of its
            // residual jobs (those with eob > 0) that sizes the launch as the summary's count would
            uint64_t ub[5] = { 0, 0, 0, 0, 0 };
            for (int i : P.frames) {
                const vp9h_frame &f = in.pkts[i];
                const FrameBuild &fb = fbs[i];
                for (uint32_t k = 0; k < f.nblocks; k++) {
                    const vp9h_block &b = f.blocks[k];
                    if (b.skip || b.bs >= VP9H_N_BS || b.tx > 3 || b.uvtx > 3) continue;
                    for (int p = 0; p < 3; p++) {
                        const PlTxGrid gr = pl_txgrid(b, p, fb.cols, fb.rows, c->ss_h, c->ss_v);
                        ub[f.lossless ? 4 : gr.txs] += (uint64_t) (gr.nx * gr.ny);
                    }
                }
            }
            for (int tc = 0; tc < 5; tc++) {
                if (!ub[tc]) continue;
                Launch L = { K_RESID, (uint32_t) (P.g_res + tc * 2), (uint32_t) std::min<uint64_t>(ub[tc], 0xffffffffu), tc,
                             g, ph, PART_RECON, 0 };
                L.devr = 1;
                s.launches.push_back(L);
            }
            const int np = P.np, nlf = P.nlf;
            const int nt = std::max(np, nlf ? nlf + PLF_LAG : 0);
            for (int t = 0; t < nt; t++) {
                const uint32_t k = P.key0 + (uint32_t) t;
                const uint32_t pn = t < np && k < s.nkey ? kc[k] : 0u;
                const int j = t - PLF_LAG;
                const std::pair<uint32_t, uint32_t> lv = j >= 0 && j < nlf ? P.lf[j] : std::make_pair(0u, 0u);
                if (!pn) {
                    if (lv.second) s.launches.push_back(Launch{ K_LF, lv.first, lv.second, 0, g, ph, PART_LF, j });
                    continue;
                }
                Launch L = { K_PLF, H + s.exp_ko[k], pn, 0, g, ph, PART_RECON, t };
                L.off2 = lv.first;
                L.n2 = lv.second;
                if (t < (int) P.pred_bytes.size()) {
                    s.alg_stat[K_PRED] -= P.pred_bytes[t];
                    s.alg_stat[K_PLF] += P.pred_bytes[t];
                }
                if (lv.second) {
                    s.alg_stat[K_LF] -= P.lf_bytes[j];
                    s.alg_stat[K_PLF] += P.lf_bytes[j];
                }
                s.launches.push_back(L);
            }
        }
    s.stat = true;
}

static int stage_dev(vp9hip_ctx *c, const DevIn &in)
{
    Staged &s = c->stg;
    const int n = in.n;
    const std::vector<FrameBuild> &fbs = *in.fbs;
    const vp9h_frame *pkts = in.pkts;
    s.dev = true;
    s.planned = false;
    s.nframes = n;
    s.jcap = s.rcap = pl_rcap(c->ss_h, c->ss_v);
    s.fuse = in.fuse;
    std::vector<uint32_t> slot0(n + 1, 0);
    s.max_blk = 0; s.max_sb = 0;
    for (int i = 0; i < n; i++) {
        slot0[i + 1] = slot0[i] + (uint32_t) (fbs[i].sb_cols * fbs[i].sb_rows);
        s.max_blk = std::max(s.max_blk, (int) pkts[i].nblocks);
        s.max_sb = std::max(s.max_sb, fbs[i].sb_cols * fbs[i].sb_rows);
    }
    const uint32_t NS = slot0[n];
    s.nslots = NS;
    std::vector<uint32_t> slot_pos(NS, 0), seg_pre4, seg_sz, seg_pre1, gidx, hl;
    s.dph.assign(in.NP, Staged::DevPhase());
    for (int i = 0; i < n; i++) s.dph[fbs[i].phase].frames.push_back(i);
    std::vector<PlanFrame> pf(n);
    memset(pf.data(), 0, pf.size() * sizeof(PlanFrame));
    uint32_t base = 0, segs = 0, keys = 0, sbs_before = 0;
    s.n_ctr = 0;
    s.lfr_ctr.clear();
    for (int ph = 0; ph < in.NP; ph++) {
        Staged::DevPhase &P = s.dph[ph];
        if (P.frames.empty()) continue;
        P.group = ph / (in.maxpos + 1);
        P.fused = (*in.res_fused)[ph];
        P.levels = (*in.lvl_ph)[ph];
        P.lfr = in.lfr_any && (c->lf_rows > 1 || (int) P.frames.size() < LFR_MAX_FRAMES);
        P.all_lf = true;
        for (int i : P.frames) P.all_lf &= fbs[i].f->filter_level != 0;
        if (P.levels && c->pred_df && c->ss_h && c->ss_v) {  // the phase's intra levels as one k_predd
            P.pred_ctr = (int) s.n_ctr;
            s.lfr_ctr.push_back(s.n_ctr);
            s.n_ctr += 4;              // ticket, finished, timeouts, spin
        }
        int nd = 0, nlfd = 0, nk = 0;
        for (int i : P.frames) {
            const FrameBuild &fb = fbs[i];
            const int l2 = fb.f->log2_tile_cols;
            int tw = 0;
            for (int t = 0; t < (1 << l2); t++)
                tw = std::max(tw, std::min(((t + 1) * fb.sb_cols) >> l2, fb.sb_cols) - std::min((t * fb.sb_cols) >> l2, fb.sb_cols));
            nd = std::max(nd, tw + fb.sb_rows - 1);
            nlfd = std::max(nlfd, fb.sb_cols + 2 * (fb.sb_rows - 1));
            nk = std::max(nk, fb.sb_cols + fb.sb_rows - 1);
        }
        P.np = nd;
        P.nseg = P.fused ? nd : 1;
        P.seg_sz.assign(P.nseg, 0);
        P.pred_bytes.assign(nd, 0.0);
        P.nkey = nk;
        P.key0 = keys;
        keys += (uint32_t) nk;
        // residual segments: the SBs' positions (frames in order, raster order)
        for (int i : P.frames) {
            const FrameBuild &fb = fbs[i];
            const bool intra = fb.f->keyframe || fb.f->intraonly;
            for (int y = 0; y < fb.sb_rows; y++)
                for (int x = 0; x < fb.sb_cols; x++) {
                    int ts0;
                    pl_tile_of(x, fb.sb_cols, fb.f->log2_tile_cols, &ts0);
                    const int d = (x - ts0) + y;
                    slot_pos[slot0[i] + (uint32_t) (y * fb.sb_cols + x)] = P.seg_sz[P.fused ? d : 0]++;
                    if (intra) P.pred_bytes[d] += sb_bytes(c, *fb.f, x, y);
                }
        }
        uint32_t S = 0;
        for (uint32_t z : P.seg_sz) S += z;
        const uint32_t s4 = 4 * S;
        P.g_res = (int) gidx.size();
        uint32_t pre = 0;
        for (int d = 0; d < P.nseg; d++) {
            seg_pre4.push_back(base + 4 * pre);
            seg_sz.push_back(P.seg_sz[d]);
            seg_pre1.push_back(sbs_before + pre);
            for (int tc = 0; tc < 5; tc++) {
                gidx.push_back(base + 4 * pre + (uint32_t) tc * s4);
                gidx.push_back(base + 4 * pre + (uint32_t) tc * s4 + 4 * P.seg_sz[d]);
            }
            pre += P.seg_sz[d];
        }
        P.g_mc = (int) gidx.size();                      // MC-count offsets (bit 31)
        gidx.push_back(0x80000000u | sbs_before);
        gidx.push_back(0x80000000u | (sbs_before + S));
        for (int i : P.frames) { pf[i].seg0 = segs; pf[i].s4 = s4; pf[i].key0 = P.key0; }
        segs += (uint32_t) P.nseg;
        base += 20 * S;                                  // 5 transform codes x 4 transform types per SB
        sbs_before += S;
        // LF diagonals x + 2y: every SB of the phase's filtered frames
        std::vector<std::vector<uint32_t>> lfd(nlfd);
        P.lf_bytes.assign(nlfd, 0.0);
        for (int i : P.frames) {
            const FrameBuild &fb = fbs[i];
            if (!fb.f->filter_level) continue;
            for (int y = 0; y < fb.sb_rows; y++)
                for (int x = 0; x < fb.sb_cols; x++) {
                    lfd[x + 2 * y].push_back(slot0[i] + (uint32_t) (y * fb.sb_cols + x));
                    P.lf_bytes[x + 2 * y] += 2.0 * sb_bytes(c, *fb.f, x, y);
                }
        }
        P.lf.assign(nlfd, { 0, 0 });
        for (int j = 0; j < nlfd; j++) {
            P.lf[j] = { (uint32_t) hl.size(), (uint32_t) lfd[j].size() };
            hl.insert(hl.end(), lfd[j].begin(), lfd[j].end());
        }
        // LF diagonals fused into the intra launches (the rest: k_lfr), as in stage()
        const int nres = P.fused ? P.nseg : 0;
        const int jlfr = std::max(0, std::max(P.np, nres - 1) - PLF_LAG);
        P.nlf = P.lfr ? std::min(jlfr, nlfd) : nlfd;
        if (P.lfr) {
            const int j0 = (!in.fuse || P.levels) ? 0 : P.nlf;
            // task table: one task per (frame, SB row), rows-major, each naming the task of
            // the row above and its SBs' LF records (= slots) left to right
            std::vector<std::vector<uint32_t>> tid;
            std::vector<int> lff;
            int maxr = 0;
            for (int i : P.frames)
                if (fbs[i].f->filter_level) { lff.push_back(i); maxr = std::max(maxr, fbs[i].sb_rows); }
            tid.resize(lff.size());
            std::vector<uint32_t> recs, offs;
            auto start = [&](int r) { return std::max(0, j0 - 2 * r); };
            for (int r = 0; r < maxr; r++)
                for (size_t k = 0; k < lff.size(); k++) {
                    const FrameBuild &fb = fbs[lff[k]];
                    if (r >= fb.sb_rows) continue;
                    const int nc = fb.sb_cols, c0 = start(r);
                    if (c0 >= nc) { tid[k].push_back(~0u); continue; }
                    tid[k].push_back((uint32_t) offs.size());
                    offs.push_back((uint32_t) recs.size());
                    const uint32_t dep = r ? tid[k][r - 1] : ~0u;
                    recs.push_back(dep);
                    recs.push_back((uint32_t) nc);
                    recs.push_back((uint32_t) c0);
                    recs.push_back(dep != ~0u ? (uint32_t) std::max(0, start(r - 1) - 1) : 0u);
                    for (int x = c0; x < nc; x++) recs.push_back(slot0[lff[k]] + (uint32_t) (r * nc + x));
                    for (int x = c0; x < nc; x++) P.lfr_bytes += 2.0 * sb_bytes(c, *fb.f, x, r);
                }
            if (!offs.empty()) {
                const uint32_t nt = (uint32_t) offs.size();
                for (uint32_t &o : offs) o += nt;
                P.lfr_off = (uint32_t) hl.size();
                P.lfr_n = nt;
                hl.insert(hl.end(), offs.begin(), offs.end());
                hl.insert(hl.end(), recs.begin(), recs.end());
                P.lfr_ctr = (int) s.n_ctr;
                s.lfr_ctr.push_back(s.n_ctr);
                s.n_ctr += 4 + nt;         // ticket, done, timeouts, spin; progress per task
            } else {
                P.lfr = false;
            }
        }
    }
    s.pdone = 0;
    for (const Staged::DevPhase &P : s.dph)
        if (P.pred_ctr >= 0) { s.pdone = s.n_ctr; s.n_ctr += NS; break; }
    s.nkey = keys;
    s.host_lists = (uint32_t) hl.size();
    s.n_gidx = (uint32_t) gidx.size();
    // frame records of the planner
    uint64_t nb = 0, ne = 0, nc = 0, nmc = 0;
    s.any_levels = false;
    s.plan_flags = 0;
    s.frame_res_bytes.assign(n, 0.0);
    s.frame_fused.assign(n, 0);
    for (int i = 0; i < n; i++) {
        const FrameBuild &fb = fbs[i];
        const vp9h_frame *f = &pkts[i];
        PlanFrame &F = pf[i];
        F.blk0 = (uint32_t) nb; F.nblk = f->nblocks;
        F.eob0 = (uint32_t) ne; F.neob = f->neobs;
        F.coef0 = (uint32_t) nc; F.ncoef = (uint32_t) f->ncoefs;
        F.slot0 = slot0[i];
        F.frame = i;
        F.sb_cols = fb.sb_cols; F.sb_rows = fb.sb_rows;
        F.log2_tc = f->log2_tile_cols; F.log2_tr = f->log2_tile_rows;
        F.tile_lo = fb.tile_lo; F.tile_hi = fb.tile_hi;
        F.lossless = f->lossless; F.filter_level = f->filter_level;
        F.intra = f->keyframe || f->intraonly;
        F.by_diag = fb.by_diag;
        F.levels = fb.levels && !F.intra;
        F.bypp = c->bypp;
        F.pitch[0] = fb.pitch[0]; F.pitch[1] = fb.pitch[1];
        F.mc = fb.mc;
        memcpy(F.lflvl, f->lflvl, sizeof(F.lflvl));
        s.any_levels |= F.levels != 0;
        s.plan_flags |= (f->filter_level ? 1 : 0) | (F.intra ? 0 : 2);
        nb += f->nblocks; ne += f->neobs; nc += f->ncoefs;
        if (!F.intra) nmc += (uint64_t) 12 * f->nblocks;
        s.frame_res_bytes[i] = (double) f->ncoefs * in.csz;
        s.frame_fused[i] = fb.by_diag;
    }
    if (nb >= 0xffffffffull || ne >= 0xffffffffull || nc >= 0xffffffffull) return VP9HIP_ENOMEM;
    s.nblk = (uint32_t) nb; s.neob = (uint32_t) ne; s.ncoef = (uint32_t) nc;
    s.ncnt = 20 * NS;
    for (int k = 0; k < K_N; k++) s.alg_base[k] = s.alg_bytes[k];
    build_static_plan(c, in, slot0);
    // arena: the uploaded part (one DMA from a pinned image), then the planner's buffers
    auto al = [](size_t x) { return (x + 255) & ~(size_t) 255; };
    size_t o = 0;
    s.o_frames = o; o = al(o + n * sizeof(FrameDesc));
    s.o_pf = o; o = al(o + n * sizeof(PlanFrame));
    s.o_slotpos = o; o = al(o + (size_t) NS * 4);
    s.o_segpre = o; o = al(o + seg_pre4.size() * 4);
    s.o_segsz = o; o = al(o + seg_sz.size() * 4);
    s.o_segpre1 = o; o = al(o + seg_pre1.size() * 4);
    s.o_gidx = o; o = al(o + gidx.size() * 4);
    s.o_lists = o; o = al(o + (hl.size() + NS) * 4);      // host lists, then the device step lists
    s.o_expko = o; o = al(o + (s.stat ? s.exp_ko.size() : 0) * 4);   // static lists' offsets (k_psort)
    s.o_ctr = o; o = al(o + (size_t) s.n_ctr * 4);
    s.o_blocks = o; o = al(o + nb * sizeof(vp9h_block));
    s.o_eobs = o; o = al(o + ne * 2);
    s.o_coefs = o; o = al(o + nc * in.csz + 64);
    const size_t up = o;
    s.o_bneob = o; o = al(o + (nb + 1) * 4);
    s.o_beob0 = o; o = al(o + (nb + 1) * 4);
    s.o_sbfirst = o; o = al(o + (size_t) 2 * NS * 4);        // sb_first, then sb_end
    s.o_sbncoef = o; o = al(o + ((size_t) NS + 1) * 4);
    s.o_sbcoef0 = o; o = al(o + ((size_t) NS + 1) * 4);
    s.o_cnt = o; o = al(o + ((size_t) s.ncnt + 1) * 4);
    s.o_cnt0 = o; o = al(o + ((size_t) s.ncnt + 1) * 4);
    s.o_cntm = o; o = al(o + ((size_t) NS + 1) * 4);
    s.o_cntm0 = o; o = al(o + ((size_t) NS + 1) * 4);
    s.o_ibits = o; o = al(o + (size_t) NS * 96);
    s.o_sbinfo = o; o = al(o + (size_t) NS * 4);
    s.o_sbkey = o; o = al(o + (size_t) NS * 4);
    s.o_sbkpos = o; o = al(o + (size_t) NS * 4);
    s.o_keyoff = o; o = al(o + ((size_t) keys + 1) * 4);
    s.o_keycnt = o;                                           // zeroed every run: counts, status, byte totals
    s.o_status = al(o + ((size_t) keys + 1) * 4);
    s.o_fbytes = s.o_status + 256;
    s.o_fbad = s.o_fbytes + (size_t) n * 16;                 // per-frame status bits
    o = al(s.o_fbad + (size_t) n * 4);
    s.zero_bytes = o - s.o_keycnt;
    // status, count offsets, key offsets, byte totals, per-frame status, status[1]
    s.summary_words = 1 + gidx.size() + keys + 1 + 5 * (size_t) n + 1;
    s.o_summary = o; o = al(o + s.summary_words * 4);
    s.o_sbs = o; o = al(o + (size_t) NS * sizeof(SBRec));
    s.o_wgs = o; o = al(o + (size_t) NS * sizeof(WGRec));
    s.o_lfs = o; o = al(o + (size_t) NS * sizeof(LFRec));
    s.o_pjobs = o; o = al(o + (size_t) NS * s.jcap * sizeof(PJob));
    s.o_passes = o; o = al(o + (size_t) NS * s.jcap * 4);
    s.o_jobw = o; o = al(o + (size_t) NS * s.jcap * 4);
    s.o_sbnj = o; o = al(o + (size_t) NS * 4);
    s.o_rjobs = o; o = al(o + (ne + 1) * sizeof(RJob));
    s.o_mcs = o; o = al(o + (nmc + 1) * sizeof(McUnit));
    s.cap_mcs = (uint32_t) (nmc + 1);
    s.scan_bytes = std::max<size_t>(vp9hip_plan_scan_bytes(std::max<uint64_t>(nb, s.ncnt) + 1), 256);
    s.o_scan = o; o = al(o + s.scan_bytes);
    if (o > s.arena_cap) {
        if (s.arena) hipFree(s.arena);
        s.arena = nullptr;
        s.arena_cap = 0;
        if (hipMalloc(&s.arena, o) != hipSuccess) return VP9HIP_ENOMEM;
        s.arena_cap = o;
    }
    if (up > s.pinned_cap) {
        if (s.pinned) hipHostFree(s.pinned);
        s.pinned = nullptr;
        s.pinned_cap = 0;
        if (hipHostMalloc((void **) &s.pinned, up, hipHostMallocDefault) != hipSuccess) return VP9HIP_ENOMEM;
        s.pinned_cap = up;
    }
    if (s.summary_words * 4 > s.summary_cap) {
        if (s.summary_h) hipHostFree(s.summary_h);
        s.summary_h = nullptr;
        s.summary_cap = 0;
        if (hipHostMalloc((void **) &s.summary_h, s.summary_words * 4, hipHostMallocDefault) != hipSuccess) return VP9HIP_ENOMEM;
        s.summary_cap = s.summary_words * 4;
    }
    const size_t rbytes = ((size_t) NS + 1) * s.rcap * 32;
    if (rbytes > s.resid_cap) {
        if (s.resid) hipFree(s.resid);
        s.resid = nullptr;
        s.resid_cap = 0;
        if (hipMalloc(&s.resid, rbytes) != hipSuccess) return VP9HIP_ENOMEM;
        s.resid_cap = rbytes;
    }
    uint8_t *img = s.pinned;
    memcpy(img + s.o_frames, s.frames.data(), n * sizeof(FrameDesc));
    memcpy(img + s.o_pf, pf.data(), n * sizeof(PlanFrame));
    memcpy(img + s.o_slotpos, slot_pos.data(), (size_t) NS * 4);
    if (!seg_pre4.empty()) memcpy(img + s.o_segpre, seg_pre4.data(), seg_pre4.size() * 4);
    if (!seg_sz.empty()) memcpy(img + s.o_segsz, seg_sz.data(), seg_sz.size() * 4);
    if (!seg_pre1.empty()) memcpy(img + s.o_segpre1, seg_pre1.data(), seg_pre1.size() * 4);
    if (!gidx.empty()) memcpy(img + s.o_gidx, gidx.data(), gidx.size() * 4);
    if (!hl.empty()) memcpy(img + s.o_lists, hl.data(), hl.size() * 4);
    if (s.stat && !s.stat_lists.empty()) {
        if (s.stat_lists.size() > NS) return VP9HIP_EBUG;
        memcpy(img + s.o_lists + hl.size() * 4, s.stat_lists.data(), s.stat_lists.size() * 4);
        memcpy(img + s.o_expko, s.exp_ko.data(), s.exp_ko.size() * 4);
    }
    init_lfr_ctr(c, s, (uint32_t *) (img + s.o_ctr));
    {   // packets: blocks, eobs, coefficients (frames copied in parallel)
        std::atomic<int> next(0);
        auto worker = [&]() {
            for (int i; (i = next.fetch_add(1)) < n;) {
                const vp9h_frame *f = &pkts[i];
                const PlanFrame &F = pf[i];
                if (f->nblocks) memcpy(img + s.o_blocks + (size_t) F.blk0 * sizeof(vp9h_block), f->blocks, (size_t) f->nblocks * sizeof(vp9h_block));
                if (f->neobs) memcpy(img + s.o_eobs + (size_t) F.eob0 * 2, f->eobs, (size_t) f->neobs * 2);
                if (f->ncoefs) memcpy(img + s.o_coefs + (size_t) F.coef0 * in.csz, f->coefs, (size_t) f->ncoefs * in.csz);
            }
        };
        const int nt = std::min(n, c->host_threads);
        std::vector<std::thread> pool;
        for (int t = 1; t < nt; t++) pool.emplace_back(worker);
        worker();
        for (auto &t : pool) t.join();
    }
    if (c->test_reject) {   // test hook (vp9hip_test_hooks): the k-th batch the context stages
        // gets an intra block with a mode the device planner rejects as the first block of its
        // frame f, so the front ends' handling of a rejected frame can be tested from real
        // bitstreams
        const int k = c->test_reject & 0xffff, f = c->test_reject >> 16;
        if (++c->nstaged == k && f < n && pf[f].nblk) {
            vp9h_block *b = (vp9h_block *) (img + s.o_blocks) + pf[f].blk0;
            b->intra = 1;
            for (int m = 0; m < 4; m++) b->mode[m] = 20;
        }
    }
    // the upload goes on the planner stream: the other batch slot's pixel kernels keep the
    // main stream busy meanwhile
    const hipStream_t us = plan_stream(c);
    HIPCHK(hipMemcpyAsync(s.arena, img, up, hipMemcpyHostToDevice, us));
    // scan sentinels (never written by the planner)
    HIPCHK(hipMemsetAsync(s.arena + s.o_bneob + nb * 4, 0, 4, us));
    HIPCHK(hipMemsetAsync(s.arena + s.o_sbncoef + (size_t) NS * 4, 0, 4, us));
    HIPCHK(hipMemsetAsync(s.arena + s.o_cnt + (size_t) s.ncnt * 4, 0, 4, us));
    HIPCHK(hipMemsetAsync(s.arena + s.o_cntm + (size_t) NS * 4, 0, 4, us));
    // no host wait: the planner and the pixel launches follow on this stream (or after it),
    // and the next staging of this slot waits for the event before rewriting the image
    if (!s.up_ev) HIPCHK(hipEventCreateWithFlags(&s.up_ev, hipEventDisableTiming));
    HIPCHK(hipEventRecord(s.up_ev, us));
    s.ready = true;
    return 0;
}

// The per-frame verdicts of a rejected batch from its summary: frames whose status bits are
// set are rejected, the others get `good` (0: reconstructed, EAGAIN: not run). A status that
// names no frame (PLS_BOUNDS: a shared buffer's capacity; PLS_TOTAL: a frame's totals shift
// the batch-wide scans) rejects every frame. Returns the number rejected.
static int frame_verdicts(Staged &s, const uint32_t *sm, int good)
{
    const uint32_t *fbad = sm + 1 + s.n_gidx + s.nkey + 1 + 4 * (size_t) s.nframes;
    const bool all = (sm[0] & (PLS_BOUNDS | PLS_TOTAL)) != 0;
    s.fstat.assign(s.nframes, good);
    int nbad = 0;
    for (int i = 0; i < s.nframes; i++)
        if (all || fbad[i]) { s.fstat[i] = VP9HIP_EINVALIDDATA; nbad++; }
    return nbad;
}

// A static-plan batch's summary, once its run is complete (the caller waited for it):
// planner status (AVERROR_INVALIDDATA: the batch was neutralised by k_pguard; kept in
// s.status and returned by every later check until the slot is restaged) and the
// algorithmic byte totals. Consistency of the step lists with the staged launch list rests
// on k_plan's PLS_SCHED check (with static lists k_plan does not count keys, so the summary's
// key offsets are only used to locate the byte totals).
static void print_plan_prof(vp9hip_ctx *c, const Staged &s);
static int finish_summary(vp9hip_ctx *c, Staged &s)
{
    if (!s.stat || !s.summary_pending) return s.status;
    s.summary_pending = false;
    if (c->plan_prof_on && c->plan_prof) print_plan_prof(c, s);
    HIPCHK(hipMemcpy(s.summary_h, s.arena + s.o_summary, s.summary_words * 4, hipMemcpyDeviceToHost));
    const uint32_t *sm = s.summary_h;
    if (sm[0]) {
        // k_pguard neutralised the rejected frames only (the whole batch if no frame is named):
        // the others ran as if alone
        const int nbad = frame_verdicts(s, sm, 0);
        fprintf(stderr, "vp9hip: %d of %d frames rejected by the device planner (status 0x%x, bounds 0x%x)\n", nbad,
                s.nframes, sm[0], sm[s.summary_words - 1]);
        s.status = VP9HIP_EINVALIDDATA;
        return s.status;
    }
    // each static k_resid_dev grid was sized from a staged bound on its job range: a range
    // beyond it would have dropped residual jobs silently
    for (const Launch &L : s.launches)
        if (L.kind == K_RESID && L.devr) {
            const uint32_t *rng = sm + 1 + L.off;
            if (rng[1] > rng[0] && rng[1] - rng[0] > L.n) {
                fprintf(stderr, "vp9hip: residual job range %u exceeds its staged bound %u\n", rng[1] - rng[0], (unsigned) L.n);
                s.fstat.assign(s.nframes, VP9HIP_EBUG);
                s.status = VP9HIP_EBUG;
                return s.status;
            }
        }
    const uint32_t *ko = sm + 1 + s.n_gidx, *fb32 = ko + s.nkey + 1;
    for (int k = 0; k < K_N; k++) s.alg_bytes[k] = s.alg_stat[k];
    s.alg_bytes[K_PLAN] = (double) s.nblk * sizeof(vp9h_block) + (double) s.neob * 2;
    for (int i = 0; i < s.nframes; i++) {
        s.alg_bytes[K_RESID] += (double) ((uint64_t) fb32[4 * i] | (uint64_t) fb32[4 * i + 1] << 32);
        s.alg_bytes[K_MC] += (double) ((uint64_t) fb32[4 * i + 2] | (uint64_t) fb32[4 * i + 3] << 32);
    }
    return 0;
}

// VP9HIP_PLAN_PROF=1: the planner's per-SB phase cycles of the last run (k_pjob phases 0-2,
// k_plan 3-10), summed over the SBs, on stderr. The caller has waited for the planner.
static void print_plan_prof(vp9hip_ctx *c, const Staged &s)
{
    unsigned long long pc[16];
    if (hipMemcpy(pc, c->plan_prof, sizeof(pc), hipMemcpyDeviceToHost) != hipSuccess) return;
    double tot = 0;
    for (int k = 0; k < 11; k++) tot += (double) pc[k];
    fprintf(stderr, "vp9hip plan phases (%% of planner SB cycles, %.3g cycles/SB%s):", tot / std::max<uint32_t>(1, s.nslots),
            s.stat ? ", static plan" : "");
    for (int k = 0; k < 11; k++) fprintf(stderr, " %d:%.1f", k, 100.0 * (double) pc[k] / std::max(1.0, tot));
    fprintf(stderr, "\n");
}

// Run the device planner of the staged batch and build its launch list from the summary.
static int plan_dev(vp9hip_ctx *c)
{
    const bool plan_trace = c->stage_trace;
    const auto pt0 = std::chrono::steady_clock::now();
    Staged &s = c->stg;
    uint8_t *A = s.arena;
    s.planned = false;
    if (!s.stat) s.launches.clear();
    // the planner runs on its own stream, after this slot's previous run (its records are
    // rewritten in place) and after whatever the main stream holds for it (the staging
    // upload); the other slot's pixel kernels run meanwhile
    const hipStream_t ps = plan_stream(c);
    if (s.done_ev) HIPCHK(hipStreamWaitEvent(ps, s.done_ev, 0));
    HIPCHK(hipMemsetAsync(A + s.o_sbfirst, 0xff, (size_t) 2 * s.nslots * 4, ps));
    HIPCHK(hipMemsetAsync(A + s.o_keycnt, 0, s.zero_bytes, ps));
    PlanDev D;
    D.frames = (const PlanFrame *) (A + s.o_pf);
    D.blocks = (const vp9h_block *) (A + s.o_blocks);
    D.eobs = (const uint16_t *) (A + s.o_eobs);
    D.total_blocks = s.nblk;
    D.total_eobs = s.neob;
    D.total_coefs = s.ncoef;
    D.slot_pos = (const uint32_t *) (A + s.o_slotpos);
    D.seg_pre4 = (const uint32_t *) (A + s.o_segpre);
    D.seg_sz = (const uint32_t *) (A + s.o_segsz);
    D.seg_pre1 = (const uint32_t *) (A + s.o_segpre1);
    D.blk_neob = (uint32_t *) (A + s.o_bneob);
    D.blk_eob0 = (uint32_t *) (A + s.o_beob0);
    D.sb_first = (uint32_t *) (A + s.o_sbfirst);
    D.sb_end = D.sb_first + s.nslots;
    D.sb_ncoef = (uint32_t *) (A + s.o_sbncoef);
    D.sb_coef0 = (uint32_t *) (A + s.o_sbcoef0);
    D.cnt = (uint32_t *) (A + s.o_cnt);
    D.cnt0 = (uint32_t *) (A + s.o_cnt0);
    D.cntm = (uint32_t *) (A + s.o_cntm);
    D.cntm0 = (uint32_t *) (A + s.o_cntm0);
    D.ibits = (uint32_t *) (A + s.o_ibits);
    D.sb_info = (uint32_t *) (A + s.o_sbinfo);
    D.sb_key = (uint32_t *) (A + s.o_sbkey);
    D.sb_kpos = (uint32_t *) (A + s.o_sbkpos);
    D.key_cnt = (uint32_t *) (A + s.o_keycnt);
    D.key_off = (uint32_t *) (A + s.o_keyoff);
    D.status = (uint32_t *) (A + s.o_status);
    D.fbytes = (unsigned long long *) (A + s.o_fbytes);
    D.fbad = (uint32_t *) (A + s.o_fbad);
    D.sbs = (SBRec *) (A + s.o_sbs);
    D.wgs = (WGRec *) (A + s.o_wgs);
    D.pjobs = (PJob *) (A + s.o_pjobs);
    D.passes = (uint32_t *) (A + s.o_passes);
    D.lfs = (LFRec *) (A + s.o_lfs);
    D.rjobs = (RJob *) (A + s.o_rjobs);
    D.mcs = (McUnit *) (A + s.o_mcs);
    D.dlists = (uint32_t *) (A + s.o_lists) + s.host_lists;
    D.jobw = (uint32_t *) (A + s.o_jobw);
    D.sb_nj = (uint32_t *) (A + s.o_sbnj);
    D.nz = c->nz;
    D.jcap = (uint32_t) s.jcap;
    D.rcap = (uint32_t) s.rcap;
    D.nslots = s.nslots;
    D.cap_cnt = s.ncnt + 1;
    D.cap_cntm = s.nslots + 1;
    D.cap_rjobs = s.neob + 1;
    D.cap_mcs = s.cap_mcs;
    D.cap_dlists = s.nslots;
    D.nkeys = s.nkey;
    D.nframes = (uint32_t) s.nframes;
    const bool pprof = c->plan_prof_on;
    D.dbg = c->plan_dbg;
    D.static_lists = s.stat ? 1 : 0;
    D.stat_ko = s.stat && !s.stat_lists.empty() && s.exp_ko.size() == (size_t) s.nkey + 1 ? (const uint32_t *) (A + s.o_expko)
                                                                                        : nullptr;
    D.prof = nullptr;
    if (pprof) {
        if (!c->plan_prof && hipMalloc(&c->plan_prof, 16 * sizeof(unsigned long long)) != hipSuccess) return VP9HIP_ENOMEM;
        HIPCHK(hipMemsetAsync(c->plan_prof, 0, 16 * sizeof(unsigned long long), ps));
        D.prof = c->plan_prof;
    }
    if (c->timing) {
        for (auto &e : c->pev)
            if (!e) HIPCHK(hipEventCreate(&e));
        HIPCHK(hipEventRecord(c->pev[0], ps));
    }
    if (vp9hip_plan_enqueue(ps, &D, c->ss_h | c->ss_v << 1, s.nframes, s.max_blk, s.max_sb, s.nblk, s.nslots,
                            s.ncnt, (int) s.nkey, (const uint32_t *) (A + s.o_gidx), (int) s.n_gidx,
                            (uint32_t *) (A + s.o_summary), A + s.o_scan, s.scan_bytes, s.any_levels, s.plan_flags,
                            s.stat ? 1 : 0))
        return VP9HIP_EEXTERNAL;
    if (c->timing) HIPCHK(hipEventRecord(c->pev[1], ps));
    c->plan_timed = c->timing;
    if (s.stat) {                  // launch list fixed at staging: the pixel launches wait on the device
        if (!s.plan_ev) HIPCHK(hipEventCreateWithFlags(&s.plan_ev, hipEventDisableTiming));
        HIPCHK(hipEventRecord(s.plan_ev, ps));
        s.summary_pending = true;
        s.planned = true;
        return 0;
    }
    HIPCHK(hipMemcpyAsync(s.summary_h, A + s.o_summary, s.summary_words * 4, hipMemcpyDeviceToHost, ps));
    HIPCHK(hipStreamSynchronize(ps));          // the pixel kernels, queued after this, read the plan
    if (pprof) print_plan_prof(c, s);
    if (plan_trace)
        fprintf(stderr, "vp9hip plan (device): %d frames: %.2f ms host wall\n", s.nframes,
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - pt0).count());
    const uint32_t *sm = s.summary_h;
    if (sm[0]) {                                              // the packets are inconsistent (PLS_*)
        // nothing was launched: the frames the planner did not reject are valid, not run
        const int nbad = frame_verdicts(s, sm, VP9HIP_EAGAIN);
        fprintf(stderr, "vp9hip: %d of %d frames rejected by the device planner (status 0x%x, bounds 0x%x)\n", nbad,
                s.nframes, sm[0], sm[s.summary_words - 1]);
        return VP9HIP_EINVALIDDATA;
    }
    const uint32_t *gv = sm + 1, *ko = sm + 1 + s.n_gidx, *fb32 = ko + s.nkey + 1;
    auto fbytes = [&](int i, int k) {
        return (double) ((uint64_t) fb32[2 * (2 * i + k)] | (uint64_t) fb32[2 * (2 * i + k) + 1] << 32);
    };
    for (int k = 0; k < K_N; k++) s.alg_bytes[k] = s.alg_base[k];
    // the planner's algorithmic bytes: the packet it plans from (blocks and eobs)
    s.alg_bytes[K_PLAN] = (double) s.nblk * sizeof(vp9h_block) + (double) s.neob * 2;
    for (int i = 0; i < s.nframes; i++) {
        s.alg_bytes[K_RESID] += fbytes(i, 0);
        s.alg_bytes[K_MC] += fbytes(i, 1);
        if (s.frame_fused[i]) {                               // residuals inside the k_plf launches
            const double b = s.frame_res_bytes[i] + fbytes(i, 0);
            s.alg_bytes[K_RESID] -= b;
            s.alg_bytes[K_PLF] += b;
        }
    }
    const uint32_t H = s.host_lists;
    const int nph = (int) s.dph.size();
    for (int g = 0; g < s.ngroups; g++)
        for (int ph = 0; ph < nph; ph++) {
            const Staged::DevPhase &P = s.dph[ph];
            if (P.frames.empty() || P.group != g) continue;
            auto push = [&](int kind, uint32_t off, uint32_t cnt, int arg, int part, int step) {
                Launch L = { kind, off, cnt, arg, g, ph, part, step };
                s.launches.push_back(L);
            };
            const uint32_t m0 = gv[P.g_mc], m1 = gv[P.g_mc + 1];
            if (m1 > m0) push(K_MC, m0, m1 - m0, 0, PART_RECON, 0);
            auto rr = [&](int d, int tc) {
                const uint32_t a = gv[P.g_res + (d * 5 + tc) * 2], b = gv[P.g_res + (d * 5 + tc) * 2 + 1];
                return std::make_pair(a, b - a);
            };
            // level-scheduled (inter chain) phases: every tx size in one launch (arg 5, the
            // ranges in roff / rn); VP9HIP_RESID_MULTI=0 keeps one launch per size
            const bool rmulti = c->resid_multi;
            if (!P.fused && P.levels && rmulti) {
                Launch L = { K_RESID, 0, 0, 5, g, ph, PART_RECON, 0 };
                for (int tc = 0; tc < 5; tc++) { L.roff[tc] = rr(0, tc).first; L.rn[tc] = rr(0, tc).second; L.n += L.rn[tc]; }
                if (L.n) s.launches.push_back(L);
            } else if (!P.fused) {
                for (int tc = 0; tc < 5; tc++)
                    if (rr(0, tc).second) push(K_RESID, rr(0, tc).first, rr(0, tc).second, tc, PART_RECON, 0);
            }
            auto step = [&](int d) {
                const uint32_t k = P.key0 + (uint32_t) d;
                return std::make_pair(H + ko[k], ko[k + 1] - ko[k]);
            };
            uint32_t in_off = 0, in_n = 0;          // intra SBs inside the k_lfro launch
            auto lfr = [&]() {
                if (!P.lfr) return;
                push(K_LFR, P.lfr_off, P.lfr_n, (int) P.lfr_ctr, PART_LF, 0);
                if (in_n) {
                    s.launches.back().off2 = in_off;
                    s.launches.back().n2 = in_n;
                    s.launches.back().flow = P.pred_ctr;
                }
                s.alg_bytes[K_LF] -= P.lfr_bytes;
                s.alg_bytes[K_LFR] += P.lfr_bytes;
            };
            if (!s.fuse || P.levels) {
                // the level lists are back to back in level order: one k_predd launch when the
                // phase has few intra SBs (its level launches are latency-bound); wide phases
                // keep the level launches, which run every SB of a level at once (C5: its 8K
                // frames' levels were faster than k_predd's capped grid, profiles/r05u)
                const uint32_t a = P.nkey ? step(0).first : 0, b = P.nkey ? step(P.nkey - 1).first + step(P.nkey - 1).second : 0;
                if (P.pred_ctr >= 0 && b - a <= (uint32_t) c->pred_df_max && P.levels && P.nkey) {
                    if (b > a && c->pred_lf_fuse && P.lfr && P.all_lf && c->kcfg.lfro) {
                        // inside the phase's k_lfro launch (VP9HIP_PRED_LF_FUSE): the LF of an
                        // SB starts once it and the SBs reading its pre-LF pixels are predicted
                        in_off = a;
                        in_n = b - a;
                    } else if (b > a) {
                        push(K_PRED, a, b - a, 0, PART_RECON, 0);
                        s.launches.back().flow = P.pred_ctr;
                    }
                } else
                for (int d = 0; d < P.nkey; d++)
                    if (step(d).second) push(K_PRED, step(d).first, step(d).second, 0, PART_RECON, d);
                if (P.lfr) lfr();
                else
                    for (size_t j = 0; j < P.lf.size(); j++)
                        if (P.lf[j].second) push(K_LF, P.lf[j].first, P.lf[j].second, 0, PART_LF, (int) j);
                continue;
            }
            // fused: launch t = intra diagonal t + LF diagonal t - PLF_LAG + residuals of t + 1
            const int np = P.np, nres = P.fused ? P.nseg : 0, nlf = P.nlf;
            const int nt = std::max(std::max(np, nlf ? nlf + PLF_LAG : 0), nres - 1);
            for (int t = -1; t < nt; t++) {
                const std::pair<uint32_t, uint32_t> pv = t >= 0 && t < np ? step(t) : std::make_pair(0u, 0u);
                const int j = t - PLF_LAG;
                const std::pair<uint32_t, uint32_t> lv = j >= 0 && j < nlf ? P.lf[j] : std::make_pair(0u, 0u);
                bool res = false;
                for (int k = 0; t + 1 < nres && k < 5; k++) res |= rr(t + 1, k).second > 0;
                if (!pv.second && !res) {
                    if (lv.second) push(K_LF, lv.first, lv.second, 0, PART_LF, j);
                    continue;
                }
                Launch L = { K_PLF, pv.first, pv.second, 0, g, ph, PART_RECON, t };
                L.off2 = lv.first;
                L.n2 = lv.second;
                if (pv.second && t < (int) P.pred_bytes.size()) {
                    s.alg_bytes[K_PRED] -= P.pred_bytes[t];
                    s.alg_bytes[K_PLF] += P.pred_bytes[t];
                }
                if (lv.second) {
                    s.alg_bytes[K_LF] -= P.lf_bytes[j];
                    s.alg_bytes[K_PLF] += P.lf_bytes[j];
                }
                for (int k = 0; res && k < 5; k++) { L.roff[k] = rr(t + 1, k).first; L.rn[k] = rr(t + 1, k).second; }
                s.launches.push_back(L);
            }
            lfr();
        }
    s.planned = true;
    return 0;
}

static int stage(vp9hip_ctx *c, const vp9h_frame *pkts, int n, const int *out_bufs, const int *ref_bufs /*n*3 or null*/,
                 int tile_lo = 0, int tile_hi = 64, int max_groups = 0, bool tiled = false)
{
    // fused intra + LF launches need the LF of a phase in the same launch sequence as its
    // reconstruction (not for tile-sharded batches: recon, exchange, then LF)
    const bool fuse = c->fuse_plf && !tiled;
    // the loop filter of a phase as one row-pipelined k_lfr launch (after the phase's
    // reconstruction) instead of x + 2y diagonal launches
    const bool lfr_any = c->lf_rows > 0 && !tiled;
    // VP9HIP_STAGE_TRACE=1: host time of the staging steps on stderr
    const bool stage_trace = c->stage_trace;
    double st_ms[6] = { 0, 0, 0, 0, 0, 0 };
    auto st_t0 = std::chrono::steady_clock::now();
#define STAGE_T(k) do { auto t_ = std::chrono::steady_clock::now(); \
        st_ms[k] = std::chrono::duration<double, std::milli>(t_ - st_t0).count(); st_t0 = t_; } while (0)
    if (!c || !pkts || n <= 0 || !out_bufs) return VP9HIP_EINVAL;
    if (c->bufs.empty()) return VP9HIP_EINVAL;
    hipSetDevice(c->dev);
    // this slot's previous batch may still read the arena (the other slot's work may go on)
    if (c->stg.done_ev) HIPCHK(hipEventSynchronize(c->stg.done_ev));
    if (c->stg.up_ev) HIPCHK(hipEventSynchronize(c->stg.up_ev));
    Staged &s = c->stg;
    if (s.graph) { hipGraphExecDestroy(s.graph); s.graph = nullptr; }
    s.frames.clear(); s.sbs.clear(); s.pjobs.clear(); s.passes.clear(); s.lfs.clear(); s.mcs.clear();
    s.wgs.clear(); s.sbh.clear(); s.sbjobs.clear(); s.jdep0.clear(); s.jdeps.clear();
    s.rjobs.clear(); s.resid16 = 0;
    s.rbucket.clear();
    s.lists.clear(); s.launches.clear(); s.coefs.clear(); s.n_ctr = 0; s.lfr_ctr.clear();
    s.frame_phase.assign(n, 0); s.frame_log2.assign(n, 0);
    s.tile_lo = tile_lo; s.tile_hi = tile_hi;
    s.stat = false;
    s.summary_pending = false;
    s.status = 0;
    s.fstat.assign(n, 0);
    for (int k = 0; k < K_N; k++) s.alg_bytes[k] = 0;
    s.ready = false;

    const int csz = c->hb ? 4 : 2;
    init_nz();
    // Frame dependencies inside the batch: an inter frame follows the frames whose output
    // it references, and a frame overwriting a buffer follows every earlier frame that
    // reads or writes that buffer. Dependent frames form chains; chains are spread over G
    // stream groups, and within a group frames of equal chain position ("phase") are
    // interleaved in every launch (a keyframe batch is one phase per group).
    std::vector<int> pos(n, 0), comp(n);
    for (int i = 0; i < n; i++) comp[i] = i;
    std::function<int(int)> find = [&](int x) { return comp[x] == x ? x : comp[x] = find(comp[x]); };
    for (int i = 0; i < n; i++) {
        const vp9h_frame *f = &pkts[i];
        const bool inter = !(f->keyframe || f->intraonly);
        if (inter && !ref_bufs) return VP9HIP_EINVAL;
        for (int j = 0; j < i; j++) {
            bool dep = out_bufs[j] == out_bufs[i];
            for (int r = 0; r < 3 && !dep; r++) {
                if (inter && ref_bufs[i * 3 + r] == out_bufs[j]) dep = true;
                const bool jinter = !(pkts[j].keyframe || pkts[j].intraonly);
                if (jinter && ref_bufs[j * 3 + r] == out_bufs[i]) dep = true;
            }
            if (dep) { pos[i] = std::max(pos[i], pos[j] + 1); comp[find(i)] = find(j); }
        }
    }
    std::vector<int> roots;
    for (int i = 0; i < n; i++) if (find(i) == i) roots.push_back(i);
    // G groups: as many as allowed, but chains split evenly (unless there are many: 4 GOP
    // chains over 3 streams run 2/1/1 and the pair sets the time)
    const int nroots = (int) roots.size();
    int G = std::max(1, std::min<int>(max_groups > 0 ? max_groups : c->max_groups, nroots));
    while (G > 1 && nroots % G && nroots < 16 * G) G--;
    s.ngroups = G;
    std::vector<int> grp(n);
    for (int i = 0; i < n; i++)
        grp[i] = (int) (std::lower_bound(roots.begin(), roots.end(), find(i)) - roots.begin()) % G;
    int maxpos = 0;
    for (int i = 0; i < n; i++) maxpos = std::max(maxpos, pos[i]);
    const int NP = G * (maxpos + 1);                   // phase id = g * (maxpos + 1) + pos
    s.nphases = NP;
    // residuals fused into the wavefront launches: per phase (RES_FUSE_MAX_FRAMES)
    std::vector<int> phase_n(NP, 0);
    for (int i = 0; i < n; i++) phase_n[grp[i] * (maxpos + 1) + pos[i]]++;
    std::vector<char> res_fused(NP);
    for (int ph = 0; ph < NP; ph++) res_fused[ph] = fuse && phase_n[ph] < RES_FUSE_MAX_FRAMES;
    // level-scheduled phases (inter frames of k_lfr phases): MC, all residuals, the intra
    // SBs by dependency level (k_pred), then the whole loop filter as one k_lfr launch
    std::vector<char> lvl_ph(NP, 0);
    if (lfr_any && c->level_sched) {
        for (int ph = 0; ph < NP; ph++) lvl_ph[ph] = c->lf_rows > 1 || phase_n[ph] < LFR_MAX_FRAMES;
        for (int i = 0; i < n; i++)
            if (pkts[i].keyframe || pkts[i].intraonly) lvl_ph[grp[i] * (maxpos + 1) + pos[i]] = 0;
        for (int ph = 0; ph < NP; ph++) if (lvl_ph[ph]) res_fused[ph] = false;
    }
    // per frame: validate, frame descriptor, reference scaling (sequential, cheap)
    std::vector<FrameBuild> fbs(n);
    std::vector<size_t> coef_off(n + 1, 0);
    uint64_t coef_base = 0;
    uint64_t edge_sbs = 0;                  // SBs of the batch's intra frames (FrameDesc.edge)
    for (int i = 0; i < n; i++) {
        const vp9h_frame *f = &pkts[i];
        // frames up to the configured size share the buffers (reference scaling, vp9.c:845-880)
        if (f->width <= 0 || f->height <= 0 || f->width > c->w || f->height > c->h || f->bpp != c->bpp ||
            f->ss_h != c->ss_h || f->ss_v != c->ss_v)
            return VP9HIP_EINVAL;
        const int cols = (f->width + 7) >> 3, rows = (f->height + 7) >> 3;
        if (out_bufs[i] < 0 || out_bufs[i] >= (int) c->bufs.size()) return VP9HIP_EINVAL;
        const bool intra = f->keyframe || f->intraonly;
        FrameDesc fd;
        memset(&fd, 0, sizeof(fd));
        uint8_t *ob = c->bufs[out_bufs[i]];
        for (int p = 0; p < 3; p++) fd.plane[p] = (uint64_t) (ob + c->plane_off[p]);
        fd.pitch[0] = c->pitch[0]; fd.pitch[1] = c->pitch[1];
        fd.w8[0] = cols * 8; fd.h8[0] = rows * 8;
        fd.w8[1] = cols * 8 >> c->ss_h; fd.h8[1] = rows * 8 >> c->ss_v;
        fd.sb_cols = (f->width + 63) >> 6; fd.sb_rows = (f->height + 63) >> 6;
        fd.bd = c->bpp;
        fd.sharp = f->sharpness;
        if (!intra) {
            for (int r = 0; r < 3; r++) {
                int rb = ref_bufs[i * 3 + r];
                if (rb < 0 || rb >= (int) c->bufs.size()) return VP9HIP_EINVAL;
                if (rb == out_bufs[i]) return VP9HIP_EINVAL;                       // in-place MC
                if (f->ref_w[r] <= 0 || f->ref_h[r] <= 0 || f->ref_w[r] > c->w || f->ref_h[r] > c->h)
                    return VP9HIP_EINVAL;
                for (int p = 0; p < 3; p++) fd.ref[r][p] = (uint64_t) (c->bufs[rb] + c->plane_off[p]);
                fd.refw[r][0] = f->ref_w[r]; fd.refh[r][0] = f->ref_h[r];
                fd.refw[r][1] = (f->ref_w[r] + c->ss_h) >> c->ss_h; fd.refh[r][1] = (f->ref_h[r] + c->ss_v) >> c->ss_v;
            }
        }
        if (intra) {                    // FrameDesc.edge: an SB index for now, a pointer below
            fd.edge = edge_sbs + 1;
            edge_sbs += (uint64_t) fd.sb_cols * fd.sb_rows;
        }
        s.frames.push_back(fd);
        c->buf_wh[out_bufs[i]] = { f->width, f->height };
        FrameBuild &fb = fbs[i];
        fb.f = f; fb.frame_idx = i;
        fb.cols = cols; fb.rows = rows; fb.sb_cols = fd.sb_cols; fb.sb_rows = fd.sb_rows;
        memset(&fb.mc, 0, sizeof(fb.mc));
        fb.mc.cols = cols; fb.mc.rows = rows; fb.mc.ss_h = c->ss_h; fb.mc.ss_v = c->ss_v;
        if (!intra) {
            // reference scale factors (vp9.c:845-880)
            int valid = 0;
            for (int r = 0; r < 3; r++) {
                const int rw = f->ref_w[r], rh = f->ref_h[r], w = f->width, h = f->height;
                if (rw == w && rh == h) { valid++; continue; }
                if (w * 2 < rw || h * 2 < rh || w > 16 * rw || h > 16 * rh) {
                    fb.mc.scale[r][0] = fb.mc.scale[r][1] = SCALE_INVALID;
                    continue;
                }
                fb.mc.scale[r][0] = (rw << 14) / w;
                fb.mc.scale[r][1] = (rh << 14) / h;
                fb.mc.step[r][0] = 16 * fb.mc.scale[r][0] >> 14;
                fb.mc.step[r][1] = 16 * fb.mc.scale[r][1] >> 14;
                valid++;
            }
            if (!valid) {               // no usable reference scale (vp9.c:845-880): this frame only
                s.fstat.assign(n, VP9HIP_EAGAIN);
                s.fstat[i] = VP9HIP_EINVALIDDATA;
                return VP9HIP_EINVALIDDATA;
            }
        }
        fb.ss_h = c->ss_h; fb.ss_v = c->ss_v; fb.coef_size = csz;
        fb.pitch[0] = c->pitch[0]; fb.pitch[1] = c->pitch[1];
        fb.coef_base = coef_base;
        fb.phase = grp[i] * (maxpos + 1) + pos[i];
        fb.tile_lo = tile_lo; fb.tile_hi = tile_hi;
        fb.by_diag = res_fused[fb.phase];
        fb.levels = lvl_ph[fb.phase];
        s.frame_phase[i] = fb.phase;
        s.frame_log2[i] = f->log2_tile_cols;
        coef_off[i + 1] = coef_off[i] + (size_t) f->ncoefs * csz;
        coef_base += f->ncoefs;
        if (coef_base > 0xffffffffull) return VP9HIP_ENOMEM;
        // algorithmic bytes: reconstruction reads C and writes P (k_resid
        // owns C, k_pred owns P; inter residuals read + write their pixels in k_resid),
        // LF reads + writes P, MC reads R*P and writes the predicted pixels
        const double pix_bytes = (double) f->width * f->height * c->bypp * (1.0 + 2.0 / ((1 << c->ss_h) * (1 << c->ss_v)));
        s.alg_bytes[K_RESID] += (double) f->ncoefs * csz;
        if (intra) s.alg_bytes[K_PRED] += pix_bytes;
        if (f->filter_level) s.alg_bytes[K_LF] += 2.0 * pix_bytes;
    }
    // the intra frames' SB right columns: written by each SB's intra workgroup, read by the
    // SB to its right in place of a column of one-pixel frame rows (128 scattered lines)
    {
        const size_t eb = (size_t) edge_sbs * EDGE_PIX * c->bypp + 256;
        // only the 4:2:0 tile loader reads the edge columns (the other chroma formats load
        // their left column from frame rows): no buffer written and never read for those
        const bool edge_off = !c->edge || !(c->ss_h && c->ss_v);
        if (edge_sbs && !edge_off && eb > s.edge_cap) {
            if (s.edge) hipFree(s.edge);
            s.edge = nullptr;
            s.edge_cap = 0;
            if (hipMalloc(&s.edge, eb) != hipSuccess) return VP9HIP_ENOMEM;
            s.edge_cap = eb;
        }
        for (FrameDesc &fd : s.frames)
            fd.edge = fd.edge && !edge_off ? (uint64_t) (s.edge + (size_t) (fd.edge - 1) * EDGE_PIX * c->bypp) : 0;
    }

    STAGE_T(0);
    // the buffers this batch writes and reads, and which other slots' batches touch them
    s.wr.assign(out_bufs, out_bufs + n);
    s.rd.clear();
    for (int i = 0; i < n && ref_bufs; i++)
        if (!(pkts[i].keyframe || pkts[i].intraonly))
            for (int r = 0; r < 3; r++) s.rd.push_back(ref_bufs[i * 3 + r]);
    for (auto *v : { &s.wr, &s.rd }) { std::sort(v->begin(), v->end()); v->erase(std::unique(v->begin(), v->end()), v->end()); }
    {
        auto meet = [](const std::vector<int> &a, const std::vector<int> &b) {
            for (size_t i = 0, j = 0; i < a.size() && j < b.size();) {
                if (a[i] == b[j]) return true;
                if (a[i] < b[j]) i++; else j++;
            }
            return false;
        };
        s.dep_mask = 0;
        for (int k = 0; k < MAX_SLOTS; k++) {
            if (k == c->slot) continue;
            const Staged &o = c->sl[k];
            if (o.ready && (meet(s.wr, o.wr) || meet(s.wr, o.rd) || meet(s.rd, o.wr))) s.dep_mask |= 1u << k;
        }
    }
    s.dev = false;
    if (!c->host_plan) {
        DevIn in;
        in.pkts = pkts; in.n = n; in.G = G; in.maxpos = maxpos; in.NP = NP; in.csz = csz;
        in.fbs = &fbs; in.res_fused = &res_fused; in.lvl_ph = &lvl_ph;
        in.fuse = fuse; in.lfr_any = lfr_any;
        const int r = stage_dev(c, in);
        if (r) return r;
        STAGE_T(1);
        if (stage_trace) fprintf(stderr, "vp9hip stage (device plan): %d frames: setup %.1f upload %.1f ms\n", n, st_ms[0], st_ms[1]);
        return 0;
    }
    // work planning of every frame (independent), on host threads: jobs, dependency
    // levels and pass packing, LF programs, MC units, coefficient copy
    std::vector<FramePlan> plans(n);
    {
        std::atomic<int> next(0);
        auto worker = [&]() {
            for (int i; (i = next.fetch_add(1)) < n;) {
                plans[i].err = plan_frame(fbs[i], plans[i]);
            }
        };
        const int nt = std::min(n, c->host_threads);
        std::vector<std::thread> pool;
        for (int t = 1; t < nt; t++) pool.emplace_back(worker);
        worker();
        for (auto &t : pool) t.join();
    }
    STAGE_T(1);
    // merge: batch offsets of every frame's records (prefix sums in frame order; residual
    // jobs in launch order: group, phase, tx code, txtp, frame). The records themselves
    // are written, with their index fixups, straight into the pinned arena image below.
    for (int i = 0; i < n; i++)
        if (plans[i].err < 0) return plans[i].err;
    struct Off { uint32_t sb, job, pass, wg, lf, mc; uint64_t res; };
    std::vector<Off> off(n);
    Off tot = {};
    for (int i = 0; i < n; i++) {
        const Staged &l = plans[i].s;
        off[i] = tot;
        tot.sb += (uint32_t) l.sbs.size(); tot.job += (uint32_t) l.pjobs.size(); tot.pass += (uint32_t) l.passes.size();
        tot.wg += (uint32_t) l.wgs.size(); tot.lf += (uint32_t) l.lfs.size(); tot.mc += (uint32_t) l.mcs.size();
        tot.res += l.resid16;
    }
    if (tot.res > 0xffffffffull) return VP9HIP_ENOMEM;
    s.resid16 = tot.res;
    std::vector<std::vector<int>> phase_frames(NP);
    for (int i = 0; i < n; i++) phase_frames[fbs[i].phase].push_back(i);
    // residual jobs per (phase, bucket = intra diagonal when fused, tx code): (off, n)
    std::vector<std::vector<std::array<std::pair<uint32_t, uint32_t>, 5>>> rj_range(NP);
    std::vector<std::vector<std::array<std::array<uint32_t, 4>, 5>>> rj_off(n);   // per frame, bucket
    for (int i = 0; i < n; i++) rj_off[i].resize(plans[i].s.rbucket.size());
    uint32_t tot_rj = 0;
    for (int ph = 0; ph < NP; ph++) {                  // phase ids are group-major, chain order
        size_t nb = 0;
        for (int i : phase_frames[ph]) nb = std::max(nb, plans[i].s.rbucket.size());
        rj_range[ph].resize(nb);
        for (size_t d = 0; d < nb; d++)
            for (int t = 0; t < 5; t++) {
                rj_range[ph][d][t].first = tot_rj;
                for (int tp = 0; tp < 4; tp++)
                    for (int i : phase_frames[ph]) {
                        if (d >= plans[i].s.rbucket.size()) continue;
                        rj_off[i][d][t][tp] = tot_rj;
                        tot_rj += (uint32_t) plans[i].s.rbucket[d][t][tp].size();
                    }
                rj_range[ph][d][t].second = tot_rj - rj_range[ph][d][t].first;
            }
    }
    // per workgroup / LF record: the algorithmic pixel bytes its SB moves (fused launches)
    std::vector<double> wg_bytes(tot.wg, 0.0), lf_bytes(tot.lf, 0.0);
    for (int i = 0; i < n; i++) {
        const Staged &l = plans[i].s;
        const bool intra = pkts[i].keyframe || pkts[i].intraonly;
        for (size_t k = 0; k < l.wgs.size() && intra; k++) {
            const SBRec &sb = l.sbs[l.wgs[k].sb[0]];
            wg_bytes[off[i].wg + k] = sb_bytes(c, pkts[i], sb.sbx, sb.sby);
        }
        for (size_t k = 0; k < l.lfs.size(); k++)
            lf_bytes[off[i].lf + k] = 2.0 * sb_bytes(c, pkts[i], l.lfs[k].sbx, l.lfs[k].sby);
    }
    std::vector<std::vector<std::vector<uint32_t>>> wsteps(NP), lsteps(NP);   // per phase: WG / LF lists
    std::vector<std::vector<std::pair<uint32_t, uint32_t>>> mcr(NP);           // MC unit ranges per phase
    for (int i = 0; i < n; i++) {
        FramePlan &fp = plans[i];
        const int ph = fbs[i].phase;
        if (!fp.s.mcs.empty()) mcr[ph].push_back({ off[i].mc, (uint32_t) fp.s.mcs.size() });
        for (const McUnit &m : fp.s.mcs) s.alg_bytes[K_MC] += (double) m.w * m.h * c->bypp * (1 + m.nref);
        if (wsteps[ph].size() < fp.wsteps.size()) wsteps[ph].resize(fp.wsteps.size());
        for (size_t d = 0; d < fp.wsteps.size(); d++)
            for (uint32_t w : fp.wsteps[d]) wsteps[ph][d].push_back(w + off[i].wg);
        if (lsteps[ph].size() < fp.lsteps.size()) lsteps[ph].resize(fp.lsteps.size());
        for (size_t d = 0; d < fp.lsteps.size(); d++)
            for (uint32_t li : fp.lsteps[d]) lsteps[ph][d].push_back(li + off[i].lf);
    }
    STAGE_T(2);
    // launch schedule per group, phases in chain order: MC, residuals by (tx code, txtp),
    // the intra SB wavefront, the LF wavefront; inter residual pixels are algorithmic
    // reads + writes of k_resid
    for (int g = 0; g < G; g++)
        for (int ph = g * (maxpos + 1); ph < (g + 1) * (maxpos + 1); ph++) {
            for (auto &mr : mcr[ph]) s.launches.push_back({ K_MC, mr.first, mr.second, 0, g, ph, PART_RECON, 0 });
            if (!res_fused[ph])                          // residual jobs placed by the merge
                for (auto &rr : rj_range[ph])
                    for (int t = 0; t < 5; t++)
                        if (rr[t].second)
                            s.launches.push_back({ K_RESID, rr[t].first, rr[t].second, t, g, ph, PART_RECON, 0 });
            auto add_list = [&](int kind, const std::vector<uint32_t> &v, int step) {
                if (v.empty()) return;
                s.launches.push_back({ kind, (uint32_t) s.lists.size(), (uint32_t) v.size(), 0, g, ph,
                                       kind == K_LF ? PART_LF : PART_RECON, step });
                s.lists.insert(s.lists.end(), v.begin(), v.end());
            };
            const std::vector<std::vector<uint32_t>> &wls = wsteps[ph];   // one workgroup per SB
            const bool lfr = lfr_any && (c->lf_rows > 1 || (int) phase_frames[ph].size() < LFR_MAX_FRAMES);
            // k_lfr task table of the phase: one task per (frame, SB row), rows-major, each
            // naming the task of the row above (dep) and its SBs' LF records left to right
            // j0: LF diagonals x + 2y < j0 ran in earlier (fused) launches
            auto add_lfr = [&](int j0) {
                std::vector<std::vector<std::vector<uint32_t>>> grid;      // per frame: [row][col]
                int maxr = 0;
                for (int i : phase_frames[ph]) {
                    const std::vector<LFRec> &lf = plans[i].s.lfs;
                    if (lf.empty()) continue;
                    int nr = 0, nc = 0;
                    for (const LFRec &r : lf) { nr = std::max(nr, r.sby + 1); nc = std::max(nc, r.sbx + 1); }
                    std::vector<std::vector<uint32_t>> gr(nr, std::vector<uint32_t>(nc, ~0u));
                    for (size_t k = 0; k < lf.size(); k++) gr[lf[k].sby][lf[k].sbx] = off[i].lf + (uint32_t) k;
                    for (auto &row : gr)
                        for (uint32_t v : row)
                            if (v == ~0u) return VP9HIP_EINVALIDDATA;
                    grid.push_back(std::move(gr));
                    maxr = std::max(maxr, nr);
                }
                if (grid.empty()) return 0;
                std::vector<std::vector<uint32_t>> tid(grid.size());   // task of (frame, row) or ~0u
                std::vector<uint32_t> recs;
                std::vector<uint32_t> offs;
                auto start = [&](int r) { return std::max(0, j0 - 2 * r); };
                for (int r = 0; r < maxr; r++)
                    for (size_t f = 0; f < grid.size(); f++) {
                        if (r >= (int) grid[f].size()) continue;
                        const int nc = (int) grid[f][r].size(), c0 = start(r);
                        if (c0 >= nc) { tid[f].push_back(~0u); continue; }
                        tid[f].push_back((uint32_t) offs.size());
                        offs.push_back((uint32_t) recs.size());
                        const uint32_t dep = r ? tid[f][r - 1] : ~0u;
                        recs.push_back(dep);
                        recs.push_back((uint32_t) nc);
                        recs.push_back((uint32_t) c0);
                        recs.push_back(dep != ~0u ? (uint32_t) std::max(0, start(r - 1) - 1) : 0u);
                        recs.insert(recs.end(), grid[f][r].begin() + c0, grid[f][r].end());
                    }
                if (offs.empty()) return 0;
                const uint32_t nt = (uint32_t) offs.size();
                Launch L = { K_LFR, (uint32_t) s.lists.size(), nt, (int) s.n_ctr, g, ph, PART_LF, 0 };
                for (uint32_t &o : offs) o += nt;
                s.lists.insert(s.lists.end(), offs.begin(), offs.end());
                s.lists.insert(s.lists.end(), recs.begin(), recs.end());
                s.lfr_ctr.push_back(s.n_ctr);
                s.n_ctr += 4 + 2 * nt;     // ticket, done, timeouts, spin; progress and row-done per task
                s.launches.push_back(L);
                for (int i : phase_frames[ph])
                    for (size_t k = 0; k < plans[i].s.lfs.size(); k++) {
                        const LFRec &r = plans[i].s.lfs[k];
                        if (r.sbx + 2 * r.sby < j0) continue;
                        s.alg_bytes[K_LF] -= lf_bytes[off[i].lf + k];
                        s.alg_bytes[K_LFR] += lf_bytes[off[i].lf + k];
                    }
                return 0;
            };
            if (!fuse || lvl_ph[ph]) {
                for (size_t d = 0; d < wls.size(); d++) add_list(K_PRED, wls[d], (int) d);
                if (lfr) {
                    if (int e = add_lfr(0)) return e;
                } else {
                    for (size_t d = 0; d < lsteps[ph].size(); d++) add_list(K_LF, lsteps[ph][d], (int) d);
                }
                continue;
            }
            // Fused schedule: launch t runs intra diagonal t and LF diagonal t - PLF_LAG.
            // LF of SB (x, y) (diagonal x + 2y = j) rewrites pre-LF pixels of SBs
            // (x - 1 .. x, y - 1 .. y) that the intra blocks of SBs (x - 1 .. x + 1, y .. y + 1)
            // read; those are on intra diagonals <= x_in_tile + y + 2 <= j + 2, i.e. in earlier
            // launches. Conversely the intra diagonal t reads SBs on diagonals t - 1, t - 2,
            // whose pixels no LF SB of diagonal t - 3 touches (that needs x - x_in_tile + y < 0).
            // This is the ordering the reference gets from its pre-LF intra_pred_data row
            // (vp9.c:1404-1416), without a second copy.
            // The residuals of intra diagonal t + 1 (inverse transforms, incl. inter
            // residuals added onto the MC prediction) run in launch t too, so no separate
            // residual pass precedes the wavefront: launch -1 holds diagonal 0's alone.
            const int np = (int) wls.size();
            const int nres = res_fused[ph] ? (int) rj_range[ph].size() : 0;
            // with k_lfr, LF diagonals fuse into the launches the intra wavefront needs anyway
            // and k_lfr filters the rest
            const int jlfr = std::max(0, std::max(np, nres - 1) - PLF_LAG);
            const int nlf = lfr ? std::min(jlfr, (int) lsteps[ph].size()) : (int) lsteps[ph].size();
            const int nt = std::max(std::max(np, nlf ? nlf + PLF_LAG : 0), nres - 1);
            for (int t = -1; t < nt; t++) {
                const std::vector<uint32_t> *pv = t >= 0 && t < np && !wls[t].empty() ? &wls[t] : nullptr;
                const int j = t - PLF_LAG;
                const std::vector<uint32_t> *lv = j >= 0 && j < nlf && !lsteps[ph][j].empty() ? &lsteps[ph][j] : nullptr;
                const std::array<std::pair<uint32_t, uint32_t>, 5> *rr = t + 1 < nres ? &rj_range[ph][t + 1] : nullptr;
                bool res = false;
                for (int k = 0; rr && k < 5; k++) res |= (*rr)[k].second > 0;
                if (!pv && !res) {
                    if (lv) add_list(K_LF, *lv, j);
                    continue;
                }
                Launch L = { K_PLF, (uint32_t) s.lists.size(), 0, 0, g, ph, PART_RECON, t };
                if (pv) {
                    L.n = (uint32_t) pv->size();
                    s.lists.insert(s.lists.end(), pv->begin(), pv->end());
                    for (uint32_t w : *pv) { s.alg_bytes[K_PRED] -= wg_bytes[w]; s.alg_bytes[K_PLF] += wg_bytes[w]; }
                }
                L.off2 = (uint32_t) s.lists.size();
                if (lv) {
                    L.n2 = (uint32_t) lv->size();
                    s.lists.insert(s.lists.end(), lv->begin(), lv->end());
                    for (uint32_t li : *lv) { s.alg_bytes[K_LF] -= lf_bytes[li]; s.alg_bytes[K_PLF] += lf_bytes[li]; }
                }
                for (int k = 0; res && k < 5; k++) { L.roff[k] = (*rr)[k].first; L.rn[k] = (*rr)[k].second; }
                s.launches.push_back(L);
            }
            if (lfr)
                if (int e = add_lfr(nlf)) return e;
        }
    if (s.resid16 > 0xffffffffull) return VP9HIP_ENOMEM;

    STAGE_T(3);
    // upload: one arena; its host image is built in pinned memory (every frame writes its
    // records there with the batch index fixups, in parallel) and copied with one DMA
    auto al = [](size_t x) { return (x + 255) & ~(size_t) 255; };
    size_t o = 0;
    s.o_frames = o; o = al(o + s.frames.size() * sizeof(FrameDesc));
    s.o_sbs = o; o = al(o + (size_t) tot.sb * sizeof(SBRec));
    s.o_pjobs = o; o = al(o + (size_t) tot.job * sizeof(PJob));
    s.o_passes = o; o = al(o + (size_t) tot.pass * sizeof(uint32_t));
    s.o_wgs = o; o = al(o + (size_t) tot.wg * sizeof(WGRec));
    s.o_rjobs = o; o = al(o + (size_t) tot_rj * sizeof(RJob));
    s.o_lfs = o; o = al(o + (size_t) tot.lf * sizeof(LFRec));
    s.o_mcs = o; o = al(o + (size_t) tot.mc * sizeof(McUnit));
    s.o_lists = o; o = al(o + s.lists.size() * sizeof(uint32_t));
    s.o_ctr = o; o = al(o + (size_t) s.n_ctr * sizeof(uint32_t));
    s.o_coefs = o; o = al(o + coef_off[n] + 64);
    s.n_sbs = tot.sb; s.n_pjobs = tot.job; s.n_passes = tot.pass; s.n_wgs = tot.wg; s.n_rjobs = tot_rj;
    s.n_lfs = tot.lf; s.n_mcs = tot.mc;
    if (o > s.arena_cap) {
        if (s.arena) hipFree(s.arena);
        s.arena = nullptr;
        s.arena_cap = 0;
        if (hipMalloc(&s.arena, o) != hipSuccess) return VP9HIP_ENOMEM;
        s.arena_cap = o;
    }
    if (o > s.pinned_cap) {
        if (s.pinned) hipHostFree(s.pinned);
        s.pinned = nullptr;
        s.pinned_cap = 0;
        if (hipHostMalloc((void **) &s.pinned, o, hipHostMallocDefault) != hipSuccess) return VP9HIP_ENOMEM;
        s.pinned_cap = o;
    }
    const size_t rbytes = (size_t) s.resid16 * 32 + 256;
    if (rbytes > s.resid_cap) {
        if (s.resid) hipFree(s.resid);
        s.resid = nullptr;
        s.resid_cap = 0;
        if (hipMalloc(&s.resid, rbytes) != hipSuccess) return VP9HIP_ENOMEM;
        s.resid_cap = rbytes;
    }
    uint8_t *img = s.pinned;
    memcpy(img + s.o_frames, s.frames.data(), s.frames.size() * sizeof(FrameDesc));
    if (!s.lists.empty()) memcpy(img + s.o_lists, s.lists.data(), s.lists.size() * sizeof(uint32_t));
    init_lfr_ctr(c, s, (uint32_t *) (img + s.o_ctr));
    std::vector<double> inplace_bytes(n, 0.0);
    {
        std::atomic<int> next(0);
        auto worker = [&]() {
            for (int i; (i = next.fetch_add(1)) < n;) {
                const Staged &l = plans[i].s;
                const Off &q = off[i];
                const uint32_t res = (uint32_t) q.res;
                if (!l.sbs.empty()) memcpy((SBRec *) (img + s.o_sbs) + q.sb, l.sbs.data(), l.sbs.size() * sizeof(SBRec));
                PJob *pj = (PJob *) (img + s.o_pjobs) + q.job;
                for (size_t k = 0; k < l.pjobs.size(); k++) {
                    PJob j = l.pjobs[k];
                    if (PJ_RES(j)) j.roff += res;
                    pj[k] = j;
                }
                if (!l.passes.empty())
                    memcpy((uint32_t *) (img + s.o_passes) + q.pass, l.passes.data(), l.passes.size() * sizeof(uint32_t));
                WGRec *wg = (WGRec *) (img + s.o_wgs) + q.wg;
                for (size_t k = 0; k < l.wgs.size(); k++) {
                    WGRec w = l.wgs[k];
                    w.job0 += q.job; w.pass0 += q.pass; w.sb[0] += q.sb;
                    wg[k] = w;
                }
                if (!l.lfs.empty()) memcpy((LFRec *) (img + s.o_lfs) + q.lf, l.lfs.data(), l.lfs.size() * sizeof(LFRec));
                if (!l.mcs.empty()) memcpy((McUnit *) (img + s.o_mcs) + q.mc, l.mcs.data(), l.mcs.size() * sizeof(McUnit));
                double ib = 0;
                for (size_t d = 0; d < l.rbucket.size(); d++)
                for (int t = 0; t < 5; t++)
                    for (int tp = 0; tp < 4; tp++) {
                        const std::vector<RJob> &bk = l.rbucket[d][t][tp];
                        RJob *dst = (RJob *) (img + s.o_rjobs) + rj_off[i][d][t][tp];
                        for (size_t k = 0; k < bk.size(); k++) {
                            RJob r = bk[k];
                            if (!(r.ptx & 32)) r.dst += res;          // intra: residual scratch offset
                            else ib += 2.0 * (16 << (2 * (t & 3))) * c->bypp;   // inter: pixels read + written
                            dst[k] = r;
                        }
                    }
                inplace_bytes[i] = ib;
                if (coef_off[i + 1] > coef_off[i])
                    memcpy(img + s.o_coefs + coef_off[i], pkts[i].coefs, coef_off[i + 1] - coef_off[i]);
                plans[i] = FramePlan();                  // release the frame's host images
            }
        };
        const int nt = std::min(n, c->host_threads);
        std::vector<std::thread> pool;
        for (int t = 1; t < nt; t++) pool.emplace_back(worker);
        worker();
        for (auto &t : pool) t.join();
    }
    for (int i = 0; i < n; i++) s.alg_bytes[K_RESID] += inplace_bytes[i];
    for (int i = 0; i < n; i++)                  // residuals that run inside the k_plf launches
        if (res_fused[fbs[i].phase]) {
            const double b = (double) pkts[i].ncoefs * csz + inplace_bytes[i];
            s.alg_bytes[K_RESID] -= b;
            s.alg_bytes[K_PLF] += b;
        }
    HIPCHK(hipMemcpyAsync(s.arena, img, o, hipMemcpyHostToDevice, c->st));
    STAGE_T(4);
    HIPCHK(hipStreamSynchronize(c->st));
    STAGE_T(5);
    if (stage_trace)
        fprintf(stderr, "vp9hip stage: %d frames: setup %.1f plan %.1f merge %.1f schedule %.1f upload %.1f sync %.1f ms\n",
                n, st_ms[0], st_ms[1], st_ms[2], st_ms[3], st_ms[4], st_ms[5]);
    s.ready = true;
    return 0;
}

extern "C" int vp9hip_stage_batch(vp9hip_ctx *c, const vp9h_frame *pkts, int n, const int *out_bufs)
{
    return stage(c, pkts, n, out_bufs, nullptr);
}

extern "C" int vp9hip_stage_batch_refs(vp9hip_ctx *c, const vp9h_frame *pkts, int n, const int *out_bufs,
                                       const int *ref_bufs)
{
    return stage(c, pkts, n, out_bufs, ref_bufs);
}

static int enqueue_batch(vp9hip_ctx *c);

static bool same_launches(const std::vector<Launch> &a, const std::vector<Launch> &b)
{
    if (a.size() != b.size()) return false;
    for (size_t i = 0; i < a.size(); i++) {
        const Launch &x = a[i], &y = b[i];
        if (x.kind != y.kind || x.off != y.off || x.n != y.n || x.arg != y.arg || x.grp != y.grp || x.ph != y.ph ||
            x.part != y.part || x.off2 != y.off2 || x.n2 != y.n2 || x.devr != y.devr || x.flow != y.flow ||
            memcmp(x.roff, y.roff, sizeof(x.roff)) ||
            memcmp(x.rn, y.rn, sizeof(x.rn)))
            return false;
    }
    return true;
}

// Run the staged batch. Without per-launch timing the ~300 launches of a 4K batch are
// captured once into a HIP graph (both frame-group streams) and replayed.
extern "C" int vp9hip_run_batch(vp9hip_ctx *c)
{
    if (!c || !c->stg.ready) return VP9HIP_EINVAL;
    hipSetDevice(c->dev);
    Staged &s = c->stg;
    if (s.dev && !(c->plan_reuse && s.stat && s.planned)) {   // plan on the device from the resident packets
        const int r = plan_dev(c);
        if (r) return r;
        if (c->plan_only) return 0;       // diagnostics: the planner alone
    }
    if (s.dev && s.stat && plan_stream(c) != c->st) {
        HIPCHK(hipStreamWaitEvent(c->st, s.plan_ev, 0));
    }
    // a batch touching another slot's buffers follows that slot's last run
    for (int k = 0; c->slot_streams && k < MAX_SLOTS; k++)
        if (((s.dep_mask >> k) & 1) && c->sl[k].done_ev) HIPCHK(hipStreamWaitEvent(c->st, c->sl[k].done_ev, 0));
    // this slot's last work on the main stream: its next planning waits for it
    if (!s.done_ev) HIPCHK(hipEventCreateWithFlags(&s.done_ev, hipEventDisableTiming));
    if (c->timing || !c->use_graph) {
        const int r = enqueue_batch(c);
        if (!r) HIPCHK(hipEventRecord(s.done_ev, c->st));
        return r;
    }
    // the graph of the previous run is reused when the launch list is the same (same
    // geometry and record counts); the records themselves were just rewritten in place
    if (s.graph && !same_launches(s.graph_launches, s.launches)) {
        hipGraphExecDestroy(s.graph);
        s.graph = nullptr;
    }
    if (!s.graph) {
        s.graph_launches = s.launches;
        hipGraph_t g = nullptr;
        HIPCHK(hipStreamBeginCapture(c->st, hipStreamCaptureModeThreadLocal));
        int r = enqueue_batch(c);
        hipError_t e = hipStreamEndCapture(c->st, &g);
        if (r || e != hipSuccess) { if (g) hipGraphDestroy(g); return r ? r : VP9HIP_EEXTERNAL; }
        e = hipGraphInstantiate(&s.graph, g, nullptr, nullptr, 0);
        hipGraphDestroy(g);
        if (e != hipSuccess) { s.graph = nullptr; return VP9HIP_EEXTERNAL; }
    }
    HIPCHK(hipGraphLaunch(s.graph, c->st));
    HIPCHK(hipEventRecord(s.done_ev, c->st));
    return 0;
}

static int launch_one(vp9hip_ctx *c, const Launch &L, hipStream_t st)
{
    Staged &s = c->stg;
    const FrameDesc *fr = (const FrameDesc *) (s.arena + s.o_frames);
    const uint32_t *lists = (const uint32_t *) (s.arena + s.o_lists);
    // timing-only ablations (tools/ablate.sh; frames are then wrong): VP9HIP_DEBUG bit 28 skips
    // the level phases' k_resid_multi launches, bit 29 the k_mcq launches
    if ((c->dbg >> 28 & 1) && L.kind == K_RESID && L.arg == 5) return 0;
    if ((c->dbg >> 29 & 1) && L.kind == K_MC) return 0;
    switch (L.kind) {
    case K_MC:
        return vp9hip_launch_mc(c->hb, st, (int) L.n, (const McUnit *) (s.arena + s.o_mcs) + L.off, fr, &c->kcfg);
    case K_RESID:
        if (L.devr)
            return vp9hip_launch_resid_dev(c->hb, st, L.arg, (int) L.n, (const RJob *) (s.arena + s.o_rjobs),
                                           (const uint32_t *) (s.arena + s.o_summary) + 1 + L.off, fr,
                                           s.arena + s.o_coefs, s.resid);
        if (L.arg == 5)
            return vp9hip_launch_resid_multi(c->hb, st, L.roff, L.rn, (const RJob *) (s.arena + s.o_rjobs), fr,
                                             s.arena + s.o_coefs, s.resid);
        return vp9hip_launch_resid(c->hb, st, L.arg, (int) L.n, (const RJob *) (s.arena + s.o_rjobs) + L.off, fr,
                                   s.arena + s.o_coefs, s.resid);
    case K_PRED:
        if (L.flow >= 0)
            return vp9hip_launch_predd(c->hb | c->ss_h << 1 | c->ss_v << 2, st, (int) L.n, c->pred_df_wgs, lists + L.off,
                                       (const uint32_t *) (s.arena + s.o_sbinfo), (const WGRec *) (s.arena + s.o_wgs),
                                       (const SBRec *) (s.arena + s.o_sbs), (const PJob *) (s.arena + s.o_pjobs),
                                       (const uint32_t *) (s.arena + s.o_passes), fr, s.resid, c->ptab,
                                       (uint32_t *) (s.arena + s.o_ctr) + L.flow, (uint32_t *) (s.arena + s.o_ctr) + s.pdone,
                                       c->dbg);
        return vp9hip_launch_pred(c->hb | c->ss_h << 1 | c->ss_v << 2, st, (int) L.n, lists + L.off, (const WGRec *) (s.arena + s.o_wgs),
                                  (const SBRec *) (s.arena + s.o_sbs), (const PJob *) (s.arena + s.o_pjobs),
                                  (const uint32_t *) (s.arena + s.o_passes), fr, s.resid, c->ptab, c->dbg);
    case K_LFR:
    {
        LfrIntra li = {};
        if (L.n2) {                    // the phase's intra SBs inside the launch
            li.list = lists + L.off2;
            li.sbinfo = (const uint32_t *) (s.arena + s.o_sbinfo);
            li.wgs = (const WGRec *) (s.arena + s.o_wgs);
            li.sbs = (const SBRec *) (s.arena + s.o_sbs);
            li.jobs = (const PJob *) (s.arena + s.o_pjobs);
            li.passes = (const uint32_t *) (s.arena + s.o_passes);
            li.resid = s.resid;
            li.ptab = c->ptab;
            li.pctr = (uint32_t *) (s.arena + s.o_ctr) + L.flow;
            li.done = (uint32_t *) (s.arena + s.o_ctr) + s.pdone;
            li.n = (int) L.n2;
            li.nblk = (int) std::min<uint32_t>((L.n2 + LFRI_WAVES - 1) / LFRI_WAVES,
                                               (uint32_t) std::max(1, c->pred_df_wgs / LFRI_WAVES));
            li.dbg = c->dbg;
        }
        return vp9hip_launch_lfr(c->hb | c->ss_h << 1 | c->ss_v << 2, st, (int) L.n, lists + L.off,
                                 (const LFRec *) (s.arena + s.o_lfs), fr, (uint32_t *) (s.arena + s.o_ctr) + L.arg,
                                 &c->kcfg, &li);
    }
    case K_LF:
        return vp9hip_launch_lf(c->hb | c->ss_h << 1 | c->ss_v << 2, st, (int) L.n, lists + L.off, (const LFRec *) (s.arena + s.o_lfs), fr, c->dbg >> 16);
    case K_PLF: {
        PlfLaunch pl;
        pl.npred = L.n; pl.nlf = L.n2;
        for (int k = 0; k < 5; k++) { pl.roff[k] = L.roff[k]; pl.rn[k] = L.rn[k]; }
        return vp9hip_launch_plf(c->hb | c->ss_h << 1 | c->ss_v << 2, st, &pl, lists + L.off, lists + L.off2,
                                 (const WGRec *) (s.arena + s.o_wgs), (const SBRec *) (s.arena + s.o_sbs),
                                 (const PJob *) (s.arena + s.o_pjobs), (const uint32_t *) (s.arena + s.o_passes),
                                 (const LFRec *) (s.arena + s.o_lfs), (const RJob *) (s.arena + s.o_rjobs), fr,
                                 s.arena + s.o_coefs, s.resid, c->ptab, c->dbg);
    }
    }
    return -1;
}

// Enqueue the staged launches: group g runs on its own stream (group 0 on the main
// stream), forked from and joined back into the main stream. (Round 1 also ran a group's
// loop filter on a second stream, LF diagonal j after intra diagonal j + LF_LAG through
// cross-stream events: 8,131 vs 11,800 fps at C3, removed; k_plf fuses the two instead.)
static int enqueue_batch(vp9hip_ctx *c)
{
    Staged &s = c->stg;
    size_t nl = s.launches.size();
    c->timed_run = c->timing;
    if (c->timing && c->ev.size() < 2 * nl) {
        size_t old = c->ev.size();
        c->ev.resize(2 * nl);
        for (size_t i = old; i < c->ev.size(); i++) HIPCHK(hipEventCreate(&c->ev[i]));
    }
    // timing runs put every launch on the main stream (serialised, as under a rocprofv3
    // kernel trace), so each launch's event duration is its own, not one inflated by the
    // other frame groups' launches
    const bool serial = c->timing;
    const int ngs = serial ? 1 : s.ngroups;
    auto rstream = [&](int g) { return g && !serial ? c->xst[g - 1] : c->st; };
    // fork: every stream of the batch starts after what is queued on the main stream
    if (ngs > 1) {
        HIPCHK(hipEventRecord(c->fork_ev, c->st));
        for (int g = 1; g < ngs; g++) HIPCHK(hipStreamWaitEvent(c->xst[g - 1], c->fork_ev, 0));
    }
    for (size_t i = 0; i < nl; i++) {
        const Launch &L = s.launches[i];
        hipStream_t st = rstream(L.grp);
        if (c->timing) HIPCHK(hipEventRecord(c->ev[2 * i], st));
        if (launch_one(c, L, st)) return VP9HIP_EEXTERNAL;
        if (c->timing) HIPCHK(hipEventRecord(c->ev[2 * i + 1], st));
    }
    // join: the main stream (downloads, sync, the next stage) waits for every stream
    for (int g = 1; g < ngs; g++) {
        HIPCHK(hipEventRecord(c->join_ev[g - 1], c->xst[g - 1]));
        HIPCHK(hipStreamWaitEvent(c->st, c->join_ev[g - 1], 0));
    }
    return 0;
}

// ---- tile-column sharding of one stream over several devices ----
extern "C" int vp9hip_stage_batch_tiles(vp9hip_ctx *c, const vp9h_frame *pkts, int n, const int *out_bufs,
                                        const int *ref_bufs, int tile_lo, int tile_hi)
{
    if (tile_lo < 0 || tile_hi < tile_lo || tile_hi > 64) return VP9HIP_EINVAL;
    return stage(c, pkts, n, out_bufs, ref_bufs, tile_lo, tile_hi, 1, true);   // one group: phases in chain order
}

extern "C" int vp9hip_batch_phases(vp9hip_ctx *c)
{
    if (!c || !c->stg.ready) return VP9HIP_EINVAL;
    return c->stg.nphases;
}

// Frame groups (concurrent HIP streams) of the staged batch.
extern "C" int vp9hip_batch_groups(vp9hip_ctx *c)
{
    if (!c || !c->stg.ready) return VP9HIP_EINVAL;
    return c->stg.ngroups;
}

extern "C" int vp9hip_phase_frames(vp9hip_ctx *c, int phase, int *frames, int cap)
{
    if (!c || !c->stg.ready || phase < 0 || phase >= c->stg.nphases || cap < 0) return VP9HIP_EINVAL;
    int n = 0;
    for (int i = 0; i < (int) c->stg.frame_phase.size(); i++)
        if (c->stg.frame_phase[i] == phase) {
            if (frames && n < cap) frames[n] = i;
            n++;
        }
    return n;
}

// Enqueue one part of one phase: PART_RECON (MC, residuals, intra of this context's
// tile columns) or PART_LF (the loop filter of the whole frames).
extern "C" int vp9hip_run_phase(vp9hip_ctx *c, int phase, int part)
{
    if (!c || !c->stg.ready || phase < 0 || phase >= c->stg.nphases || (part != PART_RECON && part != PART_LF))
        return VP9HIP_EINVAL;
    hipSetDevice(c->dev);
    Staged &s = c->stg;
    // a pass over the batch starts at phase 0's reconstruction: plan it again (decoding the
    // batch includes planning it), after the previous pass's launches
    if (s.dev && (!s.planned || (phase == 0 && part == PART_RECON))) {
        const int r = plan_dev(c);
        if (r) return r;
    }
    c->timed_run = false;
    for (const Launch &L : s.launches)
        if (L.ph == phase && L.part == part && launch_one(c, L, c->st)) return VP9HIP_EEXTERNAL;
    if (!s.done_ev) HIPCHK(hipEventCreateWithFlags(&s.done_ev, hipEventDisableTiming));
    HIPCHK(hipEventRecord(s.done_ev, c->st));
    return 0;
}

// Copy the pixel columns of tile columns [tile_lo, tile_hi) of batch frame `frame` (all
// 8-aligned rows; Y, then U, then V, each packed row by row) between the frame's buffer
// and contiguous device memory `dev`: to_frame = 0 packs, 1 unpacks. dev == NULL only
// returns the byte count. Tile columns follow set_tile_offset (vp9.c:1244-1250).
extern "C" int64_t vp9hip_stripe(vp9hip_ctx *c, int frame, int tile_lo, int tile_hi, void *dev, int to_frame)
{
    if (!c || !c->stg.ready || frame < 0 || frame >= (int) c->stg.frames.size() || tile_lo < 0 || tile_hi < tile_lo)
        return VP9HIP_EINVAL;
    const FrameDesc &fd = c->stg.frames[frame];
    const int log2 = c->stg.frame_log2[frame], nt = 1 << log2;
    auto sbx = [&](int t) { return std::min(std::min(t, nt) * fd.sb_cols >> log2, fd.sb_cols); };
    const int x0 = std::min(sbx(tile_lo) * 64, (int) fd.w8[0]), x1 = std::min(sbx(tile_hi) * 64, (int) fd.w8[0]);
    int64_t off = 0;
    for (int p = 0; p < 3; p++) {
        const int sh = p ? c->ss_h : 0, h = p ? fd.h8[1] : fd.h8[0];
        const size_t w = (size_t) ((x1 >> sh) - (x0 >> sh)) * c->bypp, pitch = (size_t) fd.pitch[p ? 1 : 0] * c->bypp;
        if (dev && w && h) {
            uint8_t *fp = (uint8_t *) fd.plane[p] + (size_t) (x0 >> sh) * c->bypp, *dp = (uint8_t *) dev + off;
            hipError_t e = to_frame ? hipMemcpy2DAsync(fp, pitch, dp, w, w, h, hipMemcpyDeviceToDevice, c->st)
                                    : hipMemcpy2DAsync(dp, w, fp, pitch, w, h, hipMemcpyDeviceToDevice, c->st);
            if (e != hipSuccess) return VP9HIP_EEXTERNAL;
        }
        off += (int64_t) w * h;
    }
    return off;
}

// k_lfr bounds its spins and counts the waits it gave up (timeout word of each launch's
// counter block): a nonzero count means the row hand-off broke, and the slot's frames are
// not trusted. The slot's work must be complete.
static int check_lfr(const Staged &g)
{
    if (!g.ready || g.lfr_ctr.empty()) return 0;
    std::vector<uint32_t> ctr(g.n_ctr);
    HIPCHK(hipMemcpy(ctr.data(), g.arena + g.o_ctr, ctr.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
    for (uint32_t o : g.lfr_ctr)
        if (ctr[o + 2]) return VP9HIP_EBUG;
    return 0;
}

extern "C" int vp9hip_sync_slot(vp9hip_ctx *c, int slot)
{
    if (!c || slot < 0 || slot >= MAX_SLOTS) return VP9HIP_EINVAL;
    hipSetDevice(c->dev);
    Staged &g = slot_ref(c, slot);
    if (g.done_ev) HIPCHK(hipEventSynchronize(g.done_ev));
    // a batch with rejected frames still ran the others: their loop-filter hand-offs count
    const int r = finish_summary(c, g);
    if (r && r != VP9HIP_EINVALIDDATA) return r;
    if (const int l = check_lfr(g)) return l;
    return r;
}

extern "C" int vp9hip_batch_frame_status(vp9hip_ctx *c, int slot, int *status, int cap)
{
    if (!c || slot < 0 || slot >= MAX_SLOTS || cap < 0 || (cap > 0 && !status)) return VP9HIP_EINVAL;
    const Staged &g = slot_ref(c, slot);
    const int n = (int) g.fstat.size();
    for (int i = 0; i < n && i < cap; i++) status[i] = g.fstat[i];
    return n;
}

extern "C" int vp9hip_slot_stream_wait(vp9hip_ctx *c, int slot, void *stream)
{
    if (!c || slot < 0 || slot >= MAX_SLOTS) return VP9HIP_EINVAL;
    hipSetDevice(c->dev);
    const Staged &g = slot_ref(c, slot);
    if (g.done_ev) HIPCHK(hipStreamWaitEvent((hipStream_t) stream, g.done_ev, 0));
    return 0;
}

extern "C" int vp9hip_slot_busy(vp9hip_ctx *c, int slot)
{
    if (!c || slot < 0 || slot >= MAX_SLOTS) return VP9HIP_EINVAL;
    hipSetDevice(c->dev);
    const Staged &g = slot_ref(c, slot);
    if (!g.done_ev) return 0;
    const hipError_t e = hipEventQuery(g.done_ev);
    return e == hipErrorNotReady ? 1 : e == hipSuccess ? 0 : VP9HIP_EEXTERNAL;
}

extern "C" int vp9hip_sync(vp9hip_ctx *c)
{
    if (!c) return VP9HIP_EINVAL;
    hipSetDevice(c->dev);
    HIPCHK(sync_all(c));
    // every slot's work is complete: their hand-off counters and summaries are final; every
    // slot is checked (each summary read once), the first error returned
    int err = 0;
    for (int k = 0; k < MAX_SLOTS; k++) {
        int r = finish_summary(c, slot_ref(c, k));
        if (!r || r == VP9HIP_EINVALIDDATA)
            if (const int l = check_lfr(slot_ref(c, k))) r = l;
        if (r && !err) err = r;
    }
    if (err) return err;
    if (c->timing && c->timed_run && c->stg.ready) {
        for (int k = 0; k < K_N; k++) { c->kms[k] = 0; c->kcount[k] = 0; }
        for (size_t i = 0; i < c->stg.launches.size() && 2 * i + 1 < c->ev.size(); i++) {
            float ms = 0;
            if (hipEventElapsedTime(&ms, c->ev[2 * i], c->ev[2 * i + 1]) == hipSuccess) {
                c->kms[c->stg.launches[i].kind] += ms;
                c->kcount[c->stg.launches[i].kind]++;
            }
        }
        float ms = 0;
        if (c->plan_timed && hipEventElapsedTime(&ms, c->pev[0], c->pev[1]) == hipSuccess) {
            c->kms[K_PLAN] = ms;
            c->kcount[K_PLAN] = 1;
        }
    }
    return 0;
}

extern "C" int vp9hip_submit_frame(vp9hip_ctx *c, const vp9h_frame *pkt, int out_buf, const int ref_buf[3])
{
    int r = stage(c, pkt, 1, &out_buf, ref_buf);
    if (r < 0) return r;
    return vp9hip_run_batch(c);
}

// Wait for the batches that write buffer `buf`: the slots whose staged batch has it in its
// write set (a slot's older batches were complete when it was restaged: stage() waits for
// them), not the whole context, whose streams may already hold newer batches.
static int wait_writers(vp9hip_ctx *c, int buf)
{
    for (int k = 0; k < MAX_SLOTS; k++) {
        const Staged &g = slot_ref(c, k);
        if (g.done_ev && std::binary_search(g.wr.begin(), g.wr.end(), buf))
            HIPCHK(hipEventSynchronize(g.done_ev));
    }
    return 0;
}

#define DL_CHUNK ((size_t) 16 << 20)    // bytes per staging chunk (D2H: 29 GB/s at 8 MB, 55 at 16, tools/d2h_bw.py)
#define DL_RING 4

extern "C" int vp9hip_download_frame(vp9hip_ctx *c, int buf, uint8_t *const planes[3], const ptrdiff_t linesize[3])
{
    if (!c || buf < 0 || buf >= (int) c->bufs.size() || !planes) return VP9HIP_EINVAL;
    hipSetDevice(c->dev);
    if (const int r = wait_writers(c, buf)) return r;
    if (!c->dst_dl) HIPCHK(hipStreamCreateWithFlags(&c->dst_dl, hipStreamNonBlocking));
    // a buffer no staged batch writes may still be under vp9hip_fill_buffers' memset (on the
    // main stream): the copies follow it
    if (c->fill_ev) HIPCHK(hipStreamWaitEvent(c->dst_dl, c->fill_ev, 0));
    if (!c->dl_pin) HIPCHK(hipHostMalloc((void **) &c->dl_pin, DL_CHUNK * DL_RING, hipHostMallocDefault));
    for (auto &e : c->dl_ev)
        if (!e) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    if (!c->dl_pool) c->dl_pool.reset(new CopyPool(c->dl_threads));
    // chunks of whole rows: D2H into ring slot k, then (once the slot after it is queued)
    // the host copy of slot k into the caller's planes
    struct Piece { int p, y0, ny; };
    std::vector<Piece> pieces;
    const int bw = c->buf_wh[buf].first, bh = c->buf_wh[buf].second;
    for (int p = 0; p < 3; p++) {
        const int pw = p ? (bw + c->ss_h) >> c->ss_h : bw, ph = p ? (bh + c->ss_v) >> c->ss_v : bh;
        const size_t row = (size_t) pw * c->bypp;
        const int per = (int) std::max<size_t>(1, DL_CHUNK / row);
        for (int y = 0; y < ph; y += per) pieces.push_back({ p, y, std::min(per, ph - y) });
    }
    auto row_bytes = [&](int p) { return (size_t) (p ? (bw + c->ss_h) >> c->ss_h : bw) * c->bypp; };
    auto issue = [&](size_t i) -> int {
        const Piece &q = pieces[i];
        const size_t row = row_bytes(q.p), pitch = (size_t) c->pitch[q.p ? 1 : 0] * c->bypp;
        const uint8_t *src = c->bufs[buf] + c->plane_off[q.p] + (size_t) q.y0 * pitch;
        if (pitch == row)   // unpadded rows (widths of 64-multiples): one linear copy
            HIPCHK(hipMemcpyAsync(c->dl_pin + (i % DL_RING) * DL_CHUNK, src, row * q.ny, hipMemcpyDeviceToHost, c->dst_dl));
        else
            HIPCHK(hipMemcpy2DAsync(c->dl_pin + (i % DL_RING) * DL_CHUNK, row, src, pitch, row, q.ny,
                                    hipMemcpyDeviceToHost, c->dst_dl));
        HIPCHK(hipEventRecord(c->dl_ev[i % DL_RING], c->dst_dl));
        return 0;
    };
    for (size_t i = 0; i < pieces.size() && i < DL_RING; i++)
        if (const int r = issue(i)) return r;
    for (size_t i = 0; i < pieces.size(); i++) {
        const Piece &q = pieces[i];
        HIPCHK(hipEventSynchronize(c->dl_ev[i % DL_RING]));
        const size_t row = row_bytes(q.p);
        const uint8_t *src = c->dl_pin + (i % DL_RING) * DL_CHUNK;
        uint8_t *dst = planes[q.p] + (ptrdiff_t) q.y0 * linesize[q.p];
        c->dl_pool->run(dst, linesize[q.p], src, row, row, q.ny);
        if (i + DL_RING < pieces.size())
            if (const int r = issue(i + DL_RING)) return r;
    }
    return 0;
}

extern "C" int vp9hip_upload_frame(vp9hip_ctx *c, int buf, const uint8_t *const planes[3], const ptrdiff_t linesize[3])
{
    if (!c || buf < 0 || buf >= (int) c->bufs.size() || !planes) return VP9HIP_EINVAL;
    hipSetDevice(c->dev);
    HIPCHK(sync_all(c));
    for (int p = 0; p < 3; p++) {
        const int bw = c->buf_wh[buf].first, bh = c->buf_wh[buf].second;
        int pw = p ? (bw + c->ss_h) >> c->ss_h : bw, ph = p ? (bh + c->ss_v) >> c->ss_v : bh;
        HIPCHK(hipMemcpy2DAsync(c->bufs[buf] + c->plane_off[p], (size_t) c->pitch[p ? 1 : 0] * c->bypp,
                                planes[p], linesize[p], (size_t) pw * c->bypp, ph, hipMemcpyHostToDevice, c->st));
    }
    HIPCHK(hipStreamSynchronize(c->st));
    return 0;
}

// Zero-copy export of a decoded frame: device pointers of the three
// planes, their pitches in bytes, the visible size, and the context's stream, which
// orders every kernel that writes the buffer. A consumer that enqueues on that stream
// (or waits for vp9hip_sync) reads the finished frame without a D2H copy. The pointers
// stay valid until vp9hip_configure / vp9hip_close; the content until the buffer is
// written again.
extern "C" int vp9hip_frame_device(vp9hip_ctx *c, int buf, void *planes[3], ptrdiff_t linesize[3], int *width,
                                   int *height, void **stream)
{
    if (!c || buf < 0 || buf >= (int) c->bufs.size() || !planes || !linesize) return VP9HIP_EINVAL;
    for (int p = 0; p < 3; p++) {
        planes[p] = c->bufs[buf] + c->plane_off[p];
        linesize[p] = (ptrdiff_t) c->pitch[p ? 1 : 0] * c->bypp;
    }
    if (width) *width = c->buf_wh[buf].first;
    if (height) *height = c->buf_wh[buf].second;
    if (stream) *stream = (void *) c->st;
    return 0;
}

extern "C" int vp9hip_flush(vp9hip_ctx *c)
{
    if (!c) return VP9HIP_EINVAL;
    hipSetDevice(c->dev);
    HIPCHK(sync_all(c));
    drop_slots(c);
    return 0;
}

extern "C" int vp9hip_fill_buffers(vp9hip_ctx *c, int buf0, int count, int value)
{
    if (!c || buf0 < 0 || count < 0 || buf0 + count > (int) c->bufs.size()) return VP9HIP_EINVAL;
    hipSetDevice(c->dev);
    HIPCHK(sync_all(c));                 // neither slot's work may still read the buffers
    for (int i = buf0; i < buf0 + count; i++) HIPCHK(hipMemsetAsync(c->bufs[i], value & 255, c->buf_bytes, c->st));
    // every slot's later work (whichever stream it runs on) follows the fill
    if (!c->fill_ev) HIPCHK(hipEventCreateWithFlags(&c->fill_ev, hipEventDisableTiming));
    HIPCHK(hipEventRecord(c->fill_ev, c->st));
    for (int k = 0; k < MAX_SLOTS; k++)
        if (c->sst[k] && c->sst[k] != c->st) HIPCHK(hipStreamWaitEvent(c->sst[k], c->fill_ev, 0));
    if (c->pst) HIPCHK(hipStreamWaitEvent(c->pst, c->fill_ev, 0));
    return 0;
}

extern "C" int vp9hip_last_timing(vp9hip_ctx *c, const char **names, double *ms, int *launches, int cap)
{
    if (!c) return VP9HIP_EINVAL;
    int n = 0;
    for (int k = 0; k < K_N && n < cap; k++, n++) {
        if (names) names[n] = kname[k];
        if (ms) ms[n] = c->kms[k];
        if (launches) launches[n] = c->kcount[k];
    }
    return n;
}

// Algorithmic bytes of the staged batch per kernel class (same order as timing).
extern "C" int vp9hip_alg_bytes(vp9hip_ctx *c, double *bytes, int cap)
{
    if (!c) return VP9HIP_EINVAL;
    if (c->stg.summary_pending) {            // a static plan's totals: after its run
        hipSetDevice(c->dev);
        HIPCHK(sync_all(c));
        if (const int r = finish_summary(c, c->stg)) return r;
    }
    int n = 0;
    for (int k = 0; k < K_N && n < cap; k++, n++) bytes[n] = c->stg.alg_bytes[k];
    return n;
}

extern "C" int vp9hip_set_timing(vp9hip_ctx *c, int on)
{
    if (!c) return VP9HIP_EINVAL;
    c->timing = on != 0;
    return 0;
}

extern "C" int vp9hip_set_graph(vp9hip_ctx *c, int on)
{
    if (!c) return VP9HIP_EINVAL;
    c->use_graph = on != 0;
    return 0;
}

extern "C" int vp9hip_abi_version(void) { return VP9HIP_ABI_VERSION; }

extern "C" int vp9hip_device_info(int device, char *pci_bus_id, int len, char *name, int name_len)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return VP9HIP_ENOSYS;
    if (pci_bus_id && len > 0) HIPCHK(hipDeviceGetPCIBusId(pci_bus_id, len, device));
    if (name && name_len > 0) {
        hipDeviceProp_t p;
        HIPCHK(hipGetDeviceProperties(&p, device));
        snprintf(name, (size_t) name_len, "%s (%s)", p.name, p.gcnArchName);
    }
    return 0;
}

// VP9HIP_MAX_SLOTS batch slots per context: stage / run / sync / phase calls act on the
// current slot. Each slot has its own arena, plan, graph and (per-slot streams) streams; the
// frame buffers are the context's. A run of one slot plans while other slots' pixel kernels
// still run.
extern "C" int vp9hip_set_batch_slot(vp9hip_ctx *c, int slot)
{
    if (!c || slot < 0 || slot >= MAX_SLOTS) return VP9HIP_EINVAL;
    if (slot != c->slot) {
        if (c->slot_streams) {
            hipSetDevice(c->dev);
            if (!slot_streams_make(c, slot)) return VP9HIP_EEXTERNAL;
        }
        std::swap(c->stg, c->sl[c->slot]);   // the current batch back into its storage
        std::swap(c->stg, c->sl[slot]);      // and the other one in
        if (c->slot_streams) {
            c->st = c->sst[slot];
            for (int i = 0; i < MAX_GROUPS - 1; i++) c->xst[i] = c->sxst[slot][i];
        }
        c->slot = slot;
    }
    return 0;
}

// Host-only planning statistics of one frame (no device needed): used by the CPU tests
// and to size kernels. out[]: 0 SBs with intra work, 1 passes, 2 intra jobs, 3 residual
// jobs, 4..7 intra jobs per tx size, 8 lane use (job lanes / 64 per pass), 9 max passes
// in one SB, 10 LF records, 11 MC units, 12 intra wavefront steps, 13 LF wavefront steps.
// Diagnostics (tools/wave_tail.py): per SB of one packet, in raster order, the pixel rows its
// intra passes loop over (sum of each pass's largest job size), as staged for the device.
extern "C" int vp9hip_plan_sb_costs(const vp9h_frame *f, double *out, int cap)
{
    if (!f || !out) return VP9HIP_EINVAL;
    if (f->ss_h > 1 || f->ss_v > 1) return VP9HIP_EINVAL;
    init_nz();
    Staged s;
    FrameBuild fb;
    fb.f = f; fb.frame_idx = 0;
    fb.cols = (f->width + 7) >> 3; fb.rows = (f->height + 7) >> 3;
    fb.sb_cols = (f->width + 63) >> 6; fb.sb_rows = (f->height + 63) >> 6;
    fb.ss_h = f->ss_h; fb.ss_v = f->ss_v; fb.coef_size = f->bpp > 8 ? 4 : 2;
    fb.pitch[0] = fb.sb_cols * 64; fb.pitch[1] = fb.sb_cols * 64 >> f->ss_h;
    fb.coef_base = 0;
    fb.phase = 0;
    memset(&fb.mc, 0, sizeof(fb.mc));
    fb.mc.cols = fb.cols; fb.mc.rows = fb.rows; fb.mc.ss_h = f->ss_h; fb.mc.ss_v = f->ss_v;
    s.rbucket.resize(1);
    std::vector<std::vector<uint32_t>> ps, ls;
    int r = build_frame(nullptr, s, fb, ps, ls);
    if (r < 0) return r;
    const int n = fb.sb_cols * fb.sb_rows;
    if (cap < n) return VP9HIP_EINVAL;
    for (int i = 0; i < n; i++) out[i] = 0;
    for (auto &v : ps)
        for (uint32_t sbi : v) {
            r = merge_mixed(s, sbi);
            if (r) return r;
        }
    for (const WGRec &wg : s.wgs) {
        const SBRec &sb = s.sbs[wg.sb[0]];
        double rows = 0;
        for (uint32_t k = 0; k < wg.npass; k++) {
            const uint32_t w = s.passes[wg.pass0 + k];
            rows += (w & 3) ? 32 : ((w >> 2) & 7) ? 16 : ((w >> 5) & 15) ? 8 : 4;
        }
        out[sb.sby * fb.sb_cols + sb.sbx] = rows;
    }
    return n;
}

extern "C" int vp9hip_plan_stats(const vp9h_frame *f, double *out, int cap)
{
    if (!f || !out || cap < 16) return VP9HIP_EINVAL;
    if (f->ss_h > 1 || f->ss_v > 1) return VP9HIP_EINVAL;
    init_nz();
    Staged s;
    FrameBuild fb;
    fb.f = f; fb.frame_idx = 0;
    fb.cols = (f->width + 7) >> 3; fb.rows = (f->height + 7) >> 3;
    fb.sb_cols = (f->width + 63) >> 6; fb.sb_rows = (f->height + 63) >> 6;
    fb.ss_h = f->ss_h; fb.ss_v = f->ss_v; fb.coef_size = f->bpp > 8 ? 4 : 2;
    fb.pitch[0] = fb.sb_cols * 64; fb.pitch[1] = fb.sb_cols * 64 >> f->ss_h;
    fb.coef_base = 0;
    fb.phase = 0;
    memset(&fb.mc, 0, sizeof(fb.mc));
    fb.mc.cols = fb.cols; fb.mc.rows = fb.rows; fb.mc.ss_h = f->ss_h; fb.mc.ss_v = f->ss_v;
    s.rbucket.resize(1);
    std::vector<std::vector<uint32_t>> ps, ls;
    int r = build_frame(nullptr, s, fb, ps, ls);
    if (r < 0) return r;
    // one k_pred workgroup per SB, mixed-size passes (as staged for the device)
    for (auto &v : ps)
        for (uint32_t sbi : v) {
            r = merge_mixed(s, sbi);
            if (r) return r;
        }
    for (int i = 0; i < std::min(cap, 23); i++) out[i] = 0;     // every value this writes, some summed
    out[0] = (double) s.sbs.size();
    out[1] = (double) s.passes.size();
    out[2] = (double) s.pjobs.size();
    size_t nr = 0;
    for (auto &bt : s.rbucket[0]) for (auto &bk : bt) nr += bk.size();
    out[3] = (double) nr;
    double lanes = 0;
    for (uint32_t w : s.passes) {
        const int c4 = (w >> 9) & 31, c8 = (w >> 5) & 15, c16 = (w >> 2) & 7, c32 = w & 3;
        out[4] += c4; out[5] += c8; out[6] += c16; out[7] += c32;      // jobs per tx size
        lanes += 4 * c4 + 8 * c8 + 16 * c16 + 32 * c32;
        out[15] += c32 ? 32 : c16 ? 16 : c8 ? 8 : 4;                     // pixel rows the pass loops over
    }
    out[8] = s.passes.empty() ? 0 : lanes / (64.0 * s.passes.size());
    for (auto &wg : s.wgs) out[9] = std::max(out[9], (double) wg.npass);
    out[10] = (double) s.lfs.size();
    out[11] = (double) s.mcs.size();
    out[12] = (double) ps.size();
    out[13] = (double) ls.size();
    for (auto &h : s.sbh) out[14] += h.nlev;                           // dependency levels (pass lower bound)
    if (cap > 17) {                     // passes of ASAP-level packing (jobs of a level, sizes descending)
        for (size_t sbi = 0; sbi < s.sbh.size(); sbi++) {
            const Staged::SBHost &h = s.sbh[sbi];
            const int N = (int) h.njobs;
            const PJob *jobs = s.sbjobs.data() + h.job0;
            const uint32_t *d0 = s.jdep0.data() + h.job0 + sbi;
            std::vector<int> lv(N, 0), lanes;
            for (int k = 0; k < N; k++) {
                for (uint32_t e = d0[k]; e < d0[k + 1]; e++) lv[k] = std::max(lv[k], lv[s.jdeps[e]] + 1);
                if ((int) lanes.size() <= lv[k]) lanes.resize(lv[k] + 1, 0);
                lanes[lv[k]] += 4 << PJ_TS(jobs[k]);
            }
            for (int l : lanes) out[17] += (l + 63) / 64;
        }
    }
    if (cap > 18) {                     // passes of first-fit packing in decode order: each job
                                        // into the first pass after its producers' with room
        for (size_t sbi = 0; sbi < s.sbh.size(); sbi++) {
            const Staged::SBHost &h = s.sbh[sbi];
            const int N = (int) h.njobs;
            const PJob *jobs = s.sbjobs.data() + h.job0;
            const uint32_t *d0 = s.jdep0.data() + h.job0 + sbi;
            std::vector<int> ps(N, 0), room, hg(N, 1), order(N);
            for (int k = N - 1; k >= 0; k--)                      // heights (producers precede consumers)
                for (uint32_t q = d0[k]; q < d0[k + 1]; q++) hg[s.jdeps[q]] = std::max(hg[s.jdeps[q]], hg[k] + 1);
            for (int k = 0; k < N; k++) order[k] = k;
            if (cap > 19) std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return hg[a] > hg[b]; });
            for (int kk = 0; kk < N; kk++) {
                const int k = order[kk];
                int e = 0;
                for (uint32_t q = d0[k]; q < d0[k + 1]; q++) e = std::max(e, ps[s.jdeps[q]] + 1);
                const int sz = 4 << PJ_TS(jobs[k]);
                while ((int) room.size() <= e) room.push_back(64);
                while (room[e] < sz) { e++; if ((int) room.size() <= e) room.push_back(64); }
                room[e] -= sz;
                ps[k] = e;
            }
            out[cap > 19 ? 19 : 18] += (double) room.size();
        }
    }
    if (cap > 16) {                     // intra steps of the level schedule (inter frames)
        Staged s2;
        FrameBuild fb2 = fb;
        fb2.levels = true;
        s2.rbucket.resize(1);
        std::vector<std::vector<uint32_t>> ps2, ls2;
        r = build_frame(nullptr, s2, fb2, ps2, ls2);
        if (r < 0) return r;
        out[16] = (double) ps2.size();
    }
    if (cap > 22) {                     // MC bytes of the frame's units: [20] predicted pixels,
                                        // [21] x (1 + references) (the roofline's algorithmic
                                        // bytes), [22] the 128-byte lines k_mcq's window rows
                                        // touch (columns x - 3 .. x + w + 4, rows y - 3 .. y + h + 3
                                        // when the vertical phase is fractional), each unit alone
        const int bypp = f->bpp > 8 ? 2 : 1;
        for (const McUnit &m : s.mcs) {
            const double ob = (double) m.w * m.h * bypp;
            out[20] += ob;
            out[21] += ob * (1 + m.nref);
            const int pw = m.plane ? ((f->width + f->ss_h) >> f->ss_h) : f->width;
            for (int k = 0; k < m.nref && k < 2; k++) {
                const McRef &r = m.r[k];
                const int rows = r.my || r.dy != 16 ? m.h + 7 : m.h;
                const int x0 = std::max(0, std::min(pw - 1, r.ix - 3));
                const int x1 = std::max(x0 + 1, std::min(pw, r.ix + m.w + 5));
                const int lines = (x1 * bypp - 1) / 128 - (x0 * bypp) / 128 + 1;
                out[22] += (double) rows * lines * 128;
            }
        }
    }
    return 0;
}
