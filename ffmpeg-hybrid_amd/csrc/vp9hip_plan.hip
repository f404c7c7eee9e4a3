// Device planner (gfx950): the per-frame work planning of the pixel path, from the pass-1
// packets resident in HBM to the records the pixel kernels consume (vp9hip_work.h). It
// replaces, on the GPU, the host planner of vp9hip_runtime.cpp and applies the same rules
// (vp9hip_planlogic.h), so a batch needs nothing from the host between its packets and its
// frames except the launch list, which depends on the record counts only.
//
//   k_pblk   one thread per block: the SB slot of each block, the slots' block ranges,
//            decode-order validation, eob entries per block
//   (scan)   eob entries -> each block's first eob
//   k_psb    one wave per SB: per-tx eobs -> coefficient total, residual-job counts per
//            (tcode, txtp), MC-unit count, the intra 4x4-unit map
//   (scan)   coefficients (decode order) -> each SB's first coefficient; counts -> record offsets
//   k_pjob   one wave per SB: the tx blocks in decode order, eobs, coefficient offsets,
//            residual jobs, intra job words with check_intra_mode resolved (vp9recon.c:37-221)
//   k_plan   one wave per SB: the intra jobs' producers, heights, list-scheduled passes (the
//            host's merge_mixed, restated wave-parallel), the SB's intra step
//   k_pllf   one wave per SB: the LF program (vp9block.c:1142-1262, vp9lpf.c:31-230)
//   k_plmc   one wave per SB of inter frames: MC units (vp9_mc_template.c:30-464)
//   k_plevel one workgroup per level-scheduled inter frame: SB dependency levels along
//            anti-diagonals
//   k_pkeys  step-list offsets; the launch summary the host reads back
//   k_plists the intra step lists
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include "vp9hip_plan.h"

#define DEV __device__ __forceinline__

namespace {

// Wave-wide scans and reductions on DPP (row shifts within 16-lane rows, then the gfx9
// row broadcasts of lanes 15 / 31): VALU-latency steps instead of ds_bpermute round trips.
// Every value of a uniform lane index is read with readlane.
enum { OP_ADD, OP_OR, OP_MAX };
template <int OP> DEV uint32_t dpp_op(uint32_t a, uint32_t b) { return OP == OP_OR ? (a | b) : OP == OP_MAX ? (a > b ? a : b) : (a + b); }
template <int OP> DEV uint32_t wscan_dpp(uint32_t v)
{
    v = dpp_op<OP>(v, (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x111, 0xf, 0xf, true));   // row_shr:1
    v = dpp_op<OP>(v, (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x112, 0xf, 0xf, true));   // row_shr:2
    v = dpp_op<OP>(v, (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x114, 0xf, 0xf, true));   // row_shr:4
    v = dpp_op<OP>(v, (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x118, 0xf, 0xf, true));   // row_shr:8
    v = dpp_op<OP>(v, (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x142, 0xa, 0xf, false));  // row_bcast:15
    v = dpp_op<OP>(v, (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x143, 0xc, 0xf, false));  // row_bcast:31
    return v;
}
DEV uint32_t wscan_incl(uint32_t v, int) { return wscan_dpp<OP_ADD>(v); }
DEV uint32_t rdl(uint32_t v, int l) { return (uint32_t) __builtin_amdgcn_readlane((int) v, l); }
DEV int rdl(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
DEV uint32_t wsum(uint32_t v) { return rdl(wscan_dpp<OP_ADD>(v), 63); }
DEV uint32_t mbcnt(uint64_t m)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t) (m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t) m, 0));
}
// Bounds guard of every planner write: false (and a status bit) when i >= cap.
DEV bool inb(const PlanDev &D, uint32_t i, uint32_t cap, uint32_t bit)
{
    if (i < cap) return true;
    atomicOr(&D.status[1], bit);
    atomicOr(&D.status[0], PLS_BOUNDS);
    return false;
}
// A frame's packet is inconsistent: its status bits, for the batch and for the frame.
DEV void plan_fail(const PlanDev &D, const PlanFrame &F, uint32_t st)
{
    atomicOr(D.status, st);
    if ((uint32_t) F.frame < D.nframes) atomicOr(&D.fbad[F.frame], st);
}
// The planner's workgroups are one wave: the LDS unit executes a wave's DS instructions in
// order, so a wave-scope fence (compiler ordering) replaces the workgroup barrier.
DEV void wsync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// A block as the planner uses it: fields out of range are clamped (the batch fails with
// PLS_BLOCK / PLS_MODE from k_pblk / k_psb, and every later index stays in bounds).
DEV vp9h_block load_block(const vp9h_block *g)
{
    vp9h_block b = *g;
    if (b.bs >= VP9H_N_BS) b.bs = VP9H_BS_4x4;
    if (b.tx > 3) b.tx = 0;
    if (b.uvtx > 3) b.uvtx = 0;
    return b;
}
// The block fields k_plan's tx enumeration reads (16 bytes in LDS instead of 52).
struct PBlk {
    uint16_t row, col;
    uint8_t bs, tx, uvtx, skip, intra, uvmode;
    uint8_t mode[4];
    uint8_t pad[2];
};
DEV PBlk pblk(const vp9h_block &b)
{
    PBlk r;
    r.row = b.row; r.col = b.col; r.bs = b.bs; r.tx = b.tx; r.uvtx = b.uvtx; r.skip = b.skip; r.intra = b.intra;
    r.uvmode = b.uvmode;
    for (int i = 0; i < 4; i++) r.mode[i] = b.mode[i];
    r.pad[0] = r.pad[1] = 0;
    return r;
}
DEV bool block_ok(const vp9h_block &b)
{
    return b.bs < VP9H_N_BS && b.tx <= 3 && b.uvtx <= 3;
}

// Per (block, plane) tx-block counts, packed all | eob << 10 | intra jobs << 20, and their
// exclusive scan over the SB's blocks in decode order (pre[3 * nb] = totals).
template <int SSH, int SSV, class B>
DEV uint32_t sb_prefix(const B *blk, int nb, int cols, int rows, bool mine, uint32_t *pre, int lane)
{
    uint32_t v[3] = { 0, 0, 0 };
    if (lane < nb) {
        const B &b = blk[lane];
        for (int p = 0; p < 3; p++) {
            const PlTxGrid g = pl_txgrid(b, p, cols, rows, SSH, SSV);
            const uint32_t n = (uint32_t) (g.nx * g.ny);
            v[p] = n | (b.skip ? 0u : n) << 10 | (b.intra && mine ? n : 0u) << 20;
        }
    }
    const uint32_t sum = v[0] + v[1] + v[2];
    const uint32_t incl = wscan_incl(sum, lane), excl = incl - sum;
    if (lane < nb) {
        pre[3 * lane] = excl;
        pre[3 * lane + 1] = excl + v[0];
        pre[3 * lane + 2] = excl + v[0] + v[1];
    }
    const uint32_t tot = rdl(incl, 63);
    if (lane == 0) pre[3 * nb] = tot;
    wsync();
    return tot;
}

// (block, plane) entry of tx t: the largest k with all-prefix(k) <= t
DEV int sb_locate(const uint32_t *pre, int n3, uint32_t t)
{
    int lo = 0, hi = n3 - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if ((pre[mid] & 1023) <= t) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

struct Tx {
    int b, p, k;            // block, plane, (block, plane) entry
    int l, x, y;            // index in the plane's tx grid, position (4x4 units in the block)
    PlTxGrid g;
};
// q = l / n for l < 4096, 1 <= n <= 16: the multiply by ceil(2^16 / n) is exact there
DEV int udiv16(int l, int n)
{
    return (int) (((uint32_t) l * ((65536u + (uint32_t) n - 1) / (uint32_t) n)) >> 16);
}
template <int SSH, int SSV, class B>
DEV Tx sb_tx_at(const B *blk, const uint32_t *pre, int k, uint32_t t, int cols, int rows)
{
    Tx r;
    r.k = k;
    r.b = (k * 171) >> 9;                    // k / 3 for k < 192
    r.p = r.k - 3 * r.b;
    r.l = (int) (t - (pre[r.k] & 1023));
    r.g = pl_txgrid(blk[r.b], r.p, cols, rows, SSH, SSV);
    const int nx = r.g.nx > 0 ? r.g.nx : 1;
    const int q = udiv16(r.l, nx);
    r.x = (r.l - q * nx) << r.g.txs;
    r.y = q << r.g.txs;
    return r;
}
template <int SSH, int SSV>
DEV Tx sb_tx(const vp9h_block *blk, const uint32_t *pre, int nb, uint32_t t, int cols, int rows)
{
    return sb_tx_at<SSH, SSV>(blk, pre, sb_locate(pre, 3 * nb, t), t, cols, rows);
}

// The eob of tx t (0 for skipped blocks), range-checked against the packet. (A frame whose
// eob count disagrees with its packet shifts the later frames' eobs: k_pkeys' totals check
// rejects the batch then, PLS_TOTAL.)
template <class B> DEV int tx_eob(const PlanDev &D, const B &b, const Tx &tx, const uint32_t *pre, uint32_t b0, uint32_t &st)
{
    if (b.skip) return 0;
    const uint32_t i = D.blk_eob0[b0 + tx.b] + ((pre[tx.k] & 1023) - (pre[3 * tx.b] & 1023)) + (uint32_t) tx.l;
    if (i >= D.total_eobs) { st |= PLS_EOB; return 0; }
    const int e = D.eobs[i];
    if (e > (16 << (2 * tx.g.txs))) { st |= PLS_EOB; return 0; }
    return e;
}

template <class B> DEV int tx_mode(const B &b, const Tx &tx, uint32_t &st)
{
    const int m = tx.p ? b.uvmode : b.mode[b.bs > VP9H_BS_8x8 && b.tx == 0 ? tx.y * 2 + tx.x : 0];
    if (m > 9) { st |= PLS_MODE; return 0; }
    return m;
}

DEV bool mc_refs_ok(const vp9h_block &b, const PlMcGeo &g)
{
    if (b.ref[0] > 2 || (b.comp && b.ref[1] > 2)) return false;
    const int r1 = b.comp ? b.ref[1] : b.ref[0];
    return g.scale[b.ref[0]][0] != 0xFFFF && g.scale[r1][0] != 0xFFFF;
}

DEV uint32_t cnt_idx(const PlanDev &D, const PlanFrame &F, uint32_t seg, uint32_t slot, int tc, int tp)
{
    return D.seg_pre4[seg] + (uint32_t) tc * F.s4 + (uint32_t) tp * D.seg_sz[seg] + D.slot_pos[slot];
}

struct SbGeo {
    int sbx, sby, tile_sb0, mine;
    uint32_t slot, seg, dord;
};
DEV SbGeo sb_geo(const PlanFrame &F, int s)
{
    SbGeo G;
    G.sbx = s % F.sb_cols;
    G.sby = s / F.sb_cols;
    const int tile = pl_tile_of(G.sbx, F.sb_cols, F.log2_tc, &G.tile_sb0);
    G.mine = tile >= F.tile_lo && tile < F.tile_hi;
    G.slot = F.slot0 + (uint32_t) s;
    G.seg = F.seg0 + (F.by_diag ? (uint32_t) ((G.sbx - G.tile_sb0) + G.sby) : 0u);
    G.dord = F.slot0 + (uint32_t) pl_sb_dorder(G.sbx, G.sby, F.sb_cols);
    return G;
}

// The SB's block range; 0 blocks if it has none (the batch is already marked invalid).
DEV int sb_blocks(const PlanDev &D, uint32_t slot, uint32_t &b0, uint32_t &st)
{
    b0 = D.sb_first[slot];
    const uint32_t b1 = D.sb_end[slot];
    if (b0 == 0xffffffffu || b1 == 0xffffffffu || b1 <= b0 || b1 > D.total_blocks) { st |= PLS_ORDER; b0 = 0; return 0; }
    if (b1 - b0 > 64) { st |= PLS_ORDER; return 64; }
    return (int) (b1 - b0);
}

// ------------------------------------------------------------------ k_pblk
__global__ __launch_bounds__(256) void k_pblk(PlanDev D)
{
    const PlanFrame &F = D.frames[blockIdx.y];
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= F.nblk) return;
    const uint32_t gi = F.blk0 + i;
    const int cols = F.mc.cols, rows = F.mc.rows;
    auto sb_of = [&](const vp9h_block &b, int &dord) {
        const int sbx = pl_min(b.col, cols - 1) >> 3, sby = pl_min(b.row, rows - 1) >> 3;
        dord = pl_sb_dorder(sbx, sby, F.sb_cols);
        return F.slot0 + (uint32_t) (sby * F.sb_cols + sbx);
    };
    const vp9h_block raw = D.blocks[gi];
    uint32_t st = 0;
    if (!block_ok(raw) || raw.row >= rows || raw.col >= cols) st |= PLS_BLOCK;
    const vp9h_block b = load_block(&D.blocks[gi]);
    int d, dp = -1, dn = -1;
    const uint32_t slot = sb_of(b, d);
    uint32_t sp = 0xffffffffu, sn = 0xffffffffu;
    if (i > 0) sp = sb_of(load_block(&D.blocks[gi - 1]), dp);
    if (i + 1 < F.nblk) sn = sb_of(load_block(&D.blocks[gi + 1]), dn);
    if (!inb(D, slot, D.nslots, 1u)) return;
    if (sp != slot) {
        D.sb_first[slot] = gi;
        if (i > 0 && dp >= d) st |= PLS_ORDER;       // SBs in decode order, each one contiguous
    }
    if (sn != slot) D.sb_end[slot] = gi + 1;
    uint32_t n = 0;
    if (!b.skip)
        for (int p = 0; p < 3; p++) {
            const PlTxGrid g = pl_txgrid(b, p, cols, rows, F.mc.ss_h, F.mc.ss_v);
            n += (uint32_t) (g.nx * g.ny);
        }
    D.blk_neob[gi] = n;
    if (st) plan_fail(D, F, st);
}

// ------------------------------------------------------------------ k_psb
// Residual-job counts: lane k holds key k's count, one ballot per distinct key of a chunk.
// Intra unit map: ORed into IBC copies of the 24 map words (copy = lane & 3), so at most a
// quarter of a chunk's lanes share an address. Round 4's per-lane map columns (6.2 KB of
// LDS) removed the conflicts but cut occupancy from 32 to 15 waves per CU and made the
// kernel 1.58x slower; the blocks are held as 16-byte PBlk for the same reason (LDS 2.2 KB
// per workgroup: the 32-waves/CU cap binds, not LDS).
#define IBC 4
template <int SSH, int SSV>
__global__ __launch_bounds__(64) void k_psb(PlanDev D)
{
    constexpr int CW = 16 >> SSH, CH = 16 >> SSV, JCAP = 256 + 2 * CW * CH;
    __shared__ PBlk blk[64];
    __shared__ uint32_t pre[3 * 64 + 1];
    __shared__ uint32_t ibw[24 * IBC];
    const PlanFrame &F = D.frames[blockIdx.y];
    const int s = blockIdx.x, lane = threadIdx.x;
    if (s >= F.sb_cols * F.sb_rows) return;
    const SbGeo G = sb_geo(F, s);
    const int cols = F.mc.cols, rows = F.mc.rows;
    uint32_t st = 0, b0;
    const int nb = sb_blocks(D, G.slot, b0, st);
    if (lane < 24 * IBC / 2) { ibw[2 * lane] = 0; ibw[2 * lane + 1] = 0; }
    vp9h_block own;
    if (lane < nb) {
        own = load_block(&D.blocks[b0 + lane]);
        blk[lane] = pblk(own);
    }
    wsync();
    const uint32_t tot = sb_prefix<SSH, SSV>(blk, nb, cols, rows, G.mine, pre, lane);
    const uint32_t T = pl_min((int) (tot & 1023), JCAP);
    uint32_t ncoef = 0, kcnt = 0;
    for (uint32_t t0 = 0; t0 < T; t0 += 64) {
        const uint32_t t = t0 + (uint32_t) lane;
        int key = -1;
        if (t < T) {
            const Tx tx = sb_tx_at<SSH, SSV>(blk, pre, sb_locate(pre, 3 * nb, t), t, cols, rows);
            const PBlk &b = blk[tx.b];
            const int e = tx_eob(D, b, tx, pre, b0, st);
            ncoef += (uint32_t) e;
            int txtp = 0;
            if (b.intra) {
                const int mode = tx_mode(b, tx, st);
                txtp = tx.p || tx.g.txs == 3 ? 0 : pl_intra_txfm_type(mode);
            }
            if (e && G.mine) key = (F.lossless ? 4 : tx.g.txs) * 4 + txtp;
            if (b.intra && G.mine) {            // the job's 4x4 units in the SB plane's unit map
                const int sh = tx.p ? SSH : 0, sv = tx.p ? SSV : 0;
                const int units = 16 >> sh, unitsv = 16 >> sv;
                const int ux0 = ((tx.g.bx - G.sbx * (64 >> sh)) >> 2) + tx.x, uy0 = ((tx.g.by - G.sby * (64 >> sv)) >> 2) + tx.y;
                uint32_t m = 0;
                for (int u = ux0; u < ux0 + tx.g.step && u < units; u++) m |= 1u << u;
                for (int v = uy0; v < uy0 + tx.g.step && v < unitsv; v++)
                    atomicOr(&ibw[(tx.p * 8 + (v >> 1)) * IBC + (lane & (IBC - 1))], m << ((v & 1) * 16));
            }
        }
        uint64_t pend = __ballot(key >= 0);
        while (pend) {
            const int kk = rdl(key, __builtin_ctzll(pend));
            const uint64_t m = __ballot(key == kk);
            if (lane == kk) kcnt += (uint32_t) __popcll(m);
            pend &= ~m;
        }
    }
    // MC units of the SB's inter blocks
    uint32_t nmc = 0;
    if (lane < nb && G.mine && !own.intra) {
        if (mc_refs_ok(own, F.mc)) nmc = (uint32_t) pl_mc_block(own, F.mc, 0, [](const McUnit &) {});
        else st |= PLS_REF;
    }
    nmc = wsum(nmc);
    ncoef = wsum(ncoef);
    wsync();
    uint32_t ib = 0;
    if (lane < 24)
#pragma unroll
        for (int j = 0; j < IBC; j++) ib |= ibw[lane * IBC + j];
    if (lane < 20) {
        const uint32_t ci = cnt_idx(D, F, G.seg, G.slot, lane >> 2, lane & 3);
        if (inb(D, ci, D.cap_cnt, 2u)) D.cnt[ci] = kcnt;
    }
    if (lane == 20) {
        const uint32_t ci = D.seg_pre1[G.seg] + D.slot_pos[G.slot];
        if (inb(D, ci, D.cap_cntm, 2u)) D.cntm[ci] = nmc;
    }
    if (lane < 24 && inb(D, G.slot, D.nslots, 4u)) D.ibits[(size_t) G.slot * 24 + lane] = ib;
    if (lane == 0 && inb(D, G.dord, D.nslots, 8u)) D.sb_ncoef[G.dord] = ncoef;
    if (st) plan_fail(D, F, st);
}

// ------------------------------------------------------------------ k_plan
// k_pjob's LDS: the SB's blocks and its tx enumeration.
template <int JCAP> struct PJobLds {
    PBlk blk[64];
    uint32_t pre[3 * 64 + 1];
    uint16_t et[JCAP];            // eob per tx (decode order)
    uint16_t co[JCAP];            // SB-relative first coefficient per tx; first the raw eobs
    uint16_t ost[JCAP];           // (block, plane) entry starting at tx t, else 0
    uint8_t  own[JCAP];           // (block, plane) entry of tx t (max-scan of ost)
    uint32_t eb[64];              // first eob entry of each block
};
// k_plan's LDS: the unit map, then the heights, then the priority order with the pass of
// each job share one region, each dead before the next is written (7.2 KB at 4:2:0; with ord
// and sch after the heights 8.75 KB: 17 instead of 21 workgroups per CU)
template <int JCAP> struct alignas(16) PlanLds {   // 16: jmap rows are stored 16 bytes at a time
    uint32_t ja[JCAP];            // PJob word per intra job (decode order), bit 30: the 4x4
                                  // top-right lies inside the block (trx)
    union {
        uint16_t jmap[3][256];    // producing job of each 4x4 unit
        struct {
            union {
                uint32_t hgt[JCAP];           // longest path to a sink (list-scheduling priority)
                struct {
                    uint16_t ord[JCAP];       // jobs by (height desc, index asc)
                    uint16_t sch[JCAP];       // pass of each job (0xffff: not yet)
                } os;
            } h;
            uint16_t doff[JCAP + 1];      // producers of job j: dep[2 (doff & 2047) ..] (count doff >> 11)
            uint16_t dep[4 * JCAP];
            uint32_t hs[64];              // height histogram -> list starts
            uint16_t tk[16];              // jobs taken by the pass being built
        } b;
    } u;
};
static_assert(sizeof(uint16_t[3][256]) <= sizeof(uint32_t[256 + 2 * 64]), "the unit map fits the heights' region");
#define JA_TRX (1u << 30)
// unit-map entry: job | units to its right edge << 10 | units to its bottom edge << 13 (0..7
// each: a job is at most 8 units wide); 0xffff (job 1023 > JCAP) marks a unit no job covers
#define JM_ENT(j, r, b) ((uint32_t) (j) | (uint32_t) (r) << 10 | (uint32_t) (b) << 13)

// edges the job's (substituted) mode reads: 1 left, 2 top, 4 top-left, 8 top-right (pl_intra_job)
DEV uint32_t needs_of(uint32_t a)
{
    return (uint32_t) pl_field(0x21371a777a12ull, (int) ((a >> 8) & 15), 4);     /* pl_intra_job's needs by slot */
}
DEV uint32_t wor(uint32_t v) { return rdl(wscan_dpp<OP_OR>(v), 63); }

// VP9HIP_PLAN_PROF: shader-clock cycles of each k_plan phase, summed over the SBs
#define PPT(k) do { if (D.prof) { const unsigned long long t_ = clock64(); \
        if (lane == 0) atomicAdd(&D.prof[k], t_ - pt0); pt0 = t_; } } while (0)

// One wave per SB: the SB's tx blocks in decode order (the (block, plane) entry of each
// by a max-scan), their eobs and coefficient offsets, the residual jobs (every coded tx,
// bucketed by transform), and the intra jobs' words with check_intra_mode resolved, for
// k_plan. Small LDS (4.8 KB at 4:2:0): a kernel of its own so this per-tx work runs at full
// occupancy instead of with k_plan's scheduling state.
// ja: k_pjplan's LDS job words (the intra job words go there, not to D.jobw); returns the
// SB's intra job count for k_plan's part, -1 past the frame
template <int SSH, int SSV>
DEV int pjob_sb(const PlanDev &D, PJobLds<256 + 2 * (16 >> SSH) * (16 >> SSV)> &S, uint32_t *ja)
{
    constexpr int CW = 16 >> SSH, CH = 16 >> SSV, JCAP = 256 + 2 * CW * CH;
    const PlanFrame &F = D.frames[blockIdx.y];
    const int s = blockIdx.x, lane = threadIdx.x;
    if (s >= F.sb_cols * F.sb_rows) return -1;
    unsigned long long pt0 = D.prof ? clock64() : 0;
    const SbGeo G = sb_geo(F, s);
    const int cols = F.mc.cols, rows = F.mc.rows;
    const uint32_t slot = G.slot;
    uint32_t st = 0, b0;
    const int nb = sb_blocks(D, slot, b0, st);
    st = 0;                                   // reported by k_psb
    if (lane < nb) S.blk[lane] = pblk(load_block(&D.blocks[b0 + lane]));
    wsync();
    const uint32_t tot = sb_prefix<SSH, SSV>(S.blk, nb, cols, rows, G.mine, S.pre, lane);
    const int T = pl_min((int) (tot & 1023), JCAP), NJ = pl_min((int) (tot >> 20), JCAP);
    // the (block, plane) entry of every tx: each non-empty entry marks its first tx (ranges
    // are disjoint), a max-scan fills the rest (= sb_locate's largest k with pre[k] <= t)
    for (int t = lane; t < T; t += 64) S.ost[t] = 0;
    wsync();
    if (lane < nb)
        for (int p = 0; p < 3; p++) {
            const int k = 3 * lane + p;
            const uint32_t a0 = S.pre[k] & 1023, a1 = S.pre[k + 1] & 1023;
            if (a1 > a0 && a0 < (uint32_t) T) S.ost[a0] = (uint16_t) k;
        }
    wsync();
    {
        uint32_t carry = 0;
        for (int c = 0; c < T; c += 64) {
            const uint32_t v = c + lane < T ? S.ost[c + lane] : 0u;
            const uint32_t incl = dpp_op<OP_MAX>(wscan_dpp<OP_MAX>(v), carry);
            if (c + lane < T) S.own[c + lane] = (uint8_t) incl;
            carry = rdl(incl, 63);
        }
    }
    wsync();
    PPT(0);

    // ---- eobs and SB-relative coefficient offsets (decode order). The SB's eob entries are
    // contiguous in the packet (its coded blocks' tx in decode order): one coalesced load
    // into LDS, then each tx picks its entry (skipped blocks have none)
    {
        const uint32_t be = lane <= nb ? D.blk_eob0[b0 + (uint32_t) lane] : 0u;      // nb + 1 entries
        if (lane < nb) S.eb[lane] = be;
        const uint32_t E0 = rdl(be, 0), E1 = rdl(be, nb);
        uint32_t E = E1 - E0;
        if (E1 < E0 || E > (uint32_t) JCAP || E1 > D.total_eobs) { st |= PLS_EOB; E = 0; }
        for (uint32_t i = (uint32_t) lane; i < E; i += 64) S.co[i] = D.eobs[E0 + i];
        wsync();
        for (int t = lane; t < T; t += 64) {
            const int k = S.own[t], b = (k * 171) >> 9;
            const PBlk &bk = S.blk[b];
            int e = 0;
            if (!bk.skip) {
                const uint32_t i = S.eb[b] - E0 + (uint32_t) t - (S.pre[3 * b] & 1023);
                const int txs = (k - 3 * b) ? bk.uvtx : bk.tx;
                if (i < E) e = S.co[i];
                else st |= PLS_EOB;
                if (e > (16 << (2 * txs))) { st |= PLS_EOB; e = 0; }
            }
            S.et[t] = (uint16_t) e;
        }
    }
    wsync();
    {
        uint32_t carry = 0;
        for (int c = 0; c < T; c += 64) {
            const uint32_t v = c + lane < T ? S.et[c + lane] : 0u;
            const uint32_t incl = wscan_incl(v, lane);
            if (c + lane < T) S.co[c + lane] = (uint16_t) (carry + incl - v);
            carry += rdl(incl, 63);
        }
    }
    // record bases of the SB: lanes 0..19 residual keys (tcode * 4 + txtp), lane 20 MC units;
    // rl: the end of the key's range (k_psb's count), which no emitted job may pass
    uint32_t rb = 0, rl = 0;
    if (lane < 20) {
        const uint32_t ci = cnt_idx(D, F, G.seg, slot, lane >> 2, lane & 3);
        if (inb(D, ci, D.cap_cnt, 16u)) { rb = D.cnt0[ci]; rl = rb + D.cnt[ci]; }
    } else if (lane == 20) {
        const uint32_t ci = D.seg_pre1[G.seg] + D.slot_pos[slot];
        rb = inb(D, ci, D.cap_cntm, 16u) ? D.cntm0[ci] : 0u;
    }
    const uint32_t coef_sb = inb(D, G.dord, D.nslots, 32u) ? D.sb_coef0[G.dord] : 0u;
    const uint32_t rbase = slot * D.rcap;
    unsigned long long ibytes = 0;
    wsync();
    PPT(1);

    // ---- residual jobs (every coded tx block) and intra jobs with their unit map
    const int tx0l = G.tile_sb0 * 64;
    for (int c = 0; c < T; c += 64) {
        const int t = c + lane;
        int key = -1;
        RJob r;
        if (t < T) {
            const Tx tx = sb_tx_at<SSH, SSV>(S.blk, S.pre, S.own[t], (uint32_t) t, cols, rows);
            const PBlk &b = S.blk[tx.b];
            const int p = tx.p, sh = p ? SSH : 0, sv = p ? SSV : 0, txs = tx.g.txs;
            const int e0 = S.et[t];
            int mode = 0, txtp = 0;
            if (b.intra) {
                mode = tx_mode(b, tx, st);
                txtp = p || txs == 3 ? 0 : pl_intra_txfm_type(mode);
            }
            const int tcode = F.lossless ? 4 : txs;
            const int ux0 = ((tx.g.bx - G.sbx * (64 >> sh)) >> 2) + tx.x, uy0 = ((tx.g.by - G.sby * (64 >> sv)) >> 2) + tx.y;
            const uint32_t roff = rbase + pl_resid_unit(p, ux0, uy0, SSH, SSV);
            if (e0 && G.mine) {
                uint32_t coef = coef_sb + S.co[t];
                int e = e0;
                if (coef + (uint32_t) e > D.total_coefs) { st |= PLS_COEF; e = 0; coef = 0; }
                r.coef = coef;
                r.eob = (uint16_t) e;
                r.frame = (uint16_t) F.frame;
                r.ptx = (uint8_t) (p | tcode << 2 | (b.intra ? 0 : 1) << 5 | txtp << 6);
                r.nzc = D.nz[(((tcode * 4 + txtp) * 1025) + e) * 2];
                r.nzr = D.nz[(((tcode * 4 + txtp) * 1025) + e) * 2 + 1];
                r.pad = 0;
                if (b.intra) r.dst = roff;
                else {
                    r.dst = (uint32_t) ((size_t) (tx.g.by + tx.y * 4) * F.pitch[p ? 1 : 0] + tx.g.bx + tx.x * 4);
                    ibytes += (unsigned long long) (2 * (16 << (2 * txs)) * F.bypp);
                }
                key = tcode * 4 + txtp;
            }
            if (b.intra && G.mine) {
                const int j = (int) (S.pre[tx.k] >> 20) + tx.l;
                const int pw8 = p ? cols * 8 >> SSH : cols * 8, ph8 = p ? rows * 8 >> SSV : rows * 8;
                const PlIntra pi = pl_intra_job(p, txs, mode, e0, tx.g.bx + tx.x * 4, tx.g.by + tx.y * 4, tx.x, tx.g.pw4,
                                                p ? tx0l >> SSH : tx0l, pw8, ph8, ux0, uy0);
                if (j < JCAP) {
                    if (ja) ja[j] = pi.a | (pi.trx ? JA_TRX : 0u);
                    else D.jobw[(size_t) slot * JCAP + (uint32_t) j] = pi.a | (pi.trx ? JA_TRX : 0u);
                }
            }
        }
        // ranks within each key, in decode order: one ballot per distinct key of the chunk
        uint64_t pend = __ballot(key >= 0);
        uint32_t pos = 0, lim = 0;
        while (pend) {
            const int l0 = __builtin_ctzll(pend);
            const int kk = rdl(key, l0);
            const uint64_t m = __ballot(key == kk);
            const uint32_t base = rdl(rb, kk), end = rdl(rl, kk);
            if (key == kk) { pos = base + mbcnt(m); lim = end; }
            if (lane == kk) rb += (uint32_t) __popcll(m);
            pend &= ~m;
        }
        if (key >= 0 && pos >= lim) { st |= PLS_EOB; key = -1; }   // more jobs than k_psb counted
        if (key >= 0 && inb(D, pos, D.cap_rjobs, 64u)) D.rjobs[pos] = r;
    }
    for (int d = 32; d; d >>= 1) ibytes += __shfl_xor(ibytes, d);
    if (lane == 0) {
        if (!ja) D.sb_nj[slot] = (uint32_t) (G.mine ? NJ : 0);
        if (ibytes && inb(D, (uint32_t) F.frame, D.nframes, 2048u)) atomicAdd(&D.fbytes[2 * F.frame], ibytes);
    }
    st = wor(st);
    if (lane == 0 && st) plan_fail(D, F, st);
    PPT(2);
    return G.mine ? NJ : 0;
}
template <int SSH, int SSV>
__global__ __launch_bounds__(64) void k_pjob(PlanDev D)
{
    __shared__ PJobLds<256 + 2 * (16 >> SSH) * (16 >> SSV)> S;
    pjob_sb<SSH, SSV>(D, S, nullptr);
}

// One wave per SB: producers of every intra job, heights, priority order, list-scheduled
// passes (the host's merge_mixed), the PJob / pass records, the SB's records, its level
// dependencies and intra step. Jobs come from k_pjob (D.jobw); the unit map is rebuilt.
// (Two SBs per wave with the second's job words loaded under the first's scheduling cut the
// first load's share of a wave's cycles from 31 to 20 %, but not the kernel: 2,880 -> 2,926 us
// per C3 batch. The waves' time goes to dependent LDS chains at 6 waves per SIMD, LDS-bound.)
// nj >= 0 (k_pjplan): the SB's job words are in S.ja already, nj of them
template <int SSH, int SSV>
DEV void plan_sb(const PlanDev &D, PlanLds<256 + 2 * (16 >> SSH) * (16 >> SSV)> &S, int nj)
{
    constexpr int CW = 16 >> SSH, CH = 16 >> SSV, JCAP = 256 + 2 * CW * CH, NCH = JCAP / 64;
    const PlanFrame &F = D.frames[blockIdx.y];
    const int s = blockIdx.x, lane = threadIdx.x;
    if (s >= F.sb_cols * F.sb_rows) return;
    unsigned long long pt0 = D.prof ? clock64() : 0;
    const SbGeo G = sb_geo(F, s);
    const uint32_t slot = G.slot;
    const uint32_t rbase = slot * D.rcap;
    uint32_t st = 0;
    const int NJ = pl_min(nj >= 0 ? nj : (int) D.sb_nj[slot], JCAP);
    for (int i = lane; i < 3 * 256 / 8; i += 64) ((uint4 *) &S.u.jmap[0][0])[i] = make_uint4(~0u, ~0u, ~0u, ~0u);
    if (nj < 0)
        for (int j = lane; j < NJ; j += 64) S.ja[j] = D.jobw[(size_t) slot * JCAP + (uint32_t) j];
    wsync();
    PPT(8);
    // the unit map: each job's 4x4 units hold JM_ENT(job, units to the job's right edge, units
    // to its bottom edge), so the producer walk below steps past a producer's extent from the
    // entry alone (one LDS read per producer instead of the entry and the job's word)
    for (int j = lane; j < NJ; j += 64) {
        const uint32_t a = S.ja[j];
        const int p = a & 3, step = 1 << ((a >> 2) & 3), ux0 = (a >> 12) & 15, uy0 = (a >> 16) & 15;
        const int units = p ? CW : 16, unitsv = p ? CH : 16;
        if (ux0 + step <= units) {
            // a job is an aligned square inside its plane's 16-unit rows, so each of its unit
            // rows is one aligned 2 / 4 / 8 / 16-byte store: a 32x32 job paints 8 rows, not 64
            // units (the loop's trip count is the largest job's of the chunk)
            uint16_t *row = &S.u.jmap[p][uy0 * 16 + ux0];
            for (int v = 0; v < step && uy0 + v < unitsv; v++, row += 16) {
                const uint32_t b = JM_ENT(j, 0, step - 1 - v);
                // two units: right distances r and r - 1 (the lower address first)
                auto e2 = [&](uint32_t r) { return (b | r << 10) | (b | (r - 1) << 10) << 16; };
                if (step == 1) *row = (uint16_t) b;
                else if (step == 2) *(uint32_t *) row = e2(1);
                else if (step == 4) *(uint2 *) row = make_uint2(e2(3), e2(1));
                else *(uint4 *) row = make_uint4(e2(7), e2(5), e2(3), e2(1));
            }
        } else {
            for (int v = uy0; v < uy0 + step && v < unitsv; v++)
                for (int u = ux0; u < ux0 + step && u < units; u++)
                    S.u.jmap[p][v * 16 + u] = (uint16_t) JM_ENT(j, ux0 + step - 1 - u, uy0 + step - 1 - v);
        }
    }
    wsync();
    PPT(9);

    // ---- producers of every intra job (the pixels its substituted mode reads)
    // The units job j reads are pl_local_reads' runs: the top row (uy0 - 1, from ux0 - 1 with
    // the top-left unit to ux0 + n + trx) and the left column (ux0 - 1, rows uy0 .. uy0 + n - 1).
    // Jobs are aligned squares, so a run's units of one producer are consecutive: the walk
    // jumps from a producer's unit past that producer's extent (one step per distinct
    // producer instead of one per unit). Only the top-left unit's producer can recur in the
    // left run. Units no intra job covers (0xffff) are stepped over one by one.
    auto deps_of = [&](int j, auto fn) {
        const uint32_t a = S.ja[j];
        const int p = a & 3, ts = (a >> 2) & 3, ux0 = (a >> 12) & 15, uy0 = (a >> 16) & 15;
        const int units = p ? CW : 16, unitsv = p ? CH : 16, n4 = 1 << ts;
        const int nd = (int) needs_of(a), trx = (a & JA_TRX) ? 1 : 0;
        int tl = -1;                                       // producer of the top-left unit
        if (uy0 > 0) {
            const int u1 = pl_min((nd & 2) ? ux0 + n4 + trx : ux0, units);
            int u = (nd & 4) ? ux0 - 1 : ux0;
            if (u < 0) u = 0;
            const uint16_t *row = S.u.jmap[p] + (uy0 - 1) * 16;
            while (u < u1) {
                const uint32_t e = row[u];
                if (e == 0xffff) { u++; continue; }
                const int d = (int) (e & 1023);
                if (u == ux0 - 1) tl = d;
                if (d < j) fn(d);
                u += (int) ((e >> 10) & 7) + 1;               // past the producer's right edge
            }
        }
        if (ux0 > 0 && (nd & 1)) {
            const int v1 = pl_min(uy0 + n4, unitsv);
            int v = uy0;
            const uint16_t *col = S.u.jmap[p] + ux0 - 1;
            while (v < v1) {
                const uint32_t e = col[v * 16];
                if (e == 0xffff) { v++; continue; }
                const int d = (int) (e & 1023);
                if (d < j && d != tl) fn(d);
                v += (int) (e >> 13) + 1;                     // past the producer's bottom edge
            }
        }
    };
    {
        // one enumeration: job j's list starts at the prefix sum of the per-size bounds (an
        // n-unit job reads at most 2n + 2 units: its left column, and the top row with the
        // top-left and top-right units; 4 * JCAP for a tiling of 4x4 jobs): every bound is
        // even, so doff[j] holds the start / 2 in bits 0-10 and the length in bits 11-15
        uint32_t carry = 0;
        for (int c = 0; c < NJ; c += 64) {
            const int j = c + lane;
            const uint32_t cap = j < NJ ? 2u * (1u << ((S.ja[j] >> 2) & 3)) + 2u : 0u;
            const uint32_t incl = wscan_incl(cap, lane);
            const uint32_t off = carry + incl - cap;
            if (j < NJ) {
                uint32_t k = off;
                if (off + cap <= 4u * JCAP) deps_of(j, [&](int d) { if (k < off + cap) S.u.b.dep[k++] = (uint16_t) d; });
                else st |= PLS_SCHED;
                S.u.b.doff[j] = (uint16_t) (off >> 1 | (k - off) << 11);
            }
            carry += rdl(incl, 63);
        }
        wsync();                              // jmap is dead: hgt overlays it
        for (int j = lane; j < NJ; j += 64) S.u.b.h.hgt[j] = 1;
    }
    wsync();
    PPT(3);
    // ---- heights (longest path to a sink). Producers precede their consumers (d < j), so
    // the chunks of 64 jobs are finished last to first: a chunk's consumers in later chunks
    // are final, and the chunk relaxes until none of its own jobs rises (at most one round
    // per job of a chain inside it); its last round pushes final heights to every producer
    for (int c = ((NJ - 1) & ~63); c >= 0; c -= 64) {
        const int j = c + lane;
        const uint32_t dw = j < NJ ? S.u.b.doff[j] : 0u;
        const int k0 = (int) (dw & 2047) << 1, k1 = k0 + (int) (dw >> 11);
        for (int it = 0; it < 65; it++) {
            bool ch = false;                  // a job of this chunk rose
            if (j < NJ) {
                const uint32_t h1 = S.u.b.h.hgt[j] + 1;
                for (int k = k0; k < k1; k++) {
                    const int d = S.u.b.dep[k];
                    if (S.u.b.h.hgt[d] < h1) { atomicMax(&S.u.b.h.hgt[d], h1); ch |= d >= c; }
                }
            }
            wsync();
            if (!__any(ch)) break;
        }
    }
    PPT(4);
    // ---- priority order: height descending, then decode order. The heights go to registers
    // first: the order and the pass words overlay them (NCH = JCAP / 64 chunks)
    int hreg[NCH];
#pragma unroll
    for (int c = 0; c < NCH; c++) {
        const int j = c * 64 + lane;
        hreg[c] = j < NJ ? pl_min((int) S.u.b.h.hgt[j], 63) : -1;
    }
    S.u.b.hs[lane] = 0;
    wsync();
#pragma unroll
    for (int c = 0; c < NCH; c++)
        if (hreg[c] >= 0) atomicAdd(&S.u.b.hs[hreg[c]], 1u);
    wsync();
    {
        const uint32_t v = S.u.b.hs[63 - lane];                // heights from the top
        const uint32_t incl = wscan_incl(v, lane);
        wsync();
        S.u.b.hs[63 - lane] = incl - v;
        wsync();
#pragma unroll
        for (int c = 0; c < NCH; c++) {
            if (c * 64 >= NJ) break;
            const int j = c * 64 + lane;
            const int h = hreg[c];
            uint64_t pend = __ballot(h >= 0);
            while (pend) {
                const int hh = rdl(h, __builtin_ctzll(pend));
                const uint64_t m = __ballot(h == hh);
                const uint32_t base = S.u.b.hs[hh];
                if (h == hh) S.u.b.h.os.ord[base + mbcnt(m)] = (uint16_t) j;
                wsync();
                if (lane == 0) S.u.b.hs[hh] = base + (uint32_t) __popcll(m);
                wsync();
                pend &= ~m;
            }
        }
    }
    wsync();
    for (int j = lane; j < NJ; j += 64) S.u.b.h.os.sch[j] = 0xffff;
    wsync();
    PPT(5);
    // ---- list scheduling (merge_mixed): each pass takes, in priority order, every ready job
    // (all producers in earlier passes) that still fits in 64 lanes; lane groups by size
    uint32_t *gpass = D.passes + (size_t) slot * JCAP;
    PJob *gjob = D.pjobs + (size_t) slot * JCAP;
    int done = 0, npass = 0;
    // Each lane holds, per chunk c of the priority order, position c * 64 + lane: its job, size,
    // and the range of its producer list still to see (k: the first producer not known to be
    // scheduled in an earlier pass; producers scheduled in earlier passes stay so), and bit c
    // of `pend` while it is unscheduled. A pass then reads LDS only for the sch[] word of each
    // waiting job's current producer.
    uint32_t jreg[NCH], kreg[NCH], k1reg[NCH], szreg[NCH];
    uint32_t pend = 0;
#pragma unroll
    for (int c = 0; c < NCH; c++) {
        const int pos = c * 64 + lane;
        jreg[c] = kreg[c] = k1reg[c] = 0;
        szreg[c] = 0;
        if (pos < NJ) {
            const uint32_t j = S.u.b.h.os.ord[pos], dw = S.u.b.doff[j];
            jreg[c] = j;
            kreg[c] = (dw & 2047) << 1;
            k1reg[c] = kreg[c] + (dw >> 11);
            szreg[c] = 4u << ((S.ja[j] >> 2) & 3);
            pend |= 1u << c;
        }
    }
    if (D.dbg & 2) done = NJ;                 // ablation (timing only): no pass building
    while (done < NJ) {
        int budget = 64, ntake = 0;
#pragma unroll
        for (int c = 0; c < NCH; c++) {
            if (budget < 4) break;
            bool cand = (pend >> c) & 1u;
            if (!__any(cand)) continue;           // every job of this chunk is scheduled
            if (cand) {
                uint32_t k = kreg[c];
                const uint32_t k1 = k1reg[c];
                while (k < k1 && S.u.b.h.os.sch[S.u.b.dep[k]] < (uint16_t) npass) k++;
                kreg[c] = k;
                cand = k == k1;
            }
            if (!__any(cand)) continue;           // nothing ready in this chunk
            const uint32_t j = jreg[c], sz = szreg[c];
            // takes in priority order by lane-size prefix sums: round 1 takes the longest
            // prefix of the chunk's ready jobs that fits, later rounds refill the remaining
            // lanes from the jobs skipped (any packing that respects the producers is exact;
            // only the pass count depends on it)
            for (int round = 0; round < 3 && budget >= 4; round++) {
                if (round && !__any(cand)) break;     // round 1 took every ready job
                const uint32_t incl = wscan_incl(cand ? sz : 0u, lane);
                const bool take = cand && incl <= (uint32_t) budget;
                const uint64_t m = __ballot(take);
                if (!m) break;
                if (take) {
                    cand = false;
                    pend &= ~(1u << c);
                    S.u.b.h.os.sch[j] = (uint16_t) npass;
                    S.u.b.tk[ntake + (int) mbcnt(m)] = (uint16_t) j;
                }
                ntake += __popcll(m);
                budget -= (int) rdl(incl, 63 - __builtin_clzll(m));
            }
        }
        wsync();
        if (ntake == 0) { st |= PLS_SCHED; break; }
        // emit: sizes 32, 16, 8, 4, take order within a size
        const int J = lane < ntake ? S.u.b.tk[lane] : 0;
        const int ts = lane < ntake ? (int) ((S.ja[J] >> 2) & 3) : -1;
        uint32_t cnt[4], at = 0;
        int mypos = 0;
        for (int q = 3; q >= 0; q--) {
            const uint64_t m = __ballot(ts == q);
            cnt[q] = (uint32_t) __popcll(m);
            if (ts == q) mypos = (int) (at + mbcnt(m));
            at += cnt[q];
        }
        if (lane < ntake) {
            const uint32_t a = S.ja[J];
            PJob pj;
            pj.a = a & ~JA_TRX;
            pj.roff = ((a >> 4) & 1) ? rbase + pl_resid_unit(a & 3, (a >> 12) & 15, (a >> 16) & 15, SSH, SSV) : 0u;
            if (inb(D, (uint32_t) (done + mypos), JCAP, 128u)) gjob[done + mypos] = pj;
        }
        if (lane == 0 && inb(D, (uint32_t) npass, JCAP, 256u)) gpass[npass] = (uint32_t) done << 14 | cnt[0] << 9 | cnt[1] << 5 | cnt[2] << 2 | cnt[3];
        done += ntake;
        npass++;
        wsync();
    }
    if (lane == 0) {
        SBRec sr;
        sr.frame = (uint32_t) F.frame; sr.sbx = (uint16_t) G.sbx; sr.sby = (uint16_t) G.sby;
        sr.tile_x0 = (uint16_t) (G.tile_sb0 << 3);
        sr.flags = F.intra ? 0 : 1;
        D.sbs[slot] = sr;
        WGRec w;
        w.job0 = slot * JCAP; w.pass0 = slot * JCAP;
        w.njobs = (uint16_t) done; w.npass = (uint16_t) npass;
        w.sb[0] = slot;
        D.wgs[slot] = w;
    }
    PPT(6);

    // ---- cross-SB reads of level-scheduled inter frames: left / top / top-left SBs whose
    // intra units this SB's jobs read (the host's umap levels)
    uint32_t dmask = 0;
    if (F.levels && !F.intra)
        for (int j = lane; j < NJ; j += 64) {
            const uint32_t a = S.ja[j];
            const int p = a & 3, ts = (a >> 2) & 3, ux0 = (a >> 12) & 15, uy0 = (a >> 16) & 15;
            const int units = p ? CW : 16, unitsv = p ? CH : 16;
            const int fx = G.sbx * units + ux0, fy = G.sby * unitsv + uy0;
            pl_cross_reads(ux0, uy0, fx, fy, 1 << ts, (int) needs_of(a), (a & JA_TRX) ? 1 : 0, [&](int ux, int uy) {
                if (ux < 0 || uy < 0 || ux >= F.sb_cols * units) return;
                const int nx = ux / units, ny = uy / unitsv, u = ux - nx * units, v = uy - ny * unitsv;
                const uint32_t ns = F.slot0 + (uint32_t) (ny * F.sb_cols + nx);
                if (!((D.ibits[(size_t) ns * 24 + p * 8 + (v >> 1)] >> ((v & 1) * 16 + u)) & 1)) return;
                dmask |= nx < G.sbx ? (ny < G.sby ? 8u : 2u) : 4u;      // TL, L, T
            });
        }
    dmask = wor(dmask);
    PPT(7);


    // ---- the SB's intra step (diagonal phases; level phases in k_plevel) and batch totals
    if (lane == 0) {
        const uint32_t has = done > 0;
        D.sb_info[slot] = has | dmask;
        if (D.static_lists) {
            if (!has && G.mine) st |= PLS_SCHED;          // the staged step list holds every SB
            D.sb_kpos[slot] = (uint32_t) npass;           // k_psort's key (no step keys here)
        } else if (has && !(F.levels && !F.intra)) {
            const uint32_t key = F.key0 + (uint32_t) ((G.sbx - G.tile_sb0) + G.sby);
            D.sb_key[slot] = key;
            D.sb_kpos[slot] = inb(D, key, D.nkeys, 1024u) ? atomicAdd(&D.key_cnt[key], 1u) : 0u;
        }
    }
    st = wor(st);
    if (lane == 0 && st) plan_fail(D, F, st);
    PPT(10);
}
template <int SSH, int SSV>
__global__ __launch_bounds__(64) void k_plan(PlanDev D)
{
    __shared__ PlanLds<256 + 2 * (16 >> SSH) * (16 >> SSV)> S;
    plan_sb<SSH, SSV>(D, S, -1);
}
// k_pjob and k_plan of one SB in one wave: the intra job words stay in LDS (no D.jobw round
// trip through HBM, one wave start instead of two). k_pjob's LDS overlays k_plan's unit
// map / schedule region, which k_plan writes only after the job words are in place, so the
// fused wave keeps k_plan's 7.2 KB (4:2:0). VP9HIP_PLAN_DBG bit 3: the two kernels.
template <int SSH, int SSV>
__global__ __launch_bounds__(64) void k_pjplan(PlanDev D)
{
    constexpr int JCAP = 256 + 2 * (16 >> SSH) * (16 >> SSV);
    typedef PlanLds<JCAP> PL;
    __shared__ union alignas(16) {
        PL pl;
        struct { uint32_t ja[JCAP]; PJobLds<JCAP> pj; } pjx;   // pj over pl.u
    } U;
    static_assert(offsetof(PL, u) == sizeof(uint32_t) * JCAP, "k_pjob's LDS overlays k_plan's union, not its job words");
    const int nj = pjob_sb<SSH, SSV>(D, U.pjx.pj, U.pl.ja);
    if (nj < 0) return;
    wsync();
    plan_sb<SSH, SSV>(D, U.pl, nj);
}

// ------------------------------------------------------------------ k_plmc
// MC units of the SB's inter blocks in decode order (vp9_mc_template.c:30-464), one wave per
// SB of the batch's inter frames. A kernel of its own: the unit emission is large code that
// keyframe batches never run, and it needs none of k_plan's LDS.
template <int SSH, int SSV>
__global__ __launch_bounds__(64) void k_plmc(PlanDev D)
{
    const PlanFrame &F = D.frames[blockIdx.y];
    const int s = blockIdx.x, lane = threadIdx.x;
    if (F.intra || s >= F.sb_cols * F.sb_rows) return;
    const SbGeo G = sb_geo(F, s);
    uint32_t st = 0, b0;
    const int nb = sb_blocks(D, G.slot, b0, st);
    const uint32_t ci = D.seg_pre1[G.seg] + D.slot_pos[G.slot];
    const uint32_t base = inb(D, ci, D.cap_cntm, 16u) ? D.cntm0[ci] : 0u;
    vp9h_block b;
    bool mc = false;
    if (lane < nb) {
        b = load_block(&D.blocks[b0 + lane]);
        mc = G.mine && !b.intra && mc_refs_ok(b, F.mc);
    }
    const uint32_t n = mc ? (uint32_t) pl_mc_block(b, F.mc, 0, [](const McUnit &) {}) : 0u;
    const uint32_t incl = wscan_incl(n, lane);
    uint32_t o = base + incl - n;
    unsigned long long mbytes = 0;
    if (mc)
        pl_mc_block(b, F.mc, (uint32_t) F.frame, [&](const McUnit &m) {
            if (inb(D, o, D.cap_mcs, 512u)) D.mcs[o] = m;
            o++;
            mbytes += (unsigned long long) m.w * m.h * F.bypp * (1 + m.nref);
        });
    for (int d = 32; d; d >>= 1) mbytes += __shfl_xor(mbytes, d);
    if (lane == 0 && mbytes && inb(D, (uint32_t) F.frame, D.nframes, 2048u)) atomicAdd(&D.fbytes[2 * F.frame + 1], mbytes);
}

// ------------------------------------------------------------------ k_pllf
// The SB's loop-filter levels, masks and program (vp9block.c:1438-1452 via mask_edges,
// vp9lpf.c:31-230 via pl_lf_item): one wave per SB, 0.7 KB of LDS.
template <int SSH, int SSV>
__global__ __launch_bounds__(64) void k_pllf(PlanDev D)
{
    __shared__ uint32_t lfm[2][2][8];        // LF masks [cls][dir][row]: kinds 0..3 in bytes
    __shared__ uint8_t lfl[64];              // LF level of each 8x8
    __shared__ uint32_t prog[LF_PROG_BYTES / 4];
    const PlanFrame &F = D.frames[blockIdx.y];
    const int s = blockIdx.x, lane = threadIdx.x;
    if (!F.filter_level || s >= F.sb_cols * F.sb_rows) return;
    const SbGeo G = sb_geo(F, s);
    const int cols = F.mc.cols, rows = F.mc.rows;
    uint32_t st = 0, b0;
    const int nb = sb_blocks(D, G.slot, b0, st);
    if (lane < 32) (&lfm[0][0][0])[lane] = 0;
    lfl[lane] = 0;
    for (int i = lane; i < LF_PROG_BYTES / 4; i += 64) prog[i] = 0;
    wsync();
    if (lane < nb) {
        const vp9h_block b = load_block(&D.blocks[b0 + lane]);
        if (const int lvl = pl_lf_level(b, F.lflvl, F.filter_level)) {
            const int bw8 = pl_bwh(1, b.bs, 0), bh8 = pl_bwh(1, b.bs, 1), col7 = b.col & 7, row7 = b.row & 7;
            for (int yy = 0; yy < bh8; yy++)
                for (int xx = 0; xx < bw8; xx++)
                    if (row7 + yy < 8 && col7 + xx < 8) lfl[(row7 + yy) * 8 + col7 + xx] = (uint8_t) lvl;
            pl_lf_block_masks(b, cols, rows, SSH, SSV, [&](int cls, int d, int y, int k, unsigned v) {
                if (y < 8) atomicOr(&lfm[cls][d][y], (v & 255u) << (8 * k));
            });
        }
    }
    wsync();
    uint8_t *pg = (uint8_t *) prog;
    for (int i = lane; i < pl_lf_items(SSH, SSV); i += 64)
        pl_lf_item(i, SSH, SSV, G.sbx == 0, G.sby == 0, [&](int pos) { return (int) lfl[pos]; },
                   [&](int cls, int d, int y, int k) { return (lfm[cls][d][y] >> (8 * k)) & 255u; },
                   [&](int off, uint8_t v) { pg[off] = v; });
    wsync();
    uint32_t *g = (uint32_t *) &D.lfs[G.slot];
    for (int i = lane; i < (int) (sizeof(LFRec) / 4); i += 64)
        g[i] = i == 0 ? (uint32_t) F.frame : i == 1 ? ((uint32_t) G.sbx | (uint32_t) G.sby << 16) : prog[i - 2];
}

// ------------------------------------------------------------------ k_plevel
// Level schedule of one inter frame: an SB with intra jobs gets 1 + the highest level of
// the left / top / top-left SBs whose intra pixels it reads (0 if none), computed along
// anti-diagonals; its key is the phase's key0 + level.
__global__ __launch_bounds__(256) void k_plevel(PlanDev D)
{
    const PlanFrame &F = D.frames[blockIdx.x];
    if (!F.levels || F.intra) return;
    const int W = F.sb_cols, H = F.sb_rows;
    for (int d = 0; d < W + H - 1; d++) {
        const int x0 = pl_max(0, d - (H - 1)), x1 = pl_min(d, W - 1);
        for (int x = x0 + (int) threadIdx.x; x <= x1; x += 256) {
            const int y = d - x;
            const uint32_t slot = F.slot0 + (uint32_t) (y * W + x);
            const uint32_t info = D.sb_info[slot];
            if (!(info & 1)) continue;
            // neighbours of earlier diagonals: agent-scope loads (not the CU's L1)
            auto lv = [&](uint32_t n) {
                return (int) (__hip_atomic_load(&D.sb_key[n], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - F.key0) + 1;
            };
            int lvl = 0;
            if ((info & 2) && x > 0) lvl = pl_max(lvl, lv(slot - 1));
            if ((info & 4) && y > 0) lvl = pl_max(lvl, lv(slot - W));
            if ((info & 8) && x > 0 && y > 0) lvl = pl_max(lvl, lv(slot - W - 1));
            const uint32_t key = F.key0 + (uint32_t) lvl;
            if (!inb(D, key, D.nkeys, 4096u)) continue;
            __hip_atomic_store(&D.sb_key[slot], key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            D.sb_kpos[slot] = atomicAdd(&D.key_cnt[key], 1u);
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------ k_pkeys
// One workgroup: exclusive scan of the step-key counts, and the launch summary:
// out[0] status, out[1 .. 1 + ng) count-matrix offsets at the host's gather indices,
// then nk + 1 key offsets, then 2 x nframes 64-bit byte totals.
__global__ __launch_bounds__(1024) void k_pkeys(PlanDev D, int nk, const uint32_t *gidx, int ng, int nframes,
                                                uint32_t *out)
{
    __shared__ uint32_t part[1024];
    const int t = threadIdx.x;
    const int per = (nk + 1023) / 1024, k0 = t * per, k1 = pl_min(nk, k0 + per);
    uint32_t s = 0;
    for (int k = k0; k < k1; k++) s += D.key_cnt[k];
    part[t] = s;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
        const uint32_t v = t >= d ? part[t - d] : 0u;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint32_t run = part[t] - s;
    uint32_t *ko = out + 1 + ng;
    for (int k = k0; k < k1; k++) {
        D.key_off[k] = run;
        ko[k] = run;
        run += D.key_cnt[k];
    }
    if (t == 1023) { D.key_off[nk] = part[1023]; ko[nk] = part[1023]; }
    for (int i = t; i < ng; i += 1024)      // bit 31: an MC-count offset
        out[1 + i] = (gidx[i] >> 31) ? D.cntm0[gidx[i] & 0x7fffffffu] : D.cnt0[gidx[i]];
    uint32_t *fb = ko + nk + 1;
    for (int i = t; i < 2 * nframes; i += 1024) {
        fb[2 * i] = (uint32_t) D.fbytes[i];
        fb[2 * i + 1] = (uint32_t) (D.fbytes[i] >> 32);
    }
    // every frame's eob and coefficient totals as the scans saw them against its packet's
    // counts: a frame that disagrees shifts the eobs / coefficients of every later frame in
    // the batch-wide scans, so the batch fails as a whole (PLS_TOTAL names no frame)
    for (int i = t; i < nframes; i += 1024) {
        const PlanFrame &F = D.frames[i];
        const uint32_t ne = D.blk_eob0[F.blk0 + F.nblk] - D.blk_eob0[F.blk0];
        const uint32_t d0 = F.slot0, d1 = F.slot0 + (uint32_t) (F.sb_cols * F.sb_rows);
        const uint32_t nc = d1 <= D.nslots ? D.sb_coef0[d1] - D.sb_coef0[d0] : ~0u;
        if (ne != F.neob || nc != F.ncoef || D.blk_eob0[F.blk0] != F.eob0 || D.sb_coef0[d0] != F.coef0)
            atomicOr(D.status, PLS_TOTAL);
    }
    __syncthreads();
    for (int i = t; i < nframes; i += 1024) fb[4 * nframes + i] = D.fbad[i];     // per-frame status
    if (t == 0) { out[0] = D.status[0]; out[1 + ng + nk + 1 + 5 * nframes] = D.status[1]; }
}

// ------------------------------------------------------------------ k_plists
__global__ __launch_bounds__(256) void k_plists(PlanDev D)
{
    const PlanFrame &F = D.frames[blockIdx.y];
    const int s = blockIdx.x * 256 + threadIdx.x;
    if (s >= F.sb_cols * F.sb_rows) return;
    const uint32_t slot = F.slot0 + (uint32_t) s;
    if (!(D.sb_info[slot] & 1)) return;
    const uint32_t key = D.sb_key[slot];
    if (!inb(D, key, D.nkeys, 8192u)) return;
    const uint32_t i = D.key_off[key] + D.sb_kpos[slot];
    if (inb(D, i, D.cap_dlists, 16384u)) D.dlists[i] = slot;
}

// ------------------------------------------------------------------ k_psort
// Static step lists (keyframe batches): one workgroup per intra step, its SBs reordered by
// the length of their pass chains, longest first (sb_kpos: the SB's passes, from k_plan; a
// per-pass row count was measured 2 % slower in k_plan's scheduling loop for the same order).
// A k_plf launch lasts until its slowest chain ends; chains dispatched in descending length
// start the long ones first, and the short ones fill the CUs behind them (longest-processing-
// time order). Counting sort over 256 bins (passes, longest first; more than 255 share the
// last), each thread's entries held in registers between the histogram and the scatter
// (one workgroup owns the segment: every read precedes every write); segments of more than
// PSORT_PER * 1024 entries keep the staged order.
#define PSORT_PER 8
__global__ __launch_bounds__(1024) void k_psort(PlanDev D, const uint32_t *ko)
{
    __shared__ uint32_t hist[256];
    const uint32_t k = blockIdx.x, t = threadIdx.x;
    const uint32_t a = ko[k], e = ko[k + 1];
    if (e <= a + 1 || e > D.nslots || e - a > PSORT_PER * 1024u) return;
    if (t < 256) hist[t] = 0;
    __syncthreads();
    uint32_t sl[PSORT_PER], bn[PSORT_PER];
#pragma unroll
    for (int j = 0; j < PSORT_PER; j++) {
        const uint32_t i = a + t + (uint32_t) j * 1024u;
        sl[j] = i < e ? D.dlists[i] : 0u;
    }
#pragma unroll
    for (int j = 0; j < PSORT_PER; j++) {
        const uint32_t i = a + t + (uint32_t) j * 1024u;
        const uint32_t c = i < e ? D.sb_kpos[sl[j]] : 0u;
        bn[j] = 255u - (c < 255u ? c : 255u);
        if (i < e) atomicAdd(&hist[bn[j]], 1u);
    }
    __syncthreads();
    const uint32_t v = t < 256 ? hist[t] : 0u;
    for (uint32_t d = 1; d < 256; d <<= 1) {           // inclusive scan of the bins
        const uint32_t x = t < 256 && t >= d ? hist[t - d] : 0u;
        __syncthreads();
        if (t < 256) hist[t] += x;
        __syncthreads();
    }
    if (t < 256) hist[t] -= v;                         // exclusive: each bin's first position
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PSORT_PER; j++) {
        const uint32_t i = a + t + (uint32_t) j * 1024u;
        if (i < e) D.dlists[a + atomicAdd(&hist[bn[j]], 1u)] = sl[j];
    }
}

// ------------------------------------------------------------------ k_pguard
// Batches whose launch list is fixed at staging (keyframe batches, runtime "static plan"):
// their pixel kernels run after the planner without a host check of its status, so the
// frames the planner rejected (fbad != 0: the frame's packet is inconsistent) are
// neutralised here: no intra passes (WGRec), and their residual jobs write nothing but
// zeros into the spare scratch slot (slot nslots) from no coefficients. The other frames'
// records address only their own data (k_pjob), so they reconstruct as if alone; a status
// that names no frame (PLS_BOUNDS, PLS_TOTAL) neutralises the whole batch (every WGRec, the summary's
// residual ranges). The status is re-copied into the summary (k_plists' bound checks come
// after k_pkeys), which the host reads when it next waits for the batch (vp9hip_sync /
// sync_slot: AVERROR_INVALIDDATA; vp9hip_batch_frame_status: which frames).
__global__ __launch_bounds__(256) void k_pguard(PlanDev D, uint32_t *summary, int ng)
{
    const uint32_t st = __builtin_amdgcn_readfirstlane(D.status[0]);
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) summary[0] = st;
    if (!st) return;
    const bool all = (st & (PLS_BOUNDS | PLS_TOTAL)) != 0;
    const PlanFrame &F = D.frames[blockIdx.y];
    const int s = blockIdx.x * 256 + threadIdx.x;
    if (all && blockIdx.y == 0)
        for (int i = s; i < ng; i += (int) gridDim.x * 256) summary[1 + i] = 0;
    if (!all) {
        const uint32_t spare = D.nslots * D.rcap;        // resid scratch has nslots + 1 slots
        const uint32_t nt = gridDim.x * gridDim.y * 256u;
        for (uint32_t i = (blockIdx.y * gridDim.x + blockIdx.x) * 256u + threadIdx.x; i + 1 < D.cap_rjobs; i += nt) {
            RJob r = D.rjobs[i];
            if (r.frame >= D.nframes || !D.fbad[r.frame]) continue;
            r.coef = 0; r.dst = spare; r.eob = 0; r.nzc = 1; r.nzr = 1;
            r.ptx &= (uint8_t) ~(1u << 5);                   // scratch, not in place
            D.rjobs[i] = r;
        }
    }
    const bool bad = all || ((uint32_t) F.frame < D.nframes && D.fbad[F.frame]);
    if (!bad || s >= F.sb_cols * F.sb_rows) return;
    const uint32_t slot = F.slot0 + (uint32_t) s;
    if (slot < D.nslots) { D.wgs[slot].njobs = 0; D.wgs[slot].npass = 0; }
}

// stage 0: k_psb; 1: k_pjob, k_plan, then k_pllf (filtered frames) and k_plmc (inter frames)
template <int SSH, int SSV>
void launch_sb_kernels(hipStream_t st, const PlanDev &D, int max_sb, int nframes, int stage, int flags)
{
    const dim3 g(max_sb, nframes);
    if (stage == 0) { hipLaunchKernelGGL((k_psb<SSH, SSV>), g, dim3(64), 0, st, D); return; }
    if (D.dbg & 8) {                                             // VP9HIP_PLAN_DBG bit 3: unfused
        hipLaunchKernelGGL((k_pjob<SSH, SSV>), g, dim3(64), 0, st, D);
        hipLaunchKernelGGL((k_plan<SSH, SSV>), g, dim3(64), 0, st, D);
    } else
        hipLaunchKernelGGL((k_pjplan<SSH, SSV>), g, dim3(64), 0, st, D);
    if (flags & 1) hipLaunchKernelGGL((k_pllf<SSH, SSV>), g, dim3(64), 0, st, D);
    if (flags & 2) hipLaunchKernelGGL((k_plmc<SSH, SSV>), g, dim3(64), 0, st, D);
}

// ss: ss_h | ss_v << 1 (as the pixel kernels' launchers)
void launch_sb(int ss, hipStream_t st, const PlanDev &D, int max_sb, int nframes, int stage, int flags)
{
    switch (ss) {
    case 3: launch_sb_kernels<1, 1>(st, D, max_sb, nframes, stage, flags); break;
    case 1: launch_sb_kernels<1, 0>(st, D, max_sb, nframes, stage, flags); break;
    case 2: launch_sb_kernels<0, 1>(st, D, max_sb, nframes, stage, flags); break;
    default: launch_sb_kernels<0, 0>(st, D, max_sb, nframes, stage, flags); break;
    }
}

} // namespace

extern "C" {
// Temporary storage of the exclusive scans over up to n elements.
size_t vp9hip_plan_scan_bytes(size_t n)
{
    size_t b = 0;
    if (hipcub::DeviceScan::ExclusiveSum(nullptr, b, (const uint32_t *) nullptr, (uint32_t *) nullptr, (int) n) != hipSuccess) return 0;
    return b;
}

// Enqueue the device planner of a staged batch on `st`. The caller has zeroed
// status / key_cnt / fbytes and set sb_first / sb_end to 0xffffffff.
// nb / nslots / ncnt: blocks, SB slots, count-matrix entries (each array + 1 zero entry).
int vp9hip_plan_enqueue(hipStream_t st, const PlanDev *Dp, int ss, int nframes, int max_blk, int max_sb, uint32_t nb,
                        uint32_t nslots, uint32_t ncnt, int nk, const uint32_t *gidx, int ng, uint32_t *summary,
                        void *scan_tmp, size_t scan_bytes, int any_levels, int flags, int guard)
{
    const PlanDev &D = *Dp;
    if (nframes <= 0) return 0;
    hipLaunchKernelGGL(k_pblk, dim3((max_blk + 255) / 256, nframes), dim3(256), 0, st, D);
    size_t tb = scan_bytes;
    if (hipcub::DeviceScan::ExclusiveSum(scan_tmp, tb, D.blk_neob, D.blk_eob0, (int) nb + 1, st) != hipSuccess) return -1;
    launch_sb(ss, st, D, max_sb, nframes, 0, 0);
    tb = scan_bytes;
    if (hipcub::DeviceScan::ExclusiveSum(scan_tmp, tb, D.sb_ncoef, D.sb_coef0, (int) nslots + 1, st) != hipSuccess) return -1;
    tb = scan_bytes;
    if (hipcub::DeviceScan::ExclusiveSum(scan_tmp, tb, D.cnt, D.cnt0, (int) ncnt + 1, st) != hipSuccess) return -1;
    tb = scan_bytes;
    if (hipcub::DeviceScan::ExclusiveSum(scan_tmp, tb, D.cntm, D.cntm0, (int) nslots + 1, st) != hipSuccess) return -1;
    launch_sb(ss, st, D, max_sb, nframes, 1, flags);
    if (any_levels) hipLaunchKernelGGL(k_plevel, dim3(nframes), dim3(256), 0, st, D);
    if (D.static_lists && D.stat_ko && !(D.dbg & 4))             // VP9HIP_PLAN_DBG bit 2: staged order
        hipLaunchKernelGGL(k_psort, dim3(nk), dim3(1024), 0, st, D, D.stat_ko);
    hipLaunchKernelGGL(k_pkeys, dim3(1), dim3(1024), 0, st, D, nk, gidx, ng, nframes, summary);
    if (!D.static_lists) hipLaunchKernelGGL(k_plists, dim3((max_sb + 255) / 256, nframes), dim3(256), 0, st, D);
    if (guard) hipLaunchKernelGGL(k_pguard, dim3((max_sb + 255) / 256, nframes), dim3(256), 0, st, D, summary, ng);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
}
