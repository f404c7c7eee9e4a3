// gfx950 (MI355X) kernels of the VP9 hybrid decoder pixel path.
//
//   k_resid / k_resid_dev / k_resid_multi — inverse DCT / ADST / WHT of every coded tx block
//              (vp9dsp_template.c:1155-1754): one lane per column, 64 / N jobs per wave,
//              LDS transpose; intra residuals to int16 scratch, inter ones added in place.
//   k_pred   — intra prediction passes of an SB (vp9recon.c:235-364, the 15 predictors of
//              vp9dsp_template.c:28-1106 as a per-pixel formula table) + residual add.
//   k_lf     — the deblocking filter of one SB (ff_vp9_loopfilter_sb, vp9lpf.c:183-230) on
//              an LDS tile, SBs launched along the t = x + 2y wavefront (raster order).
//   k_plf    — fused keyframe launches: intra diagonal t and LF diagonal t - 3.
//   k_lfrd / k_lfro — the row-pipelined loop filter of narrow phases: one workgroup per SB
//              row, hand-offs between rows through sc1 stores and progress words.
//   k_mcq    — sub-pel motion compensation, unscaled and scaled references, compound
//              (vp9dsp_template.c:1969-2569), edge clamping (videodsp_template.c:27-105).
//
// Arithmetic restates vp9dsp_template.c bit-exactly: 8-bit transforms run in
// wrapping 32-bit arithmetic with int16 intermediates (dctint int / dctcoef int16,
// vp9dsp_8bpp.c), high bit depth in int64 with int32 intermediates.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>

#define VP9T_STORAGE static __constant__ const
#include "vp9_tables.h"
#include "vp9hip_work.h"

// The Makefile compiles this file once per KPART (0..5), each object holding a subset of
// the launchers below and so of the kernel instantiations (parallel builds); without KPART
// (profiling builds) one object holds everything.
#ifdef KPART
#define KP(n) (KPART == (n))
#else
#define KP(n) 1
#endif
#if !defined(KPART) || KPART == 0
#define KP_DEV __device__
#else
#define KP_DEV static __device__
#endif

#define DEV __device__ __forceinline__

// ------------------------------------------------------------------ helpers
DEV int clipbd(int v, int bd) { int m = (1 << bd) - 1; return v < 0 ? 0 : (v > m ? m : v); }

// clamp to [0, mx] in one v_med3_i32 (mx wave-uniform)
DEV int med3_0(int v, int mx)
{
    int r;
    asm("v_med3_i32 %0, %1, 0, %2" : "=v"(r) : "v"(v), "s"(mx));
    return r;
}

DEV void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Transform arithmetic policy. 8-bit: uint32 bit patterns (defined wrap-around,
// identical to the reference's `x * 11585U` products cast back to int) with an
// arithmetic rounding shift. High bit depth: int64.
struct M32 {
    typedef uint32_t T;
    static DEV T in(int32_t v) { return (uint32_t) v; }
    static DEV T r14(T v) { return (uint32_t) ((int32_t) (v + 8192u) >> 14); }
};
struct M64 {
    typedef int64_t T;
    static DEV T in(int32_t v) { return (int64_t) v; }
    static DEV T r14(T v) { return (v + 8192) >> 14; }
};

#define R(x) M::r14(x)
#define C(k) ((T) (k))

// vp9dsp_template.c:1202-1216
template <class M> DEV void idct4(typename M::T *io)
{
    typedef typename M::T T;
    T t0 = R((io[0] + io[2]) * C(11585)), t1 = R((io[0] - io[2]) * C(11585));
    T t2 = R(io[1] * C(6270) - io[3] * C(15137)), t3 = R(io[1] * C(15137) + io[3] * C(6270));
    io[0] = t0 + t3; io[1] = t1 + t2; io[2] = t1 - t2; io[3] = t0 - t3;
}
// vp9dsp_template.c:1218-1232
template <class M> DEV void iadst4(typename M::T *io)
{
    typedef typename M::T T;
    T t0 = C(5283) * io[0] + C(15212) * io[2] + C(9929) * io[3];
    T t1 = C(9929) * io[0] - C(5283) * io[2] - C(15212) * io[3];
    T t2 = C(13377) * (io[0] - io[2] + io[3]);
    T t3 = C(13377) * io[1];
    io[0] = R(t0 + t3); io[1] = R(t1 + t3); io[2] = R(t2); io[3] = R(t0 + t1 - t3);
}
// vp9dsp_template.c:1236-1270
template <class M> DEV void idct8(typename M::T *io)
{
    typedef typename M::T T;
    T t0a = R((io[0] + io[4]) * C(11585)), t1a = R((io[0] - io[4]) * C(11585));
    T t2a = R(io[2] * C(6270) - io[6] * C(15137)), t3a = R(io[2] * C(15137) + io[6] * C(6270));
    T t4a = R(io[1] * C(3196) - io[7] * C(16069)), t5a = R(io[5] * C(13623) - io[3] * C(9102));
    T t6a = R(io[5] * C(9102) + io[3] * C(13623)), t7a = R(io[1] * C(16069) + io[7] * C(3196));
    T t0 = t0a + t3a, t1 = t1a + t2a, t2 = t1a - t2a, t3 = t0a - t3a;
    T t4 = t4a + t5a, t7 = t7a + t6a;
    t5a = t4a - t5a; t6a = t7a - t6a;
    T t5 = R((t6a - t5a) * C(11585)), t6 = R((t6a + t5a) * C(11585));
    io[0] = t0 + t7; io[1] = t1 + t6; io[2] = t2 + t5; io[3] = t3 + t4;
    io[4] = t3 - t4; io[5] = t2 - t5; io[6] = t1 - t6; io[7] = t0 - t7;
}
// vp9dsp_template.c:1272-1314
template <class M> DEV void iadst8(typename M::T *io)
{
    typedef typename M::T T;
    T t0a = C(16305) * io[7] + C(1606) * io[0], t1a = C(1606) * io[7] - C(16305) * io[0];
    T t2a = C(14449) * io[5] + C(7723) * io[2], t3a = C(7723) * io[5] - C(14449) * io[2];
    T t4a = C(10394) * io[3] + C(12665) * io[4], t5a = C(12665) * io[3] - C(10394) * io[4];
    T t6a = C(4756) * io[1] + C(15679) * io[6], t7a = C(15679) * io[1] - C(4756) * io[6];
    T t0 = R(t0a + t4a), t1 = R(t1a + t5a), t2 = R(t2a + t6a), t3 = R(t3a + t7a);
    T t4 = R(t0a - t4a), t5 = R(t1a - t5a), t6 = R(t2a - t6a), t7 = R(t3a - t7a);
    t4a = C(15137) * t4 + C(6270) * t5;
    t5a = C(6270) * t4 - C(15137) * t5;
    t6a = C(15137) * t7 - C(6270) * t6;
    t7a = C(6270) * t7 + C(15137) * t6;
    io[0] = t0 + t2;
    io[7] = C(0) - (t1 + t3);
    t2 = t0 - t2;
    t3 = t1 - t3;
    io[1] = C(0) - R(t4a + t6a);
    io[6] = R(t5a + t7a);
    t6 = R(t4a - t6a);
    t7 = R(t5a - t7a);
    io[3] = C(0) - R((t2 + t3) * C(11585));
    io[4] = R((t2 - t3) * C(11585));
    io[2] = R((t6 + t7) * C(11585));
    io[5] = C(0) - R((t6 - t7) * C(11585));
}
// vp9dsp_template.c:1318-1404
template <class M> DEV void idct16(typename M::T *io)
{
    typedef typename M::T T;
    T t0, t1, t2, t3, t4, t5, t6, t7, t8, t9, t10, t11, t12, t13, t14, t15;
    T t0a, t1a, t2a, t3a, t4a, t5a, t6a, t7a, t8a, t9a, t10a, t11a, t12a, t13a, t14a, t15a;
    t0a = R((io[0] + io[8]) * C(11585));
    t1a = R((io[0] - io[8]) * C(11585));
    t2a = R(io[4] * C(6270) - io[12] * C(15137));
    t3a = R(io[4] * C(15137) + io[12] * C(6270));
    t4a = R(io[2] * C(3196) - io[14] * C(16069));
    t7a = R(io[2] * C(16069) + io[14] * C(3196));
    t5a = R(io[10] * C(13623) - io[6] * C(9102));
    t6a = R(io[10] * C(9102) + io[6] * C(13623));
    t8a = R(io[1] * C(1606) - io[15] * C(16305));
    t15a = R(io[1] * C(16305) + io[15] * C(1606));
    t9a = R(io[9] * C(12665) - io[7] * C(10394));
    t14a = R(io[9] * C(10394) + io[7] * C(12665));
    t10a = R(io[5] * C(7723) - io[11] * C(14449));
    t13a = R(io[5] * C(14449) + io[11] * C(7723));
    t11a = R(io[13] * C(15679) - io[3] * C(4756));
    t12a = R(io[13] * C(4756) + io[3] * C(15679));
    t0 = t0a + t3a; t1 = t1a + t2a; t2 = t1a - t2a; t3 = t0a - t3a;
    t4 = t4a + t5a; t5 = t4a - t5a; t6 = t7a - t6a; t7 = t7a + t6a;
    t8 = t8a + t9a; t9 = t8a - t9a; t10 = t11a - t10a; t11 = t11a + t10a;
    t12 = t12a + t13a; t13 = t12a - t13a; t14 = t15a - t14a; t15 = t15a + t14a;
    t5a = R((t6 - t5) * C(11585));
    t6a = R((t6 + t5) * C(11585));
    t9a = R(t14 * C(6270) - t9 * C(15137));
    t14a = R(t14 * C(15137) + t9 * C(6270));
    t10a = R(C(0) - (t13 * C(15137) + t10 * C(6270)));
    t13a = R(t13 * C(6270) - t10 * C(15137));
    t0a = t0 + t7; t1a = t1 + t6a; t2a = t2 + t5a; t3a = t3 + t4;
    t4 = t3 - t4; t5 = t2 - t5a; t6 = t1 - t6a; t7 = t0 - t7;
    t8a = t8 + t11; t9 = t9a + t10a; t10 = t9a - t10a; t11a = t8 - t11;
    t12a = t15 - t12; t13 = t14a - t13a; t14 = t14a + t13a; t15a = t15 + t12;
    t10a = R((t13 - t10) * C(11585));
    t13a = R((t13 + t10) * C(11585));
    t11 = R((t12a - t11a) * C(11585));
    t12 = R((t12a + t11a) * C(11585));
    io[0] = t0a + t15a; io[1] = t1a + t14; io[2] = t2a + t13a; io[3] = t3a + t12;
    io[4] = t4 + t11; io[5] = t5 + t10a; io[6] = t6 + t9; io[7] = t7 + t8a;
    io[8] = t7 - t8a; io[9] = t6 - t9; io[10] = t5 - t10a; io[11] = t4 - t11;
    io[12] = t3a - t12; io[13] = t2a - t13a; io[14] = t1a - t14; io[15] = t0a - t15a;
}
// vp9dsp_template.c:1406-1507
template <class M> DEV void iadst16(typename M::T *io)
{
    typedef typename M::T T;
    T t0, t1, t2, t3, t4, t5, t6, t7, t8, t9, t10, t11, t12, t13, t14, t15;
    T t0a, t1a, t2a, t3a, t4a, t5a, t6a, t7a, t8a, t9a, t10a, t11a, t12a, t13a, t14a, t15a;
    t0 = io[15] * C(16364) + io[0] * C(804);
    t1 = io[15] * C(804) - io[0] * C(16364);
    t2 = io[13] * C(15893) + io[2] * C(3981);
    t3 = io[13] * C(3981) - io[2] * C(15893);
    t4 = io[11] * C(14811) + io[4] * C(7005);
    t5 = io[11] * C(7005) - io[4] * C(14811);
    t6 = io[9] * C(13160) + io[6] * C(9760);
    t7 = io[9] * C(9760) - io[6] * C(13160);
    t8 = io[7] * C(11003) + io[8] * C(12140);
    t9 = io[7] * C(12140) - io[8] * C(11003);
    t10 = io[5] * C(8423) + io[10] * C(14053);
    t11 = io[5] * C(14053) - io[10] * C(8423);
    t12 = io[3] * C(5520) + io[12] * C(15426);
    t13 = io[3] * C(15426) - io[12] * C(5520);
    t14 = io[1] * C(2404) + io[14] * C(16207);
    t15 = io[1] * C(16207) - io[14] * C(2404);
    t0a = R(t0 + t8); t1a = R(t1 + t9); t2a = R(t2 + t10); t3a = R(t3 + t11);
    t4a = R(t4 + t12); t5a = R(t5 + t13); t6a = R(t6 + t14); t7a = R(t7 + t15);
    t8a = R(t0 - t8); t9a = R(t1 - t9); t10a = R(t2 - t10); t11a = R(t3 - t11);
    t12a = R(t4 - t12); t13a = R(t5 - t13); t14a = R(t6 - t14); t15a = R(t7 - t15);
    t8 = t8a * C(16069) + t9a * C(3196);
    t9 = t8a * C(3196) - t9a * C(16069);
    t10 = t10a * C(9102) + t11a * C(13623);
    t11 = t10a * C(13623) - t11a * C(9102);
    t12 = t13a * C(16069) - t12a * C(3196);
    t13 = t13a * C(3196) + t12a * C(16069);
    t14 = t15a * C(9102) - t14a * C(13623);
    t15 = t15a * C(13623) + t14a * C(9102);
    t0 = t0a + t4a; t1 = t1a + t5a; t2 = t2a + t6a; t3 = t3a + t7a;
    t4 = t0a - t4a; t5 = t1a - t5a; t6 = t2a - t6a; t7 = t3a - t7a;
    t8a = R(t8 + t12); t9a = R(t9 + t13); t10a = R(t10 + t14); t11a = R(t11 + t15);
    t12a = R(t8 - t12); t13a = R(t9 - t13); t14a = R(t10 - t14); t15a = R(t11 - t15);
    t4a = t4 * C(15137) + t5 * C(6270);
    t5a = t4 * C(6270) - t5 * C(15137);
    t6a = t7 * C(15137) - t6 * C(6270);
    t7a = t7 * C(6270) + t6 * C(15137);
    t12 = t12a * C(15137) + t13a * C(6270);
    t13 = t12a * C(6270) - t13a * C(15137);
    t14 = t15a * C(15137) - t14a * C(6270);
    t15 = t15a * C(6270) + t14a * C(15137);
    io[0] = t0 + t2;
    io[15] = C(0) - (t1 + t3);
    t2a = t0 - t2;
    t3a = t1 - t3;
    io[3] = C(0) - R(t4a + t6a);
    io[12] = R(t5a + t7a);
    t6 = R(t4a - t6a);
    t7 = R(t5a - t7a);
    io[1] = C(0) - (t8a + t10a);
    io[14] = t9a + t11a;
    t10 = t8a - t10a;
    t11 = t9a - t11a;
    io[2] = R(t12 + t14);
    io[13] = C(0) - R(t13 + t15);
    t14a = R(t12 - t14);
    t15a = R(t13 - t15);
    io[7] = R((C(0) - (t2a + t3a)) * C(11585));
    io[8] = R((t2a - t3a) * C(11585));
    io[4] = R((t7 + t6) * C(11585));
    io[11] = R((t7 - t6) * C(11585));
    io[6] = R((t11 + t10) * C(11585));
    io[9] = R((t11 - t10) * C(11585));
    io[5] = R((C(0) - (t14a + t15a)) * C(11585));
    io[10] = R((t14a - t15a) * C(11585));
}
// vp9dsp_template.c:1511-1715
template <class M> DEV void idct32(typename M::T *io)
{
    typedef typename M::T T;
    T t0a = R((io[0] + io[16]) * C(11585));
    T t1a = R((io[0] - io[16]) * C(11585));
    T t2a = R(io[8] * C(6270) - io[24] * C(15137));
    T t3a = R(io[8] * C(15137) + io[24] * C(6270));
    T t4a = R(io[4] * C(3196) - io[28] * C(16069));
    T t7a = R(io[4] * C(16069) + io[28] * C(3196));
    T t5a = R(io[20] * C(13623) - io[12] * C(9102));
    T t6a = R(io[20] * C(9102) + io[12] * C(13623));
    T t8a = R(io[2] * C(1606) - io[30] * C(16305));
    T t15a = R(io[2] * C(16305) + io[30] * C(1606));
    T t9a = R(io[18] * C(12665) - io[14] * C(10394));
    T t14a = R(io[18] * C(10394) + io[14] * C(12665));
    T t10a = R(io[10] * C(7723) - io[22] * C(14449));
    T t13a = R(io[10] * C(14449) + io[22] * C(7723));
    T t11a = R(io[26] * C(15679) - io[6] * C(4756));
    T t12a = R(io[26] * C(4756) + io[6] * C(15679));
    T t16a = R(io[1] * C(804) - io[31] * C(16364));
    T t31a = R(io[1] * C(16364) + io[31] * C(804));
    T t17a = R(io[17] * C(12140) - io[15] * C(11003));
    T t30a = R(io[17] * C(11003) + io[15] * C(12140));
    T t18a = R(io[9] * C(7005) - io[23] * C(14811));
    T t29a = R(io[9] * C(14811) + io[23] * C(7005));
    T t19a = R(io[25] * C(15426) - io[7] * C(5520));
    T t28a = R(io[25] * C(5520) + io[7] * C(15426));
    T t20a = R(io[5] * C(3981) - io[27] * C(15893));
    T t27a = R(io[5] * C(15893) + io[27] * C(3981));
    T t21a = R(io[21] * C(14053) - io[11] * C(8423));
    T t26a = R(io[21] * C(8423) + io[11] * C(14053));
    T t22a = R(io[13] * C(9760) - io[19] * C(13160));
    T t25a = R(io[13] * C(13160) + io[19] * C(9760));
    T t23a = R(io[29] * C(16207) - io[3] * C(2404));
    T t24a = R(io[29] * C(2404) + io[3] * C(16207));

    T t0 = t0a + t3a, t1 = t1a + t2a, t2 = t1a - t2a, t3 = t0a - t3a;
    T t4 = t4a + t5a, t5 = t4a - t5a, t6 = t7a - t6a, t7 = t7a + t6a;
    T t8 = t8a + t9a, t9 = t8a - t9a, t10 = t11a - t10a, t11 = t11a + t10a;
    T t12 = t12a + t13a, t13 = t12a - t13a, t14 = t15a - t14a, t15 = t15a + t14a;
    T t16 = t16a + t17a, t17 = t16a - t17a, t18 = t19a - t18a, t19 = t19a + t18a;
    T t20 = t20a + t21a, t21 = t20a - t21a, t22 = t23a - t22a, t23 = t23a + t22a;
    T t24 = t24a + t25a, t25 = t24a - t25a, t26 = t27a - t26a, t27 = t27a + t26a;
    T t28 = t28a + t29a, t29 = t28a - t29a, t30 = t31a - t30a, t31 = t31a + t30a;

    t5a = R((t6 - t5) * C(11585));
    t6a = R((t6 + t5) * C(11585));
    t9a = R(t14 * C(6270) - t9 * C(15137));
    t14a = R(t14 * C(15137) + t9 * C(6270));
    t10a = R(C(0) - (t13 * C(15137) + t10 * C(6270)));
    t13a = R(t13 * C(6270) - t10 * C(15137));
    t17a = R(t30 * C(3196) - t17 * C(16069));
    t30a = R(t30 * C(16069) + t17 * C(3196));
    t18a = R(C(0) - (t29 * C(16069) + t18 * C(3196)));
    t29a = R(t29 * C(3196) - t18 * C(16069));
    t21a = R(t26 * C(13623) - t21 * C(9102));
    t26a = R(t26 * C(9102) + t21 * C(13623));
    t22a = R(C(0) - (t25 * C(9102) + t22 * C(13623)));
    t25a = R(t25 * C(13623) - t22 * C(9102));

    t0a = t0 + t7; t1a = t1 + t6a; t2a = t2 + t5a; t3a = t3 + t4;
    t4a = t3 - t4; t5 = t2 - t5a; t6 = t1 - t6a; t7a = t0 - t7;
    t8a = t8 + t11; t9 = t9a + t10a; t10 = t9a - t10a; t11a = t8 - t11;
    t12a = t15 - t12; t13 = t14a - t13a; t14 = t14a + t13a; t15a = t15 + t12;
    t16a = t16 + t19; t17 = t17a + t18a; t18 = t17a - t18a; t19a = t16 - t19;
    t20a = t23 - t20; t21 = t22a - t21a; t22 = t22a + t21a; t23a = t23 + t20;
    t24a = t24 + t27; t25 = t25a + t26a; t26 = t25a - t26a; t27a = t24 - t27;
    t28a = t31 - t28; t29 = t30a - t29a; t30 = t30a + t29a; t31a = t31 + t28;

    t10a = R((t13 - t10) * C(11585));
    t13a = R((t13 + t10) * C(11585));
    t11 = R((t12a - t11a) * C(11585));
    t12 = R((t12a + t11a) * C(11585));
    t18a = R(t29 * C(6270) - t18 * C(15137));
    t29a = R(t29 * C(15137) + t18 * C(6270));
    t19 = R(t28a * C(6270) - t19a * C(15137));
    t28 = R(t28a * C(15137) + t19a * C(6270));
    t20 = R(C(0) - (t27a * C(15137) + t20a * C(6270)));
    t27 = R(t27a * C(6270) - t20a * C(15137));
    t21a = R(C(0) - (t26 * C(15137) + t21 * C(6270)));
    t26a = R(t26 * C(6270) - t21 * C(15137));

    t0 = t0a + t15a; t1 = t1a + t14; t2 = t2a + t13a; t3 = t3a + t12;
    t4 = t4a + t11; t5a = t5 + t10a; t6a = t6 + t9; t7 = t7a + t8a;
    t8 = t7a - t8a; t9a = t6 - t9; t10 = t5 - t10a; t11a = t4a - t11;
    t12a = t3a - t12; t13 = t2a - t13a; t14a = t1a - t14; t15 = t0a - t15a;
    t16 = t16a + t23a; t17a = t17 + t22; t18 = t18a + t21a; t19a = t19 + t20;
    t20a = t19 - t20; t21 = t18a - t21a; t22a = t17 - t22; t23 = t16a - t23a;
    t24 = t31a - t24a; t25a = t30 - t25; t26 = t29a - t26a; t27a = t28 - t27;
    t28a = t28 + t27; t29 = t29a + t26a; t30a = t30 + t25; t31 = t31a + t24a;

    t20 = R((t27a - t20a) * C(11585));
    t27 = R((t27a + t20a) * C(11585));
    t21a = R((t26 - t21) * C(11585));
    t26a = R((t26 + t21) * C(11585));
    t22 = R((t25a - t22a) * C(11585));
    t25 = R((t25a + t22a) * C(11585));
    t23a = R((t24 - t23) * C(11585));
    t24a = R((t24 + t23) * C(11585));

    io[0] = t0 + t31; io[1] = t1 + t30a; io[2] = t2 + t29; io[3] = t3 + t28a;
    io[4] = t4 + t27; io[5] = t5a + t26a; io[6] = t6a + t25; io[7] = t7 + t24a;
    io[8] = t8 + t23a; io[9] = t9a + t22; io[10] = t10 + t21a; io[11] = t11a + t20;
    io[12] = t12a + t19a; io[13] = t13 + t18; io[14] = t14a + t17a; io[15] = t15 + t16;
    io[16] = t15 - t16; io[17] = t14a - t17a; io[18] = t13 - t18; io[19] = t12a - t19a;
    io[20] = t11a - t20; io[21] = t10 - t21a; io[22] = t9a - t22; io[23] = t8 - t23a;
    io[24] = t7 - t24a; io[25] = t6a - t25; io[26] = t5a - t26a; io[27] = t4 - t27;
    io[28] = t3 - t28a; io[29] = t2 - t29; io[30] = t1 - t30a; io[31] = t0 - t31;
}
#undef R
#undef C

// iwht4_1d (vp9dsp_template.c:1719-1748), int temporaries
DEV void iwht4(int32_t *io, int pass)
{
    uint32_t t0, t1, t2, t3, t4;
    if (pass == 0) { t0 = io[0] >> 2; t1 = io[3] >> 2; t2 = io[1] >> 2; t3 = io[2] >> 2; }
    else { t0 = io[0]; t1 = io[3]; t2 = io[1]; t3 = io[2]; }
    t0 += t2; t3 -= t1; t4 = (uint32_t) ((int32_t) (t0 - t3) >> 1); t1 = t4 - t1; t2 = t4 - t2; t0 -= t1; t3 += t2;
    io[0] = (int32_t) t0; io[1] = (int32_t) t1; io[2] = (int32_t) t2; io[3] = (int32_t) t3;
}

// One 1-D inverse transform of compile-time length N (adst: 0 dct, 1 adst).
template <int N, class M> DEV void tx1n(typename M::T *v, int adst)
{
    if (N == 4) { if (adst) iadst4<M>(v); else idct4<M>(v); }
    else if (N == 8) { if (adst) iadst8<M>(v); else idct8<M>(v); }
    else if (N == 16) { if (adst) iadst16<M>(v); else idct16<M>(v); }
    else idct32<M>(v);
}

// ------------------------------------------------------------ intra predict
// Edge array layout per wave (`e`): e[0..n) = left column bottom-to-top (top-to-
// bottom for HOR_UP), e[n] = top-left, e[n+1 ..] = top row incl. top-right.
// Per-pixel closed forms of the predictors of vp9dsp_template.c:28-1106.
#define A2(a, b) (((a) + (b) + 1) >> 1)
#define A3(a, b, c) (((a) + 2 * (b) + (c) + 2) >> 2)

DEV int pred_px(int mode, int n, int x, int y, const uint16_t *e, int dc, int bd)
{
    const uint16_t *L = e, *T = e + n + 1;
    switch (mode) {
    case 0: return T[x];                                           // VERT
    case 1: return L[n - 1 - y];                                   // HOR
    case 9: return clipbd(T[x] + L[n - 1 - y] - T[-1], bd);        // TM_VP8
    case 3: {                                                      // DIAG_DOWN_LEFT
        int k = x + y;
        if (n == 4) return k < 6 ? A3(T[k], T[k + 1], T[k + 2]) : T[7];
        if (k < n - 2) return A3(T[k], T[k + 1], T[k + 2]);
        if (k == n - 2) return (T[n - 2] + T[n - 1] * 3 + 2) >> 2;
        return T[n - 1];
    }
    case 4: { int j = n - 1 - y + x; return A3(e[j], e[j + 1], e[j + 2]); }   // DIAG_DOWN_RIGHT
    case 5: {                                                      // VERT_RIGHT
        int h = n >> 1, m = h - 1 - (y >> 1) + x;
        if (!(y & 1)) {
            if (m <= h - 2) return A3(e[2 * m + 2], e[2 * m + 3], e[2 * m + 4]);
            return A2(e[n + m - h + 1], e[n + m - h + 2]);
        }
        if (m <= h - 2) return A3(e[2 * m + 1], e[2 * m + 2], e[2 * m + 3]);
        return A3(e[n + m - h], e[n + m - h + 1], e[n + m - h + 2]);
    }
    case 6: {                                                      // HOR_DOWN
        int m = 2 * n - 2 - 2 * y + x;
        if (m >= 2 * n) { int i = m - 2 * n; return A3(e[n + i], e[n + i + 1], e[n + i + 2]); }
        int i = m >> 1;
        return (m & 1) ? A3(e[i], e[i + 1], e[i + 2]) : A2(e[i], e[i + 1]);
    }
    case 7: {                                                      // VERT_LEFT
        int k = (y >> 1) + x;
        if (n == 4) return (y & 1) ? A3(T[k], T[k + 1], T[k + 2]) : A2(T[k], T[k + 1]);
        if (x >= n - (y >> 1) - 1) return T[n - 1];
        if (!(y & 1)) return A2(T[k], T[k + 1]);
        return k < n - 2 ? A3(T[k], T[k + 1], T[k + 2]) : (T[n - 2] + T[n - 1] * 3 + 2) >> 2;
    }
    case 8: {                                                      // HOR_UP (L top-to-bottom)
        if (y >= (n >> 1) && x >= 2 * n - 2 - 2 * y) return L[n - 1];
        int m = 2 * y + x, i = m >> 1;
        if (!(m & 1)) return A2(L[i], L[i + 1]);
        return i < n - 2 ? A3(L[i], L[i + 1], L[i + 2]) : (L[n - 2] + L[n - 1] * 3 + 2) >> 2;
    }
    default: return dc;                                            // DC variants
    }
}

// ------------------------------------------------------------- k_resid
// Inverse transform of every coded tx block of a batch (vp9dsp_template.c:1139-1750),
// one launch per tx code, no dependencies: a wave holds 64/N jobs, N lanes per job
// (one per column). The residual (out + (1 << (bits - 1))) >> bits is either added in
// place onto the motion-compensated prediction (inter blocks) or stored column-major
// as int16 for k_pred (intra blocks; 10/12-bit values saturate to int16, which leaves
// clip(pred + r) unchanged since |pred| < 4096).
#define RWAVES 4

DEV const int16_t *scan_for(int tcode, int txtp)
{
    const int ts = tcode & 3;
    if (tcode == 4) return vp9t_scan_default_4x4;                 // lossless (vp9data.c:600-618)
    return ts == 0 ? (txtp == 1 ? vp9t_scan_col_4x4 : txtp == 2 ? vp9t_scan_row_4x4 : vp9t_scan_default_4x4)
         : ts == 1 ? (txtp == 1 ? vp9t_scan_col_8x8 : txtp == 2 ? vp9t_scan_row_8x8 : vp9t_scan_default_8x8)
         : ts == 2 ? (txtp == 1 ? vp9t_scan_col_16x16 : txtp == 2 ? vp9t_scan_row_16x16 : vp9t_scan_default_16x16)
         : vp9t_scan_default_32x32;
}

template <int N> DEV void store_col(int16_t *dst, const int (&r)[N])
{
    uint32_t w[N / 2];
#pragma unroll
    for (int k = 0; k < N / 2; k++) w[k] = ((uint32_t) r[2 * k] & 0xffff) | ((uint32_t) r[2 * k + 1] << 16);
    if (N == 4) *(uint2 *) dst = make_uint2(w[0], w[1]);
    else
#pragma unroll
        for (int k = 0; k < N / 8; k++) ((uint4 *) dst)[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
}

// LDS row stride (coefficients) of an N x N block: padded so that the transposed store
// (lane li writes row li) spreads over the banks: an odd number of dwords per row
template <int N, typename COEF> struct RStride { static constexpr int S = N + (sizeof(COEF) == 2 ? 2 : 1); };
// LDS coefficients of one residual wave: 64 / N blocks of N rows
template <int N, typename COEF> struct RWave { static constexpr int E = (64 / N) * N * RStride<N, COEF>::S; };

// One wave of residual work: jobs [wj * 64/N, (wj + 1) * 64/N) of `jobs`, n lanes per
// job; cbw = the wave's LDS block (RWave<N, COEF>::E coefficients, rows padded to S).
// PREQ: in-place jobs load their prediction pixels before the transform (the inter
// launches); the keyframe launches (k_resid_dev) write scratch and keep their registers:
// they run beside the other slot's k_plf chains, whose co-resident waves the extra
// registers cost (r04's PREQ everywhere: C3 10,245 -> 9,863 fps on one box, profiles/r05b).
template <int N, int TCODE, typename PIX, class M, typename COEF, bool PREQ = true>
DEV void resid_wave(const RJob *__restrict__ jobs, int njobs, int wj, int lane, const FrameDesc *__restrict__ frames,
                    const COEF *__restrict__ coefs, int16_t *__restrict__ resid, COEF *cbw)
{
    typedef typename M::T T;
    constexpr int CAP = 64 / N;
    constexpr int LG = N == 4 ? 2 : N == 8 ? 3 : N == 16 ? 4 : 5;
    constexpr int TS = LG - 2;
    constexpr int BITS = N == 32 ? 6 : TS + 4;
    constexpr int S = RStride<N, COEF>::S;
    const int grp = lane >> LG, li = lane & (N - 1);
    const int j = wj * CAP + grp;
    const bool act = j < njobs;
    COEF *cb = cbw + grp * N * S;

    RJob r;
    if (act) r = jobs[j];
    else { r.coef = 0; r.dst = 0; r.eob = 0; r.frame = 0; r.ptx = 0; r.nzc = 1; r.nzr = 1; }
    const int eob = r.eob, txtp = TCODE == 3 || TCODE == 4 ? 0 : RJ_TXTP(r);
    const int nzc = TCODE == 4 ? 4 : r.nzc, nzr = TCODE == 4 ? 4 : r.nzr;   // the WHT reads every row
    const COEF *src = coefs + r.coef;
    const bool dconly = TCODE != 4 && act && eob == 1 && txtp == 0;
    const bool full = act && !dconly;
    // in place (inter residuals, N <= 16): the destination column's prediction pixels are
    // loaded here, under the coefficient loads and the transform, not after it (one global
    // round trip less on the wave's chain; 32-point columns keep the late load: registers)
    constexpr bool PRE = PREQ && N <= 16;
    int pq[PRE ? N : 1];
    PIX *q = nullptr;
    size_t qp = 0;
    if (act && RJ_INPLACE(r)) {
        const FrameDesc &fd = frames[r.frame];
        const int p = RJ_PLANE(r);
        q = (PIX *) fd.plane[p] + r.dst + li;
        qp = (size_t) fd.pitch[p ? 1 : 0];
        if (PRE) {
#pragma unroll
            for (int k = 0; k < (PRE ? N : 1); k++) pq[k] = q[k * qp];
        }
    }

    // zero the nonzero bounding box, then scatter scan-order coefficients
    if (full)
        for (int k = 0; k < nzr; k++) cb[k * S + li] = 0;
    wave_sync();
    if (full) {
        const int16_t *scan = scan_for(TCODE, txtp);
        for (int k0 = 0; k0 < eob; k0 += 8 * N) {
            COEF c[8];
            int pos[8];
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const int k = k0 + li + u * N;
                if (k < eob) { c[u] = src[k]; pos[u] = scan[k]; pos[u] += (pos[u] >> LG) * (S - N); }
            }
#pragma unroll
            for (int u = 0; u < 8; u++)
                if (k0 + li + u * N < eob) cb[pos[u]] = c[u];
        }
    }
    wave_sync();

    int res[N];
    if (TCODE == 4) {
        // lossless WHT (vp9dsp_template.c:1719-1750); in-place transpose through LDS
        int32_t v[4];
        if (full) for (int k = 0; k < 4; k++) v[k] = cb[k * S + li];
        wave_sync();
        if (full) { iwht4(v, 0); for (int k = 0; k < 4; k++) cb[li * S + k] = (COEF) v[k]; }
        wave_sync();
        if (full) { for (int k = 0; k < 4; k++) v[k] = cb[k * S + li]; iwht4(v, 1); }
#pragma unroll
        for (int k = 0; k < N; k++) res[k] = full ? (int) (COEF) v[k & 3] : 0;
    } else {
        T v[N];
        // column pass (type_a): lane c < nzc transforms column c into row c
        const bool colp = full && li < nzc;
#pragma unroll
        for (int k = 0; k < N; k++) v[k] = colp && k < nzr ? M::in(cb[k * S + li]) : (T) 0;
        wave_sync();
        if (colp) {
            tx1n<N, M>(v, txtp & 1);
#pragma unroll
            for (int k = 0; k < N; k++) cb[li * S + k] = (COEF) (int64_t) v[k];
        }
        wave_sync();
        // row pass (type_b): lane i transforms column i of the transposed block
        if (full) {
#pragma unroll
            for (int k = 0; k < N; k++) v[k] = k < nzc ? M::in(cb[k * S + li]) : (T) 0;
            tx1n<N, M>(v, txtp >> 1);
#pragma unroll
            for (int k = 0; k < N; k++) {
                const int32_t ov = (COEF) (int64_t) v[k];
                res[k] = (int32_t) ((uint32_t) ov + (1u << (BITS - 1))) >> BITS;
            }
        } else {
            // DC-only shortcut (vp9dsp_template.c:1165-1178)
            int add = 0;
            if (dconly) {
                const T t1 = M::r14(M::in((int32_t) src[0]) * (T) 11585);
                const int32_t tdc = (int32_t) M::r14(t1 * (T) 11585);
                add = (int32_t) ((uint32_t) tdc + (1u << (BITS - 1))) >> BITS;
            }
#pragma unroll
            for (int k = 0; k < N; k++) res[k] = add;
        }
    }
    if (!act) return;
    if (RJ_INPLACE(r)) {
        const int bd = frames[r.frame].bd;
#pragma unroll
        for (int k = 0; k < N; k++) {
            const int pv = PRE ? pq[PRE ? k : 0] : (int) q[k * qp];
            q[k * qp] = (PIX) clipbd(pv + res[k], bd);
        }
    } else {
#pragma unroll
        for (int k = 0; k < N; k++) res[k] = res[k] < -32768 ? -32768 : res[k] > 32767 ? 32767 : res[k];
        store_col<N>(resid + (size_t) r.dst * 16 + li * N, res);
    }
}

template <int N, int TCODE, typename PIX, class M, typename COEF>
__global__ __launch_bounds__(64 * RWAVES) void k_resid(const RJob *__restrict__ jobs, int njobs,
                                                       const FrameDesc *__restrict__ frames,
                                                       const COEF *__restrict__ coefs, int16_t *__restrict__ resid)
{
    __shared__ COEF cbs[RWAVES][RWave<N, COEF>::E];
    const int wave = threadIdx.x >> 6;
    resid_wave<N, TCODE, PIX, M, COEF>(jobs, njobs, blockIdx.x * RWAVES + wave, threadIdx.x & 63, frames, coefs, resid,
                                       cbs[wave]);
}

// k_resid of a launch list fixed at staging (runtime "static plan"): the job range comes
// from the planner's summary in HBM (rng = {first, end}); the grid is sized from a staged
// bound on the range (every tx block of the coded blocks), so one wave per 64 / N jobs as
// in k_resid, the waves past the range returning at once (a strided loop here costs 15-20
// VGPRs and measurably slower launches beside the other frame group's).
template <int N, int TCODE, typename PIX, class M, typename COEF>
__global__ __launch_bounds__(64 * RWAVES) void k_resid_dev(const RJob *__restrict__ jobs, const uint32_t *__restrict__ rng,
                                                           const FrameDesc *__restrict__ frames,
                                                           const COEF *__restrict__ coefs, int16_t *__restrict__ resid)
{
    __shared__ COEF cbs[RWAVES][RWave<N, COEF>::E];
    constexpr int CAP = 64 / N;
    const uint32_t j0 = __builtin_amdgcn_readfirstlane(rng[0]), j1 = __builtin_amdgcn_readfirstlane(rng[1]);
    const int njobs = j1 > j0 ? (int) (j1 - j0) : 0;
    const int wave = threadIdx.x >> 6, wj = (int) blockIdx.x * RWAVES + wave;
    if (wj * CAP >= njobs) return;
    resid_wave<N, TCODE, PIX, M, COEF, false>(jobs + j0, njobs, wj, threadIdx.x & 63, frames, coefs, resid, cbs[wave]);
}

// Every transform size of a phase in ONE launch (narrow, level-scheduled phases: the chain
// positions of inter streams, whose launches are latency-bound): waves [w0[t], w0[t + 1])
// run tx code t's jobs, each wave with an LDS block sized for the largest transform. The
// five per-size launches ran one after another on the phase's stream.
struct ResidMulti { uint32_t off[5], n[5], w0[6]; };
template <typename PIX, class M, typename COEF>
__global__ __launch_bounds__(64 * RWAVES) void k_resid_multi(ResidMulti a, const RJob *__restrict__ jobs,
                                                             const FrameDesc *__restrict__ frames,
                                                             const COEF *__restrict__ coefs, int16_t *__restrict__ resid)
{
    constexpr int E = RWave<32, COEF>::E > RWave<16, COEF>::E ? RWave<32, COEF>::E : RWave<16, COEF>::E;
    static_assert(E >= RWave<8, COEF>::E && E >= RWave<4, COEF>::E, "LDS block of the largest transform");
    __shared__ COEF cbs[RWAVES][E];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t gw = blockIdx.x * RWAVES + wave;
    if (gw >= a.w0[5]) return;
    int t = 0;
#pragma unroll
    for (int k = 1; k < 5; k++) t += gw >= a.w0[k];
    const int wj = (int) (gw - a.w0[t]);
    const RJob *j = jobs + a.off[t];
    const int n = (int) a.n[t];
    switch (t) {
    case 0: resid_wave<4, 0, PIX, M, COEF>(j, n, wj, lane, frames, coefs, resid, cbs[wave]); break;
    case 1: resid_wave<8, 1, PIX, M, COEF>(j, n, wj, lane, frames, coefs, resid, cbs[wave]); break;
    case 2: resid_wave<16, 2, PIX, M, COEF>(j, n, wj, lane, frames, coefs, resid, cbs[wave]); break;
    case 3: resid_wave<32, 3, PIX, M, COEF>(j, n, wj, lane, frames, coefs, resid, cbs[wave]); break;
    default: resid_wave<4, 4, PIX, M, COEF>(j, n, wj, lane, frames, coefs, resid, cbs[wave]); break;
    }
}

// ------------------------------------------------------------- k_pred
// One wavefront predicts one 64x64 superblock (luma + 4:2:0 chroma) in LDS. The host
// packs the SB's intra tx blocks into passes of independent jobs of one size (same
// dependency level): 64/n jobs side by side, n lanes per job, lane = pixel column.
// A pass is branch-free: edges are filled from host-resolved clamps (check_intra_mode,
// vp9recon.c:37-221), every predictor pixel is one formula-table word
// (vp9dsp_template.c:28-1106 restated per pixel), then + residual from k_resid, clip.
// A tile's row 0 / column 0 hold the pixels above / left of the SB; pixel (x, y) of
// plane p lives at tile_p[(y + 1) * pitch_p + x + PX0]: pixel rows start 4-pixel aligned,
// so the SB interior moves between LDS and HBM in 16-byte chunks.
#ifndef PRED_LTAB_LDS
#define PRED_LTAB_LDS 1       // 4x4 / 8x8 formula words: LDS copy (1) or the global table via L1 (0)
#endif
#ifndef PRED_ABL
#define PRED_ABL 0            // timing-only ablations of a pass (build flag, tools/ablate.sh): 8 no
                              // predictor rows, 16 no edge writes (frames are then wrong)
#endif
#define LP 68            // luma tile pitch (17 dwords at 8-bit: column reads are bank-conflict free)
#define PX0 4            // tile column of pixel x = 0 (x = -1 at column 3)
#define LT_SIZE (65 * LP)
// chroma tile geometry of a subsampling (4:2:0 = Geo<1, 1>): CW x CH pixels per SB,
// tile pitch CP, CT elements per chroma tile, TILE elements per SB (Y, U, V)
template <int SSH, int SSV> struct Geo {
    static constexpr int SH = SSH, SV = SSV;
    static constexpr int CW = 64 >> SSH, CH = 64 >> SSV, CP = CW + PX0, CT = (CH + 1) * CP;
    static constexpr int TILE = LT_SIZE + 2 * CT;
};
typedef Geo<1, 1> G420;

// Lane map of a mixed pass (pass word: first << 14 | c4 << 9 | c8 << 5 | c16 << 2 | c32):
// lanes [0, 32 c32) serve 32x32 jobs, then 16x16, 8x8, 4x4 -- every group aligned to its
// size n, one lane per pixel column.
struct LaneMap { int ts, li, jidx, gstart; bool act; };
DEV LaneMap lane_map(uint32_t w, int lane)
{
    const int c32 = w & 3, c16 = (w >> 2) & 7, c8 = (w >> 5) & 15, c4 = (w >> 9) & 31;
    const int b32 = 32 * c32, b16 = b32 + 16 * c16, b8 = b16 + 8 * c8, b4 = b8 + 4 * c4;
    LaneMap m;
    const int ts = lane < b32 ? 3 : lane < b16 ? 2 : lane < b8 ? 1 : 0;
    const int base = ts == 3 ? 0 : ts == 2 ? b32 : ts == 1 ? b16 : b8;
    const int j0 = ts == 3 ? 0 : ts == 2 ? c32 : ts == 1 ? c32 + c16 : c32 + c16 + c8;
    const int lg = ts + 2, rel = lane - base;
    m.ts = ts;
    m.li = rel & ((1 << lg) - 1);
    m.jidx = j0 + (rel >> lg);
    m.gstart = lane - m.li;
    m.act = lane < b4;
    if (!m.act) m.jidx = 0;
    return m;
}
#define PASS_FIRST_M(w) ((w) >> 14)
#define PASS_MAXN(w) (((w) & 3) ? 32 : (((w) >> 2) & 7) ? 16 : (((w) >> 5) & 15) ? 8 : 4)

// Prefetched per-lane inputs of one pass: the lane's job record and the first 8 rows
// of its residual column (named fields, so the set stays in registers). The job records
// (global, L1/L2) are read two passes ahead, the residual rows (whose address needs the
// job record) one pass ahead; every load is unconditional (clamped pass index), so no
// control-flow join forces an early s_waitcnt.
struct PSet { uint32_t ja, jr; uint4 r0; };
struct JSet { uint32_t ja, jr, lt; };     // job record + (li | ts << 8) of the lane
DEV uint32_t pr_word(const PSet &s, int k)
{
    return k == 0 ? s.r0.x : k == 1 ? s.r0.y : k == 2 ? s.r0.z : s.r0.w;
}

DEV void load_job(uint32_t w, int lane, const PJob *__restrict__ lj, JSet &j)
{
    const LaneMap m = lane_map(w, lane);
    const PJob jb = lj[PASS_FIRST_M(w) + m.jidx];
    j.ja = jb.a;
    j.jr = jb.roff;
    j.lt = (uint32_t) m.li | (uint32_t) m.ts << 8;
}

DEV void load_resid(const JSet &j, const int16_t *__restrict__ resid, PSet &ps)
{
    ps.ja = j.ja;
    ps.jr = j.jr;
    const uint32_t li = j.lt & 255, ts = j.lt >> 8;
    ps.r0 = *(const uint4 *) (resid + (((j.ja >> 4) & 1) ? (size_t) j.jr * 16 + (li << (ts + 2)) : 0));
}

// Load the pixels above / left of an SB (and, for inter frames, its interior: the
// MC prediction + inter residuals) into the LDS tile. All global loads of a batch are
// issued before any LDS write so their latencies overlap.
// 16-byte chunks between global memory and an LDS tile (16 pixels at 8-bit, 8 at 16-bit):
// one dwordx4 load / store each, 16-byte aligned in the frame buffer
struct Chunk16 {
    typedef uint4 T;
    static DEV T zero() { return make_uint4(0, 0, 0, 0); }
    static DEV void to_lds(T v, void *t)
    {
        uint32_t *d = (uint32_t *) t;
        d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
    }
    static DEV T from_lds(const void *t)
    {
        const uint32_t *s = (const uint32_t *) t;
        return make_uint4(s[0], s[1], s[2], s[3]);
    }
};

// The SB interior (all planes) between HBM and the LDS tile in 16-byte chunks (16 px at
// 8-bit, 8 at 16-bit): STORE = false loads (inter frames: MC prediction + inter residuals),
// true stores the reconstructed SB. All loads of a lane are issued before its LDS writes.
typedef __attribute__((address_space(1))) uint64_t gpx64;
// SC (stores only): written through with sc1 (intra workers inside k_lfro: its loader on
// another XCD reads them in the same launch)
template <typename PIX, class G, bool STORE, bool SC = false>
DEV void sb_interior(const FrameDesc &fd, int sbx, int sby, int lane, PIX *tile)
{
    constexpr int CPX = 16 / sizeof(PIX);
    constexpr int YK = 64 / CPX, CKX = G::CW / CPX;              // chunks per row
    constexpr int NY = 64 * YK, NC = G::CH * CKX, NT = NY + 2 * NC;
    constexpr int NB = 2;                                         // 16-byte loads in flight per lane (VGPR budget)
    auto where = [&](int c, PIX *&g, PIX *&t) {
        int p, r, k;
        if (c < NY) { p = 0; r = c / YK; k = c - r * YK; }
        else { const int cc = c - NY; p = 1 + (cc >= NC); const int q = cc - (p - 1) * NC; r = q / CKX; k = q - r * CKX; }
        g = (PIX *) fd.plane[p] + (size_t) ((p ? sby * G::CH : sby * 64) + r) * fd.pitch[p ? 1 : 0] +
            (p ? sbx * G::CW : sbx * 64) + k * CPX;
        t = tile + (p == 0 ? 0 : p == 1 ? LT_SIZE : LT_SIZE + G::CT) + (r + 1) * (p ? G::CP : LP) + PX0 + k * CPX;
    };
#pragma unroll 1
    for (int c0 = 0; c0 < NT; c0 += 64 * NB) {
        uint4 v[NB];
#pragma unroll
        for (int u = 0; u < NB; u++) {
            const int c = c0 + lane + 64 * u;
            if (c >= NT) break;
            PIX *g, *t;
            where(c, g, t);
            if (STORE && SC) {
                const uint4 w = Chunk16::from_lds(t);
                __hip_atomic_store((gpx64 *) g, (uint64_t) w.x | (uint64_t) w.y << 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store((gpx64 *) g + 1, (uint64_t) w.z | (uint64_t) w.w << 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else if (STORE) {
                *(uint4 *) g = Chunk16::from_lds(t);
            } else {
                v[u] = *(const uint4 *) g;
            }
        }
        if (STORE) continue;
#pragma unroll
        for (int u = 0; u < NB; u++) {
            const int c = c0 + lane + 64 * u;
            if (c >= NT) break;
            PIX *g, *t;
            where(c, g, t);
            Chunk16::to_lds(v[u], t);
        }
    }
}

// Pixel loads / stores of the intra hand-off inside one k_predd launch: sc1 (agent scope), so
// a workgroup on another XCD reads what the producer wrote through, without an L2 write-back
// or invalidate (the k_lfro row hand-off's protocol). SC = false: plain.
typedef __attribute__((address_space(1))) uint8_t gpx8;
typedef __attribute__((address_space(1))) uint16_t gpx16;
template <bool SC, typename PIX> DEV PIX ld_px(const PIX *p)
{
    if constexpr (!SC) return *p;
    else if constexpr (sizeof(PIX) == 1) return __hip_atomic_load((gpx8 *) p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return __hip_atomic_load((gpx16 *) p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <bool SC, typename PIX> DEV void st_px(PIX *p, PIX v)
{
    if constexpr (!SC) *p = v;
    else if constexpr (sizeof(PIX) == 1) __hip_atomic_store((gpx8 *) p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else __hip_atomic_store((gpx16 *) p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// SC: the halo (the row above, the left column) with sc1 loads (k_predd; 4:2:0)
template <typename PIX, class G, bool SC = false>
DEV void load_sb_tile(const FrameDesc &fd, int sbx, int sby, bool interior, int lane, PIX *tile)
{
    if (G::SH != 1 || G::SV != 1) {
        // 4:2:2 / 4:4:0 / 4:4:4: plain loops (same tile layout, chroma CW x CH)
        const int lx = sbx * 64, ly = sby * 64, cx = sbx * G::CW, cy = sby * G::CH;
        const int py = fd.pitch[0], pc = fd.pitch[1];
        for (int p = 0; p < 3; p++) {
            const PIX *g = (const PIX *) fd.plane[p];
            const int pitch = p ? pc : py, x0 = p ? cx : lx, y0 = p ? cy : ly;
            const int w = p ? G::CW : 64, h = p ? G::CH : 64, tp = p ? G::CP : LP;
            PIX *t = tile + (p == 0 ? 0 : p == 1 ? LT_SIZE : LT_SIZE + G::CT);
            if (y0 > 0)
                for (int i = lane; i <= w; i += 64) t[i + PX0 - 1] = x0 - 1 + i >= 0 ? g[(size_t) (y0 - 1) * pitch + x0 - 1 + i] : 0;
            if (x0 > 0)
                for (int i = lane; i < h; i += 64) t[(i + 1) * tp + PX0 - 1] = g[(size_t) (y0 + i) * pitch + x0 - 1];
        }
        if (interior) sb_interior<PIX, G, false>(fd, sbx, sby, lane, tile);
        return;
    }
    constexpr int CP = G::CP, CT_SIZE = G::CT;
    const PIX *gy = (const PIX *) fd.plane[0], *gu = (const PIX *) fd.plane[1], *gv = (const PIX *) fd.plane[2];
    const int py = fd.pitch[0], pc = fd.pitch[1];
    const int lx = sbx * 64, ly = sby * 64, cx = sbx * 32, cy = sby * 32;
    // lanes 0..32 read U top x = -1..31, lanes 33..63 V top x = -1..29, lanes 0..1 V x = 30..31
    PIX v0 = 0, v1 = 0, v2 = 0, v3 = 0, v4 = 0, v5 = 0;
    const bool top = ly > 0, left = lx > 0;
    const PIX *gc = lane < 33 ? gu : gv;
    const int ci = lane < 33 ? lane : lane - 33;
    if (top) {
        if (lx - 1 + lane >= 0) v0 = ld_px<SC>(gy + (size_t) (ly - 1) * py + lx - 1 + lane);
        if (lane == 0) v4 = ld_px<SC>(gy + (size_t) (ly - 1) * py + lx + 63);
        if (cx - 1 + ci >= 0) v2 = ld_px<SC>(gc + (size_t) (cy - 1) * pc + cx - 1 + ci);
        if (lane < 2) v5 = ld_px<SC>(gv + (size_t) (cy - 1) * pc + cx + 30 + lane);
    }
    if (left && fd.edge) {
        // the left SB's right column as its intra workgroup saved it (FrameDesc.edge):
        // two 64-pixel runs instead of 128 one-pixel frame rows
        const PIX *e = (const PIX *) fd.edge + (size_t) (sby * fd.sb_cols + sbx - 1) * EDGE_PIX;
        v1 = ld_px<SC>(e + lane);
        v3 = ld_px<SC>(e + 64 + lane);
    } else if (left) {
        v1 = ld_px<SC>(gy + (size_t) (ly + lane) * py + lx - 1);
        v3 = ld_px<SC>((lane < 32 ? gu : gv) + (size_t) (cy + (lane & 31)) * pc + cx - 1);
    }
    PIX *tu = tile + LT_SIZE, *tv = tile + LT_SIZE + CT_SIZE;
    if (top) {
        tile[PX0 - 1 + lane] = v0;
        if (lane == 0) tile[PX0 + 63] = v4;
        (lane < 33 ? tu : tv)[PX0 - 1 + ci] = v2;
        if (lane < 2) tv[PX0 + 30 + lane] = v5;
    }
    if (left) { tile[(lane + 1) * LP + PX0 - 1] = v1; (lane < 32 ? tu : tv)[((lane & 31) + 1) * CP + PX0 - 1] = v3; }
    if (interior) sb_interior<PIX, G, false>(fd, sbx, sby, lane, tile);
}

// one predictor pixel from its formula word and the three edge values it names
DEV int pix_formula_apply(uint32_t fw, int a, int b, int c, int mx)
{
    const int wb = (fw >> 24) & 3, s = (fw >> 28) & 3, rnd = fw >> 30;
    const int wc = __builtin_amdgcn_sbfe((int) fw, 26, 2);
    return med3_0(((a + rnd) + wb * b + wc * c) >> s, mx);
}

// The rows of a pass of 4x4 / 8x8 jobs. The edge array and the tile are disjoint LDS
// (restrict): the compiler issues the edge reads of every row before the first tile store,
// one LDS round trip for the column; inline in pred_pass each row's reads waited for the
// previous row's store (C2 k_plf 4.10 -> 3.99 ms, C3 6.62 -> 6.50 ms per step, profiles/r05l).
template <int N, typename PIX>
DEV void pass_rows(const char *__restrict__ e8, PIX *__restrict__ o, int tpch, int li, int n, int mx, int hr,
                   const uint32_t (&f)[N], const PSet &ps)
{
#pragma unroll
    for (int y = 0; y < N; y++) {
        if (N > 4 && y >= n) continue;
        const uint32_t fw = f[y];
        const int a = *(const uint16_t *) (e8 + (fw & 255)), b = *(const uint16_t *) (e8 + ((fw >> 8) & 255)),
                  c = *(const uint16_t *) (e8 + ((fw >> 16) & 255));
        int v = pix_formula_apply(fw, a, b, c, mx);
        const int r = (int) (int16_t) (pr_word(ps, y >> 1) >> ((y & 1) * 16));
        v = med3_0(v + (hr ? r : 0), mx);
        o[y * tpch + li] = (PIX) v;
    }
}

// One mixed pass: lane li of an n x n job predicts pixel column li (rows 0..n-1); the
// row loop runs to the pass's largest n (MAXN, unrolled), rows >= n are masked.
// pf() issues the next passes' global prefetches: after this pass's own global loads, so
// that waiting for those (vmcnt counts in issue order) never waits for the prefetches.
typedef __attribute__((address_space(3))) const uint32_t lds_u32;
typedef __attribute__((address_space(1))) const uint32_t glb_u32;
template <int MAXN, typename PIX, class G, class PF>
DEV void pred_pass(uint32_t w, int lane, PIX *tile, uint16_t *eb, int bd, const PSet &ps, const uint32_t *ltab,
                   const int16_t *__restrict__ resid, const uint32_t *__restrict__ ptab, int dbg, PF &&pf)
{
    const LaneMap m = lane_map(w, lane);
    PJob jb;
    jb.a = ps.ja;
    jb.roff = ps.jr;
    const int ts = m.ts, n = 4 << ts, li = m.li;
    const bool act = m.act;
    const int p = PJ_PLANE(jb);
    const int tpch = p ? G::CP : LP;
    PIX *o = tile + PJ_SLOT(jb) * G::TILE + (p == 0 ? 0 : p == 1 ? LT_SIZE : LT_SIZE + G::CT) +
             (PJ_Y4(jb) * 4 + 1) * tpch + PJ_X4(jb) * 4 + PX0;
    const int ms = PJ_MSLOT(jb), slot = ms < 9 ? ms : 9;
    const int toff = ts == 3 ? 336 : (int) __builtin_amdgcn_ubfe(16u << 10 | 80u << 20, 10 * ts, 10);
    // formula words of this column: rows of 4x4 / 8x8 from the LDS copy, larger from L1/L2.
    // Rows 0-7 here; rows >= 8 of 16x16 / 32x32 (formula + residual words) per 8-row chunk,
    // one chunk ahead, so at most two chunks are live
    constexpr int F0 = MAXN < 8 ? MAXN : 8;
    uint32_t f[F0];
    // passes of 4x4 / 8x8 jobs read the LDS copy, passes with a 16 / 32 job the global table
    // for every job (explicit address spaces: a per-lane choice between the two was a flat
    // pointer, and a flat load's wait covers every outstanding load, the prefetches included)
    lds_u32 *ftl = (lds_u32 *) (ltab + slot * 80 + toff + li);
    glb_u32 *ftg = (glb_u32 *) (ptab + slot * PTAB_SLOT + toff + li);
    auto fword = [&](int row) -> uint32_t { return PRED_LTAB_LDS && MAXN <= 8 ? ftl[row * n] : ftg[row * n]; };
#pragma unroll
    for (int y = 0; y < F0; y++) f[y] = fword(y < n ? y : 0);
    const uint32_t *rr = (const uint32_t *) (resid + (PJ_RES(jb) && ts >= 2 ? (size_t) jb.roff * 16 + li * n : 0));
    uint32_t fa[8], ra[4], fb[8], rb[4];
    if (MAXN > 8) {
#pragma unroll
        for (int y = 0; y < 8; y++) fa[y] = fword(8 + y < n ? 8 + y : 0);
#pragma unroll
        for (int k = 0; k < 4; k++) ra[k] = rr[4 + k < n / 2 ? 4 + k : 0];
    }
    pf();

    // edges (fills: vp9recon.c:103-210): every load hits a valid tile address, the
    // host-resolved availability selects between pixel and fill value (no branches)
    const int base = 128 << (bd - 8);
    const int htop = PJ_HTOP(jb), hleft = PJ_HLEFT(jb), ct = PJ_CT(jb), cl = PJ_CL(jb);
    const PIX *orow = o - tpch;
    const int t_px = orow[li < ct ? li : ct];
    const int l_px = o[(n - 1 - li < cl ? n - 1 - li : cl) * tpch - 1];
    const int tl_px = orow[-1];
    const int tr_px = orow[PJ_TRREAL(jb) ? 4 + li : ct];
    const int tv = htop ? t_px : base - 1;
    const int lv = hleft ? l_px : base + 1;
    const int tl = (hleft & htop) ? tl_px : base + (htop ? 1 : -1);
    const int tr = htop ? tr_px : base - 1;
    uint16_t *e = eb + 2 * m.gstart + 10 * m.jidx;  // 2n + 10 entries per job: n + 5 dwords, odd
    if (act && !(PRED_ABL & 16)) {
        e[li] = (uint16_t) lv;
        e[n + 1 + li] = (uint16_t) tv;
        if (ts == 0) e[n + 5 + li] = (uint16_t) tr;
        e[n] = (uint16_t) tl;                  // every lane of the group writes the same value
    }
    // DC family: sums over the job's n lanes (only when the pass holds a DC / LEFT_DC /
    // TOP_DC job), the value stored at edge index 2n + 7 for the formula table's copy
    int dc = ms == 12 ? base : ms == 13 ? base - 1 : base + 1;
    if (__any(act && ms >= 9 && ms <= 11)) {
        int sl = lv, st = tv;
#pragma unroll
        for (int k = 1; k < MAXN; k <<= 1) {
            const int a = __shfl_xor(sl, k), b = __shfl_xor(st, k);
            if (k < n) { sl += a; st += b; }
        }
        const int d9 = (sl + st + n) >> (ts + 3), d10 = (sl + (n >> 1)) >> (ts + 2), d11 = (st + (n >> 1)) >> (ts + 2);
        dc = ms == 9 ? d9 : ms == 10 ? d10 : ms == 11 ? d11 : dc;
    }
    if (act && ms >= 9 && li == 0 && !(PRED_ABL & 16)) e[2 * n + 7] = (uint16_t) dc;
    wave_sync();
    if (act && !(PRED_ABL & 8)) {
        const int mx = (1 << bd) - 1;
        const int hr = PJ_RES(jb);
        if constexpr (MAXN <= 8) {
            pass_rows<MAXN, PIX>((const char *) e, o, tpch, li, n, mx, hr, f, ps);
            return;
        }
        const char *e8 = (const char *) e;
#pragma unroll
        for (int y = 0; y < MAXN; y++) {
            if (MAXN > 8 && (y & 7) == 0 && y >= 8 && y + 8 < MAXN) {   // prefetch the chunk after this one
                uint32_t *fn = ((y >> 3) & 1) ? fb : fa, *rn = ((y >> 3) & 1) ? rb : ra;
#pragma unroll
                for (int k = 0; k < 8; k++) fn[k] = fword(y + 8 + k < n ? y + 8 + k : 0);
#pragma unroll
                for (int k = 0; k < 4; k++) rn[k] = rr[(y + 8) / 2 + k < n / 2 ? (y + 8) / 2 + k : 0];
            }
            if (y >= n) continue;
            const uint32_t fw = y < 8 ? f[y < F0 ? y : 0] : ((y >> 3) & 1) ? fa[y & 7] : fb[y & 7];
            const int a = *(const uint16_t *) (e8 + (fw & 255)), b = *(const uint16_t *) (e8 + ((fw >> 8) & 255)),
                      c = *(const uint16_t *) (e8 + ((fw >> 16) & 255));
            int v = pix_formula_apply(fw, a, b, c, mx);
            const uint32_t rw = y < 8 ? pr_word(ps, y >> 1) : ((y >> 3) & 1) ? ra[(y >> 1) & 3] : rb[(y >> 1) & 3];
            const int r = (int) (int16_t) (rw >> ((y & 1) * 16));
            v = med3_0(v + (hr ? r : 0), mx);
            o[y * tpch + li] = (PIX) v;
        }
    }
}

template <typename PIX, class G, class PF>
DEV void run_pass(uint32_t w, int lane, PIX *tile, uint16_t *eb, int bd, const PSet &ps, const uint32_t *ltab,
                  const int16_t *__restrict__ resid, const uint32_t *__restrict__ ptab, int dbg, PF &&pf)
{
    switch (PASS_MAXN(w)) {
    case 4: pred_pass<4, PIX, G>(w, lane, tile, eb, bd, ps, ltab, resid, ptab, dbg, pf); break;
    case 8: pred_pass<8, PIX, G>(w, lane, tile, eb, bd, ps, ltab, resid, ptab, dbg, pf); break;
    case 16: pred_pass<16, PIX, G>(w, lane, tile, eb, bd, ps, ltab, resid, ptab, dbg, pf); break;
    default: pred_pass<32, PIX, G>(w, lane, tile, eb, bd, ps, ltab, resid, ptab, dbg, pf); break;
    }
    wave_sync();
}

// The intra wave's job records and pass words, copied to LDS in the prologue (k_pred, 4:2:0):
// a pass then finds its job records by an LDS read instead of a global load whose address
// waited on another global load (the pass word), so only the residual loads are global in
// the pass chain. JL = the planner's job cap per SB (4x4 units of all planes, vp9hip_plan.hip
// JCAP). Measured (profiles/r05d): C2 11,808 -> 12,018 fps; in k_plf the extra 4.6 KB of LDS
// (10.8 -> 15.2 KB per workgroup of the fused launch) cost more than it saved (C3 10,219 ->
// 9,797 fps, k_plf 7.27 -> 7.69 ms per step), so k_plf keeps the global lists.
template <class G, bool LISTS> struct PredLists {
    static constexpr bool ON = LISTS && G::SH == 1 && G::SV == 1;
    static constexpr int JL = 256 + 2 * (16 >> G::SH) * (16 >> G::SV);
    static constexpr int N = ON ? JL : 1;
};
// LDS of one k_pred workgroup (one wavefront).
template <typename PIX, class G, bool LISTS> struct PredLds {
    PIX tile[PRED_K * G::TILE];
    uint16_t eb[288];                 // per job 2n+8 edge pixels at a pitch of 2n+10 (an odd dword
                                      // count: the jobs' arrays start in different banks)
#if PRED_LTAB_LDS
    uint32_t ltab[10 * 80];           // formula words of 4x4 and 8x8, all slots
#endif
    PJob jl[PredLists<G, LISTS>::N];  // job records (pass order)
    uint32_t pw[PredLists<G, LISTS>::N];   // pass words
};

template <typename PIX>
DEV void load_ltab(uint32_t *ltab, const uint32_t *__restrict__ ptab, int lane)
{
    uint32_t t[13];
#pragma unroll
    for (int u = 0; u < 13; u++) {
        const int i = lane + 64 * u;
        t[u] = i < 800 ? ptab[(i / 80) * PTAB_SLOT + i % 80] : 0;
    }
#pragma unroll
    for (int u = 0; u < 13; u++)
        if (lane + 64 * u < 800) ltab[lane + 64 * u] = t[u];
}

// PRED_PROF builds (profiling only, tools/pred_prof.py): lane 0 of each intra workgroup
// sums shader-clock cycles: [0] tile loads, [1] all passes, [2] interior stores, [3] passes,
// [4] workgroups, [5 + i] cycles and [9 + i] count of passes with MAXN = 4 << i; k_plf's LF
// workgroups: [13] cycles, [14] count; [15] the slowest intra workgroup's cycles
#ifndef PRED_PROF
#define PRED_PROF 0
#endif
KP_DEV unsigned long long pred_prof[16];
// Intra prediction of one workgroup record (the ltab copy must be loaded). HO (4:2:0): the
// halo loads are sc1, and 1 (k_predd): the SB's own right column / bottom row (what the SBs to
// the right and below read) are written through again; 2 (intra workers inside k_lfro): its
// whole interior is written through.
template <typename PIX, class G, bool LISTS, int HO = 0>
DEV void pred_wg(const WGRec *wgp, const SBRec *__restrict__ sbs, const PJob *__restrict__ jobs,
                 const uint32_t *__restrict__ passes, const FrameDesc *__restrict__ frames,
                 const int16_t *__restrict__ resid, const uint32_t *__restrict__ ptab, PredLds<PIX, G, LISTS> &S, int lane,
                 int dbg)
{
    PIX *tile = S.tile;
    uint16_t *eb = S.eb;
#if PRED_LTAB_LDS
    const uint32_t *ltab = S.ltab;
#else
    const uint32_t *ltab = nullptr;
#endif
    typedef PredLists<G, LISTS> PL;
    const uint32_t wjob0 = wgp->job0, wpass0 = wgp->pass0;
    const uint32_t wnjobs = PL::ON ? min((uint32_t) wgp->njobs, (uint32_t) PL::JL) : wgp->njobs;
    const uint32_t wnpass = PL::ON ? min((uint32_t) wgp->npass, wnjobs) : wgp->npass;
    const PJob *gj = jobs + wjob0;         // job records (global)
    const uint32_t *gp = passes + wpass0;  // pass words (global)
    const int bd = frames[sbs[wgp->sb[0]].frame].bd;
    uint64_t pp0 = PRED_PROF ? clock64() : 0, pp[13] = {0};

    // ---- prologue: job list, pass words, SB neighbourhoods (pre-LF pixels) ----
    constexpr int LU = PL::ON ? (PL::JL + 63) / 64 : 1;
    PJob lv[LU];
    uint32_t pv[LU];
    if (PL::ON) {                          // issued first: they land under the tile loads
#pragma unroll
        for (int u = 0; u < LU; u++) {
            const uint32_t i = (uint32_t) (lane + 64 * u);
            if (i < wnjobs) lv[u] = gj[i];
            if (i < wnpass) pv[u] = gp[i];
        }
    }
#pragma unroll 1
    for (int k = 0; k < PRED_K; k++) {
        const uint32_t sbi = __builtin_amdgcn_readfirstlane(wgp->sb[k]);
        if (sbi != 0xffffffffu) {
            const SBRec sb = sbs[sbi];
            if (!(dbg & 4)) load_sb_tile<PIX, G, HO != 0>(frames[sb.frame], sb.sbx, sb.sby, sb.flags & 1, lane, tile + k * G::TILE);
        }
    }
    if (PL::ON) {
#pragma unroll
        for (int u = 0; u < LU; u++) {
            const uint32_t i = (uint32_t) (lane + 64 * u);
            if (i < wnjobs) S.jl[i] = lv[u];
            if (i < wnpass) S.pw[i] = pv[u];
        }
    }
    const PJob *lj = PL::ON ? S.jl : gj;   // job records: read a pass ahead
    const uint32_t *lp = PL::ON ? S.pw : gp;   // pass words: wave-uniform
    wave_sync();
    if (PRED_PROF) { const uint64_t t = clock64(); pp[0] += t - pp0; pp0 = t; }

    // passes: residual sets A / B alternate (loop unrolled by two), job records J run a
    // pass ahead of them; pass words are wave-uniform scalar loads (index clamped)
    const int npass = (dbg & 1) ? 0 : wnpass;
    // pass words: wave-uniform; from the global list through the constant address space, so
    // they are scalar loads (a vector load of a uniform address was waited on at once)
    typedef __attribute__((address_space(4))) const uint32_t cst_u32;
    const cst_u32 *lpc = (const cst_u32 *) gp;
#define LPW(k) (PL::ON ? __builtin_amdgcn_readfirstlane(lp[(k) < npass ? (k) : npass - 1]) \
                       : lpc[(k) < npass ? (k) : npass - 1])
    if (npass) {
        PSet A, B;
        JSet J;
        // pass words one iteration ahead: this iteration's pair was read by the previous
        // one, the next pair (needed by this iteration's prefetches only) is read here
        uint32_t w0 = LPW(0), w1 = LPW(1);
        load_job(w0, lane, lj, J);
        load_resid(J, resid, A);
        load_job(w1, lane, lj, J);
        for (int pi = 0; pi < npass; pi += 2) {
            const uint32_t w2 = LPW(pi + 2), w3 = LPW(pi + 3);
            uint64_t tq = PRED_PROF ? clock64() : 0;
            run_pass<PIX, G>(w0, lane, tile, eb, bd, A, ltab, resid, ptab, dbg, [&] {
                load_resid(J, resid, B);
                load_job(w2, lane, lj, J);
            });
            if (PRED_PROF) {
                const uint64_t t = clock64();
                const int b = PASS_MAXN(w0) == 4 ? 0 : PASS_MAXN(w0) == 8 ? 1 : PASS_MAXN(w0) == 16 ? 2 : 3;
                pp[5 + b] += t - tq; pp[9 + b]++; tq = t;
            }
            if (pi + 1 >= npass) break;
            if (PRED_PROF) tq = clock64();
            run_pass<PIX, G>(w1, lane, tile, eb, bd, B, ltab, resid, ptab, dbg, [&] {
                load_resid(J, resid, A);
                load_job(w3, lane, lj, J);
            });
            if (PRED_PROF) {
                const uint64_t t = clock64();
                const int b = PASS_MAXN(w1) == 4 ? 0 : PASS_MAXN(w1) == 8 ? 1 : PASS_MAXN(w1) == 16 ? 2 : 3;
                pp[5 + b] += t - tq; pp[9 + b]++;
            }
            w0 = w2;
            w1 = w3;
        }
    }
#undef LPW
    if (PRED_PROF) { const uint64_t t = clock64(); pp[1] += t - pp0; pp0 = t; pp[3] = (uint64_t) npass; }

    // ---- store the SB interiors ----
    if (!(dbg & 2))
#pragma unroll 1
    for (int k = 0; k < PRED_K; k++) {
        const uint32_t sbi = __builtin_amdgcn_readfirstlane(wgp->sb[k]);
        if (sbi == 0xffffffffu) continue;
        const SBRec sb = sbs[sbi];
        const FrameDesc &fd = frames[sb.frame];
        sb_interior<PIX, G, true, HO == 2>(fd, sb.sbx, sb.sby, lane, tile + k * G::TILE);
        if constexpr (HO == 1) {       // right column and bottom row again, written through
            static_assert(G::SH == 1 && G::SV == 1, "k_predd: 4:2:0");
            const PIX *t = tile + k * G::TILE;
            PIX *gy = (PIX *) fd.plane[0];
            const int p = 1 + (lane >> 5), x = lane & 31;
            PIX *gc = (PIX *) fd.plane[p];
            const PIX *tc = t + (p == 1 ? LT_SIZE : LT_SIZE + G::CT);
            const size_t ly = (size_t) sb.sby * 64, cy = (size_t) sb.sby * 32;
            st_px<true>(gy + (ly + 63) * fd.pitch[0] + sb.sbx * 64 + lane, t[64 * LP + PX0 + lane]);
            st_px<true>(gy + (ly + lane) * fd.pitch[0] + sb.sbx * 64 + 63, t[(lane + 1) * LP + PX0 + 63]);
            st_px<true>(gc + (cy + 31) * fd.pitch[1] + sb.sbx * 32 + x, tc[32 * G::CP + PX0 + x]);
            st_px<true>(gc + (cy + x) * fd.pitch[1] + sb.sbx * 32 + 31, tc[(x + 1) * G::CP + PX0 + 31]);
        }
        if (fd.edge) {                 // the right column of each plane, for the SB to the right
            PIX *e = (PIX *) fd.edge + (size_t) (sb.sby * fd.sb_cols + sb.sbx) * EDGE_PIX;
            const PIX *t = tile + k * G::TILE;
#pragma unroll
            for (int i = lane; i < 64 + 2 * G::CH; i += 64) {
                const int p = i < 64 ? 0 : i < 64 + G::CH ? 1 : 2, r = p == 0 ? i : p == 1 ? i - 64 : i - 64 - G::CH;
                st_px<HO != 0>(e + i, t[(p == 0 ? 0 : p == 1 ? LT_SIZE : LT_SIZE + G::CT) + (r + 1) * (p ? G::CP : LP) + PX0 +
                                   (p ? G::CW : 64) - 1]);
            }
        }
    }
    if (PRED_PROF && lane == 0) {
        pp[2] += clock64() - pp0;
        pp[4] = 1;
        for (int i = 0; i < 13; i++) atomicAdd(&pred_prof[i], pp[i]);
        atomicMax(&pred_prof[15], pp[0] + pp[1] + pp[2]);    // the slowest intra workgroup
    }
}

template <typename PIX, class G>
__global__ __launch_bounds__(64) void k_pred(const uint32_t *__restrict__ list, const WGRec *__restrict__ wgs,
                                             const SBRec *__restrict__ sbs, const PJob *__restrict__ jobs,
                                             const uint32_t *__restrict__ passes, const FrameDesc *__restrict__ frames,
                                             const int16_t *__restrict__ resid, const uint32_t *__restrict__ ptab, int dbg)
{
    __shared__ PredLds<PIX, G, true> S;
#if PRED_LTAB_LDS
    load_ltab<PIX>(S.ltab, ptab, threadIdx.x);
#endif
    pred_wg<PIX, G, true>(wgs + list[blockIdx.x], sbs, jobs, passes, frames, resid, ptab, S, threadIdx.x, dbg);
}

// LF tile geometry. A tile row starts XL pixels left of the SB (16 at 8-bit, 8 at 16-bit,
// so chunks stay 16-byte aligned) and holds XL + 64 (luma) / XL + CW (chroma) pixels; the
// filters see x = -8 .. at offset XO = XL - 8. Rows: y = -8 .. 63 (luma) / CH - 1. Pitches
// in pixels, rows dword-aligned with an odd dword count (lanes of the column pass read
// dword i of consecutive rows: no bank conflicts).
template <typename PIX, class G> struct LfP {
    static constexpr int CPX = 16 / sizeof(PIX);    // pixels per chunk
    static constexpr int XL = CPX;                  // left halo loaded (8 used)
    static constexpr int XO = XL - 8;               // tile offset of x = -8
    static constexpr int YP = sizeof(PIX) == 1 ? 84 : 74;
    static constexpr int UVP = G::CW + XL + (sizeof(PIX) == 1 ? 4 : 2);
    static constexpr int PPW = 4 / sizeof(PIX);     // pixels per dword
    static constexpr int YK = (64 + XL) / CPX;      // chunks per luma tile row
    static constexpr int CK = (G::CW + XL) / CPX;   // chunks per chroma tile row
    static constexpr int CR = G::CH + 8;            // chroma tile rows
    static constexpr int NY = 72 * YK;
    static constexpr int NCHUNK = NY + 2 * CR * CK;
    static constexpr int PROG = LF_PROG_OF(G::SH, G::SV);
};

// chunk index -> (plane, tile row, chunk column): luma 72 rows x YK, then U, V CR x CK
template <typename PIX, class G> DEV void lf_chunk(int ci, int &p, int &r, int &k)
{
    typedef LfP<PIX, G> L;
    if (ci < L::NY) { p = 0; r = ci / L::YK; k = ci - r * L::YK; }
    else { const int c = ci - L::NY; p = 1 + (c >= L::CR * L::CK); const int cc = c - (p - 1) * L::CR * L::CK; r = cc / L::CK; k = cc - r * L::CK; }
}

// --------------------------------------------------------------- k_lf
DEV int ad16(int a, int b) { return (int) __builtin_amdgcn_sad_u16((uint32_t) a, (uint32_t) b, 0u); }
DEV int max3i(int a, int b, int c) { return max(max(a, b), c); }


// loop_filter (vp9dsp_template.c:1780-1889) on a line held in registers: q0 = px[C],
// compile-time positions, so a row's chain of edges (vp9lpf.c:31-104 order) runs
// without LDS round trips.
// `code` = filter width (1: 4, 2: 8, 3: 16), `eih` = the E | I << 12 | H << 22 word of
// the edge's level (lf_lut).
// Instruction economy (a line's chain of edges is the loop filter's critical path):
// - decisions branch-free: |a - b| is one v_sad_u16 (pixels < 2^12), reductions by max3,
//   one compare per condition;
// - the 4-wide results are computed by every filtered lane, both hev forms in one
//   sequence (lanes differ in hev), clamps as v_med3_i32 / min + max;
// - a wave none of whose lanes is flat (the common case) writes them in place and is done;
//   otherwise the 8- and 16-wide outputs are running sums (each output = the previous sum
//   + two entering - two leaving taps: the reference's sums term for term, exact) and every
//   position takes its lane's result by a select, so no branch leaves copies of the line's
//   registers at its join.
template <int C, int NPX>
DEV void lf_reg(int (&px)[NPX], int code, uint32_t eih, int bd)
{
    const int E = eih & 4095, I = (eih >> 12) & 1023, H = eih >> 22;
    const int F = 1 << (bd - 8), pmax = (1 << bd) - 1, smx = (1 << (bd - 1)) - 1, smn = -smx - 1;
    const int p3 = px[C - 4], p2 = px[C - 3], p1 = px[C - 2], p0 = px[C - 1];
    const int q0 = px[C], q1 = px[C + 1], q2 = px[C + 2], q3 = px[C + 3];
    const int ap1p0 = ad16(p1, p0), aq1q0 = ad16(q1, q0);
    const int mi = max3i(max3i(ad16(p3, p2), ad16(p2, p1), ap1p0), max3i(aq1q0, ad16(q2, q1), ad16(q3, q2)), 0);
    const bool fm = (mi <= I) & (ad16(p0, q0) * 2 + (ad16(p1, q1) >> 1) <= E);
    if (!fm) return;
    const bool f8 = (code >= 2) &
                    (max3i(max3i(ad16(p3, p0), ad16(p2, p0), ap1p0), max3i(aq1q0, ad16(q2, q0), ad16(q3, q0)), 0) <= F);
    // 4-wide (vp9dsp_template.c:1865-1885): with hev the p1 - q1 term enters f and p1 / q1
    // stay, without it f = 3 (q0 - p0) and p1 / q1 move by (f1 + 1) >> 1
    const bool hev = max(ap1p0, aq1q0) > H;
    const int fh = min(max(p1 - q1, smn), smx);
    int f = __mul24(q0 - p0, 3) + (hev ? fh : 0);        // v_mad_i32_i24 (|q0 - p0| < 2^12)
    f = min(max(f, smn), smx);
    const int f1 = min(f + 4, smx) >> 3, f2 = min(f + 3, smx) >> 3, f3 = (f1 + 1) >> 1;
    // v_med3_i32 clamps, evaluated for every lane (the asm is not speculated into a branch)
    const int a_p0 = med3_0(p0 + f2, pmax), a_q0 = med3_0(q0 - f1, pmax);
    const int t_p1 = med3_0(p1 + f3, pmax), t_q1 = med3_0(q1 - f3, pmax);
    const int a_p1 = hev ? p1 : t_p1, a_q1 = hev ? q1 : t_q1;
    if (!__builtin_amdgcn_ballot_w64(f8)) {              // wave-uniform: no lane is flat
        px[C - 2] = a_p1;
        px[C - 1] = a_p0;
        px[C] = a_q0;
        px[C + 1] = a_q1;
        return;
    }
    // 7-tap (vp9dsp_template.c:1859-1864) as a running sum, + 4 rounding
    int b[6];
    {
        int sm = (int) __umul24((uint32_t) p3, 3u) + 4 + (p2 + p2 + p1) + (p0 + q0);
        b[0] = sm >> 3;
        sm = sm + (p1 - p3) + (q1 - p2);
        b[1] = sm >> 3;
        sm = sm + (p0 - p3) + (q2 - p1);
        b[2] = sm >> 3;
        sm = sm + (q0 - p3) + (q3 - p0);
        b[3] = sm >> 3;
        sm = sm + (q1 - p2) + (q3 - q0);
        b[4] = sm >> 3;
        sm = sm + (q2 - p1) + (q3 - q1);
        b[5] = sm >> 3;
    }
    // positions p2 .. q2: the lane's 8- or 4-wide result (selects: no join copies)
    px[C - 3] = f8 ? b[0] : p2;
    px[C - 2] = f8 ? b[1] : a_p1;
    px[C - 1] = f8 ? b[2] : a_p0;
    px[C] = f8 ? b[3] : a_q0;
    px[C + 1] = f8 ? b[4] : a_q1;
    px[C + 2] = f8 ? b[5] : q2;
    if (C >= 8 && C + 7 < NPX) {
        const int p7 = px[C - 8 >= 0 ? C - 8 : 0], p6 = px[C - 7 >= 0 ? C - 7 : 0], p5 = px[C - 6 >= 0 ? C - 6 : 0],
                  p4 = px[C - 5 >= 0 ? C - 5 : 0];
        const int q4 = px[C + 4 < NPX ? C + 4 : NPX - 1], q5 = px[C + 5 < NPX ? C + 5 : NPX - 1],
                  q6 = px[C + 6 < NPX ? C + 6 : NPX - 1], q7 = px[C + 7 < NPX ? C + 7 : NPX - 1];
        const bool f16 = f8 & (code == 3) &
                         (max3i(max3i(ad16(p7, p0), ad16(p6, p0), ad16(p5, p0)), max3i(ad16(p4, p0), ad16(q4, q0), ad16(q5, q0)),
                                max3i(ad16(q6, q0), ad16(q7, q0), 0)) <= F);
        if (__builtin_amdgcn_ballot_w64(f16)) {
            // 15-tap (vp9dsp_template.c:1836-1857): the window sum of output k (+ the rounding
            // 8) slides by v[k + 8] - v[k - 7] + v[k + 1] - v[k], ends replicated; inputs
            // are the values before this edge (p7 .. q7 and p3 .. q3 above)
            const int v[16] = { p7, p6, p5, p4, p3, p2, p1, p0, q0, q1, q2, q3, q4, q5, q6, q7 };
            int o[14];
            int sum = (int) __umul24((uint32_t) p7, 7u) + 8 + (p6 + p6 + p5) + (p4 + p3 + p2) + (p1 + p0 + q0);
            o[0] = sum >> 4;
#pragma unroll
            for (int k = 1; k < 14; k++) {
                const int lo = k - 7 < 0 ? 0 : k - 7, hi = k + 8 > 15 ? 15 : k + 8;
                sum = sum + (v[hi] - v[lo]) + (v[k + 1] - v[k]);
                o[k] = sum >> 4;
            }
#pragma unroll
            for (int k = 0; k < 14; k++)
                px[C - 7 + k] = f16 ? o[k] : px[C - 7 + k];
        }
    }
}

template <typename PIX, int N> DEV void lf_unpack(const uint32_t *w, int (&px)[N], int i0, int i1, int o)
{
    constexpr int PPW = 4 / sizeof(PIX);
#pragma unroll
    for (int i = i0; i < i1; i++)
#pragma unroll
        for (int j = 0; j < PPW; j++)
            px[o + (i - i0) * PPW + j] = (w[i] >> (8 * sizeof(PIX) * j)) & ((1u << (8 * sizeof(PIX))) - 1);
}
template <typename PIX, int N> DEV void lf_pack(uint32_t *w, const int (&px)[N], int i0, int i1, int o)
{
    constexpr int PPW = 4 / sizeof(PIX);
#pragma unroll
    for (int i = i0; i < i1; i++) {
        uint32_t v = 0;
#pragma unroll
        for (int j = 0; j < PPW; j++) v |= (uint32_t) px[o + (i - i0) * PPW + j] << (8 * sizeof(PIX) * j);
        w[i] = v;
    }
}

// Edge chains of one line held in registers (vp9lpf.c:31-181 order), program words pw
// of the line's band. "wide": a 64-pixel plane dimension, line x = -8..63, 8 edges 8
// apart each with an inner 4-wide edge, processed in two 40-pixel register halves
// (an edge touches 8 pixels either side: x = -8..31 for edges 0-3, then x = 24..63 for
// edges 4-7, x = 24..31 carried over). "narrow": a subsampled 32-pixel chroma dimension,
// x = -8..31, 8 edges 4 apart.
// PF (k_lfrd: one wave per SIMD, nothing hides an LDS read's latency): the E | I | H words
// of a line's edges are read from the LDS table before its first edge (lf_eih_wide /
// _narrow: every load in flight at once), so no edge waits on an LDS read. Without PF (the
// diagonal kernels, several waves per SIMD) each edge reads its word: fewer live registers.
template <bool PF, int N> struct LfEv {
    uint32_t v[PF ? N : 1];
    const uint32_t *lut;
    DEV uint32_t operator()(int i, uint32_t lvl) const
    {
        if constexpr (PF) return v[i];
        else return lut[lvl & 63];
    }
};
#define LF_EDGE_WIDE(k, C0)                                                                              \
    {                                                                                                    \
        const uint32_t ww = (k) < 2 ? pw0 : (k) < 4 ? pw1 : (k) < 6 ? pw2 : pw3;                         \
        const uint32_t m = (ww >> (16 * ((k) & 1))) & 255, in = (ww >> (16 * ((k) & 1) + 8)) & 255;      \
        if (m >> 6) lf_reg<8 * (k) + 8 - (C0)>(px, m >> 6, ev(2 * (k), m), bd);                          \
        if (in) lf_reg<8 * (k) + 12 - (C0)>(px, 1, ev(2 * (k) + 1, in), bd);                             \
    }
#define LF_EDGE_NARROW(k)                                                                                \
    {                                                                                                    \
        const uint32_t m = (((k) < 4 ? pc0 : pc1) >> (8 * ((k) & 3))) & 255;                             \
        if (m >> 6) lf_reg<4 * (k) + 8>(px, m >> 6, ev(k, m), bd);                                       \
    }
// the 16 edge words of a 64-pixel line (8 edges + their inner 4-wide edges), program words pw0..3
template <bool PF>
DEV void lf_eih_wide(LfEv<PF, 16> &ev, uint32_t pw0, uint32_t pw1, uint32_t pw2, uint32_t pw3, const uint32_t *lut)
{
    ev.lut = lut;
    if constexpr (PF) {
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const uint32_t ww = k < 2 ? pw0 : k < 4 ? pw1 : k < 6 ? pw2 : pw3;
            ev.v[2 * k] = lut[(ww >> (16 * (k & 1))) & 63];
            ev.v[2 * k + 1] = lut[(ww >> (16 * (k & 1) + 8)) & 63];
        }
    }
}
// the 8 edge words of a subsampled 32-pixel chroma line
template <bool PF, int N>
DEV void lf_eih_narrow(LfEv<PF, N> &ev, uint32_t pc0, uint32_t pc1, const uint32_t *lut)
{
    ev.lut = lut;
    if constexpr (PF) {
#pragma unroll
        for (int k = 0; k < 8; k++) ev.v[k] = lut[((k < 4 ? pc0 : pc1) >> (8 * (k & 3))) & 63];
    }
}
// column edges of one pixel row (packed dwords in LDS)
template <typename PIX, bool PF = false>
DEV void lf_line_row_wide(uint32_t *rowp, const uint32_t *pw, const uint32_t *lut, int bd)
{
    constexpr int PPW = 4 / sizeof(PIX);
    const uint32_t pw0 = pw[0], pw1 = pw[1], pw2 = pw[2], pw3 = pw[3];
    LfEv<PF, 16> ev;
    lf_eih_wide<PF>(ev, pw0, pw1, pw2, pw3, lut);
    int px[40];
    lf_unpack<PIX>(rowp, px, 0, 40 / PPW, 0);
    LF_EDGE_WIDE(0, 0) LF_EDGE_WIDE(1, 0) LF_EDGE_WIDE(2, 0) LF_EDGE_WIDE(3, 0)
    lf_pack<PIX>(rowp, px, 0, 32 / PPW, 0);
#pragma unroll
    for (int i = 0; i < 8; i++) px[i] = px[32 + i];
    lf_unpack<PIX>(rowp, px, 40 / PPW, 72 / PPW, 8);
    LF_EDGE_WIDE(4, 32) LF_EDGE_WIDE(5, 32) LF_EDGE_WIDE(6, 32) LF_EDGE_WIDE(7, 32)
    lf_pack<PIX>(rowp, px, 32 / PPW, 72 / PPW, 0);
}
template <typename PIX, bool PF = false>
DEV void lf_line_row_narrow(uint32_t *rowp, const uint32_t *pw, const uint32_t *lut, int bd)
{
    constexpr int PPW = 4 / sizeof(PIX);
    const uint32_t pc0 = pw[0], pc1 = pw[1];
    LfEv<PF, 8> ev;
    lf_eih_narrow<PF>(ev, pc0, pc1, lut);
    int px[40];
    lf_unpack<PIX>(rowp, px, 0, 40 / PPW, 0);
    LF_EDGE_NARROW(0) LF_EDGE_NARROW(1) LF_EDGE_NARROW(2) LF_EDGE_NARROW(3)
    LF_EDGE_NARROW(4) LF_EDGE_NARROW(5) LF_EDGE_NARROW(6) LF_EDGE_NARROW(7)
    lf_pack<PIX>(rowp, px, 0, 40 / PPW, 0);
}
// k_lfrd's column pass in two parts around a barrier: part 1 filters a row's first edge
// (x = 0, the only one that reaches x < 0: later edges modify x >= 1) and writes
// x = -8..-1 back, so the previous SB's last columns are final in LDS after it; part 2
// runs the row's other edges on the same registers (and edge words: ev, read in part 1).
template <typename PIX>
DEV void lf_row_wide_1(uint32_t *rowp, const uint32_t *pw, const uint32_t *lut, int bd, int (&px)[40], LfEv<true, 16> &ev)
{
    constexpr int PPW = 4 / sizeof(PIX);
    lf_eih_wide<true>(ev, pw[0], pw[1], pw[2], pw[3], lut);
    lf_unpack<PIX>(rowp, px, 0, 40 / PPW, 0);
    const uint32_t m = pw[0] & 255;
    if (m >> 6) lf_reg<8>(px, m >> 6, ev(0, m), bd);
    lf_pack<PIX>(rowp, px, 0, 8 / PPW, 0);
}
template <typename PIX>
DEV void lf_row_wide_2(uint32_t *rowp, const uint32_t *pw, const uint32_t *lut, int bd, int (&px)[40], const LfEv<true, 16> &ev)
{
    constexpr int PPW = 4 / sizeof(PIX);
    const uint32_t pw0 = pw[0], pw1 = pw[1], pw2 = pw[2], pw3 = pw[3];
    const uint32_t in0 = (pw0 >> 8) & 255;
    if (in0) lf_reg<12>(px, 1, ev(1, in0), bd);
    LF_EDGE_WIDE(1, 0) LF_EDGE_WIDE(2, 0) LF_EDGE_WIDE(3, 0)
    lf_pack<PIX>(rowp, px, 8 / PPW, 32 / PPW, 8);
#pragma unroll
    for (int i = 0; i < 8; i++) px[i] = px[32 + i];
    lf_unpack<PIX>(rowp, px, 40 / PPW, 72 / PPW, 8);
    LF_EDGE_WIDE(4, 32) LF_EDGE_WIDE(5, 32) LF_EDGE_WIDE(6, 32) LF_EDGE_WIDE(7, 32)
    lf_pack<PIX>(rowp, px, 32 / PPW, 72 / PPW, 0);
}
template <typename PIX>
DEV void lf_row_narrow_1(uint32_t *rowp, const uint32_t *pw, const uint32_t *lut, int bd, int (&px)[40], LfEv<true, 16> &ev)
{
    constexpr int PPW = 4 / sizeof(PIX);
    lf_eih_narrow<true, 16>(ev, pw[0], pw[1], lut);
    lf_unpack<PIX>(rowp, px, 0, 40 / PPW, 0);
    const uint32_t m = pw[0] & 255;
    if (m >> 6) lf_reg<8>(px, m >> 6, ev(0, m), bd);
    lf_pack<PIX>(rowp, px, 0, 8 / PPW, 0);
}
template <typename PIX>
DEV void lf_row_narrow_2(uint32_t *rowp, const uint32_t *pw, const uint32_t *lut, int bd, int (&px)[40], const LfEv<true, 16> &ev)
{
    constexpr int PPW = 4 / sizeof(PIX);
    const uint32_t pc0 = pw[0], pc1 = pw[1];
    LF_EDGE_NARROW(1) LF_EDGE_NARROW(2) LF_EDGE_NARROW(3)
    LF_EDGE_NARROW(4) LF_EDGE_NARROW(5) LF_EDGE_NARROW(6) LF_EDGE_NARROW(7)
    lf_pack<PIX>(rowp, px, 8 / PPW, 40 / PPW, 8);
}
// row edges of one pixel column (tile pitch P)
template <typename PIX, int P, bool PF = false>
DEV void lf_line_col_wide(PIX *colp, const uint32_t *pw, const uint32_t *lut, int bd)
{
    const uint32_t pw0 = pw[0], pw1 = pw[1], pw2 = pw[2], pw3 = pw[3];
    LfEv<PF, 16> ev;
    lf_eih_wide<PF>(ev, pw0, pw1, pw2, pw3, lut);
    int px[40];                    // rows -8..31, then 24..63 (as the column pass)
#pragma unroll
    for (int i = 0; i < 40; i++) px[i] = colp[i * P];
    LF_EDGE_WIDE(0, 0) LF_EDGE_WIDE(1, 0) LF_EDGE_WIDE(2, 0) LF_EDGE_WIDE(3, 0)
#pragma unroll
    for (int i = 1; i < 32; i++) colp[i * P] = (PIX) px[i];
#pragma unroll
    for (int i = 0; i < 8; i++) px[i] = px[32 + i];
#pragma unroll
    for (int i = 8; i < 40; i++) px[i] = colp[(32 + i) * P];
    LF_EDGE_WIDE(4, 32) LF_EDGE_WIDE(5, 32) LF_EDGE_WIDE(6, 32) LF_EDGE_WIDE(7, 32)
#pragma unroll
    for (int i = 0; i < 40; i++) colp[(32 + i) * P] = (PIX) px[i];
}
template <typename PIX, int P, bool PF = false>
DEV void lf_line_col_narrow(PIX *colp, const uint32_t *pw, const uint32_t *lut, int bd)
{
    const uint32_t pc0 = pw[0], pc1 = pw[1];
    LfEv<PF, 8> ev;
    lf_eih_narrow<PF>(ev, pc0, pc1, lut);
    int px[40];
#pragma unroll
    for (int i = 0; i < 40; i++) px[i] = colp[i * P];
    LF_EDGE_NARROW(0) LF_EDGE_NARROW(1) LF_EDGE_NARROW(2) LF_EDGE_NARROW(3)
    LF_EDGE_NARROW(4) LF_EDGE_NARROW(5) LF_EDGE_NARROW(6) LF_EDGE_NARROW(7)
#pragma unroll
    for (int i = 1; i < 40; i++) colp[i * P] = (PIX) px[i];
}
#undef LF_EDGE_WIDE
#undef LF_EDGE_NARROW

// One SB of loop filter by NT threads (128 for 4:2:0: luma and chroma lines in parallel).
// Planes are independent (vp9lpf.c:183-230), so lanes take luma and chroma lines
// together; each plane filters all column edges, then all row edges.
template <typename PIX, class G> struct LfLds {
    PIX lt[72 * LfP<PIX, G>::YP];
    PIX ct[2][LfP<PIX, G>::CR * LfP<PIX, G>::UVP];
    uint32_t prog[LfP<PIX, G>::PROG / 4];    // the SB's edge decisions (LFRec.prog)
    uint32_t lut[64];                         // level -> E | I << 12 | H << 22
};

// E / I / H of a filter level (vp9.c:669-687 limit LUTs; loop_filter's F / E / I / H
// scaling by bit depth, vp9dsp_template.c:1780-1800)
DEV uint32_t lf_eih(int L, int sharp, int bd)
{
    int limit = L;
    if (sharp > 0) { limit >>= (sharp + 3) >> 2; limit = limit < 9 - sharp ? limit : 9 - sharp; }
    limit = limit > 1 ? limit : 1;
    const uint32_t E = (2 * (L + 2) + limit) << (bd - 8), I = limit << (bd - 8), H = (L >> 4) << (bd - 8);
    return E | I << 12 | H << 22;
}

// The filter passes of one SB over its LDS tile: all column edges of every plane (lanes =
// pixel rows), then all row edges (lanes = pixel columns). Ends with a barrier.
template <typename PIX, class G, int NT, int PASSES = 3, bool PF = false>
DEV void lf_passes_v(PIX *lt, PIX (*ct)[LfP<PIX, G>::CR * LfP<PIX, G>::UVP], const uint32_t *prog, const uint32_t *lut,
                     int lane, int bd)
{
#define LF_SYNC() do { if (NT == 64) wave_sync(); else __syncthreads(); } while (0)
    typedef LfP<PIX, G> L;
    constexpr int FLP = L::YP, FCP = L::UVP, CW = G::CW, CH = G::CH;
    constexpr int XL = L::XL, XO = L::XO;
    // ---- column edges (filter_plane_cols, vp9lpf.c:31-104): one lane per pixel row ----
    if (PASSES & 1) {
    for (int tid = lane; tid < 64 + 2 * CH; tid += NT) {
        if (tid < 64) {
            lf_line_row_wide<PIX, PF>((uint32_t *) (lt + (tid + 8) * FLP + XO), prog + (LFP_YC + (tid >> 3) * 16) / 4, lut, bd);
        } else {
            const int p = 1 + (tid - 64 >= CH), r = tid - 64 - (p - 1) * CH;
            uint32_t *rowp = (uint32_t *) (ct[p - 1] + (r + 8) * FCP + XO);
            const uint32_t *pw = prog + (LFP_CC + (r >> 3) * LFP_CSTRIDE(G::SH)) / 4;
            if (G::SH) lf_line_row_narrow<PIX, PF>(rowp, pw, lut, bd);
            else lf_line_row_wide<PIX, PF>(rowp, pw, lut, bd);
        }
    }
    LF_SYNC();
    }
    // ---- row edges (filter_plane_rows, vp9lpf.c:106-181): one lane per pixel column ----
    if (PASSES & 2) {
    for (int tid = lane; tid < 64 + 2 * CW; tid += NT) {
        if (tid < 64) {
            lf_line_col_wide<PIX, FLP, PF>(lt + XL + tid, prog + (LFP_YR + (tid >> 3) * 16) / 4, lut, bd);
        } else {
            const int p = 1 + (tid - 64 >= CW), c = tid - 64 - (p - 1) * CW;
            PIX *colp = ct[p - 1] + XL + c;
            const uint32_t *pw = prog + (LFP_CR(G::SH, G::SV) + (c >> 3) * LFP_CSTRIDE(G::SV)) / 4;
            if (G::SV) lf_line_col_narrow<PIX, FCP, PF>(colp, pw, lut, bd);
            else lf_line_col_wide<PIX, FCP, PF>(colp, pw, lut, bd);
        }
    }
    LF_SYNC();
    }
#undef LF_SYNC
}

template <typename PIX, class G, int NT, int PASSES = 3>
DEV void lf_passes(LfLds<PIX, G> &S, int lane, int bd)
{
    lf_passes_v<PIX, G, NT, PASSES>(S.lt, S.ct, S.prog, S.lut, lane, bd);
}

template <typename PIX, class G, int NT>
DEV void lf_sb(const LFRec &rec, const FrameDesc *__restrict__ frames, LfLds<PIX, G> &S, int lane, int dbg)
{
#define LF_SYNC() do { if (NT == 64) wave_sync(); else __syncthreads(); } while (0)
    typedef LfP<PIX, G> L;
    constexpr int FLP = L::YP, FCP = L::UVP, CW = G::CW, CH = G::CH;
    PIX *lt = S.lt;
    PIX (*ct)[L::CR * FCP] = S.ct;
    const uint32_t *lut = S.lut;
    const FrameDesc &fd = frames[rec.frame];
    const int bd = fd.bd, sharp = fd.sharp;
    const int sbx = rec.sbx, sby = rec.sby;
    for (int i = lane; i < L::PROG / 4; i += NT) S.prog[i] = ((const uint32_t *) rec.prog)[i];
    for (int i = lane; i < 64; i += NT) S.lut[i] = lf_eih(i, sharp, bd);

    // load: luma rows [y0-8, y0+64) x cols [x0-XL, x0+64), chroma [-8, CH) x [-XL, CW), in
    // aligned 16-byte chunks (4:2:0 8-bit: luma 72 x 5, chroma 2 x 40 x 3 = 600 chunks, <= 5
    // per thread), all global loads of a thread in flight before its LDS writes
    typedef Chunk16::T CT;
    constexpr int CPX = L::CPX, XL = L::XL, XO = L::XO;
    constexpr int NU = (L::NCHUNK + NT - 1) / NT;
    CT v[NU];
#pragma unroll
    for (int u = 0; u < NU; u++) {
        const int ci = lane + u * NT;
        int p, r, k;
        lf_chunk<PIX, G>(ci, p, r, k);
        const int gx = (p ? sbx * CW : sbx * 64) - XL + CPX * k, gy = (p ? sby * CH : sby * 64) - 8 + r;
        v[u] = Chunk16::zero();
        if (!(dbg & 4) && ci < L::NCHUNK && gx >= 0 && gy >= 0)
            v[u] = *(const CT *) ((const PIX *) fd.plane[p] + (size_t) gy * fd.pitch[p ? 1 : 0] + gx);
    }
#pragma unroll
    for (int u = 0; u < NU; u++) {
        const int ci = lane + u * NT;
        int p, r, k;
        lf_chunk<PIX, G>(ci, p, r, k);
        if (ci < L::NCHUNK) {
            PIX *t = p ? ct[p - 1] + r * FCP : lt + r * FLP;
            Chunk16::to_lds(v[u], t + CPX * k);
        }
    }
    LF_SYNC();

    if (!(dbg & 1)) lf_passes<PIX, G, NT>(S, lane, bd);
    // ---- store the modified region: rows [0,h) x cols [-8,w) and rows [-8,0) x cols [0,w).
    // Other SBs of the same wavefront step never touch this region, so whole chunks are
    // written back (pixels beyond the 8-aligned frame size are unchanged padding). ----
#pragma unroll
    for (int u = 0; u < NU; u++) {
        const int ci = lane + u * NT;
        int p, r, k;
        lf_chunk<PIX, G>(ci, p, r, k);
        const int gx = (p ? sbx * CW : sbx * 64) - XL + CPX * k, gy = (p ? sby * CH : sby * 64) - 8 + r;
        if (!(dbg & 2) && ci < L::NCHUNK && gx >= 0 && gy >= 0 && (r >= 8 || k > 0)) {
            const PIX *t = p ? ct[p - 1] + r * FCP : lt + r * FLP;
            *(CT *) ((PIX *) fd.plane[p] + (size_t) gy * fd.pitch[p ? 1 : 0] + gx) = Chunk16::from_lds(t + CPX * k);
        }
    }
#undef LF_SYNC
}

// threads per k_lf workgroup: 128 for 4:2:0, 192 when a chroma dimension is 64
template <class G> struct LfNT { static constexpr int NT = (G::SH && G::SV) ? 128 : 192; };

template <typename PIX, class G>
__global__ __launch_bounds__(LfNT<G>::NT) void k_lf(const uint32_t *__restrict__ list, const LFRec *__restrict__ recs,
                                                    const FrameDesc *__restrict__ frames, int dbg)
{
    __shared__ LfLds<PIX, G> S;
    lf_sb<PIX, G, LfNT<G>::NT>(recs[list[blockIdx.x]], frames, S, threadIdx.x, dbg);
}

// ------------------------------------------------------------- k_lfrd / k_lfro
// Row-pipelined loop filter: one workgroup filters one SB row of one frame, SB by SB left to
// right (the raster SB order of ff_vp9_loopfilter_sb's callers, vp9.c:1522-1551 /
// vp9lpf.c:183-230), instead of one launch per x + 2y wavefront diagonal.
// - The left halo (x = -XL..-1) of SB c is the previous SB's right columns, already final
//   for this row and still in LDS: copied within LDS, never re-read from HBM.
// - The top halo (y = -8..-1) is the bottom of SB row r - 1, finished by another workgroup
//   of this launch. SB (r, c) needs row r - 1 through SB c + 1 (whose left-edge column
//   filtering rewrites x = 64c + 57..63 of that row). progress[r] = p says the bottom
//   rows of SBs 0..p-1 are final: row r publishes p = c right after SB c's column pass
//   (SB c - 1's last columns are then final and stored), before its row pass, and p = ncols
//   after its last SB; SB (r + 1, c) waits for progress[r] >= c + 1 before its ROW pass
//   (the column pass rewrites rows 0..63 only, so it runs ahead of the hand-off: the lag
//   between rows is one SB's column + row pass instead of two column passes + a row pass).
//   Hand-off (MI355X_MICROARCH.md, inter-workgroup visibility, Valid forms row 1): every
//   byte of the bottom 8 rows is stored sc1 (write-through) by the workgroup's store wave
//   (lanes NT.., the only wave that stores), which drains (s_waitcnt vmcnt(0)) before ONE
//   of its lanes stores the progress word; the consumer polls with sc1
//   loads and loads those rows only with sc1 loads. Every other load reads bytes written by
//   earlier launches, or by this launch only after the load (row r + 1 rewrites row r's
//   bottom rows once row r has published them).
// - Workgroups take their task (frame, SB row) from a ticket counter in the order they
//   start, and tasks are numbered rows-major, so a workgroup waits only on tasks already
//   held by running workgroups: no assumption about dispatch order or XCD placement.
//   Spins are bounded (timeout word ctr[2]). The last workgroup to finish zeroes the
//   counters for the next launch (graph replay).
// A task may start at SB column c0 > 0 (the SBs left of it filtered by earlier diagonal
// launches: the k_plf launches of the same phase); its first left halo then comes from HBM.
// progress[] counts absolute SB columns; a dep task starting at c0' > 0 has the bottom rows
// of SBs < c0' - 1 final before the launch.
// Task table (lists): tasks[k] = offset of task k's record {dep task or ~0u, ncols, c0,
// dep's final columns at the start, LFRec index of SB c0 .. ncols - 1}. ctr: {ticket, done, timeouts,
// spin bound, progress[ntasks]}.
typedef __attribute__((address_space(1))) uint64_t gu64;
typedef __attribute__((address_space(1))) uint32_t gu32;
DEV uint64_t ld_sc1(const void *p) { return __hip_atomic_load((gu64 *) p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
DEV void st_sc1(void *p, uint64_t v) { __hip_atomic_store((gu64 *) p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// ------------------------------------------------------------- k_predd
// The intra SBs of a level-scheduled phase (inter frames: their intra blocks read the
// reconstructed pixels of the left / top / top-left SBs, the planner's dependency mask) in ONE
// launch instead of one k_pred launch per dependency level (C5: ~5 per frame). The list is
// the phase's level lists back to back (level order). Workgroups take list entries from a
// ticket counter (ctr[0]) and take the next one when done, so an SB waits only on SBs of lower
// levels held by running workgroups: no assumption about dispatch order. The grid is capped
// (a waiting workgroup holds its CU slot: uncapped, C5's thousands of waiting SBs crowded the
// other chain's kernels). An SB polls its producers' done flags (slot-indexed, sc1), then runs
// pred_wg with sc1 halo loads; the producer wrote its right column and bottom row through
// with sc1 stores and drained them (s_waitcnt vmcnt(0)) before its flag: the k_lfro row
// hand-off's protocol. Waits are bounded (ctr[2] counts the ones given up: the batch fails
// with VP9HIP_EBUG, like a k_lfr timeout); the last workgroup zeroes the flags and counters
// for the next launch (graph replay). ctr: {ticket, finished workgroups, timeouts, spin bound}.
template <typename PIX, class G>
__global__ __launch_bounds__(64) void k_predd(const uint32_t *__restrict__ list, int n, const uint32_t *__restrict__ sbinfo,
                                              const WGRec *__restrict__ wgs, const SBRec *__restrict__ sbs,
                                              const PJob *__restrict__ jobs, const uint32_t *__restrict__ passes,
                                              const FrameDesc *__restrict__ frames, const int16_t *__restrict__ resid,
                                              const uint32_t *__restrict__ ptab, uint32_t *ctr, uint32_t *done, int dbg)
{
    static_assert(G::SH == 1 && G::SV == 1, "k_predd: 4:2:0");
    __shared__ PredLds<PIX, G, true> S;
    __shared__ uint32_t s_task, s_last;
    const int lane = threadIdx.x;
#if PRED_LTAB_LDS
    load_ltab<PIX>(S.ltab, ptab, lane);
#endif
    const uint32_t spin = ctr[3] ? ctr[3] : (1u << 22);
    for (;;) {
        if (lane == 0) s_task = atomicAdd(&ctr[0], 1u);
        wave_sync();
        const uint32_t task = __builtin_amdgcn_readfirstlane(s_task);
        if (task >= (uint32_t) n) break;
        const uint32_t slot = __builtin_amdgcn_readfirstlane(list[task]);
        const WGRec *wg = wgs + slot;
        const uint32_t info = sbinfo[slot];
        const SBRec sb = sbs[wg->sb[0]];
        const uint32_t W = (uint32_t) frames[sb.frame].sb_cols;
        // lanes 0 / 1 / 2: the left / top / top-left producer
        uint32_t dep = ~0u;
        if (lane == 0 && (info & 2) && sb.sbx > 0) dep = slot - 1;
        if (lane == 1 && (info & 4) && sb.sby > 0) dep = slot - W;
        if (lane == 2 && (info & 8) && sb.sbx > 0 && sb.sby > 0) dep = slot - W - 1;
        for (uint32_t t = 0;; t++) {
            const bool ok = dep == ~0u || __hip_atomic_load((gu32 *) &done[dep], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
            if (__all(ok)) break;
            if (t > spin) {
                if (lane == 0) atomicAdd(&ctr[2], 1u);
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        pred_wg<PIX, G, true, 1>(wg, sbs, jobs, passes, frames, resid, ptab, S, lane, dbg);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) __hip_atomic_store((gu32 *) &done[slot], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        wave_sync();                   // pred_wg's LDS reads before the next SB's tile writes
    }
    if (lane == 0) s_last = atomicAdd(&ctr[1], 1u) == gridDim.x - 1;
    wave_sync();
    if (__builtin_amdgcn_readfirstlane(s_last)) {
        for (int i = lane; i < n; i += 64) done[list[i]] = 0;
        if (lane == 0) { ctr[0] = 0; ctr[1] = 0; }
    }
}

// row-LF pieces: chunk (p, r, k) of SB (sbx, sby) in its plane. Plane bases are offsets from
// plane 0 chosen by selects (an indexed array of pointers would live in scratch).
struct LfrPlanes {
    uint64_t b0, d1, d2;
    int pit0, pit1;
};
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) v4u gv4u;        // global_ (not flat_) loads / stores
template <typename PIX, class G> DEV PIX *lfr_addr(const LfrPlanes &P, int sbx, int sby, int p, int r, int k)
{
    typedef LfP<PIX, G> L;
    const int gx = (p ? sbx * G::CW : sbx * 64) - L::XL + L::CPX * k, gy = (p ? sby * G::CH : sby * 64) - 8 + r;
    const uint64_t a = P.b0 + (p == 1 ? P.d1 : 0) + (p == 2 ? P.d2 : 0);
    return (PIX *) a + (ptrdiff_t) gy * (p ? P.pit1 : P.pit0) + gx;
}
// LFR_PROF builds (profiling only, tools/lfr_prof.sh): lane 0 of each row-LF workgroup sums
// the shader-clock cycles of its SB-step phases into lfr_prof[] (vp9hip_lfr_prof_read)
#ifndef LFR_PROF
#define LFR_PROF 0
#endif
KP_DEV unsigned long long lfr_prof[16];
// LFR_PROF builds: one k_lfro workgroup's event timeline (lfro_tl[event][sb - TL_SB0],
// shader clock), the first workgroup of row task TL_TASK to claim it (lfro_tl_claim)
#define TL_SB0 40
#define TL_NSB 8
#define TL_TASK 30
KP_DEV unsigned long long lfro_tl[24][TL_NSB];
KP_DEV unsigned int lfro_tl_claim;
#define LFR_T(i)                                                                                  \
    do {                                                                                          \
        if (LFR_PROF) { const uint64_t tn = clock64(); pacc[i] += tn - tp; tp = tn; }             \
    } while (0)
// k_lfrd: the row-pipelined loop filter with two LDS tiles (SB c in tile (c - c0) & 1). The store wave writes SB
// c - 1's tile to HBM while the filtering waves run SB c's column pass, instead of between
// SB c - 1's row pass and SB c's first barrier (where every lane of the workgroup waited
// for its ~17 serialised LDS-read + store rounds); SB c + 1's interior loads and program
// words are issued during SB c (after its top halo is in LDS, so waiting for the halo never
// waits for them), and SB c's left halo is copied LDS to LDS from tile c - 1's last
// chunk column. The last chunk column of tile c - 1 (rows >= 8) is not stored from tile
// c - 1: tile c's left halo holds the same pixels after SB c's column pass (the final
// ones) and is stored from there (bottom rows at the hand-off, the rest with tile c).
// Hand-off, task table, spin bound and counter reset as described at the top of this section.
template <typename PIX, class G> DEV void lfrd_chunk_rows(int ci, int ry0, int nry, int rc0, int nrc, int &p, int &r, int &k)
{
    typedef LfP<PIX, G> L;
    if (ci < nry * L::YK) { p = 0; r = ci / L::YK; k = ci - r * L::YK; r += ry0; }
    else { const int c = ci - nry * L::YK; p = 1 + (c >= nrc * L::CK); const int cc = c - (p - 1) * nrc * L::CK; r = cc / L::CK; k = cc - r * L::CK; r += rc0; }
}
template <typename PIX, class G> DEV void lfrd_chunk(int ci, bool top, int &p, int &r, int &k)
{
    if (top) lfrd_chunk_rows<PIX, G>(ci, 0, 8, 0, 8, p, r, k);
    else lfrd_chunk_rows<PIX, G>(ci, 8, 64, 8, G::CH, p, r, k);
}
template <typename PIX, class G, int NTB = 2> struct LfrLds {
    typedef LfP<PIX, G> L;
    PIX lt[NTB][72 * L::YP];
    PIX ct[NTB][2][L::CR * L::UVP];
    uint32_t prog[NTB][L::PROG / 4];
    uint32_t lut[64];
};

// store wave: SB (sbx, sby)'s tile from LDS, except the bytes other steps store (the left
// halo's bottom rows, published at the hand-off; its top-left corner, never modified;
// unless `last`, the last chunk column's rows >= 8, stored from the next tile's left halo).
// part 0: the bottom 8 rows only (sc1: the row below reads them), 1: the other rows, 2: all.
// one plane's tile rows [ra, rb) (NK chunks per row, tile pitch TP), chunk-parallel over
// the 64 store lanes; g0 = the plane at the tile's origin (x = -XL, y = -8)
template <typename PIX, int NK, int TP>
DEV void lfrd_store_rows(const PIX *tile, PIX *g0, int pitch, int ra, int rb, int ml, int sbx, int sby, bool last, bool bot)
{
    typedef Chunk16::T CT;
    constexpr int CPX = 16 / sizeof(PIX);
    const int n = (rb - ra) * NK;
    for (int ci = ml; ci < n; ci += 64) {
        const int rr = ci / NK, k = ci - rr * NK, r = ra + rr;
        if ((k == 0 && (sbx == 0 || r < 8 || bot)) || (r < 8 && sby == 0) || (!last && k == NK - 1 && r >= 8)) continue;
        const CT w = Chunk16::from_lds(tile + r * TP + CPX * k);
        PIX *g = g0 + (ptrdiff_t) r * pitch + CPX * k;
        if (bot) {
            st_sc1(g, (uint64_t) w.x | (uint64_t) w.y << 32);
            st_sc1((char *) g + 8, (uint64_t) w.z | (uint64_t) w.w << 32);
        } else {
            v4u x; x.x = w.x; x.y = w.y; x.z = w.z; x.w = w.w;
            *(gv4u *) g = x;
        }
    }
}
template <typename PIX, class G, class LDS>
DEV void lfrd_store(const LDS &S, int tb, const LfrPlanes &P, int sbx, int sby, int ml, bool last, int part)
{
    typedef LfP<PIX, G> L;
    // part 0: the bottom 8 rows of each plane (sc1: the row below reads them), 1: the other
    // rows, 2: both
    PIX *g0 = lfr_addr<PIX, G>(P, sbx, sby, 0, 0, 0), *g1 = lfr_addr<PIX, G>(P, sbx, sby, 1, 0, 0),
        *g2 = lfr_addr<PIX, G>(P, sbx, sby, 2, 0, 0);
#pragma unroll
    for (int q = 0; q < 2; q++) {
        if ((part == 0 && q == 1) || (part == 1 && q == 0)) continue;
        const bool bot = !q;
        const int ya = bot ? 64 : 0, yb = bot ? 72 : 64, ca = bot ? L::CR - 8 : 0, cb = bot ? L::CR : L::CR - 8;
        lfrd_store_rows<PIX, L::YK, L::YP>(S.lt[tb], g0, P.pit0, ya, yb, ml, sbx, sby, last, bot);
        lfrd_store_rows<PIX, L::CK, L::UVP>(S.ct[tb][0], g1, P.pit1, ca, cb, ml, sbx, sby, last, bot);
        lfrd_store_rows<PIX, L::CK, L::UVP>(S.ct[tb][1], g2, P.pit1, ca, cb, ml, sbx, sby, last, bot);
    }
}

template <typename PIX, class G> struct LfrdN {
    typedef LfP<PIX, G> L;
    static constexpr int NTOP = 8 * (L::YK + 2 * L::CK), NINT = L::NCHUNK - NTOP;
    static constexpr int NUT = (NTOP + LfNT<G>::NT - 1) / LfNT<G>::NT, NUI = (NINT + LfNT<G>::NT - 1) / LfNT<G>::NT;
};
// interior loads of SB (sbx, sby) (left halo from HBM only when `halo`)
template <typename PIX, class G, int NUI>
DEV void lfrd_issue(Chunk16::T (&v)[NUI], const LfrPlanes &P, int sbx, int sby, int lane, bool halo)
{
    typedef LfrdN<PIX, G> N;
    static_assert(NUI == N::NUI, "interior chunk registers");
#pragma unroll
    for (int u = 0; u < NUI; u++) {
        const int ci = lane + u * LfNT<G>::NT;
        int p, r, k;
        lfrd_chunk<PIX, G>(ci, false, p, r, k);
        if (ci < N::NINT && (k > 0 || halo)) {
            const v4u x = *(const gv4u *) lfr_addr<PIX, G>(P, sbx, sby, p, r, k);
            v[u] = make_uint4(x.x, x.y, x.z, x.w);
        }
    }
}
// top halo (rows handed off by the row above, sc1 loads)
template <typename PIX, class G, int NUT>
DEV void lfrd_top(Chunk16::T (&v)[NUT], const LfrPlanes &P, int sbx, int sby, int lane)
{
    typedef LfrdN<PIX, G> N;
    static_assert(NUT == N::NUT, "top-halo chunk registers");
#pragma unroll
    for (int u = 0; u < NUT; u++) {
        const int ci = lane + u * LfNT<G>::NT;
        int p, r, k;
        lfrd_chunk<PIX, G>(ci, true, p, r, k);
        if (ci >= N::NTOP || k == 0 || sby == 0) continue;
        const PIX *g = lfr_addr<PIX, G>(P, sbx, sby, p, r, k);
        const uint64_t lo = ld_sc1(g), hi = ld_sc1((const char *) g + 8);
        v[u] = make_uint4((uint32_t) lo, (uint32_t) (lo >> 32), (uint32_t) hi, (uint32_t) (hi >> 32));
    }
}

// the last workgroup of a row-LF launch zeroes its counters and row progress words for the
// next launch (graph replay)
DEV void lfrd_retire(uint32_t *ctr, int ntasks, int lane, int nth, uint32_t *s_last)
{
    __syncthreads();
    if (lane == 0) *s_last = atomicAdd(&ctr[1], 1u) == (uint32_t) ntasks - 1;
    __syncthreads();
    if (*s_last) {
        for (int i = lane; i < ntasks; i += nth) ctr[4 + i] = 0;
        if (lane == 0) { ctr[0] = 0; ctr[1] = 0; }
    }
}

template <typename PIX, class G>
__global__ __launch_bounds__(LfNT<G>::NT + 64) void k_lfrd(const uint32_t *__restrict__ tasks, const LFRec *__restrict__ recs,
                                                      const FrameDesc *__restrict__ frames, uint32_t *ctr, int ntasks)
{
    constexpr int NT = LfNT<G>::NT;
    typedef LfP<PIX, G> L;
    typedef Chunk16::T CT;
    constexpr int FLP = L::YP, FCP = L::UVP, CW = G::CW, CPX = L::CPX;
    typedef LfrdN<PIX, G> N;
    constexpr int NUM = (L::NCHUNK + 63) / 64;
    __shared__ LfrLds<PIX, G> S;
    __shared__ uint32_t s_task, s_last, s_pre;
    const int lane = threadIdx.x;
    uint32_t *const progress = ctr + 4;
    __builtin_amdgcn_s_setprio(3);
    uint64_t pacc[14] = {0}, tp = LFR_PROF ? clock64() : 0;
    const uint64_t tk0 = tp;
    if (lane == 0) s_task = atomicAdd(&ctr[0], 1u);
    __syncthreads();
    // spin bound of a wait (ctr[3], 0 = 2^22 polls; a small bound is a test hook)
    const uint32_t spin = ctr[3] ? ctr[3] : (1u << 22);
    const uint32_t *T = tasks + tasks[s_task];
    const uint32_t dep = T[0], ncols = T[1], c0 = T[2];
    uint32_t seen = T[3];
    const LFRec &rec0 = recs[T[4]];
    const FrameDesc &fd = frames[rec0.frame];
    const int bd = fd.bd, sby = rec0.sby;
    LfrPlanes P;
    P.b0 = fd.plane[0]; P.d1 = fd.plane[1] - P.b0; P.d2 = fd.plane[2] - P.b0;
    P.pit0 = fd.pitch[0]; P.pit1 = fd.pitch[1];
    for (int i = lane; i < 64; i += NT) S.lut[i] = lf_eih(i, fd.sharp, bd);
    static_assert(L::PROG / 4 <= NT, "one program word per filtering lane");
    CT vi[N::NUI], vt[N::NUT];
#pragma unroll
    for (int u = 0; u < N::NUI; u++) vi[u] = Chunk16::zero();
#pragma unroll
    for (int u = 0; u < N::NUT; u++) vt[u] = Chunk16::zero();
    const bool mover = lane >= NT;
    const int ml = lane - NT;
    uint32_t pwv = 0;                           // the next SB's program word
    if (!mover) {
        lfrd_issue<PIX, G>(vi, P, c0, sby, lane, c0 > 0);
        if (lane < L::PROG / 4) pwv = ((const uint32_t *) rec0.prog)[lane];
    }
    LFR_T(7);
    for (uint32_t c = c0; c < ncols; c++) {
        const int sbx = (int) c, tb = (int) ((c - c0) & 1);
        PIX *lt = S.lt[tb];
        PIX (*ct)[L::CR * FCP] = S.ct[tb];
        // interior (loaded during the previous SB) and left halo into this SB's tile
        // the progress probe on the store wave (idle here): its round trip runs under the
        // filtering waves' tile writes
        if (lane == NT) {
            if (dep != ~0u && seen < c + 1)
                seen = __hip_atomic_load((gu32 *) &progress[dep], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_pre = dep == ~0u || seen >= c + 1;
        }
        if (!mover) {
            if (lane < L::PROG / 4) S.prog[tb][lane] = pwv;
#pragma unroll
            for (int u = 0; u < N::NUI; u++) {
                const int ci = lane + u * NT;
                int p, r, k;
                lfrd_chunk<PIX, G>(ci, false, p, r, k);
                if (ci < N::NINT) {
                    PIX *t = (p ? ct[p - 1] + r * FCP : lt + r * FLP) + CPX * k;
                    if (k == 0 && c > c0) {
                        const PIX *src = (p ? S.ct[tb ^ 1][p - 1] + r * FCP : S.lt[tb ^ 1] + r * FLP) + (p ? CW : 64);
                        Chunk16::to_lds(Chunk16::from_lds(src), t);
                    } else {
                        Chunk16::to_lds(vi[u], t);
                    }
                }
            }
        }
        LFR_T(8);
        // the hand-off ordering above; wavefront-scope fence
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        __syncthreads();
        LFR_T(0);
        const bool pre = s_pre;
        if (!mover) {
            if (pre) lfrd_top<PIX, G>(vt, P, sbx, sby, lane);
        } else if (c > c0) {
            lfrd_store<PIX, G>(S, tb ^ 1, P, sbx - 1, sby, ml, false, 0);  // SB c - 1's bottom rows first
        }
        LFR_T(9);
        // column pass part 1: every row's edge x = 0 (one row per lane)
        static_assert(64 + 2 * G::CH <= NT, "one column-pass row per filtering lane");
        int lpx[40];
        LfEv<true, 16> lev;
        const bool cl = !mover && lane < 64 + 2 * G::CH, cwide = lane < 64 || !G::SH;
        uint32_t *rowp = nullptr;
        const uint32_t *pwl = nullptr;
        if (cl) {
            if (lane < 64) {
                rowp = (uint32_t *) (lt + (lane + 8) * FLP + L::XO);
                pwl = S.prog[tb] + (LFP_YC + (lane >> 3) * 16) / 4;
            } else {
                const int p = 1 + (lane - 64 >= G::CH), r = lane - 64 - (p - 1) * G::CH;
                rowp = (uint32_t *) (ct[p - 1] + (r + 8) * FCP + L::XO);
                pwl = S.prog[tb] + (LFP_CC + (r >> 3) * LFP_CSTRIDE(G::SH)) / 4;
            }
            if (cwide) lf_row_wide_1<PIX>(rowp, pwl, S.lut, bd, lpx, lev);
            else lf_row_narrow_1<PIX>(rowp, pwl, S.lut, bd, lpx, lev);
        }
        __syncthreads();
        LFR_T(13);
        // SB c - 1's last columns are final: publish its bottom rows (the hand-off above) while
        // the filtering waves run the rest of the column pass
        if (mover && sbx > 0) {
            // the left halo's bottom 8 rows of each plane: one chunk per lane 0..23
            if (ml < 24) {
                const int p = ml >> 3, r = (p ? L::CR : 72) - 8 + (ml & 7);
                const PIX *t = p ? ct[p - 1] + r * FCP : lt + r * FLP;
                PIX *g = lfr_addr<PIX, G>(P, sbx, sby, p, r, 0);
                const CT w = Chunk16::from_lds(t);
                st_sc1(g, (uint64_t) w.x | (uint64_t) w.y << 32);
                st_sc1((char *) g + 8, (uint64_t) w.z | (uint64_t) w.w << 32);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (ml == 0) __hip_atomic_store((gu32 *) &progress[s_task], c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (mover && c > c0) lfrd_store<PIX, G>(S, tb ^ 1, P, sbx - 1, sby, ml, false, 1);   // the rest of SB c - 1
        // column pass part 2
        if (cl) {
            if (cwide) lf_row_wide_2<PIX>(rowp, pwl, S.lut, bd, lpx, lev);
            else lf_row_narrow_2<PIX>(rowp, pwl, S.lut, bd, lpx, lev);
        }
        __syncthreads();
        LFR_T(2);
        if (!pre) {
            if (lane == NT && dep != ~0u) {
                const uint32_t need = c + 1;
                for (uint32_t n = 0; seen < need; n++) {
                    seen = __hip_atomic_load((gu32 *) &progress[dep], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (seen >= need) break;
                    if (n > spin) { atomicAdd(&ctr[2], 1u); seen = need; break; }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            if (c == c0) LFR_T(12); else LFR_T(10);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            __syncthreads();
            LFR_T(11);
            if (!mover) lfrd_top<PIX, G>(vt, P, sbx, sby, lane);
        }
        if (!mover) {
#pragma unroll
            for (int u = 0; u < N::NUT; u++) {
                const int ci = lane + u * NT;
                int p, r, k;
                lfrd_chunk<PIX, G>(ci, true, p, r, k);
                if (ci >= N::NTOP || k == 0) continue;
                PIX *t = p ? ct[p - 1] + r * FCP : lt + r * FLP;
                Chunk16::to_lds(vt[u], t + CPX * k);
            }
            // the next SB's interior and program word, in flight under the row pass (issued
            // after the top halo's LDS writes: their waits never cover these loads)
            if (c + 1 < ncols) {
                lfrd_issue<PIX, G>(vi, P, sbx + 1, sby, lane, false);
                if (lane < L::PROG / 4) pwv = ((const uint32_t *) recs[T[4 + c + 1 - c0]].prog)[lane];
            }
        }
        __syncthreads();
        LFR_T(3);
        lf_passes_v<PIX, G, NT, 2, true>(lt, ct, S.prog[tb], S.lut, lane, bd);
        LFR_T(4);
        if (LFR_PROF && !pre) pacc[5]++;
        if (LFR_PROF) pacc[6]++;
    }
    // the row's last SB: its whole tile, then its bottom rows are final
    if (mover) {
        lfrd_store<PIX, G>(S, (int) ((ncols - 1 - c0) & 1), P, (int) ncols - 1, sby, ml, true, 2);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (ml == 0) __hip_atomic_store((gu32 *) &progress[s_task], ncols, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (LFR_PROF && lane == 0) {
        pacc[7] = clock64() - tk0;
        for (int i = 0; i < 14; i++) atomicAdd(&lfr_prof[i], pacc[i]);
        atomicAdd(&lfr_prof[14], 1ull);
    }
    lfrd_retire(ctr, ntasks, lane, NT + 64, &s_last);
}

// k_lfro: k_lfrd with SB c's luma row pass overlapped with SB c + 1's luma column pass
// (4:2:0). Within one SB row the SBs are serial (vp9lpf.c:183-230 order: SB c + 1's first
// column edge reads SB c's right columns after SB c's row edges), but the dependency is per
// pixel row: the column pass of pixel rows 0..31 of SB c + 1 needs SB c's row pass only
// through its row edges y = 32 / 36 (later row edges read rows >= 32), rows 32..63 all of
// it; SB c + 1's row edges y <= 28 read rows <= 35 only after the column pass of rows
// 0..31... (and its edges y >= 32 the rest). So the luma column pass runs as two waves of 32
// rows each (H0: rows 0..31, H1: rows 32..63) and the row pass as one wave (R), each
// starting as soon as the pixel rows it reads are final: the luma chain per SB is about
// half a row pass + a column pass instead of a column pass + a row pass. Chroma (both
// planes, both passes: half the luma edges) runs on one wave of its own (C), a loader wave
// (L) stages interiors, program words and top halos, the store wave (S) writes the tiles
// and publishes the row hand-off as k_lfrd does. The waves order through monotonic
// per-workgroup counters in LDS (a wave's DS operations execute in order, so a counter
// written after a tile write and read before the tile read orders them; the fences are
// compiler-only, wavefront scope). Every wait is bounded: one that gives up is counted in
// ctr[2] like a hand-off timeout (the batch fails with VP9HIP_EBUG), never hangs.
// One intra worker wave inside a k_lfro launch (LfrIntra): k_predd's ticket loop, whole
// interiors written through (the LF loader reads them with sc1 loads in the same launch).
// The last wave zeroes the tickets; the LF's last workgroup zeroes the done flags (it waited
// for every one of them).
// Bounded waits of k_lfro and its intra workers measure time, not polls: a poll's cost
// differs by orders of magnitude between an LDS counter and an agent-scope flag in HBM under
// load, so poll counts gave the waits on intra done flags (2^22 global polls) seconds where
// their sibling waves' LDS waits (2^20 polls) gave up within ~50 ms, and a long intra wait
// could end in a spurious timeout. Every wait gives up after LFRO_WAIT_TICKS of the 100 MHz
// realtime clock; waits on intra done flags after half that, and then abort their workgroup,
// so they give up first. A wait that gives up is counted (ctr[2] / pctr[2]: the batch fails
// with VP9HIP_EBUG), never hangs. The test hook (ctr[3] / pctr[3] = n) bounds every wait to
// n polls instead.
// Dispatch order: an LF workgroup's waits on done flags assume the intra worker workgroups
// (blockIdx < nblk, dispatched first as the hardware dispatches in blockIdx order) are
// resident; if they were starved the waits would give up (EBUG) rather than hang.
#define LFRO_WAIT_TICKS 20000000ull               // 200 ms
DEV bool wait_expired(uint32_t n, uint32_t spin, uint64_t &t0, uint64_t ticks)
{
    if (spin) return n > spin;
    if (n == 0) { t0 = __builtin_amdgcn_s_memrealtime(); return false; }
    return (n & 63) == 0 && __builtin_amdgcn_s_memrealtime() - t0 > ticks;
}

template <typename PIX, class G>
DEV void lfri_worker(const LfrIntra &li, const FrameDesc *__restrict__ frames, PredLds<PIX, G, true> &S, int lane)
{
#if PRED_LTAB_LDS
    load_ltab<PIX>(S.ltab, li.ptab, lane);
#endif
    const uint32_t spin = li.pctr[3];                 // 0: LFRO_WAIT_TICKS / 2
    for (;;) {
        uint32_t task = 0;
        if (lane == 0) task = atomicAdd(&li.pctr[0], 1u);
        task = __builtin_amdgcn_readfirstlane(task);
        if (task >= (uint32_t) li.n) break;
        const uint32_t slot = __builtin_amdgcn_readfirstlane(li.list[task]);
        const WGRec *wg = li.wgs + slot;
        const uint32_t info = li.sbinfo[slot];
        const SBRec sb = li.sbs[wg->sb[0]];
        const uint32_t W = (uint32_t) frames[sb.frame].sb_cols;
        uint32_t dep = ~0u;
        if (lane == 0 && (info & 2) && sb.sbx > 0) dep = slot - 1;
        if (lane == 1 && (info & 4) && sb.sby > 0) dep = slot - W;
        if (lane == 2 && (info & 8) && sb.sbx > 0 && sb.sby > 0) dep = slot - W - 1;
        uint64_t tw = 0;
        for (uint32_t t = 0;; t++) {
            const bool ok = dep == ~0u || __hip_atomic_load((gu32 *) &li.done[dep], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
            if (__all(ok)) break;
            if (wait_expired(t, spin, tw, LFRO_WAIT_TICKS / 2)) {
                if (lane == 0) atomicAdd(&li.pctr[2], 1u);
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        pred_wg<PIX, G, true, 2>(wg, li.sbs, li.jobs, li.passes, frames, li.resid, li.ptab, S, lane, li.dbg);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) __hip_atomic_store((gu32 *) &li.done[slot], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        wave_sync();
    }
    if (lane == 0 && atomicAdd(&li.pctr[1], 1u) == (uint32_t) (li.nblk * LFRI_WAVES) - 1) {
        li.pctr[0] = 0;
        li.pctr[1] = 0;
    }
}

#define LFRO_NTH 512                              // R, H0, H1, C, L1, L2, S1, S2
#define LFRO_NTB 3                                // LDS tiles: SB i + 3 reuses SB i's
#ifndef LFRO_ROLES
#define LFRO_ROLES 0x76543210u                    // roles of waves 7..0, one nibble each
#endif
struct LfroSync { uint32_t ld_int, ld_top, ra, rb, h0x, h1x, h0, h1, cx, c, st1, st2, abort, pad[3]; };
DEV void lfro_pub(uint32_t *f, uint32_t v)
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// (after a wait gives up, `abort` makes every later wait of the workgroup return at once:
// the task drains in one bounded wait instead of one per SB and counter)
DEV void lfro_wait(uint32_t *f, uint32_t need, uint32_t *ctr, uint32_t *abort, uint64_t &wc, uint32_t spin)
{
    const uint64_t t0 = LFR_PROF ? clock64() : 0;
    uint64_t tw = 0;
    for (uint32_t n = 0; __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < need; n++) {
        if (wait_expired(n, spin, tw, LFRO_WAIT_TICKS) ||
            __hip_atomic_load(abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
            if ((threadIdx.x & 63) == 0 && !__hip_atomic_exchange(abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))
                atomicAdd(&ctr[2], 1u);
            break;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (LFR_PROF) wc += clock64() - t0;
}
// the store wave's tile parts: 0 the left chunk column's bottom 8 rows (SB sbx - 1's last
// columns, final after this SB's first column edges; sc1; one chunk per lane 0..23),
// 1 the other bottom rows (sc1; the last chunk column only for the row's last SB:
// otherwise the next tile's part 0) = lfrd_store part 0, 2 everything else (the top
// halo's corner chunk is never modified) = lfrd_store part 1: compile-time row walks
template <typename PIX, class G, class LDS>
DEV void lfro_store(const LDS &S, int tb, const LfrPlanes &P, int sbx, int sby, int ml, bool last, int part)
{
    typedef LfP<PIX, G> L;
    typedef Chunk16::T CT;
    if (part == 0) {
        if (sbx > 0 && ml < 24) {
            const int p = ml >> 3, r = (p ? L::CR : 72) - 8 + (ml & 7);
            const PIX *t = p ? S.ct[tb][p - 1] + r * L::UVP : S.lt[tb] + r * L::YP;
            PIX *g = lfr_addr<PIX, G>(P, sbx, sby, p, r, 0);
            const CT w = Chunk16::from_lds(t);
            st_sc1(g, (uint64_t) w.x | (uint64_t) w.y << 32);
            st_sc1((char *) g + 8, (uint64_t) w.z | (uint64_t) w.w << 32);
        }
        return;
    }
    lfrd_store<PIX, G>(S, tb, P, sbx, sby, ml, last, part - 1);
}
#define LFRO_EDGE_WIDE(k, C0)                                                                            \
    {                                                                                                    \
        const uint32_t ww = (k) < 2 ? pw0 : (k) < 4 ? pw1 : (k) < 6 ? pw2 : pw3;                         \
        const uint32_t m = (ww >> (16 * ((k) & 1))) & 255, in = (ww >> (16 * ((k) & 1) + 8)) & 255;      \
        if (m >> 6) lf_reg<8 * (k) + 8 - (C0)>(px, m >> 6, ev(2 * (k), m), bd);                          \
        if (in) lf_reg<8 * (k) + 12 - (C0)>(px, 1, ev(2 * (k) + 1, in), bd);                             \
    }
// FI: intra worker workgroups in front of the LF tasks (LfrIntra; a separate instantiation,
// so the plain kernel keeps its registers and LDS)
template <typename PIX, class G, bool FI>
__global__ __launch_bounds__(LFRO_NTH) __attribute__((amdgpu_waves_per_eu(4))) void k_lfro(const uint32_t *__restrict__ tasks, const LFRec *__restrict__ recs,
                                                   const FrameDesc *__restrict__ frames, uint32_t *ctr, int ntasks,
                                                   LfrIntra li)
{
    static_assert(G::SH == 1 && G::SV == 1, "4:2:0: one chroma wave holds both planes' 32 lines");
    typedef LfP<PIX, G> L;
    typedef Chunk16::T CT;
    typedef LfrdN<PIX, G> N;
    constexpr int FLP = L::YP, FCP = L::UVP, CW = G::CW, CH = G::CH;
    constexpr int NUI = (N::NINT + 63) / 64, NUT = (N::NTOP + 63) / 64, NPW = (L::PROG / 4 + 63) / 64;
    // the LF tiles, or (intra worker workgroups) LFRI_WAVES intra tiles
    __shared__ union {
        struct { LfrLds<PIX, G, LFRO_NTB> S; LfroSync F; } lf;
        PredLds<PIX, G, true> pr[FI ? LFRI_WAVES : 1];
    } U;
    LfrLds<PIX, G, LFRO_NTB> &S = U.lf.S;
    LfroSync &F = U.lf.F;
    __shared__ uint32_t s_task, s_last;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    if constexpr (FI) {
        if ((int) blockIdx.x < li.nblk) {         // an intra worker workgroup
            if (w < LFRI_WAVES) lfri_worker<PIX, G>(li, frames, U.pr[w], lane);
            return;
        }
    }
    // wave -> role (R 0, H0 1, H1 2, C 3, L1 4, L2 5, S1 6, S2 7), one nibble per wave; wave
    // w runs on SIMD w % 4 (-DLFRO_ROLES=...: another permutation, for A/B builds; pairing
    // each filtering wave with the lightest helper measured equal, profiles/r04l)
    const int role = (int) ((LFRO_ROLES >> (4 * w)) & 15);
    uint32_t *const progress = ctr + 4;
    __builtin_amdgcn_s_setprio(3);
    // LFR_PROF builds: per wave role, cycles waiting on the workgroup's counters (lfr_prof[w]);
    // R's lifetime [8], L2's waits for the row above [9], SB steps [10], workgroups [11],
    // R's steady-state span (SBs n/4 .. 3n/4) [12] over [13] SBs, L2's first-SB wait [14],
    // R's waits for the top halo [15]
    uint64_t wc = 0, wrow = 0, wfill = 0, wtop = 0, tq1 = 0, tspan = 0, nspan = 0;
    const uint64_t tk0 = LFR_PROF ? clock64() : 0;
    __shared__ uint32_t s_tl;
    if (tid == 0) {
        s_task = atomicAdd(&ctr[0], 1u);
        s_tl = LFR_PROF && s_task == TL_TASK && atomicCAS(&lfro_tl_claim, 0u, 1u) == 0u;
    }
    if (tid < 16) (&F.ld_int)[tid] = 0;
    __syncthreads();
    const bool tl = LFR_PROF && s_tl;
#define TLE(e, i) do { if (tl && lane == 0 && (i) >= TL_SB0 && (i) < TL_SB0 + TL_NSB) lfro_tl[e][(i) - TL_SB0] = clock64(); } while (0)
    const uint32_t spin = ctr[3];                     // 0: the waits' time budgets (wait_expired)
    const uint32_t *T = tasks + tasks[s_task];
    const uint32_t dep = T[0], ncols = T[1], c0 = T[2];
    const LFRec &rec0 = recs[T[4]];
    const FrameDesc &fd = frames[rec0.frame];
    const int bd = fd.bd, sby = rec0.sby;
    LfrPlanes P;
    P.b0 = fd.plane[0]; P.d1 = fd.plane[1] - P.b0; P.d2 = fd.plane[2] - P.b0;
    P.pit0 = fd.pitch[0]; P.pit1 = fd.pitch[1];
    for (int i = tid; i < 64; i += LFRO_NTH) S.lut[i] = lf_eih(i, fd.sharp, bd);
    __syncthreads();
    const int n = (int) (ncols - c0);
    if (role == 0) {
        // ---- R: luma row edges, one lane per pixel column (lf_line_col_wide split at its
        // halves, each waiting for the column pass of the rows it loads)
        for (int i = 0; i < n; i++) {
            const int tb = i % LFRO_NTB, tp = tb ? tb - 1 : LFRO_NTB - 1;
            PIX *colp = S.lt[tb] + L::XL + lane;
            const uint64_t wt0 = wc;
            lfro_wait(&F.ld_top, (uint32_t) i + 1, ctr, &F.abort, wc, spin);
            if (LFR_PROF) wtop += wc - wt0;
            TLE(0, i);
            lfro_wait(&F.h0, (uint32_t) i + 1, ctr, &F.abort, wc, spin);
            TLE(1, i);
            const uint32_t *pw = S.prog[tb] + (LFP_YR + (lane >> 3) * 16) / 4;
            const uint32_t pw0 = pw[0], pw1 = pw[1], pw2 = pw[2], pw3 = pw[3];
            LfEv<true, 16> ev;
            lf_eih_wide<true>(ev, pw0, pw1, pw2, pw3, S.lut);
            int px[40];
#pragma unroll
            for (int r = 0; r < 40; r++) px[r] = colp[r * FLP];
            LFRO_EDGE_WIDE(0, 0) LFRO_EDGE_WIDE(1, 0) LFRO_EDGE_WIDE(2, 0) LFRO_EDGE_WIDE(3, 0)
#pragma unroll
            for (int r = 1; r < 32; r++) colp[r * FLP] = (PIX) px[r];
#pragma unroll
            for (int r = 0; r < 8; r++) px[r] = px[32 + r];
            TLE(2, i);
            lfro_wait(&F.h1, (uint32_t) i + 1, ctr, &F.abort, wc, spin);
            TLE(3, i);
#pragma unroll
            for (int r = 8; r < 40; r++) px[r] = colp[(32 + r) * FLP];
            LFRO_EDGE_WIDE(4, 32)
            // pixel rows 24..31 are final (later row edges read rows >= 32): SB c + 1's
            // column pass of rows 0..31 may start
#pragma unroll
            for (int r = 0; r < 8; r++) colp[(32 + r) * FLP] = (PIX) px[r];
            lfro_pub(&F.ra, (uint32_t) i + 1);
            LFRO_EDGE_WIDE(5, 32) LFRO_EDGE_WIDE(6, 32) LFRO_EDGE_WIDE(7, 32)
#pragma unroll
            for (int r = 8; r < 40; r++) colp[(32 + r) * FLP] = (PIX) px[r];
            lfro_pub(&F.rb, (uint32_t) i + 1);
            TLE(4, i);
            if (LFR_PROF && i == n / 4) tq1 = clock64();
            if (LFR_PROF && i == (3 * n) / 4 && i > n / 4) { tspan = clock64() - tq1; nspan = (uint64_t) (i - n / 4); }
        }
    } else if (role <= 2) {
        // ---- H0 / H1: luma column edges of pixel rows 0..31 / 32..63, one lane per row
        const int h = role - 1;
        if (lane < 32) {
            const int row = h * 32 + lane;
            for (int i = 0; i < n; i++) {
                const int tb = i % LFRO_NTB, tp = tb ? tb - 1 : LFRO_NTB - 1;
                lfro_wait(&F.ld_int, (uint32_t) i + 1, ctr, &F.abort, wc, spin);
                if (i > 0) lfro_wait(h ? &F.rb : &F.ra, (uint32_t) i, ctr, &F.abort, wc, spin);
                TLE(5 + 2 * h, i);
                PIX *trow = S.lt[tb] + (row + 8) * FLP;
                // left halo: SB c - 1's last chunk, final for these rows now
                if (i > 0) Chunk16::to_lds(Chunk16::from_lds(S.lt[tp] + (row + 8) * FLP + 64), trow);
                uint32_t *rowp = (uint32_t *) (trow + L::XO);
                const uint32_t *pwl = S.prog[tb] + (LFP_YC + (row >> 3) * 16) / 4;
                int lpx[40];
                LfEv<true, 16> lev;
                lf_row_wide_1<PIX>(rowp, pwl, S.lut, bd, lpx, lev);
                lfro_pub(h ? &F.h1x : &F.h0x, (uint32_t) i + 1);
                lf_row_wide_2<PIX>(rowp, pwl, S.lut, bd, lpx, lev);
                lfro_pub(h ? &F.h1 : &F.h0, (uint32_t) i + 1);
                TLE(6 + 2 * h, i);
            }
        }
    } else if (role == 3) {
        // ---- C: chroma, both planes: column edges (lane = row), then row edges (lane = column)
        const int p = 1 + (lane >= CH), r = lane & (CH - 1);
        for (int i = 0; i < n; i++) {
            const int tb = i % LFRO_NTB, tp = tb ? tb - 1 : LFRO_NTB - 1;
            lfro_wait(&F.ld_int, (uint32_t) i + 1, ctr, &F.abort, wc, spin);
            TLE(9, i);
            PIX *trow = S.ct[tb][p - 1] + (r + 8) * FCP;
            if (i > 0) Chunk16::to_lds(Chunk16::from_lds(S.ct[tp][p - 1] + (r + 8) * FCP + CW), trow);
            uint32_t *rowp = (uint32_t *) (trow + L::XO);
            const uint32_t *pwc = S.prog[tb] + (LFP_CC + (r >> 3) * LFP_CSTRIDE(1)) / 4;
            int lpx[40];
            LfEv<true, 16> lev;
            lf_row_narrow_1<PIX>(rowp, pwc, S.lut, bd, lpx, lev);
            lfro_pub(&F.cx, (uint32_t) i + 1);
            lf_row_narrow_2<PIX>(rowp, pwc, S.lut, bd, lpx, lev);
            wave_sync();
            TLE(10, i);
            lfro_wait(&F.ld_top, (uint32_t) i + 1, ctr, &F.abort, wc, spin);
            TLE(11, i);
            PIX *colp = S.ct[tb][p - 1] + L::XL + r;
            const uint32_t *pwr = S.prog[tb] + (LFP_CR(1, 1) + (r >> 3) * LFP_CSTRIDE(1)) / 4;
            lf_line_col_narrow<PIX, FCP, true>(colp, pwr, S.lut, bd);
            lfro_pub(&F.c, (uint32_t) i + 1);
            TLE(12, i);
        }
    } else if (role == 4) {
        // ---- L1: interiors and program words, one SB ahead: SB i's are staged into tile
        // i % LFRO_NTB once SB i - LFRO_NTB is stored (S1, S2) and SB i - LFRO_NTB + 1's waves
        // have copied their left halos out of that tile; SB i + 1's loads are issued right after
        CT vi[NUI];
        uint32_t pwv[NPW];
        constexpr bool intra = FI;
        auto issue = [&](int c, bool halo) {
            if constexpr (intra) {
                // intra workers in this launch: SB (r, c)'s own intra and its pre-LF readers'
                // (LfrIntra), then sc1 loads of what they wrote through
                const int dx = lane == 1 ? 1 : lane >= 2 ? lane - 3 : 0, dy = lane >= 2 ? 1 : 0;
                uint32_t s = ~0u;
                if (lane < 5 && c + dx >= 0 && c + dx < fd.sb_cols && sby + dy < fd.sb_rows) {
                    s = T[4 + c - c0] + (uint32_t) (dy * fd.sb_cols + dx);
                    if (!(li.sbinfo[s] & 1)) s = ~0u;
                }
                uint64_t tw = 0;
                for (uint32_t t = 0;; t++) {
                    const bool ok = s == ~0u || __hip_atomic_load((gu32 *) &li.done[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
                    if (__all(ok)) break;
                    // half the siblings' budget, then the workgroup aborts: its other waves'
                    // waits on this wave end at once instead of timing out on their own
                    if (wait_expired(t, spin, tw, LFRO_WAIT_TICKS / 2)) {
                        if (lane == 0 && !__hip_atomic_exchange(&F.abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))
                            atomicAdd(&ctr[2], 1u);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
#pragma unroll
            for (int u = 0; u < NUI; u++) {
                const int ci = lane + 64 * u;
                int pp, rr, kk;
                lfrd_chunk<PIX, G>(ci, false, pp, rr, kk);
                if (ci < N::NINT && (kk > 0 || halo)) {
                    const PIX *g = lfr_addr<PIX, G>(P, c, sby, pp, rr, kk);
                    if constexpr (intra) {
                        const uint64_t lo = ld_sc1(g), hi = ld_sc1((const char *) g + 8);
                        vi[u] = make_uint4((uint32_t) lo, (uint32_t) (lo >> 32), (uint32_t) hi, (uint32_t) (hi >> 32));
                    } else {
                        const v4u x = *(const gv4u *) g;
                        vi[u] = make_uint4(x.x, x.y, x.z, x.w);
                    }
                }
            }
            const LFRec &rc = recs[T[4 + c - c0]];
#pragma unroll
            for (int q = 0; q < NPW; q++)
                if (lane + 64 * q < L::PROG / 4) pwv[q] = ((const uint32_t *) rc.prog)[lane + 64 * q];
        };
        issue((int) c0, c0 > 0);
        for (int i = 0; i < n; i++) {
            const int tb = i % LFRO_NTB, tp = tb ? tb - 1 : LFRO_NTB - 1;
            const bool halo = i == 0 && c0 > 0;
            if (i >= LFRO_NTB) {
                lfro_wait(&F.st1, (uint32_t) (i - LFRO_NTB + 1), ctr, &F.abort, wc, spin);
                lfro_wait(&F.st2, (uint32_t) (i - LFRO_NTB + 1), ctr, &F.abort, wc, spin);
            }
            if (i >= LFRO_NTB - 1) {
                lfro_wait(&F.h0x, (uint32_t) (i - LFRO_NTB + 2), ctr, &F.abort, wc, spin);
                lfro_wait(&F.h1x, (uint32_t) (i - LFRO_NTB + 2), ctr, &F.abort, wc, spin);
                lfro_wait(&F.cx, (uint32_t) (i - LFRO_NTB + 2), ctr, &F.abort, wc, spin);
            }
            TLE(13, i);
#pragma unroll
            for (int u = 0; u < NUI; u++) {
                const int ci = lane + 64 * u;
                int pp, rr, kk;
                lfrd_chunk<PIX, G>(ci, false, pp, rr, kk);
                if (ci < N::NINT && (kk > 0 || halo))
                    Chunk16::to_lds(vi[u], (pp ? S.ct[tb][pp - 1] + rr * FCP : S.lt[tb] + rr * FLP) + L::CPX * kk);
            }
#pragma unroll
            for (int q = 0; q < NPW; q++)
                if (lane + 64 * q < L::PROG / 4) S.prog[tb][lane + 64 * q] = pwv[q];
            lfro_pub(&F.ld_int, (uint32_t) i + 1);
            TLE(14, i);
            if (i + 1 < n) issue((int) (c0 + i) + 1, false);
        }
    } else if (role == 5) {
        // ---- L2: top halos, handed over by the row above (its progress reaches c + 1; the row LF's
        // hand-off: sc1 stores drained before the progress word, sc1 loads here), into tile
        // i % LFRO_NTB once SB i - LFRO_NTB is stored
        CT vt[NUT];
        uint32_t seen = T[3];
        for (int i = 0; i < n; i++) {
            const uint32_t c = c0 + (uint32_t) i;
            const int tb = i % LFRO_NTB, tp = tb ? tb - 1 : LFRO_NTB - 1;
            if (sby > 0) {
                if (dep != ~0u && seen < c + 1) {
                    const uint64_t tw0 = LFR_PROF ? clock64() : 0;
                    uint64_t tw = 0;
                    for (uint32_t k = 0;; k++) {
                        seen = __builtin_amdgcn_readfirstlane(
                            __hip_atomic_load((gu32 *) &progress[dep], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                        if (seen >= c + 1) break;
                        if (wait_expired(k, spin, tw, LFRO_WAIT_TICKS)) {
                            if (lane == 0) atomicAdd(&ctr[2], 1u);
                            seen = c + 1;
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                    }
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    if (LFR_PROF) { wrow += clock64() - tw0; if (i == 0) wfill += clock64() - tw0; }
                }
                TLE(15, i);
#pragma unroll
                for (int u = 0; u < NUT; u++) {
                    const int ci = lane + 64 * u;
                    int pp, rr, kk;
                    lfrd_chunk<PIX, G>(ci, true, pp, rr, kk);
                    if (ci >= N::NTOP || kk == 0) continue;
                    const PIX *g = lfr_addr<PIX, G>(P, (int) c, sby, pp, rr, kk);
                    const uint64_t lo = ld_sc1(g), hi = ld_sc1((const char *) g + 8);
                    vt[u] = make_uint4((uint32_t) lo, (uint32_t) (lo >> 32), (uint32_t) hi, (uint32_t) (hi >> 32));
                }
                if (i >= LFRO_NTB) {
                    lfro_wait(&F.st1, (uint32_t) (i - LFRO_NTB + 1), ctr, &F.abort, wc, spin);
                    lfro_wait(&F.st2, (uint32_t) (i - LFRO_NTB + 1), ctr, &F.abort, wc, spin);
                }
#pragma unroll
                for (int u = 0; u < NUT; u++) {
                    const int ci = lane + 64 * u;
                    int pp, rr, kk;
                    lfrd_chunk<PIX, G>(ci, true, pp, rr, kk);
                    if (ci >= N::NTOP || kk == 0) continue;
                    Chunk16::to_lds(vt[u], (pp ? S.ct[tb][pp - 1] + rr * FCP : S.lt[tb] + rr * FLP) + L::CPX * kk);
                }
            }
            lfro_pub(&F.ld_top, (uint32_t) i + 1);
            TLE(16, i);
        }
    } else if (role == 6) {
        // ---- S1: the bottom rows (sc1) and the row hand-off (progress word of this task)
        for (int i = 0; i < n; i++) {
            const int c = (int) c0 + i, tb = i % LFRO_NTB;
            const bool last = i == n - 1;
            if (c > 0) {
                // SB c - 1's last columns (this tile's left halo) are final after this SB's
                // first column edges: its bottom rows are then complete
                lfro_wait(&F.h1x, (uint32_t) i + 1, ctr, &F.abort, wc, spin);
                lfro_wait(&F.cx, (uint32_t) i + 1, ctr, &F.abort, wc, spin);
                TLE(17, i);
                lfro_store<PIX, G>(S, tb, P, c, sby, lane, false, 0);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (lane == 0) __hip_atomic_store((gu32 *) &progress[s_task], (uint32_t) c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                TLE(18, i);
            }
            lfro_wait(&F.rb, (uint32_t) i + 1, ctr, &F.abort, wc, spin);
            lfro_wait(&F.c, (uint32_t) i + 1, ctr, &F.abort, wc, spin);
            lfro_store<PIX, G>(S, tb, P, c, sby, lane, last, 1);
            if (last) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (lane == 0) __hip_atomic_store((gu32 *) &progress[s_task], ncols, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            lfro_pub(&F.st1, (uint32_t) i + 1);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
        // ---- S2: the tile's other rows
        for (int i = 0; i < n; i++) {
            const int c = (int) c0 + i, tb = i % LFRO_NTB;
            lfro_wait(&F.rb, (uint32_t) i + 1, ctr, &F.abort, wc, spin);
            lfro_wait(&F.c, (uint32_t) i + 1, ctr, &F.abort, wc, spin);
            lfro_wait(&F.h0x, (uint32_t) i + 1, ctr, &F.abort, wc, spin);
            TLE(19, i);
            lfro_store<PIX, G>(S, tb, P, c, sby, lane, i == n - 1, 2);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            lfro_pub(&F.st2, (uint32_t) i + 1);
            TLE(20, i);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (LFR_PROF && lane == 0) {
        atomicAdd(&lfr_prof[role], wc);
        if (role == 0) {
            atomicAdd(&lfr_prof[8], clock64() - tk0); atomicAdd(&lfr_prof[10], (unsigned long long) n); atomicAdd(&lfr_prof[11], 1ull);
            atomicAdd(&lfr_prof[12], tspan); atomicAdd(&lfr_prof[13], nspan); atomicAdd(&lfr_prof[15], wtop);
        }
        if (role == 5) { atomicAdd(&lfr_prof[9], wrow); atomicAdd(&lfr_prof[14], wfill); }
    }
    lfrd_retire(ctr, ntasks, tid, LFRO_NTH, &s_last);
    if (FI && s_last)
        for (int i = tid; i < li.n; i += LFRO_NTH) li.done[li.list[i]] = 0;
#undef TLE
}
#undef LFRO_EDGE_WIDE

// Residual arithmetic types per pixel type: 8-bit int16 coefficients / 32-bit math,
// high bit depth int32 coefficients / 64-bit math (vp9dsp_template.c dctcoef / dctint)
template <typename PIX> struct RT;
template <> struct RT<uint8_t> { typedef M32 M; typedef int16_t C; };
template <> struct RT<uint16_t> { typedef M64 M; typedef int32_t C; };

// PRED_PROF builds: a workgroup timeline of k_plf launches of one shape: per workgroup its
// start / end on the device real-time clock (s_memrealtime, 100 MHz) | kind << 62 (0 intra,
// 1 LF, 2 residual), for the launches whose npred equals that of the first launch seen with
// npred >= PLF_TL_MIN (tools/pred_prof.py --timeline)
#define PLF_TL_N 65536
#define PLF_TL_MIN 2000
KP_DEV unsigned long long plf_tl[PLF_TL_N][2];
KP_DEV unsigned int plf_tl_n, plf_tl_key;

// Fused wavefront launch (runtime schedule, stage()): launch t holds intra diagonal t, LF
// diagonal t - 3 (disjoint pixels) and the residuals of intra diagonal t + 1.
// Workgroups [0, npred) predict one SB each with wave 0 (the other waves exit), the next
// nlf loop-filter one SB each, the rest run residual jobs by transform code, NT/64 waves
// of 64/n jobs each.
template <typename PIX, class G>
__global__ __launch_bounds__(LfNT<G>::NT) void k_plf(PlfLaunch a, const uint32_t *__restrict__ plist,
                                                     const uint32_t *__restrict__ llist, const WGRec *__restrict__ wgs,
                                                     const SBRec *__restrict__ sbs, const PJob *__restrict__ jobs,
                                                     const uint32_t *__restrict__ passes, const LFRec *__restrict__ recs,
                                                     const RJob *__restrict__ rjobs, const FrameDesc *__restrict__ frames,
                                                     const void *__restrict__ coefs, int16_t *__restrict__ resid,
                                                     const uint32_t *__restrict__ ptab, int dbg)
{
    typedef typename RT<PIX>::M M;
    typedef typename RT<PIX>::C COEF;
    constexpr int NW = LfNT<G>::NT / 64;
    __shared__ union PlfLds { PredLds<PIX, G, false> p; LfLds<PIX, G> l; COEF r[NW][RWave<32, COEF>::E]; } S;
    const int b = blockIdx.x;
    bool tl_rec = false;
    uint64_t tl_t0 = 0;
    if (PRED_PROF && threadIdx.x == 0 && a.npred >= PLF_TL_MIN) {
        const uint32_t k = atomicCAS(&plf_tl_key, 0u, a.npred);
        tl_rec = k == 0 || k == a.npred;
        tl_t0 = __builtin_amdgcn_s_memrealtime();
    }
    auto tl_end = [&](uint64_t kind) {
        if (PRED_PROF && tl_rec) {
            const uint32_t i = atomicAdd(&plf_tl_n, 1u);
            if (i < PLF_TL_N) { plf_tl[i][0] = tl_t0 | kind << 62; plf_tl[i][1] = __builtin_amdgcn_s_memrealtime(); }
        }
    };
    if (b < (int) a.npred) {
        if (threadIdx.x >= 64) return;
#if PRED_LTAB_LDS
        load_ltab<PIX>(S.p.ltab, ptab, threadIdx.x);
#endif
        pred_wg<PIX, G, false>(wgs + plist[b], sbs, jobs, passes, frames, resid, ptab, S.p, threadIdx.x, dbg);
        tl_end(0);
        return;
    }
    if (b < (int) (a.npred + a.nlf)) {
        const uint64_t t0 = PRED_PROF ? clock64() : 0;
        lf_sb<PIX, G, LfNT<G>::NT>(recs[llist[b - a.npred]], frames, S.l, threadIdx.x, dbg >> 16);
        if (PRED_PROF && threadIdx.x == 0) { atomicAdd(&pred_prof[13], clock64() - t0); atomicAdd(&pred_prof[14], 1ull); }
        tl_end(1);
        return;
    }
    // residual workgroups: transform code k owns ceil(rn[k] / (NW * 64 / n)) of them
    int rb = b - (int) (a.npred + a.nlf);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const COEF *cf = (const COEF *) coefs;
#define RES_CASE(K, N, TC)                                                                                  \
    {                                                                                                       \
        const int nwg = ((int) a.rn[K] + NW * (64 / N) - 1) / (NW * (64 / N));                             \
        if (rb < nwg) {                                                                                     \
            resid_wave<N, TC, PIX, M, COEF>(rjobs + a.roff[K], a.rn[K], rb * NW + wave, lane, frames, cf,    \
                                            resid, S.r[wave]);                                              \
            tl_end(2);                                                                                      \
            return;                                                                                         \
        }                                                                                                   \
        rb -= nwg;                                                                                          \
    }
    RES_CASE(0, 4, 0) RES_CASE(1, 8, 1) RES_CASE(2, 16, 2) RES_CASE(3, 32, 3) RES_CASE(4, 4, 4)
#undef RES_CASE
}

// --------------------------------------------------------------- MC (k_mcq)
template <typename PIX>
DEV int mc_ref(const PIX *r, int pitch, int w, int h, int x, int y)
{
    x = x < 0 ? 0 : x >= w ? w - 1 : x;
    y = y < 0 ? 0 : y >= h ? h - 1 : y;
    return r[(size_t) y * pitch + x];
}

template <typename PIX>
DEV int mc_sample(const PIX *r, int pitch, int w, int h, int X, int Y, int mx, int my, int filter, int bd)
{
    if (!mx && !my) return mc_ref(r, pitch, w, h, X, Y);
    if (filter == 3) {   // bilinear (vp9dsp_template.c:2150-2227)
        if (mx && my) {
            int a0 = mc_ref(r, pitch, w, h, X, Y), a1 = mc_ref(r, pitch, w, h, X + 1, Y);
            int b0 = mc_ref(r, pitch, w, h, X, Y + 1), b1 = mc_ref(r, pitch, w, h, X + 1, Y + 1);
            int t0 = a0 + ((mx * (a1 - a0) + 8) >> 4), t1 = b0 + ((mx * (b1 - b0) + 8) >> 4);
            return t0 + ((my * (t1 - t0) + 8) >> 4);
        }
        int a0 = mc_ref(r, pitch, w, h, X, Y);
        int a1 = mx ? mc_ref(r, pitch, w, h, X + 1, Y) : mc_ref(r, pitch, w, h, X, Y + 1);
        int m = mx ? mx : my;
        return a0 + ((m * (a1 - a0) + 8) >> 4);
    }
    const int16_t *fx = vp9t_subpel_filters[filter][mx], *fy = vp9t_subpel_filters[filter][my];
    if (mx && my) {   // 2-D: pixel-clipped horizontal pass (vp9dsp_template.c:2076-2113)
        int acc = 0;
        for (int k = 0; k < 8; k++) {
            int s = 0;
            for (int t = 0; t < 8; t++) s += fx[t] * mc_ref(r, pitch, w, h, X - 3 + t, Y - 3 + k);
            acc += fy[k] * clipbd((s + 64) >> 7, bd);
        }
        return clipbd((acc + 64) >> 7, bd);
    }
    int s = 0;
    if (mx) for (int t = 0; t < 8; t++) s += fx[t] * mc_ref(r, pitch, w, h, X - 3 + t, Y);
    else    for (int t = 0; t < 8; t++) s += fy[t] * mc_ref(r, pitch, w, h, X, Y - 3 + t);
    return clipbd((s + 64) >> 7, bd);
}

// MC unit packing: the units of a workgroup as one flat list of lane tasks (so a 4x4 chroma
// unit takes a few lanes instead of a wave and every wave is full; at C5 an 8K frame is
// ~243k units). One separable 8-tap form gives every unscaled case exactly: an identity
// phase is the tap 128 (an exact copy), so the copy and 1-D paths of
// vp9dsp_template.c:1971-2059 equal the pixel-clipped 2-D form (2076-2113) with one
// identity pass; the bilinear filter (2150-2227) is the 8-tap (0, 0, 0, 8(16 - m), 8m, 0,
// 0, 0): a + ((m(b - a) + 8) >> 4) = ((16 - m)a + mb + 8) >> 4, scaled by 8, and its
// values lie between a and b (the clip is an identity). Scaled references keep the
// per-pixel sampler (mc_sample), one pixel per task.
#define MCP_U 64                                  // units per workgroup
struct McL {                                      // a unit as its tasks read it (LDS)
    uint64_t ref[2], dst;
    int32_t ix[2], iy[2];
    int32_t pitch;
    uint16_t x, y, rw[2], rh[2];
    uint8_t lw, h, mx[2], my[2], filter, nref, direct, bd, cat, pad[3];
};

// the last unit k < n with off[k] <= g (units without tasks of this category share the
// next one's offset and are stepped over)
DEV int mcp_find(const uint32_t *off, int n, uint32_t g)
{
    int k = 0;
#pragma unroll
    for (int st = MCP_U / 2; st; st >>= 1)
        if (k + st < n && off[k + st] <= g) k += st;
    return k;
}

// a unit as its tasks read it; cat 0: unscaled, height a multiple of 8; 1: unscaled, 4
// rows; 2: a scaled reference. direct (per reference): the filter window of every pixel
// lies inside the visible reference (no clamping)
DEV void mcp_unit(const McUnit &m, const FrameDesc *__restrict__ frames, McL &L)
{
    const FrameDesc &fd = frames[m.frame];
    const int p = m.plane, c = p ? 1 : 0;
    L.dst = fd.plane[p];
    L.pitch = fd.pitch[c];
    L.x = m.x; L.y = m.y;
    L.lw = (uint8_t) (31 - __builtin_clz((unsigned) m.w));
    L.h = m.h;
    L.filter = m.filter > 3 ? 3 : m.filter;
    L.nref = m.nref;
    L.bd = (uint8_t) fd.bd;
    L.direct = 0;
    bool scaled = false;
    for (int k = 0; k < 2; k++) {
        const int rf = m.ref[k] > 2 ? 0 : m.ref[k];
        const McRef r = m.r[k];
        L.ref[k] = fd.ref[rf][p];
        L.ix[k] = r.ix; L.iy[k] = r.iy;
        L.mx[k] = r.mx & 15; L.my[k] = r.my & 15;
        L.rw[k] = (uint16_t) fd.refw[rf][c]; L.rh[k] = (uint16_t) fd.refh[rf][c];
        if (k < m.nref) {
            scaled |= r.dx != 16 || r.dy != 16;
            if (r.ix >= 3 && r.iy >= 3 && r.ix + (int) m.w + 4 < fd.refw[rf][c] && r.iy + (int) m.h + 4 < fd.refh[rf][c])
                L.direct |= (uint8_t) (1 << k);
        }
    }
    L.cat = scaled ? 2 : (m.h & 7) ? 1 : 0;
}
// exclusive task offsets per category over the workgroup's units (wave 0)
DEV void mcp_offsets(uint32_t (*off)[MCP_U + 1], const uint32_t (&cnt)[3], int tid)
{
    if (tid < 64) {
#pragma unroll
        for (int c = 0; c < 3; c++) {
            uint32_t v = cnt[c];
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t o = __shfl_up(v, d);
                if (tid >= d) v += o;
            }
            off[c][tid + 1] = v;
            if (tid == 0) off[c][0] = 0;
        }
    }
}
// scaled references: one pixel per task (mc_unit_pixels)
template <typename PIX>
DEV void mcp_scaled(const McUnit *__restrict__ units, const uint32_t *off, int nu, const FrameDesc *__restrict__ frames, int tid,
                    int g0 = 0, int gs = 256)
{
    const uint32_t T2 = off[nu];
    for (uint32_t g = tid + g0; g < T2; g += gs) {
        const int k = mcp_find(off, nu, g);
        const McUnit m = units[k];
        const FrameDesc &fd = frames[m.frame];
        const int p = m.plane, c = p ? 1 : 0, W = m.w;
        const uint32_t ti = g - off[k];
        const int yy = (int) ti / W, xx = (int) ti - yy * W;
        int out = 0;
        for (int r = 0; r < m.nref; r++) {
            const int rf = m.ref[r];
            const McRef q = m.r[r];
            const int px = q.mx + xx * q.dx, py = q.my + yy * q.dy;
            const int v = mc_sample<PIX>((const PIX *) fd.ref[rf][p], fd.pitch[c], fd.refw[rf][c], fd.refh[rf][c],
                                         q.ix + (px >> 4), q.iy + (py >> 4), px & 15, py & 15, m.filter, fd.bd);
            out = r ? (out + v + 1) >> 1 : v;
        }
        ((PIX *) fd.plane[p])[(size_t) (m.y + yy) * fd.pitch[c] + m.x + xx] = (PIX) out;
    }
}

// --------------------------------------------------------------- k_mcq
// 4-column lane tasks: a lane filters 4 adjacent output columns x R rows (R = 8; 4 for
// units 4 rows tall) from ONE load per window row (12 pixels, x - 3 .. x + 8: 8-bit a
// 12-byte load, 16-bit 24 bytes), where round 4's one-column tasks (k_mcp) loaded 8 pixels
// per row and output pixel (4x the load instructions, 2.7x the bytes through the L1). The
// horizontal 8-tap sums are packed dot products: 8-bit v_dot4_i32_i8 on the pixels biased
// by -128 (every VP9 8-tap and the bilinear-as-8-tap sum to 128, so + 128 * 128 restores
// the bias; an identity phase, tap 128, does not fit an int8 and selects the pixel), 16-bit
// v_dot2_i32_i16 on the pixel pairs (odd columns from byte-aligned pairs). The vertical pass
// accumulates each horizontally filtered row into the <= 8 outputs whose taps cover it.
// Arithmetic exactly vp9dsp_template.c:2076-2113 (the pixel-clipped 2-D form, equal to the
// 1-D / copy forms through identity phases, see above); compound averages
// (a + b + 1) >> 1 per packed pixel as (a | b) - ((a ^ b) >> 1).
struct McqLds {
    alignas(16) int16_t taps[64][8];              // [filter * 16 + phase], bilinear = filter 3
    uint32_t tap8[64][2];                         // the same taps as int8 quads (identity phases: 0)
    alignas(16) uint32_t tapp[64][12];            // vertical tap pairs (f[q], f[q + 1]), q = -1..7 (f[-1] = f[8] = 0)
    McL u[MCP_U];
    uint32_t off[3][MCP_U + 1];
};
typedef struct __attribute__((packed, aligned(1))) { uint32_t d[3]; } McqW8;   // 12 window bytes
typedef struct __attribute__((packed, aligned(2))) { uint32_t d[6]; } McqW16;  // 12 window pixels
typedef short mcq_s2 __attribute__((ext_vector_type(2)));

template <typename PIX> struct McqW { static constexpr int N = sizeof(PIX) == 1 ? 3 : 6; };

// one window row: direct (inside the visible reference) or with every pixel clamped
template <typename PIX>
DEV void mcq_load(const PIX *rp, const PIX *wrow, int pitch, int X, int Y, bool direct, int rw, int rh,
                  uint32_t (&d)[McqW<PIX>::N])
{
    if (direct) {                                      // wrow: the window row's first pixel
        if constexpr (sizeof(PIX) == 1) {
            const __attribute__((address_space(1))) McqW8 *q = (const __attribute__((address_space(1))) McqW8 *) wrow;
            d[0] = q->d[0]; d[1] = q->d[1]; d[2] = q->d[2];
        } else {
            const __attribute__((address_space(1))) McqW16 *q = (const __attribute__((address_space(1))) McqW16 *) wrow;
#pragma unroll
            for (int i = 0; i < 6; i++) d[i] = q->d[i];
        }
        return;
    }
    const int yc = Y < 0 ? 0 : Y >= rh ? rh - 1 : Y;
    const PIX *row = rp + (size_t) yc * pitch;
    constexpr int PPW = 4 / sizeof(PIX);
#pragma unroll
    for (int i = 0; i < McqW<PIX>::N; i++) {
        uint32_t w = 0;
#pragma unroll
        for (int b = 0; b < PPW; b++) {
            const int x = X + i * PPW + b, xc = x < 0 ? 0 : x >= rw ? rw - 1 : x;
            w |= (uint32_t) row[xc] << (8 * sizeof(PIX) * b);
        }
        d[i] = w;
    }
}

// the 4 horizontal 8-tap outputs of one window row (clipped pixels)
template <typename PIX>
DEV void mcq_h(const uint32_t (&d)[McqW<PIX>::N], const uint32_t (&th)[4], bool ident, int pmax, int (&h)[4])
{
    if constexpr (sizeof(PIX) == 1) {
        const uint32_t e0 = d[0] ^ 0x80808080u, e1 = d[1] ^ 0x80808080u, e2 = d[2] ^ 0x80808080u;
#pragma unroll
        for (int o = 0; o < 4; o++) {
            const uint32_t lo = o ? __builtin_amdgcn_alignbyte(e1, e0, o) : e0;
            const uint32_t hi = o ? __builtin_amdgcn_alignbyte(e2, e1, o) : e1;
            const int s = __builtin_amdgcn_sdot4((int) lo, (int) th[0],
                                                 __builtin_amdgcn_sdot4((int) hi, (int) th[1], 16384 + 64, false), false);
            h[o] = ident ? (int) ((lo >> 24) ^ 0x80u) : med3_0(s >> 7, 255);
        }
    } else {
        uint32_t sh[5];
#pragma unroll
        for (int k = 0; k < 5; k++) sh[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], 2);
#pragma unroll
        for (int o = 0; o < 4; o++) {
            int s = 64;
#pragma unroll
            for (int q = 3; q >= 0; q--) {
                const uint32_t w = (o & 1) ? sh[(o >> 1) + q] : d[(o >> 1) + q];
                s = __builtin_amdgcn_sdot2(__builtin_bit_cast(mcq_s2, w), __builtin_bit_cast(mcq_s2, th[q]), s, false);
            }
            h[o] = med3_0(s >> 7, pmax);
        }
    }
}

template <typename PIX, int R, bool V, bool DIRECT>
DEV void mcq_rows(const McL &u, const McqLds &S, int xx, int yy)
{
    constexpr int NW = sizeof(PIX) == 1 ? 1 : 2;          // output dwords per row
    constexpr int NR = V ? R + 7 : R, R0 = V ? 0 : 3;      // window rows the vertical pass reads
    const int pmax = (1 << u.bd) - 1, pitch = u.pitch;
    uint32_t outp[R][NW];
    for (int k = 0; k < u.nref; k++) {
        const int fh = u.filter * 16 + u.mx[k], fv = u.filter * 16 + u.my[k];
        uint32_t th[4];
        if constexpr (sizeof(PIX) == 1) {
            th[0] = S.tap8[fh][0]; th[1] = S.tap8[fh][1]; th[2] = th[3] = 0;
        } else {
            const uint4 hw = *(const uint4 *) S.taps[fh];
            th[0] = hw.x; th[1] = hw.y; th[2] = hw.z; th[3] = hw.w;
        }
        uint32_t fp[9];                                    // fp[q + 1] = (f[q], f[q + 1])
        if (V) {
            const uint4 v0 = *(const uint4 *) &S.tapp[fv][0], v1 = *(const uint4 *) &S.tapp[fv][4];
            fp[0] = v0.x; fp[1] = v0.y; fp[2] = v0.z; fp[3] = v0.w;
            fp[4] = v1.x; fp[5] = v1.y; fp[6] = v1.z; fp[7] = v1.w; fp[8] = S.tapp[fv][8];
        }
        const bool ident = u.mx[k] == 0;
        const int X = u.ix[k] + xx - 3, Y = u.iy[k] + yy - 3 + R0;
        const PIX *rp = (const PIX *) u.ref[k];
        const int rw = u.rw[k], rh = u.rh[k];
        const PIX *wrow = DIRECT ? rp + (ptrdiff_t) Y * pitch + X : rp;
        int acc[R][4];
#pragma unroll
        for (int t = 0; t < R; t++)
#pragma unroll
            for (int o = 0; o < 4; o++) acc[t][o] = 64;
        // window rows in pairs (2 jp, 2 jp + 1): the vertical pass as one v_dot2 per output
        // and pair, the rows' filtered pixels packed (h[2 jp], h[2 jp + 1]) per column
#pragma unroll
        for (int jp = 0; jp < (NR + 1) / 2; jp++) {
            int h[2][4];
#pragma unroll
            for (int e = 0; e < 2; e++) {
                const int j = 2 * jp + e;
                if (j >= NR) {
#pragma unroll
                    for (int o = 0; o < 4; o++) h[e][o] = 0;
                    continue;
                }
                uint32_t d[McqW<PIX>::N];
                mcq_load<PIX>(rp, wrow, pitch, X, Y + j, DIRECT, rw, rh, d);
                if (DIRECT) wrow += pitch;
                mcq_h<PIX>(d, th, ident, pmax, h[e]);
            }
            if (V) {
                uint32_t pk[4];
#pragma unroll
                for (int o = 0; o < 4; o++) pk[o] = (uint32_t) h[0][o] | (uint32_t) h[1][o] << 16;
                const int j = 2 * jp;
#pragma unroll
                for (int t = (j > 7 ? j - 7 : 0); t <= (j + 1 < R - 1 ? j + 1 : R - 1); t++)
#pragma unroll
                    for (int o = 0; o < 4; o++)
                        acc[t][o] = __builtin_amdgcn_sdot2(__builtin_bit_cast(mcq_s2, pk[o]), __builtin_bit_cast(mcq_s2, fp[j - t + 1]),
                                                           acc[t][o], false);
            } else {
#pragma unroll
                for (int e = 0; e < 2; e++)
                    if (2 * jp + e < NR)
#pragma unroll
                        for (int o = 0; o < 4; o++) acc[2 * jp + e][o] = h[e][o];
            }
        }
#pragma unroll
        for (int t = 0; t < R; t++) {
            int v[4];
#pragma unroll
            for (int o = 0; o < 4; o++) v[o] = V ? med3_0(acc[t][o] >> 7, pmax) : acc[t][o];
            uint32_t w[NW];
            if constexpr (sizeof(PIX) == 1) w[0] = (uint32_t) v[0] | (uint32_t) v[1] << 8 | (uint32_t) v[2] << 16 | (uint32_t) v[3] << 24;
            else { w[0] = (uint32_t) v[0] | (uint32_t) v[1] << 16; w[1] = (uint32_t) v[2] | (uint32_t) v[3] << 16; }
            constexpr uint32_t HM = sizeof(PIX) == 1 ? 0x7f7f7f7fu : 0x7fff7fffu;
#pragma unroll
            for (int i = 0; i < NW; i++) outp[t][i] = k ? (outp[t][i] | w[i]) - (((outp[t][i] ^ w[i]) >> 1) & HM) : w[i];
        }
    }
    typedef __attribute__((address_space(1))) PIX gpo;
    gpo *dst = (gpo *) u.dst + (size_t) (u.y + yy) * pitch + u.x + xx;
#pragma unroll
    for (int t = 0; t < R; t++) {
        if constexpr (sizeof(PIX) == 1) *(__attribute__((address_space(1))) uint32_t *) (dst + (size_t) t * pitch) = outp[t][0];
        else {
            typedef uint32_t v2u __attribute__((ext_vector_type(2)));
            v2u w2; w2.x = outp[t][0]; w2.y = outp[t][1];
            *(__attribute__((address_space(1))) v2u *) (dst + (size_t) t * pitch) = w2;
        }
    }
}

template <typename PIX, int R>
DEV void mcq_task(const McL &u, const McqLds &S, int xx, int yy)
{
    const bool v = u.my[0] | (u.nref > 1 ? u.my[1] : 0);
    const bool dir = (u.direct & ((1 << u.nref) - 1)) == ((1 << u.nref) - 1);
    if (__all(dir)) {
        if (__any(v)) mcq_rows<PIX, R, true, true>(u, S, xx, yy);
        else mcq_rows<PIX, R, false, true>(u, S, xx, yy);
    } else {
        if (__any(v)) mcq_rows<PIX, R, true, false>(u, S, xx, yy);
        else mcq_rows<PIX, R, false, false>(u, S, xx, yy);
    }
}

template <typename PIX>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_mcq(const McUnit *__restrict__ units, int nunits,
                                             const FrameDesc *__restrict__ frames)
{
    __shared__ McqLds S;
    const int tid = threadIdx.x;
    const int u0 = blockIdx.x * MCP_U, nu = nunits - u0 < MCP_U ? nunits - u0 : MCP_U;
    {
        // filter rows: 3 x 16 8-tap phases, then the bilinear ones as 8-taps; int8 quads of
        // the non-identity phases (every tap of phases 1-15 lies in [-128, 127])
        const int r = tid >> 2, q = (tid & 3) * 2;
        int16_t a, b;
        if (r < 48) { a = vp9t_subpel_filters[r >> 4][r & 15][q]; b = vp9t_subpel_filters[r >> 4][r & 15][q + 1]; }
        else {
            const int m = r & 15;
            a = (int16_t) (q == 2 ? 0 : q == 4 ? 8 * m : 0);
            b = (int16_t) (q == 2 ? 8 * (16 - m) : 0);
        }
        S.taps[r][q] = a;
        S.taps[r][q + 1] = b;
        S.tapp[r][q + 1] = (uint32_t) (uint16_t) a | (uint32_t) (uint16_t) b << 16;   // (f[q], f[q + 1])
        // tap8 dword (q >> 2): bytes q & 3, (q & 3) + 1 of it from this thread's pair
        const uint32_t pr = (r & 15) ? ((uint32_t) (uint8_t) a | (uint32_t) (uint8_t) b << 8) << (8 * (q & 3)) : 0u;
        const uint32_t other = __shfl_xor(pr, 1);
        if (!(tid & 1)) S.tap8[r][q >> 2] = pr | other;
    }
    __syncthreads();
    {
        // the odd-q pairs (f[q], f[q + 1]), q = -1, 1, 3, 5, 7, from the int16 rows
        const int r = tid >> 2;
        for (int q = 2 * (tid & 3) - 1; q < 8; q += 8) {
            const int lo = q < 0 ? 0 : S.taps[r][q], hi = q + 1 > 7 ? 0 : S.taps[r][q + 1];
            S.tapp[r][q + 1] = (uint32_t) (uint16_t) lo | (uint32_t) (uint16_t) hi << 16;
        }
    }
    uint32_t cnt[3] = { 0, 0, 0 };
    if (tid < nu) {
        McL L;
        const McUnit m = units[u0 + tid];
        mcp_unit(m, frames, L);
        // 4 x 8 (4 x 4) pixels per task
        cnt[L.cat] = L.cat == 2 ? (uint32_t) m.w * m.h : (uint32_t) m.w * m.h >> (L.cat ? 4 : 5);
        S.u[tid] = L;
    }
    mcp_offsets(S.off, cnt, tid);
    __syncthreads();
    // blockIdx.y: one of gridDim.y slices of the tasks (a workgroup of 64 large units is
    // otherwise the launch's tail: units per workgroup are counted, not their pixels)
    const int g0 = (int) blockIdx.y * 256, gs = 256 * (int) gridDim.y;
    for (int c = 0; c < 2; c++) {
        const uint32_t T = S.off[c][nu];
        for (uint32_t g = tid + g0; g < T; g += gs) {
            const int k = mcp_find(S.off[c], nu, g);
            const McL &u = S.u[k];
            const uint32_t ti = g - S.off[c][k];
            const int lq = u.lw - 2;                      // 4-column groups per row: w / 4
            const int xx = (int) (ti & ((1u << lq) - 1)) * 4;
            const int yy = (int) (ti >> lq) << (c ? 2 : 3);
            if (c == 0) mcq_task<PIX, 8>(u, S, xx, yy);
            else mcq_task<PIX, 4>(u, S, xx, yy);
        }
    }
    mcp_scaled<PIX>(units + u0, S.off[2], nu, frames, tid, g0, gs);
}

// ------------------------------------------------------------ launchers
template <int N, int TC>
static void launch_resid_n(int hb, hipStream_t st, int n, const RJob *jobs, const FrameDesc *frames,
                           const void *coefs, int16_t *resid)
{
    const int per = RWAVES * (64 / N);
    const int nb = (n + per - 1) / per;
    if (hb)
        hipLaunchKernelGGL((k_resid<N, TC, uint16_t, M64, int32_t>), dim3(nb), dim3(64 * RWAVES), 0, st,
                           jobs, n, frames, (const int32_t *) coefs, resid);
    else
        hipLaunchKernelGGL((k_resid<N, TC, uint8_t, M32, int16_t>), dim3(nb), dim3(64 * RWAVES), 0, st,
                           jobs, n, frames, (const int16_t *) coefs, resid);
}
template <int N, int TC>
static void launch_resid_dev_n(int hb, hipStream_t st, int ub, const RJob *jobs, const uint32_t *rng,
                               const FrameDesc *frames, const void *coefs, int16_t *resid)
{
    const int per = RWAVES * (64 / N);
    const int nb = (ub + per - 1) / per;
    if (hb)
        hipLaunchKernelGGL((k_resid_dev<N, TC, uint16_t, M64, int32_t>), dim3(nb), dim3(64 * RWAVES), 0, st,
                           jobs, rng, frames, (const int32_t *) coefs, resid);
    else
        hipLaunchKernelGGL((k_resid_dev<N, TC, uint8_t, M32, int16_t>), dim3(nb), dim3(64 * RWAVES), 0, st,
                           jobs, rng, frames, (const int16_t *) coefs, resid);
}
template <typename PIX, class G>
static void launch_pred_g(hipStream_t st, int nwg, size_t pad, const uint32_t *list, const WGRec *wgs, const SBRec *sbs,
                          const PJob *jobs, const uint32_t *passes, const FrameDesc *frames, const int16_t *resid,
                          const uint32_t *ptab, int dbg)
{
    hipLaunchKernelGGL((k_pred<PIX, G>), dim3(nwg), dim3(64), pad, st, list, wgs, sbs, jobs, passes, frames, resid, ptab, dbg);
}
template <typename PIX>
static void launch_pred_p(int ss, hipStream_t st, int nwg, size_t pad, const uint32_t *list, const WGRec *wgs,
                          const SBRec *sbs, const PJob *jobs, const uint32_t *passes, const FrameDesc *frames,
                          const int16_t *resid, const uint32_t *ptab, int dbg)
{
    switch (ss) {
    case 3: launch_pred_g<PIX, Geo<1, 1>>(st, nwg, pad, list, wgs, sbs, jobs, passes, frames, resid, ptab, dbg); break;
    case 1: launch_pred_g<PIX, Geo<1, 0>>(st, nwg, pad, list, wgs, sbs, jobs, passes, frames, resid, ptab, dbg); break;
    case 2: launch_pred_g<PIX, Geo<0, 1>>(st, nwg, pad, list, wgs, sbs, jobs, passes, frames, resid, ptab, dbg); break;
    default: launch_pred_g<PIX, Geo<0, 0>>(st, nwg, pad, list, wgs, sbs, jobs, passes, frames, resid, ptab, dbg); break;
    }
}
template <typename PIX>
static void launch_predd_p(hipStream_t st, int n, int wgcap, const uint32_t *list, const uint32_t *sbinfo, const WGRec *wgs,
                           const SBRec *sbs, const PJob *jobs, const uint32_t *passes, const FrameDesc *frames,
                           const int16_t *resid, const uint32_t *ptab, uint32_t *ctr, uint32_t *done, int dbg)
{
    hipLaunchKernelGGL((k_predd<PIX, Geo<1, 1>>), dim3(std::min(n, wgcap)), dim3(64), 0, st, list, n, sbinfo, wgs, sbs, jobs,
                       passes, frames, resid, ptab, ctr, done, dbg);
}
template <typename PIX, class G>
static void launch_lf_g(hipStream_t st, int nsb, const uint32_t *list, const LFRec *recs, const FrameDesc *frames, int dbg)
{
    hipLaunchKernelGGL((k_lf<PIX, G>), dim3(nsb), dim3(LfNT<G>::NT), 0, st, list, recs, frames, dbg);
}
template <typename PIX, class G>
static void launch_lfr_g(hipStream_t st, int ntasks, const uint32_t *tasks, const LFRec *recs, const FrameDesc *frames, uint32_t *ctr,
                         const KCfg &k, const LfrIntra &li)
{
    if constexpr (G::SH == 1 && G::SV == 1) {
        // the band-overlapped k_lfro (4:2:0 default; KCfg::lfro = 0: k_lfrd). Measured
        // (profiles/r04l): C5 k_lfr 1,403 -> 1,021 us per 8K frame, C2 300 -> 238 us
        if (k.lfro) {
            if (li.nblk)
                hipLaunchKernelGGL((k_lfro<PIX, G, true>), dim3(li.nblk + ntasks), dim3(LFRO_NTH), 0, st, tasks, recs, frames,
                                   ctr, ntasks, li);
            else
                hipLaunchKernelGGL((k_lfro<PIX, G, false>), dim3(ntasks), dim3(LFRO_NTH), 0, st, tasks, recs, frames, ctr,
                                   ntasks, li);
            return;
        }
    }
    hipLaunchKernelGGL((k_lfrd<PIX, G>), dim3(ntasks), dim3(LfNT<G>::NT + 64), 0, st, tasks, recs, frames, ctr, ntasks);
}
template <typename PIX>
static void launch_lfr_p(int ss, hipStream_t st, int ntasks, const uint32_t *tasks, const LFRec *recs, const FrameDesc *frames,
                         uint32_t *ctr, const KCfg &k, const LfrIntra &li)
{
    switch (ss) {
    case 3: launch_lfr_g<PIX, Geo<1, 1>>(st, ntasks, tasks, recs, frames, ctr, k, li); break;
    case 1: launch_lfr_g<PIX, Geo<1, 0>>(st, ntasks, tasks, recs, frames, ctr, k, li); break;
    case 2: launch_lfr_g<PIX, Geo<0, 1>>(st, ntasks, tasks, recs, frames, ctr, k, li); break;
    default: launch_lfr_g<PIX, Geo<0, 0>>(st, ntasks, tasks, recs, frames, ctr, k, li); break;
    }
}
template <typename PIX>
static void launch_lf_p(int ss, hipStream_t st, int nsb, const uint32_t *list, const LFRec *recs, const FrameDesc *frames,
                        int dbg)
{
    switch (ss) {
    case 3: launch_lf_g<PIX, Geo<1, 1>>(st, nsb, list, recs, frames, dbg); break;
    case 1: launch_lf_g<PIX, Geo<1, 0>>(st, nsb, list, recs, frames, dbg); break;
    case 2: launch_lf_g<PIX, Geo<0, 1>>(st, nsb, list, recs, frames, dbg); break;
    default: launch_lf_g<PIX, Geo<0, 0>>(st, nsb, list, recs, frames, dbg); break;
    }
}
template <typename PIX, class G>
static void launch_plf_g(hipStream_t st, const PlfLaunch &pl, const uint32_t *plist, const uint32_t *llist, const WGRec *wgs,
                         const SBRec *sbs, const PJob *jobs, const uint32_t *passes, const LFRec *recs, const RJob *rjobs,
                         const FrameDesc *frames, const void *coefs, int16_t *resid, const uint32_t *ptab, int dbg)
{
    constexpr int NW = LfNT<G>::NT / 64;
    static const int n_of[5] = { 4, 8, 16, 32, 4 };
    int nblk = (int) (pl.npred + pl.nlf);
    for (int k = 0; k < 5; k++) nblk += ((int) pl.rn[k] + NW * (64 / n_of[k]) - 1) / (NW * (64 / n_of[k]));
    if (nblk <= 0) return;
    hipLaunchKernelGGL((k_plf<PIX, G>), dim3(nblk), dim3(LfNT<G>::NT), 0, st, pl, plist, llist, wgs, sbs, jobs, passes,
                       recs, rjobs, frames, coefs, resid, ptab, dbg);
}
template <typename PIX>
static void launch_plf_p(int ss, hipStream_t st, const PlfLaunch &pl, const uint32_t *plist, const uint32_t *llist,
                         const WGRec *wgs, const SBRec *sbs, const PJob *jobs, const uint32_t *passes, const LFRec *recs,
                         const RJob *rjobs, const FrameDesc *frames, const void *coefs, int16_t *resid,
                         const uint32_t *ptab, int dbg)
{
    switch (ss) {
    case 3: launch_plf_g<PIX, Geo<1, 1>>(st, pl, plist, llist, wgs, sbs, jobs, passes, recs, rjobs, frames, coefs, resid, ptab, dbg); break;
    case 1: launch_plf_g<PIX, Geo<1, 0>>(st, pl, plist, llist, wgs, sbs, jobs, passes, recs, rjobs, frames, coefs, resid, ptab, dbg); break;
    case 2: launch_plf_g<PIX, Geo<0, 1>>(st, pl, plist, llist, wgs, sbs, jobs, passes, recs, rjobs, frames, coefs, resid, ptab, dbg); break;
    default: launch_plf_g<PIX, Geo<0, 0>>(st, pl, plist, llist, wgs, sbs, jobs, passes, recs, rjobs, frames, coefs, resid, ptab, dbg); break;
    }
}
extern "C" {
#if KP(0)
// PRED_PROF builds: read and clear the intra workgroup phase sums (profiling only)
int vp9hip_pred_prof_read(unsigned long long *out)
{
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(pred_prof), 16 * sizeof(unsigned long long)) != hipSuccess) return -1;
    static const unsigned long long z[16] = {0};
    return hipMemcpyToSymbol(HIP_SYMBOL(pred_prof), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
// PRED_PROF builds: the k_plf workgroup timeline (n = entries, then 2 words each; profiling
// only, not in the ABI), cleared after the read
int vp9hip_plf_tl_read(unsigned long long *out, int cap, int *n)
{
    unsigned int k = 0;
    if (hipMemcpyFromSymbol(&k, HIP_SYMBOL(plf_tl_n), 4) != hipSuccess) return -1;
    *n = (int) std::min<unsigned int>(k, PLF_TL_N);
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(plf_tl), (size_t) std::min(*n, cap) * 16) != hipSuccess) return -1;
    const unsigned int z = 0;
    return hipMemcpyToSymbol(HIP_SYMBOL(plf_tl_n), &z, 4) == hipSuccess && hipMemcpyToSymbol(HIP_SYMBOL(plf_tl_key), &z, 4) == hipSuccess ? 0 : -1;
}
// LFR_PROF builds: read and clear the row-LF phase sums (profiling only, not in the ABI)
// LFR_PROF builds: the k_lfro event timeline (24 x 8 shader-clock values; profiling only)
int vp9hip_lfro_tl_read(unsigned long long *out)
{
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(lfro_tl), sizeof(lfro_tl)) == hipSuccess ? 0 : -1;
}
int vp9hip_lfr_prof_read(unsigned long long *out)
{
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(lfr_prof), 16 * sizeof(unsigned long long)) != hipSuccess) return -1;
    static const unsigned long long z[16] = {0};
    return hipMemcpyToSymbol(HIP_SYMBOL(lfr_prof), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
int vp9hip_launch_resid(int hb, hipStream_t st, int tcode, int n, const RJob *jobs, const FrameDesc *frames,
                        const void *coefs, int16_t *resid)
{
    if (n <= 0) return 0;
    switch (tcode) {
    case 0: launch_resid_n<4, 0>(hb, st, n, jobs, frames, coefs, resid); break;
    case 1: launch_resid_n<8, 1>(hb, st, n, jobs, frames, coefs, resid); break;
    case 2: launch_resid_n<16, 2>(hb, st, n, jobs, frames, coefs, resid); break;
    case 3: launch_resid_n<32, 3>(hb, st, n, jobs, frames, coefs, resid); break;
    case 4: launch_resid_n<4, 4>(hb, st, n, jobs, frames, coefs, resid); break;
    default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
int vp9hip_launch_resid_dev(int hb, hipStream_t st, int tcode, int ub, const RJob *jobs, const uint32_t *rng,
                            const FrameDesc *frames, const void *coefs, int16_t *resid)
{
    if (ub <= 0) return 0;
    switch (tcode) {
    case 0: launch_resid_dev_n<4, 0>(hb, st, ub, jobs, rng, frames, coefs, resid); break;
    case 1: launch_resid_dev_n<8, 1>(hb, st, ub, jobs, rng, frames, coefs, resid); break;
    case 2: launch_resid_dev_n<16, 2>(hb, st, ub, jobs, rng, frames, coefs, resid); break;
    case 3: launch_resid_dev_n<32, 3>(hb, st, ub, jobs, rng, frames, coefs, resid); break;
    case 4: launch_resid_dev_n<4, 4>(hb, st, ub, jobs, rng, frames, coefs, resid); break;
    default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
int vp9hip_launch_resid_multi(int hb, hipStream_t st, const uint32_t *off, const uint32_t *n, const RJob *jobs,
                              const FrameDesc *frames, const void *coefs, int16_t *resid)
{
    static const int tn[5] = { 4, 8, 16, 32, 4 };
    ResidMulti a;
    a.w0[0] = 0;
    for (int t = 0; t < 5; t++) {
        a.off[t] = off[t]; a.n[t] = n[t];
        const uint32_t per = 64 / tn[t];
        a.w0[t + 1] = a.w0[t] + (n[t] + per - 1) / per;
    }
    if (!a.w0[5]) return 0;
    const int nb = (int) ((a.w0[5] + RWAVES - 1) / RWAVES);
    if (hb)
        hipLaunchKernelGGL((k_resid_multi<uint16_t, M64, int32_t>), dim3(nb), dim3(64 * RWAVES), 0, st, a, jobs, frames,
                           (const int32_t *) coefs, resid);
    else
        hipLaunchKernelGGL((k_resid_multi<uint8_t, M32, int16_t>), dim3(nb), dim3(64 * RWAVES), 0, st, a, jobs, frames,
                           (const int16_t *) coefs, resid);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
#endif
#if KP(1)
// fmt: bit 0 high bit depth, bit 1 ss_h, bit 2 ss_v
int vp9hip_launch_pred(int fmt, hipStream_t st, int nwg, const uint32_t *list, const WGRec *wgs, const SBRec *sbs,
                       const PJob *jobs, const uint32_t *passes, const FrameDesc *frames, const int16_t *resid,
                       const uint32_t *ptab, int dbg)
{
    if (nwg <= 0) return 0;
    const size_t pad = (size_t) ((dbg >> 8) & 255) * 1024;     // profiling: occupancy sweep via LDS padding
    if (fmt & 1) launch_pred_p<uint16_t>(fmt >> 1, st, nwg, pad, list, wgs, sbs, jobs, passes, frames, resid, ptab, dbg);
    else         launch_pred_p<uint8_t>(fmt >> 1, st, nwg, pad, list, wgs, sbs, jobs, passes, frames, resid, ptab, dbg);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
// k_predd (4:2:0 only: fmt bits 1..2 must be 3): n = the list length, wgcap the grid's cap
int vp9hip_launch_predd(int fmt, hipStream_t st, int n, int wgcap, const uint32_t *list, const uint32_t *sbinfo, const WGRec *wgs,
                        const SBRec *sbs, const PJob *jobs, const uint32_t *passes, const FrameDesc *frames,
                        const int16_t *resid, const uint32_t *ptab, uint32_t *ctr, uint32_t *done, int dbg)
{
    if (n <= 0) return 0;
    if ((fmt >> 1) != 3 || wgcap <= 0) return -1;
    if (fmt & 1) launch_predd_p<uint16_t>(st, n, wgcap, list, sbinfo, wgs, sbs, jobs, passes, frames, resid, ptab, ctr, done, dbg);
    else         launch_predd_p<uint8_t>(st, n, wgcap, list, sbinfo, wgs, sbs, jobs, passes, frames, resid, ptab, ctr, done, dbg);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
int vp9hip_launch_lf(int fmt, hipStream_t st, int nsb, const uint32_t *list, const LFRec *recs,
                     const FrameDesc *frames, int dbg)
{
    if (nsb <= 0) return 0;
    if (fmt & 1) launch_lf_p<uint16_t>(fmt >> 1, st, nsb, list, recs, frames, dbg);
    else         launch_lf_p<uint8_t>(fmt >> 1, st, nsb, list, recs, frames, dbg);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
#endif
int vp9hip_launch_lfr_8(int ss, hipStream_t st, int ntasks, const uint32_t *tasks, const LFRec *recs, const FrameDesc *frames,
                        uint32_t *ctr, const KCfg &k, const LfrIntra &li);
#if KP(2)
int vp9hip_launch_lfr_8(int ss, hipStream_t st, int ntasks, const uint32_t *tasks, const LFRec *recs, const FrameDesc *frames,
                        uint32_t *ctr, const KCfg &k, const LfrIntra &li)
{
    launch_lfr_p<uint8_t>(ss, st, ntasks, tasks, recs, frames, ctr, k, li);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
#endif
int vp9hip_launch_lfr_16(int ss, hipStream_t st, int ntasks, const uint32_t *tasks, const LFRec *recs, const FrameDesc *frames,
                        uint32_t *ctr, const KCfg &k, const LfrIntra &li);
#if KP(3)
int vp9hip_launch_lfr_16(int ss, hipStream_t st, int ntasks, const uint32_t *tasks, const LFRec *recs, const FrameDesc *frames,
                        uint32_t *ctr, const KCfg &k, const LfrIntra &li)
{
    launch_lfr_p<uint16_t>(ss, st, ntasks, tasks, recs, frames, ctr, k, li);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
#endif
int vp9hip_launch_plf_8(int ss, hipStream_t st, const PlfLaunch *pl, const uint32_t *plist, const uint32_t *llist, const WGRec *wgs,
                        const SBRec *sbs, const PJob *jobs, const uint32_t *passes, const LFRec *recs, const RJob *rjobs,
                        const FrameDesc *frames, const void *coefs, int16_t *resid, const uint32_t *ptab, int dbg);
#if KP(4)
int vp9hip_launch_plf_8(int ss, hipStream_t st, const PlfLaunch *pl, const uint32_t *plist, const uint32_t *llist, const WGRec *wgs,
                        const SBRec *sbs, const PJob *jobs, const uint32_t *passes, const LFRec *recs, const RJob *rjobs,
                        const FrameDesc *frames, const void *coefs, int16_t *resid, const uint32_t *ptab, int dbg)
{
    launch_plf_p<uint8_t>(ss, st, *pl, plist, llist, wgs, sbs, jobs, passes, recs, rjobs, frames, coefs, resid, ptab, dbg);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
#endif
int vp9hip_launch_plf_16(int ss, hipStream_t st, const PlfLaunch *pl, const uint32_t *plist, const uint32_t *llist, const WGRec *wgs,
                        const SBRec *sbs, const PJob *jobs, const uint32_t *passes, const LFRec *recs, const RJob *rjobs,
                        const FrameDesc *frames, const void *coefs, int16_t *resid, const uint32_t *ptab, int dbg);
#if KP(5)
int vp9hip_launch_plf_16(int ss, hipStream_t st, const PlfLaunch *pl, const uint32_t *plist, const uint32_t *llist, const WGRec *wgs,
                        const SBRec *sbs, const PJob *jobs, const uint32_t *passes, const LFRec *recs, const RJob *rjobs,
                        const FrameDesc *frames, const void *coefs, int16_t *resid, const uint32_t *ptab, int dbg)
{
    launch_plf_p<uint16_t>(ss, st, *pl, plist, llist, wgs, sbs, jobs, passes, recs, rjobs, frames, coefs, resid, ptab, dbg);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
#endif
#if KP(0)
// li: intra workers inside the launch (null or nblk = 0: none; k_lfro, 4:2:0 only)
int vp9hip_launch_lfr(int fmt, hipStream_t st, int ntasks, const uint32_t *tasks, const LFRec *recs,
                      const FrameDesc *frames, uint32_t *ctr, const KCfg *k, const LfrIntra *li)
{
    if (ntasks <= 0) return 0;
    const LfrIntra none = {};
    if (li && li->nblk && (!k->lfro || (fmt >> 1) != 3 || li->n <= 0)) return -1;
    return (fmt & 1 ? vp9hip_launch_lfr_16 : vp9hip_launch_lfr_8)(fmt >> 1, st, ntasks, tasks, recs, frames, ctr, *k,
                                                                  li && li->nblk ? *li : none);
}
int vp9hip_launch_plf(int fmt, hipStream_t st, const PlfLaunch *pl, const uint32_t *plist, const uint32_t *llist,
                      const WGRec *wgs, const SBRec *sbs, const PJob *jobs, const uint32_t *passes, const LFRec *recs,
                      const RJob *rjobs, const FrameDesc *frames, const void *coefs, int16_t *resid, const uint32_t *ptab,
                      int dbg)
{
    return (fmt & 1 ? vp9hip_launch_plf_16 : vp9hip_launch_plf_8)(fmt >> 1, st, pl, plist, llist, wgs, sbs, jobs, passes,
                                                                  recs, rjobs, frames, coefs, resid, ptab, dbg);
}
int vp9hip_launch_mc(int hb, hipStream_t st, int n, const McUnit *units, const FrameDesc *frames, const KCfg *k)
{
    if (n <= 0) return 0;
    // k_mcq: 64 units per workgroup, each unit group's tasks split into slices (grid y):
    // ~4k workgroups at least, 2 to 8 slices (KCfg::mcq_slices overrides; profiles/r04k)
    const int nb = (n + MCP_U - 1) / MCP_U;
    const int ns = k->mcq_slices > 0 ? std::min(16, k->mcq_slices) : std::max(2, std::min(8, 4096 / nb));
    if (hb) hipLaunchKernelGGL((k_mcq<uint16_t>), dim3(nb, ns), dim3(256), 0, st, units, n, frames);
    else    hipLaunchKernelGGL((k_mcq<uint8_t>), dim3(nb, ns), dim3(256), 0, st, units, n, frames);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
#endif
}
