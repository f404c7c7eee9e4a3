/*
 * ORACLE (test infrastructure only) — scalar C restatement of the reference VP9
 * DSP functions, instantiated twice by vp9_oracle.c:
 *   OB == 8 : pixel uint8_t, dctcoef int16_t, dctint int32_t (vp9dsp_8bpp.c:23-25,
 *             bit_depth_template.c:79-82)
 *   OB == 16: pixel uint16_t, dctcoef int32_t, dctint int64_t, runtime bit depth bd
 *             (vp9dsp_10bpp.c / vp9dsp_12bpp.c, bit_depth_template.c:51-54)
 * Compiled with -fwrapv: the reference's unsigned products (e.g. `x * 11585U`)
 * wrap modulo 2^32 and are converted back to int, which -fwrapv int32 arithmetic
 * reproduces exactly. Never linked into the product.
 */
#if OB == 8
#define PIX uint8_t
#define COEF int16_t
#define DINT int32_t
#define F(n) n##_8
#else
#define PIX uint16_t
#define COEF int32_t
#define DINT int64_t
#define F(n) n##_16
#endif

static inline int F(clip_px)(int v, int bd) { int m = (1 << bd) - 1; return v < 0 ? 0 : v > m ? m : v; }

/* ------------------------------------------------------------------ itxfm
 * vp9dsp_template.c:1155-1778. IN(x) = (dctint) in[x * stride]; outputs are
 * stored to dctcoef (truncating) exactly like the reference `out[]`. */
#define IN(x) ((DINT) in[(x) * s])
#define RND(v) (((v) + (1 << 13)) >> 14)

static void F(idct4)(const COEF *in, ptrdiff_t s, COEF *out)
{
    DINT t0 = RND((IN(0) + IN(2)) * 11585);
    DINT t1 = RND((IN(0) - IN(2)) * 11585);
    DINT t2 = RND(IN(1) * 6270 - IN(3) * 15137);
    DINT t3 = RND(IN(1) * 15137 + IN(3) * 6270);
    out[0] = t0 + t3; out[1] = t1 + t2; out[2] = t1 - t2; out[3] = t0 - t3;
}

static void F(iadst4)(const COEF *in, ptrdiff_t s, COEF *out)
{
    DINT t0 = 5283 * IN(0) + 15212 * IN(2) + 9929 * IN(3);
    DINT t1 = 9929 * IN(0) - 5283 * IN(2) - 15212 * IN(3);
    DINT t2 = 13377 * (IN(0) - IN(2) + IN(3));
    DINT t3 = 13377 * IN(1);
    out[0] = RND(t0 + t3); out[1] = RND(t1 + t3); out[2] = RND(t2); out[3] = RND(t0 + t1 - t3);
}

static void F(idct8)(const COEF *in, ptrdiff_t s, COEF *out)
{
    DINT t0a = RND((IN(0) + IN(4)) * 11585), t1a = RND((IN(0) - IN(4)) * 11585);
    DINT t2a = RND(IN(2) * 6270 - IN(6) * 15137), t3a = RND(IN(2) * 15137 + IN(6) * 6270);
    DINT t4a = RND(IN(1) * 3196 - IN(7) * 16069), t5a = RND(IN(5) * 13623 - IN(3) * 9102);
    DINT t6a = RND(IN(5) * 9102 + IN(3) * 13623), t7a = RND(IN(1) * 16069 + IN(7) * 3196);
    DINT t0 = t0a + t3a, t1 = t1a + t2a, t2 = t1a - t2a, t3 = t0a - t3a;
    DINT t4 = t4a + t5a, t7 = t7a + t6a;
    t5a = t4a - t5a; t6a = t7a - t6a;
    DINT t5 = RND((t6a - t5a) * 11585), t6 = RND((t6a + t5a) * 11585);
    out[0] = t0 + t7; out[1] = t1 + t6; out[2] = t2 + t5; out[3] = t3 + t4;
    out[4] = t3 - t4; out[5] = t2 - t5; out[6] = t1 - t6; out[7] = t0 - t7;
}

static void F(iadst8)(const COEF *in, ptrdiff_t s, COEF *out)
{
    DINT t0a = 16305 * IN(7) + 1606 * IN(0), t1a = 1606 * IN(7) - 16305 * IN(0);
    DINT t2a = 14449 * IN(5) + 7723 * IN(2), t3a = 7723 * IN(5) - 14449 * IN(2);
    DINT t4a = 10394 * IN(3) + 12665 * IN(4), t5a = 12665 * IN(3) - 10394 * IN(4);
    DINT t6a = 4756 * IN(1) + 15679 * IN(6), t7a = 15679 * IN(1) - 4756 * IN(6);
    DINT t0 = RND(t0a + t4a), t1 = RND(t1a + t5a), t2 = RND(t2a + t6a), t3 = RND(t3a + t7a);
    DINT t4 = RND(t0a - t4a), t5 = RND(t1a - t5a), t6 = RND(t2a - t6a), t7 = RND(t3a - t7a);
    t4a = 15137 * t4 + 6270 * t5;
    t5a = 6270 * t4 - 15137 * t5;
    t6a = 15137 * t7 - 6270 * t6;
    t7a = 6270 * t7 + 15137 * t6;
    out[0] = t0 + t2;
    out[7] = -(t1 + t3);
    t2 = t0 - t2;
    t3 = t1 - t3;
    out[1] = -RND(t4a + t6a);
    out[6] = RND(t5a + t7a);
    t6 = RND(t4a - t6a);
    t7 = RND(t5a - t7a);
    out[3] = -RND((t2 + t3) * 11585);
    out[4] = RND((t2 - t3) * 11585);
    out[2] = RND((t6 + t7) * 11585);
    out[5] = -RND((t6 - t7) * 11585);
}

static void F(idct16)(const COEF *in, ptrdiff_t s, COEF *out)
{
    DINT t0, t1, t2, t3, t4, t5, t6, t7, t8, t9, t10, t11, t12, t13, t14, t15;
    DINT t0a, t1a, t2a, t3a, t4a, t5a, t6a, t7a, t8a, t9a, t10a, t11a, t12a, t13a, t14a, t15a;
    t0a = RND((IN(0) + IN(8)) * 11585);
    t1a = RND((IN(0) - IN(8)) * 11585);
    t2a = RND(IN(4) * 6270 - IN(12) * 15137);
    t3a = RND(IN(4) * 15137 + IN(12) * 6270);
    t4a = RND(IN(2) * 3196 - IN(14) * 16069);
    t7a = RND(IN(2) * 16069 + IN(14) * 3196);
    t5a = RND(IN(10) * 13623 - IN(6) * 9102);
    t6a = RND(IN(10) * 9102 + IN(6) * 13623);
    t8a = RND(IN(1) * 1606 - IN(15) * 16305);
    t15a = RND(IN(1) * 16305 + IN(15) * 1606);
    t9a = RND(IN(9) * 12665 - IN(7) * 10394);
    t14a = RND(IN(9) * 10394 + IN(7) * 12665);
    t10a = RND(IN(5) * 7723 - IN(11) * 14449);
    t13a = RND(IN(5) * 14449 + IN(11) * 7723);
    t11a = RND(IN(13) * 15679 - IN(3) * 4756);
    t12a = RND(IN(13) * 4756 + IN(3) * 15679);

    t0 = t0a + t3a; t1 = t1a + t2a; t2 = t1a - t2a; t3 = t0a - t3a;
    t4 = t4a + t5a; t5 = t4a - t5a; t6 = t7a - t6a; t7 = t7a + t6a;
    t8 = t8a + t9a; t9 = t8a - t9a; t10 = t11a - t10a; t11 = t11a + t10a;
    t12 = t12a + t13a; t13 = t12a - t13a; t14 = t15a - t14a; t15 = t15a + t14a;

    t5a = RND((t6 - t5) * 11585);
    t6a = RND((t6 + t5) * 11585);
    t9a = RND(t14 * 6270 - t9 * 15137);
    t14a = RND(t14 * 15137 + t9 * 6270);
    t10a = RND(-(t13 * 15137 + t10 * 6270));
    t13a = RND(t13 * 6270 - t10 * 15137);

    t0a = t0 + t7; t1a = t1 + t6a; t2a = t2 + t5a; t3a = t3 + t4;
    t4 = t3 - t4; t5 = t2 - t5a; t6 = t1 - t6a; t7 = t0 - t7;
    t8a = t8 + t11; t9 = t9a + t10a; t10 = t9a - t10a; t11a = t8 - t11;
    t12a = t15 - t12; t13 = t14a - t13a; t14 = t14a + t13a; t15a = t15 + t12;

    t10a = RND((t13 - t10) * 11585);
    t13a = RND((t13 + t10) * 11585);
    t11 = RND((t12a - t11a) * 11585);
    t12 = RND((t12a + t11a) * 11585);

    out[0] = t0a + t15a; out[1] = t1a + t14; out[2] = t2a + t13a; out[3] = t3a + t12;
    out[4] = t4 + t11; out[5] = t5 + t10a; out[6] = t6 + t9; out[7] = t7 + t8a;
    out[8] = t7 - t8a; out[9] = t6 - t9; out[10] = t5 - t10a; out[11] = t4 - t11;
    out[12] = t3a - t12; out[13] = t2a - t13a; out[14] = t1a - t14; out[15] = t0a - t15a;
}

static void F(iadst16)(const COEF *in, ptrdiff_t s, COEF *out)
{
    DINT t0, t1, t2, t3, t4, t5, t6, t7, t8, t9, t10, t11, t12, t13, t14, t15;
    DINT t0a, t1a, t2a, t3a, t4a, t5a, t6a, t7a, t8a, t9a, t10a, t11a, t12a, t13a, t14a, t15a;
    t0 = IN(15) * 16364 + IN(0) * 804;
    t1 = IN(15) * 804 - IN(0) * 16364;
    t2 = IN(13) * 15893 + IN(2) * 3981;
    t3 = IN(13) * 3981 - IN(2) * 15893;
    t4 = IN(11) * 14811 + IN(4) * 7005;
    t5 = IN(11) * 7005 - IN(4) * 14811;
    t6 = IN(9) * 13160 + IN(6) * 9760;
    t7 = IN(9) * 9760 - IN(6) * 13160;
    t8 = IN(7) * 11003 + IN(8) * 12140;
    t9 = IN(7) * 12140 - IN(8) * 11003;
    t10 = IN(5) * 8423 + IN(10) * 14053;
    t11 = IN(5) * 14053 - IN(10) * 8423;
    t12 = IN(3) * 5520 + IN(12) * 15426;
    t13 = IN(3) * 15426 - IN(12) * 5520;
    t14 = IN(1) * 2404 + IN(14) * 16207;
    t15 = IN(1) * 16207 - IN(14) * 2404;

    t0a = RND(t0 + t8); t1a = RND(t1 + t9); t2a = RND(t2 + t10); t3a = RND(t3 + t11);
    t4a = RND(t4 + t12); t5a = RND(t5 + t13); t6a = RND(t6 + t14); t7a = RND(t7 + t15);
    t8a = RND(t0 - t8); t9a = RND(t1 - t9); t10a = RND(t2 - t10); t11a = RND(t3 - t11);
    t12a = RND(t4 - t12); t13a = RND(t5 - t13); t14a = RND(t6 - t14); t15a = RND(t7 - t15);

    t8 = t8a * 16069 + t9a * 3196;
    t9 = t8a * 3196 - t9a * 16069;
    t10 = t10a * 9102 + t11a * 13623;
    t11 = t10a * 13623 - t11a * 9102;
    t12 = t13a * 16069 - t12a * 3196;
    t13 = t13a * 3196 + t12a * 16069;
    t14 = t15a * 9102 - t14a * 13623;
    t15 = t15a * 13623 + t14a * 9102;

    t0 = t0a + t4a; t1 = t1a + t5a; t2 = t2a + t6a; t3 = t3a + t7a;
    t4 = t0a - t4a; t5 = t1a - t5a; t6 = t2a - t6a; t7 = t3a - t7a;
    t8a = RND(t8 + t12); t9a = RND(t9 + t13); t10a = RND(t10 + t14); t11a = RND(t11 + t15);
    t12a = RND(t8 - t12); t13a = RND(t9 - t13); t14a = RND(t10 - t14); t15a = RND(t11 - t15);

    t4a = t4 * 15137 + t5 * 6270;
    t5a = t4 * 6270 - t5 * 15137;
    t6a = t7 * 15137 - t6 * 6270;
    t7a = t7 * 6270 + t6 * 15137;
    t12 = t12a * 15137 + t13a * 6270;
    t13 = t12a * 6270 - t13a * 15137;
    t14 = t15a * 15137 - t14a * 6270;
    t15 = t15a * 6270 + t14a * 15137;

    out[0] = t0 + t2;
    out[15] = -(t1 + t3);
    t2a = t0 - t2;
    t3a = t1 - t3;
    out[3] = -RND(t4a + t6a);
    out[12] = RND(t5a + t7a);
    t6 = RND(t4a - t6a);
    t7 = RND(t5a - t7a);
    out[1] = -(t8a + t10a);
    out[14] = t9a + t11a;
    t10 = t8a - t10a;
    t11 = t9a - t11a;
    out[2] = RND(t12 + t14);
    out[13] = -RND(t13 + t15);
    t14a = RND(t12 - t14);
    t15a = RND(t13 - t15);

    out[7] = RND(-(t2a + t3a) * 11585);
    out[8] = RND((t2a - t3a) * 11585);
    out[4] = RND((t7 + t6) * 11585);
    out[11] = RND((t7 - t6) * 11585);
    out[6] = RND((t11 + t10) * 11585);
    out[9] = RND((t11 - t10) * 11585);
    out[5] = RND(-(t14a + t15a) * 11585);
    out[10] = RND((t14a - t15a) * 11585);
}

static void F(idct32)(const COEF *in, ptrdiff_t s, COEF *out)
{
    DINT t0a = RND((IN(0) + IN(16)) * 11585);
    DINT t1a = RND((IN(0) - IN(16)) * 11585);
    DINT t2a = RND(IN(8) * 6270 - IN(24) * 15137);
    DINT t3a = RND(IN(8) * 15137 + IN(24) * 6270);
    DINT t4a = RND(IN(4) * 3196 - IN(28) * 16069);
    DINT t7a = RND(IN(4) * 16069 + IN(28) * 3196);
    DINT t5a = RND(IN(20) * 13623 - IN(12) * 9102);
    DINT t6a = RND(IN(20) * 9102 + IN(12) * 13623);
    DINT t8a = RND(IN(2) * 1606 - IN(30) * 16305);
    DINT t15a = RND(IN(2) * 16305 + IN(30) * 1606);
    DINT t9a = RND(IN(18) * 12665 - IN(14) * 10394);
    DINT t14a = RND(IN(18) * 10394 + IN(14) * 12665);
    DINT t10a = RND(IN(10) * 7723 - IN(22) * 14449);
    DINT t13a = RND(IN(10) * 14449 + IN(22) * 7723);
    DINT t11a = RND(IN(26) * 15679 - IN(6) * 4756);
    DINT t12a = RND(IN(26) * 4756 + IN(6) * 15679);
    DINT t16a = RND(IN(1) * 804 - IN(31) * 16364);
    DINT t31a = RND(IN(1) * 16364 + IN(31) * 804);
    DINT t17a = RND(IN(17) * 12140 - IN(15) * 11003);
    DINT t30a = RND(IN(17) * 11003 + IN(15) * 12140);
    DINT t18a = RND(IN(9) * 7005 - IN(23) * 14811);
    DINT t29a = RND(IN(9) * 14811 + IN(23) * 7005);
    DINT t19a = RND(IN(25) * 15426 - IN(7) * 5520);
    DINT t28a = RND(IN(25) * 5520 + IN(7) * 15426);
    DINT t20a = RND(IN(5) * 3981 - IN(27) * 15893);
    DINT t27a = RND(IN(5) * 15893 + IN(27) * 3981);
    DINT t21a = RND(IN(21) * 14053 - IN(11) * 8423);
    DINT t26a = RND(IN(21) * 8423 + IN(11) * 14053);
    DINT t22a = RND(IN(13) * 9760 - IN(19) * 13160);
    DINT t25a = RND(IN(13) * 13160 + IN(19) * 9760);
    DINT t23a = RND(IN(29) * 16207 - IN(3) * 2404);
    DINT t24a = RND(IN(29) * 2404 + IN(3) * 16207);

    DINT t0 = t0a + t3a, t1 = t1a + t2a, t2 = t1a - t2a, t3 = t0a - t3a;
    DINT t4 = t4a + t5a, t5 = t4a - t5a, t6 = t7a - t6a, t7 = t7a + t6a;
    DINT t8 = t8a + t9a, t9 = t8a - t9a, t10 = t11a - t10a, t11 = t11a + t10a;
    DINT t12 = t12a + t13a, t13 = t12a - t13a, t14 = t15a - t14a, t15 = t15a + t14a;
    DINT t16 = t16a + t17a, t17 = t16a - t17a, t18 = t19a - t18a, t19 = t19a + t18a;
    DINT t20 = t20a + t21a, t21 = t20a - t21a, t22 = t23a - t22a, t23 = t23a + t22a;
    DINT t24 = t24a + t25a, t25 = t24a - t25a, t26 = t27a - t26a, t27 = t27a + t26a;
    DINT t28 = t28a + t29a, t29 = t28a - t29a, t30 = t31a - t30a, t31 = t31a + t30a;

    t5a = RND((t6 - t5) * 11585);
    t6a = RND((t6 + t5) * 11585);
    t9a = RND(t14 * 6270 - t9 * 15137);
    t14a = RND(t14 * 15137 + t9 * 6270);
    t10a = RND(-(t13 * 15137 + t10 * 6270));
    t13a = RND(t13 * 6270 - t10 * 15137);
    t17a = RND(t30 * 3196 - t17 * 16069);
    t30a = RND(t30 * 16069 + t17 * 3196);
    t18a = RND(-(t29 * 16069 + t18 * 3196));
    t29a = RND(t29 * 3196 - t18 * 16069);
    t21a = RND(t26 * 13623 - t21 * 9102);
    t26a = RND(t26 * 9102 + t21 * 13623);
    t22a = RND(-(t25 * 9102 + t22 * 13623));
    t25a = RND(t25 * 13623 - t22 * 9102);

    t0a = t0 + t7; t1a = t1 + t6a; t2a = t2 + t5a; t3a = t3 + t4;
    t4a = t3 - t4; t5 = t2 - t5a; t6 = t1 - t6a; t7a = t0 - t7;
    t8a = t8 + t11; t9 = t9a + t10a; t10 = t9a - t10a; t11a = t8 - t11;
    t12a = t15 - t12; t13 = t14a - t13a; t14 = t14a + t13a; t15a = t15 + t12;
    t16a = t16 + t19; t17 = t17a + t18a; t18 = t17a - t18a; t19a = t16 - t19;
    t20a = t23 - t20; t21 = t22a - t21a; t22 = t22a + t21a; t23a = t23 + t20;
    t24a = t24 + t27; t25 = t25a + t26a; t26 = t25a - t26a; t27a = t24 - t27;
    t28a = t31 - t28; t29 = t30a - t29a; t30 = t30a + t29a; t31a = t31 + t28;

    t10a = RND((t13 - t10) * 11585);
    t13a = RND((t13 + t10) * 11585);
    t11 = RND((t12a - t11a) * 11585);
    t12 = RND((t12a + t11a) * 11585);
    t18a = RND(t29 * 6270 - t18 * 15137);
    t29a = RND(t29 * 15137 + t18 * 6270);
    t19 = RND(t28a * 6270 - t19a * 15137);
    t28 = RND(t28a * 15137 + t19a * 6270);
    t20 = RND(-(t27a * 15137 + t20a * 6270));
    t27 = RND(t27a * 6270 - t20a * 15137);
    t21a = RND(-(t26 * 15137 + t21 * 6270));
    t26a = RND(t26 * 6270 - t21 * 15137);

    t0 = t0a + t15a; t1 = t1a + t14; t2 = t2a + t13a; t3 = t3a + t12;
    t4 = t4a + t11; t5a = t5 + t10a; t6a = t6 + t9; t7 = t7a + t8a;
    t8 = t7a - t8a; t9a = t6 - t9; t10 = t5 - t10a; t11a = t4a - t11;
    t12a = t3a - t12; t13 = t2a - t13a; t14a = t1a - t14; t15 = t0a - t15a;
    t16 = t16a + t23a; t17a = t17 + t22; t18 = t18a + t21a; t19a = t19 + t20;
    t20a = t19 - t20; t21 = t18a - t21a; t22a = t17 - t22; t23 = t16a - t23a;
    t24 = t31a - t24a; t25a = t30 - t25; t26 = t29a - t26a; t27a = t28 - t27;
    t28a = t28 + t27; t29 = t29a + t26a; t30a = t30 + t25; t31 = t31a + t24a;

    t20 = RND((t27a - t20a) * 11585);
    t27 = RND((t27a + t20a) * 11585);
    t21a = RND((t26 - t21) * 11585);
    t26a = RND((t26 + t21) * 11585);
    t22 = RND((t25a - t22a) * 11585);
    t25 = RND((t25a + t22a) * 11585);
    t23a = RND((t24 - t23) * 11585);
    t24a = RND((t24 + t23) * 11585);

    out[0] = t0 + t31; out[1] = t1 + t30a; out[2] = t2 + t29; out[3] = t3 + t28a;
    out[4] = t4 + t27; out[5] = t5a + t26a; out[6] = t6a + t25; out[7] = t7 + t24a;
    out[8] = t8 + t23a; out[9] = t9a + t22; out[10] = t10 + t21a; out[11] = t11a + t20;
    out[12] = t12a + t19a; out[13] = t13 + t18; out[14] = t14a + t17a; out[15] = t15 + t16;
    out[16] = t15 - t16; out[17] = t14a - t17a; out[18] = t13 - t18; out[19] = t12a - t19a;
    out[20] = t11a - t20; out[21] = t10 - t21a; out[22] = t9a - t22; out[23] = t8 - t23a;
    out[24] = t7 - t24a; out[25] = t6a - t25; out[26] = t5a - t26a; out[27] = t4 - t27;
    out[28] = t3 - t28a; out[29] = t2 - t29; out[30] = t1 - t30a; out[31] = t0 - t31;
}

/* vp9dsp_template.c:1719-1748: note the int (not dctint) temporaries. */
static void F(iwht4)(const COEF *in, ptrdiff_t s, COEF *out, int pass)
{
    int t0, t1, t2, t3, t4;
    if (pass == 0) { t0 = IN(0) >> 2; t1 = IN(3) >> 2; t2 = IN(1) >> 2; t3 = IN(2) >> 2; }
    else           { t0 = IN(0);      t1 = IN(3);      t2 = IN(1);      t3 = IN(2); }
    t0 += t2; t3 -= t1; t4 = (t0 - t3) >> 1; t1 = t4 - t1; t2 = t4 - t2; t0 -= t1; t3 += t2;
    out[0] = t0; out[1] = t1; out[2] = t2; out[3] = t3;
}
#undef IN
#undef RND

typedef void (*F(tx1d_fn))(const COEF *, ptrdiff_t, COEF *);

/* itxfm_wrapper (vp9dsp_template.c:1155-1192) + the dispatch table
 * vp9dsp_itxfm_init (1756-1778): itxfm_add[tx][DCT_ADST] = iadst_idct, i.e. type_a
 * (first pass, over block columns) is the ADST for txtp 1 and 3. tx 4 = lossless. */
static void F(itxfm_add)(PIX *dst, ptrdiff_t stride, COEF *block, int eob, int tx, int txtp, int bd)
{
    static const F(tx1d_fn) dct[4] = { F(idct4), F(idct8), F(idct16), F(idct32) };
    static const F(tx1d_fn) adst[3] = { F(iadst4), F(iadst8), F(iadst16) };
    COEF tmp[32 * 32], out[32];
    int i, j;
    if (tx == 4) {
        for (i = 0; i < 4; i++) F(iwht4)(block + i, 4, tmp + i * 4, 0);
        memset(block, 0, 16 * sizeof(*block));
        for (i = 0; i < 4; i++) {
            F(iwht4)(tmp + i, 4, out, 1);
            for (j = 0; j < 4; j++)
                dst[j * stride + i] = F(clip_px)(dst[j * stride + i] + out[j], bd);
        }
        return;
    }
    int sz = 4 << tx, bits = tx == 3 ? 6 : tx + 4;
    if (tx == 3) txtp = 0;
    F(tx1d_fn) ta = (txtp == 1 || txtp == 3) ? adst[tx] : dct[tx];
    F(tx1d_fn) tb = (txtp == 2 || txtp == 3) ? adst[tx] : dct[tx];
    if (txtp == 0 && eob == 1) {
        int t = (int) ((((((DINT) block[0] * 11585 + (1 << 13)) >> 14) * 11585) + (1 << 13)) >> 14);
        block[0] = 0;
        for (i = 0; i < sz; i++)
            for (j = 0; j < sz; j++)
                dst[j * stride + i] = F(clip_px)(dst[j * stride + i] +
                                                 ((int) (t + (1u << (bits - 1))) >> bits), bd);
        return;
    }
    for (i = 0; i < sz; i++) ta(block + i, sz, tmp + i * sz);
    memset(block, 0, sz * sz * sizeof(*block));
    for (i = 0; i < sz; i++) {
        tb(tmp + i, sz, out);
        for (j = 0; j < sz; j++)
            dst[j * stride + i] = F(clip_px)(dst[j * stride + i] +
                                             ((int) (out[j] + (1u << (bits - 1))) >> bits), bd);
    }
}

/* ------------------------------------------------------------- intra pred
 * vp9dsp_template.c:28-1153. left[] is bottom-to-top (left[n-1] is the top-most
 * pixel) except for HOR_UP (invert_left, vp9recon.c:89,196-204). top[-1] = top-left. */
#define D(x, y) dst[(x) + (y) * stride]
#define A2(a, b) (((a) + (b) + 1) >> 1)
#define A3(a, b, c) (((a) + 2 * (b) + (c) + 2) >> 2)

static void F(ipred)(PIX *dst, ptrdiff_t stride, const PIX *left, const PIX *top,
                     int tx, int mode, int bd)
{
    const int n = 4 << tx;
    int x, y, i, sum;
    PIX v[3 * 32];
    switch (mode) {
    case 0: /* VERT */
        for (y = 0; y < n; y++) for (x = 0; x < n; x++) D(x, y) = top[x];
        break;
    case 1: /* HOR */
        for (y = 0; y < n; y++) for (x = 0; x < n; x++) D(x, y) = left[n - 1 - y];
        break;
    case 2: /* DC */
        for (sum = 0, i = 0; i < n; i++) sum += left[i] + top[i];
        sum = (sum + n) >> (tx + 3);
        for (y = 0; y < n; y++) for (x = 0; x < n; x++) D(x, y) = sum;
        break;
    case 10: /* LEFT_DC */
        for (sum = 0, i = 0; i < n; i++) sum += left[i];
        sum = (sum + (n >> 1)) >> (tx + 2);
        for (y = 0; y < n; y++) for (x = 0; x < n; x++) D(x, y) = sum;
        break;
    case 11: /* TOP_DC */
        for (sum = 0, i = 0; i < n; i++) sum += top[i];
        sum = (sum + (n >> 1)) >> (tx + 2);
        for (y = 0; y < n; y++) for (x = 0; x < n; x++) D(x, y) = sum;
        break;
    case 12: case 13: case 14: /* DC_128 / DC_127 / DC_129 */
        sum = (128 << (bd - 8)) + (mode == 13 ? -1 : mode == 14 ? 1 : 0);
        for (y = 0; y < n; y++) for (x = 0; x < n; x++) D(x, y) = sum;
        break;
    case 9: { /* TM_VP8 */
        int tl = top[-1];
        for (y = 0; y < n; y++) {
            int l_m_tl = left[n - 1 - y] - tl;
            for (x = 0; x < n; x++) D(x, y) = F(clip_px)(top[x] + l_m_tl, bd);
        }
        break;
    }
    case 3: /* DIAG_DOWN_LEFT */
        if (n == 4) {
            const PIX *a = top;
            D(0,0) = A3(a[0], a[1], a[2]);
            D(1,0) = D(0,1) = A3(a[1], a[2], a[3]);
            D(2,0) = D(1,1) = D(0,2) = A3(a[2], a[3], a[4]);
            D(3,0) = D(2,1) = D(1,2) = D(0,3) = A3(a[3], a[4], a[5]);
            D(3,1) = D(2,2) = D(1,3) = A3(a[4], a[5], a[6]);
            D(3,2) = D(2,3) = A3(a[5], a[6], a[7]);
            D(3,3) = a[7];
        } else {
            for (i = 0; i < n - 2; i++) v[i] = A3(top[i], top[i + 1], top[i + 2]);
            v[n - 2] = (top[n - 2] + top[n - 1] * 3 + 2) >> 2;
            for (y = 0; y < n; y++)
                for (x = 0; x < n; x++) D(x, y) = x < n - 1 - y ? v[y + x] : top[n - 1];
        }
        break;
    case 4: /* DIAG_DOWN_RIGHT */
        if (n == 4) {
            int tl = top[-1], a0 = top[0], a1 = top[1], a2 = top[2], a3 = top[3];
            int l0 = left[3], l1 = left[2], l2 = left[1], l3 = left[0];
            D(0,3) = A3(l1, l2, l3);
            D(0,2) = D(1,3) = A3(l0, l1, l2);
            D(0,1) = D(1,2) = D(2,3) = A3(tl, l0, l1);
            D(0,0) = D(1,1) = D(2,2) = D(3,3) = A3(l0, tl, a0);
            D(1,0) = D(2,1) = D(3,2) = A3(tl, a0, a1);
            D(2,0) = D(3,1) = A3(a0, a1, a2);
            D(3,0) = A3(a1, a2, a3);
        } else {
            for (i = 0; i < n - 2; i++) {
                v[i] = A3(left[i], left[i + 1], left[i + 2]);
                v[n + 1 + i] = A3(top[i], top[i + 1], top[i + 2]);
            }
            v[n - 2] = A3(left[n - 2], left[n - 1], top[-1]);
            v[n - 1] = A3(left[n - 1], top[-1], top[0]);
            v[n] = A3(top[-1], top[0], top[1]);
            for (y = 0; y < n; y++) for (x = 0; x < n; x++) D(x, y) = v[n - 1 - y + x];
        }
        break;
    case 5: /* VERT_RIGHT */
        if (n == 4) {
            int tl = top[-1], a0 = top[0], a1 = top[1], a2 = top[2], a3 = top[3];
            int l0 = left[3], l1 = left[2], l2 = left[1];
            D(0,3) = A3(l0, l1, l2);
            D(0,2) = A3(tl, l0, l1);
            D(0,0) = D(1,2) = A2(tl, a0);
            D(0,1) = D(1,3) = A3(l0, tl, a0);
            D(1,0) = D(2,2) = A2(a0, a1);
            D(1,1) = D(2,3) = A3(tl, a0, a1);
            D(2,0) = D(3,2) = A2(a1, a2);
            D(2,1) = D(3,3) = A3(a0, a1, a2);
            D(3,0) = A2(a2, a3);
            D(3,1) = A3(a1, a2, a3);
        } else {
            PIX ve[32 + 16], vo[32 + 16];
            int h = n / 2;
            for (i = 0; i < h - 2; i++) {
                vo[i] = A3(left[i * 2 + 3], left[i * 2 + 2], left[i * 2 + 1]);
                ve[i] = A3(left[i * 2 + 4], left[i * 2 + 3], left[i * 2 + 2]);
            }
            vo[h - 2] = A3(left[n - 1], left[n - 2], left[n - 3]);
            ve[h - 2] = A3(top[-1], left[n - 1], left[n - 2]);
            ve[h - 1] = A2(top[-1], top[0]);
            vo[h - 1] = A3(left[n - 1], top[-1], top[0]);
            for (i = 0; i < n - 1; i++) {
                ve[h + i] = A2(top[i], top[i + 1]);
                vo[h + i] = A3(top[i - 1], top[i], top[i + 1]);
            }
            for (y = 0; y < h; y++)
                for (x = 0; x < n; x++) {
                    D(x, 2 * y) = ve[h - 1 - y + x];
                    D(x, 2 * y + 1) = vo[h - 1 - y + x];
                }
        }
        break;
    case 6: /* HOR_DOWN */
        if (n == 4) {
            int l0 = left[3], l1 = left[2], l2 = left[1], l3 = left[0];
            int tl = top[-1], a0 = top[0], a1 = top[1], a2 = top[2];
            D(2,0) = A3(tl, a0, a1);
            D(3,0) = A3(a0, a1, a2);
            D(0,0) = D(2,1) = A2(tl, l0);
            D(1,0) = D(3,1) = A3(a0, tl, l0);
            D(0,1) = D(2,2) = A2(l0, l1);
            D(1,1) = D(3,2) = A3(tl, l0, l1);
            D(0,2) = D(2,3) = A2(l1, l2);
            D(1,2) = D(3,3) = A3(l0, l1, l2);
            D(0,3) = A2(l2, l3);
            D(1,3) = A3(l1, l2, l3);
        } else {
            for (i = 0; i < n - 2; i++) {
                v[i * 2] = A2(left[i + 1], left[i]);
                v[i * 2 + 1] = A3(left[i + 2], left[i + 1], left[i]);
                v[n * 2 + i] = A3(top[i - 1], top[i], top[i + 1]);
            }
            v[n * 2 - 2] = A2(top[-1], left[n - 1]);
            v[n * 2 - 4] = A2(left[n - 1], left[n - 2]);
            v[n * 2 - 1] = A3(top[0], top[-1], left[n - 1]);
            v[n * 2 - 3] = A3(top[-1], left[n - 1], left[n - 2]);
            for (y = 0; y < n; y++) for (x = 0; x < n; x++) D(x, y) = v[n * 2 - 2 - y * 2 + x];
        }
        break;
    case 7: /* VERT_LEFT */
        if (n == 4) {
            int a0 = top[0], a1 = top[1], a2 = top[2], a3 = top[3], a4 = top[4], a5 = top[5], a6 = top[6];
            D(0,0) = A2(a0, a1);
            D(0,1) = A3(a0, a1, a2);
            D(1,0) = D(0,2) = A2(a1, a2);
            D(1,1) = D(0,3) = A3(a1, a2, a3);
            D(2,0) = D(1,2) = A2(a2, a3);
            D(2,1) = D(1,3) = A3(a2, a3, a4);
            D(3,0) = D(2,2) = A2(a3, a4);
            D(3,1) = D(2,3) = A3(a3, a4, a5);
            D(3,2) = A2(a4, a5);
            D(3,3) = A3(a4, a5, a6);
        } else {
            PIX ve[32], vo[32];
            for (i = 0; i < n - 2; i++) {
                ve[i] = A2(top[i], top[i + 1]);
                vo[i] = A3(top[i], top[i + 1], top[i + 2]);
            }
            ve[n - 2] = A2(top[n - 2], top[n - 1]);
            vo[n - 2] = (top[n - 2] + top[n - 1] * 3 + 2) >> 2;
            for (y = 0; y < n / 2; y++)
                for (x = 0; x < n; x++) {
                    D(x, 2 * y) = x < n - y - 1 ? ve[y + x] : top[n - 1];
                    D(x, 2 * y + 1) = x < n - y - 1 ? vo[y + x] : top[n - 1];
                }
        }
        break;
    case 8: /* HOR_UP (left[] top-to-bottom) */
        if (n == 4) {
            int l0 = left[0], l1 = left[1], l2 = left[2], l3 = left[3];
            D(0,0) = A2(l0, l1);
            D(1,0) = A3(l0, l1, l2);
            D(0,1) = D(2,0) = A2(l1, l2);
            D(1,1) = D(3,0) = A3(l1, l2, l3);
            D(0,2) = D(2,1) = A2(l2, l3);
            D(1,2) = D(3,1) = (l2 + l3 * 3 + 2) >> 2;
            D(0,3) = D(1,3) = D(2,2) = D(2,3) = D(3,2) = D(3,3) = l3;
        } else {
            for (i = 0; i < n - 2; i++) {
                v[i * 2] = A2(left[i], left[i + 1]);
                v[i * 2 + 1] = A3(left[i], left[i + 1], left[i + 2]);
            }
            v[n * 2 - 4] = A2(left[n - 2], left[n - 1]);
            v[n * 2 - 3] = (left[n - 2] + left[n - 1] * 3 + 2) >> 2;
            for (y = 0; y < n; y++)
                for (x = 0; x < n; x++)
                    D(x, y) = (y < n / 2 || x < n * 2 - 2 - y * 2) ? v[y * 2 + x] : left[n - 1];
        }
        break;
    }
}
#undef D
#undef A2
#undef A3

/* ------------------------------------------------------------ loop filter
 * vp9dsp_template.c:1780-1889 (loop_filter) with the 8-line wrappers 1891-1967. */
static inline int F(iabs)(int v) { return v < 0 ? -v : v; }
static inline int F(clip_intp2)(int v, int p) { int lo = -(1 << p), hi = (1 << p) - 1; return v < lo ? lo : v > hi ? hi : v; }

static void F(loop_filter)(PIX *dst, int E, int I, int H, ptrdiff_t stridea, ptrdiff_t strideb,
                           int wd, int bd)
{
    int i, Fl = 1 << (bd - 8);
    E <<= (bd - 8); I <<= (bd - 8); H <<= (bd - 8);
    for (i = 0; i < 8; i++, dst += stridea) {
        int p7 = 0, p6 = 0, p5 = 0, p4 = 0, q4 = 0, q5 = 0, q6 = 0, q7 = 0;
        int p3 = dst[strideb * -4], p2 = dst[strideb * -3], p1 = dst[strideb * -2], p0 = dst[strideb * -1];
        int q0 = dst[strideb * +0], q1 = dst[strideb * +1], q2 = dst[strideb * +2], q3 = dst[strideb * +3];
        int fm = F(iabs)(p3 - p2) <= I && F(iabs)(p2 - p1) <= I && F(iabs)(p1 - p0) <= I &&
                 F(iabs)(q1 - q0) <= I && F(iabs)(q2 - q1) <= I && F(iabs)(q3 - q2) <= I &&
                 F(iabs)(p0 - q0) * 2 + (F(iabs)(p1 - q1) >> 1) <= E;
        int flat8out = 0, flat8in = 0;
        if (!fm) continue;
        if (wd >= 16) {
            p7 = dst[strideb * -8]; p6 = dst[strideb * -7]; p5 = dst[strideb * -6]; p4 = dst[strideb * -5];
            q4 = dst[strideb * +4]; q5 = dst[strideb * +5]; q6 = dst[strideb * +6]; q7 = dst[strideb * +7];
            flat8out = F(iabs)(p7 - p0) <= Fl && F(iabs)(p6 - p0) <= Fl && F(iabs)(p5 - p0) <= Fl &&
                       F(iabs)(p4 - p0) <= Fl && F(iabs)(q4 - q0) <= Fl && F(iabs)(q5 - q0) <= Fl &&
                       F(iabs)(q6 - q0) <= Fl && F(iabs)(q7 - q0) <= Fl;
        }
        if (wd >= 8)
            flat8in = F(iabs)(p3 - p0) <= Fl && F(iabs)(p2 - p0) <= Fl && F(iabs)(p1 - p0) <= Fl &&
                      F(iabs)(q1 - q0) <= Fl && F(iabs)(q2 - q0) <= Fl && F(iabs)(q3 - q0) <= Fl;
        if (wd >= 16 && flat8out && flat8in) {
            /* 15-tap smoothing: out[k] = (sum of the 16-tap window around k + 8) >> 4 */
            int px[16] = { p7, p6, p5, p4, p3, p2, p1, p0, q0, q1, q2, q3, q4, q5, q6, q7 };
            int k;
            for (k = 1; k < 15; k++) {
                int acc = 8, t;
                for (t = k - 7; t <= k + 7; t++) acc += px[t < 0 ? 0 : t > 15 ? 15 : t];
                acc += px[k];
                dst[strideb * (k - 8)] = acc >> 4;
            }
        } else if (wd >= 8 && flat8in) {
            dst[strideb * -3] = (p3 + p3 + p3 + 2 * p2 + p1 + p0 + q0 + 4) >> 3;
            dst[strideb * -2] = (p3 + p3 + p2 + 2 * p1 + p0 + q0 + q1 + 4) >> 3;
            dst[strideb * -1] = (p3 + p2 + p1 + 2 * p0 + q0 + q1 + q2 + 4) >> 3;
            dst[strideb * +0] = (p2 + p1 + p0 + 2 * q0 + q1 + q2 + q3 + 4) >> 3;
            dst[strideb * +1] = (p1 + p0 + q0 + 2 * q1 + q2 + q3 + q3 + 4) >> 3;
            dst[strideb * +2] = (p0 + q0 + q1 + 2 * q2 + q3 + q3 + q3 + 4) >> 3;
        } else {
            int hev = F(iabs)(p1 - p0) > H || F(iabs)(q1 - q0) > H;
            int mx = (1 << (bd - 1)) - 1;
            if (hev) {
                int f = F(clip_intp2)(p1 - q1, bd - 1), f1, f2;
                f = F(clip_intp2)(3 * (q0 - p0) + f, bd - 1);
                f1 = (f + 4 < mx ? f + 4 : mx) >> 3;
                f2 = (f + 3 < mx ? f + 3 : mx) >> 3;
                dst[strideb * -1] = F(clip_px)(p0 + f2, bd);
                dst[strideb * +0] = F(clip_px)(q0 - f1, bd);
            } else {
                int f = F(clip_intp2)(3 * (q0 - p0), bd - 1), f1, f2;
                f1 = (f + 4 < mx ? f + 4 : mx) >> 3;
                f2 = (f + 3 < mx ? f + 3 : mx) >> 3;
                dst[strideb * -1] = F(clip_px)(p0 + f2, bd);
                dst[strideb * +0] = F(clip_px)(q0 - f1, bd);
                f = (f1 + 1) >> 1;
                dst[strideb * -2] = F(clip_px)(p1 + f, bd);
                dst[strideb * +1] = F(clip_px)(q1 - f, bd);
            }
        }
    }
}

/* loop_filter_8[wd][dir], loop_filter_16[dir], loop_filter_mix2[wd1][wd2][dir]
 * (vp9dsp_template.c:1891-1945); dir 0 = h (column edge), 1 = v (row edge);
 * stride in pixels. */
static void F(lf8)(PIX *dst, ptrdiff_t stride, int wdi, int dir, int E, int I, int H, int bd)
{
    int wd = 4 << wdi;
    if (dir == 0) F(loop_filter)(dst, E, I, H, stride, 1, wd, bd);
    else          F(loop_filter)(dst, E, I, H, 1, stride, wd, bd);
}
static void F(lf16)(PIX *dst, ptrdiff_t stride, int dir, int E, int I, int H, int bd)
{
    F(lf8)(dst, stride, 2, dir, E, I, H, bd);
    F(lf8)(dst + 8 * (dir == 0 ? stride : 1), stride, 2, dir, E, I, H, bd);
}
static void F(lfmix2)(PIX *dst, ptrdiff_t stride, int w1, int w2, int dir, int E, int I, int H, int bd)
{
    F(lf8)(dst, stride, w1, dir, E & 0xff, I & 0xff, H & 0xff, bd);
    F(lf8)(dst + 8 * (dir == 0 ? stride : 1), stride, w2, dir, E >> 8, I >> 8, H >> 8, bd);
}

/* ------------------------------------------------------------------- MC
 * vp9dsp_template.c:1969-2361 (copy/avg, 8-tap 1-D/2-D, bilinear 1-D/2-D).
 * mx/my: 1/16-pel phase. filter: 0..2 = 8-tap smooth/regular/sharp, 3 = bilinear. */
#define FILT8(src, x, f, st) F(clip_px)((f[0] * src[x - 3 * (st)] + f[1] * src[x - 2 * (st)] + \
                                       f[2] * src[x - 1 * (st)] + f[3] * src[x] + \
                                       f[4] * src[x + 1 * (st)] + f[5] * src[x + 2 * (st)] + \
                                       f[6] * src[x + 3 * (st)] + f[7] * src[x + 4 * (st)] + 64) >> 7, bd)
#define BILIN(src, x, m, st) (src[x] + ((m * (src[x + (st)] - src[x]) + 8) >> 4))

static void F(mc)(PIX *dst, ptrdiff_t ds, const PIX *src, ptrdiff_t ss, int w, int h,
                  int mx, int my, int filter, int avg, int bd)
{
    int x, y;
    if (!mx && !my) {
        for (y = 0; y < h; y++)
            for (x = 0; x < w; x++)
                dst[y * ds + x] = avg ? (dst[y * ds + x] + src[y * ss + x] + 1) >> 1 : src[y * ss + x];
        return;
    }
    if (filter == 3) {
        if (mx && my) {
            PIX tmp[64 * 65];
            for (y = 0; y < h + 1; y++)
                for (x = 0; x < w; x++) tmp[y * 64 + x] = BILIN(src, y * ss + x, mx, 1);
            for (y = 0; y < h; y++)
                for (x = 0; x < w; x++) {
                    int v = BILIN(tmp, y * 64 + x, my, 64);
                    dst[y * ds + x] = avg ? (dst[y * ds + x] + v + 1) >> 1 : v;
                }
        } else {
            int m = mx ? mx : my;
            ptrdiff_t st = mx ? 1 : ss;
            for (y = 0; y < h; y++)
                for (x = 0; x < w; x++) {
                    int v = BILIN(src, y * ss + x, m, st);
                    dst[y * ds + x] = avg ? (dst[y * ds + x] + v + 1) >> 1 : v;
                }
        }
        return;
    }
    if (mx && my) {
        PIX tmp[64 * 71];
        const int16_t *fx = vp9t_subpel_filters[filter][mx], *fy = vp9t_subpel_filters[filter][my];
        const PIX *s0 = src - 3 * ss;
        for (y = 0; y < h + 7; y++)
            for (x = 0; x < w; x++) tmp[y * 64 + x] = FILT8(s0, y * ss + x, fx, 1);
        for (y = 0; y < h; y++)
            for (x = 0; x < w; x++) {
                int v = FILT8(tmp, (y + 3) * 64 + x, fy, 64);
                dst[y * ds + x] = avg ? (dst[y * ds + x] + v + 1) >> 1 : v;
            }
    } else {
        const int16_t *f = vp9t_subpel_filters[filter][mx ? mx : my];
        ptrdiff_t st = mx ? 1 : ss;
        for (y = 0; y < h; y++)
            for (x = 0; x < w; x++) {
                int v = FILT8(src, y * ss + x, f, st);
                dst[y * ds + x] = avg ? (dst[y * ds + x] + v + 1) >> 1 : v;
            }
    }
}
/* Scaled MC, vp9dsp_template.c:2363-2482 (do_scaled_8tap_c / do_scaled_bilin_c): the
 * horizontal pass steps the source phase by dx per output pixel into a pixel-clipped
 * 64-wide tmp, the vertical pass steps by dy. 12-bit bilinear uses the 10-bit code
 * (ff_vp9dsp_scaled_mc_init, vp9dsp_template.c:2533-2541), identical for uint16 pixels. */
static void F(mc_scaled)(PIX *dst, ptrdiff_t ds, const PIX *src, ptrdiff_t ss, int w, int h,
                         int mx, int my, int dx, int dy, int filter, int avg, int bd)
{
    int x, y;
    if (filter == 3) {
        static PIX tmp[64 * 129];
        int tmp_h = (((h - 1) * dy + my) >> 4) + 2;
        PIX *tp = tmp;
        do {
            int imx = mx, ioff = 0;
            for (x = 0; x < w; x++) {
                tp[x] = BILIN(src, ioff, imx, 1);
                imx += dx;
                ioff += imx >> 4;
                imx &= 0xf;
            }
            tp += 64;
            src += ss;
        } while (--tmp_h);
        tp = tmp;
        for (y = 0; y < h; y++) {
            for (x = 0; x < w; x++) {
                int v = BILIN(tp, x, my, 64);
                dst[x] = avg ? (dst[x] + v + 1) >> 1 : v;
            }
            my += dy;
            tp += (my >> 4) * 64;
            my &= 0xf;
            dst += ds;
        }
        return;
    }
    static PIX tmp[64 * 135];
    const int16_t (*filters)[8] = vp9t_subpel_filters[filter];
    int tmp_h = (((h - 1) * dy + my) >> 4) + 8;
    PIX *tp = tmp;
    src -= ss * 3;
    do {
        int imx = mx, ioff = 0;
        for (x = 0; x < w; x++) {
            tp[x] = FILT8(src, ioff, filters[imx], 1);
            imx += dx;
            ioff += imx >> 4;
            imx &= 0xf;
        }
        tp += 64;
        src += ss;
    } while (--tmp_h);
    tp = tmp + 64 * 3;
    for (y = 0; y < h; y++) {
        const int16_t *fy = filters[my];
        for (x = 0; x < w; x++) {
            int v = FILT8(tp, x, fy, 64);
            dst[x] = avg ? (dst[x] + v + 1) >> 1 : v;
        }
        my += dy;
        tp += (my >> 4) * 64;
        my &= 0xf;
        dst += ds;
    }
}
#undef FILT8
#undef BILIN

/* ff_emulated_edge_mc (videodsp_template.c:27-105): replicate the frame border of
 * a w x h source into a block_w x block_h buffer. src/src_x/src_y point at the
 * block's top-left; strides in pixels. */
static void F(emu_edge)(PIX *buf, const PIX *src, ptrdiff_t bls, ptrdiff_t sls,
                        int bw, int bh, int sx, int sy, int w, int h)
{
    int x, y, start_y, start_x, end_y, end_x;
    if (!w || !h) return;
    if (sy >= h) { src -= sy * sls; src += (h - 1) * sls; sy = h - 1; }
    else if (sy <= -bh) { src -= sy * sls; src += (1 - bh) * sls; sy = 1 - bh; }
    if (sx >= w) { src -= (1 + sx - w); sx = w - 1; }
    else if (sx <= -bw) { src += (1 - bw - sx); sx = 1 - bw; }
    start_y = sy < 0 ? -sy : 0; start_x = sx < 0 ? -sx : 0;
    end_y = bh < h - sy ? bh : h - sy; end_x = bw < w - sx ? bw : w - sx;
    w = end_x - start_x;
    src += start_y * sls + start_x;
    buf += start_x;
    for (y = 0; y < start_y; y++) { memcpy(buf, src, w * sizeof(PIX)); buf += bls; }
    for (; y < end_y; y++) { memcpy(buf, src, w * sizeof(PIX)); src += sls; buf += bls; }
    src -= sls;
    for (; y < bh; y++) { memcpy(buf, src, w * sizeof(PIX)); buf += bls; }
    buf -= bh * bls + start_x;
    while (bh--) {
        for (x = 0; x < start_x; x++) buf[x] = buf[start_x];
        for (x = end_x; x < bw; x++) buf[x] = buf[end_x - 1];
        buf += bls;
    }
}

#undef PIX
#undef COEF
#undef DINT
#undef F
