// rtg_crmath.h -- fast, divergence-free versions of two scalar kernels on the
// solver's hottest path (the exp-map of every DOF link), bit-identical to the
// reference-faithful versions they replace.  Host + device: the host build is
// what tools/check_crmath.cpp verifies exhaustively against glibc.
//
//  * crm_sincos(x): correctly rounded float sin(x), cos(x) of a double x.
//    One Cody-Waite reduction by pi/2 (four-part constant), fdlibm's
//    __kernel_sin / __kernel_cos polynomials (|r| <= pi/4, error < 2^-58), all
//    in f64, then a rounding test: if y*(1-2^-44) and y*(1+2^-44) round to the
//    same float, that float is the correctly rounded result (the f64 error is
//    < 2^-50 |y|).  Otherwise -- about one call in 2^20 -- the caller's exact
//    fallback runs (libm sin/cos in f64, rounded once), so the result equals
//    (float)sin(x) / (float)cos(x) whenever that is correctly rounded.
//  * crm_atan2f(y, x): glibc 2.35 e_atan2f.c / s_atanf.c (fdlibm) with every
//    data-dependent branch of the finite, non-zero case turned into selects:
//    all lanes of a wave run one instruction stream instead of up to five
//    range-reduction paths x four quadrants.  The special cases (NaN, +-0,
//    +-inf, x == 1) keep the branchy restatement (g_atan2f).
#pragma once
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define RTG_HD __host__ __device__ __forceinline__
#define RTG_FMA(a, b, c) __builtin_fma((a), (b), (c))
#define RTG_RINT(a) __builtin_rint(a)
#else
#include <math.h>
#define RTG_HD static inline
#define RTG_FMA(a, b, c) fma((a), (b), (c))
#define RTG_RINT(a) rint(a)
#endif

namespace rtg {
namespace crm {

RTG_HD int32_t fbits(float f)
{
    int32_t i;
    memcpy(&i, &f, sizeof i);
    return i;
}

// ---------------------------------------------------------------- sincos
struct SinCos {
    float s, c;
    bool s_ok, c_ok;   // false: the caller must use its exact fallback for that value
};

// Round 5: the test reads the 29 bits f32 rounding drops from y's representation instead of rounding y(1 -+ 2^-44)
// twice (integer work only): accepted when they are not within 512 f64 ulps of the midpoint 2^28 -- at least the old
// margin (|y| 2^-44 is 256..512 ulps), so every accepted value is still correctly rounded -- and |y| is in the f32
// normal range (0 and subnormal results take the exact fallback).
RTG_HD bool round_ok(double y, float &out)
{
    out = (float)y;
    uint64_t b;
    memcpy(&b, &y, sizeof b);
    const uint32_t lo = (uint32_t)b & 0x1FFFFFFFu;
    const uint32_t ex = (uint32_t)(b >> 52) & 0x7FFu;
    return ((uint32_t)(lo - (0x10000000u - 512u)) > 1024u) & (ex >= 1023u - 126u) & (ex <= 1023u + 127u);
}

RTG_HD SinCos crm_sincos(double x)
{
    SinCos r;
    const double ax0 = x < 0 ? -x : x;
    // NaN / inf / huge: fallback; +-0: exact.  Selected at the end (no branch): the reduction below runs on a finite
    // stand-in for those x and its values are discarded.
    const bool special = !(ax0 <= 0x1p17) | (x == 0.0);
    const double x0 = x;
    x = special ? 0.5 : x;
    // pi/2 = P1 + P2 + P3 + P3T (fdlibm pio2_1, pio2_2, pio2_3: 33 significant bits each)
    const double P1 = 1.57079632673412561417e+00, P2 = 6.07710050630396597660e-11,
                 P3 = 2.02226624871116645580e-21, P3T = 8.47842766036889956997e-32;
    const double k = RTG_RINT(x * 6.36619772367581382433e-01);   // x * 2/pi
    double t = RTG_FMA(-k, P1, x);   // exact: k*P1 fits 53 bits and is within 2x of x
    t = RTG_FMA(-k, P2, t);
    t = RTG_FMA(-k, P3, t);
    t = RTG_FMA(-k, P3T, t);
    const double z = t * t;
    // fdlibm __kernel_sin / __kernel_cos coefficients
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    double ps = RTG_FMA(z, S6, S5);
    ps = RTG_FMA(z, ps, S4);
    ps = RTG_FMA(z, ps, S3);
    ps = RTG_FMA(z, ps, S2);
    ps = RTG_FMA(z, ps, S1);
    const double sn = RTG_FMA(t * z, ps, t);
    double pc = RTG_FMA(z, C6, C5);
    pc = RTG_FMA(z, pc, C4);
    pc = RTG_FMA(z, pc, C3);
    pc = RTG_FMA(z, pc, C2);
    pc = RTG_FMA(z, pc, C1);
    const double cs = RTG_FMA(z * z, pc, RTG_FMA(-0.5, z, 1.0));
    // quadrant n: sin = (sn, cs, -sn, -cs)[n], cos = (cs, -sn, -cs, sn)[n] -- one swap and two sign flips
    const int n = (int)(int64_t)k & 3;
    const bool swap = (n & 1) != 0;
    const double sa = swap ? cs : sn, ca = swap ? sn : cs;
    const double vs = (n & 2) ? -sa : sa;
    const double vc = ((n + 1) & 2) ? -ca : ca;
    r.s_ok = round_ok(vs, r.s);
    r.c_ok = round_ok(vc, r.c);
    r.s = special ? (float)x0 : r.s;
    r.c = special ? 1.0f : r.c;
    r.s_ok = special ? (x0 == 0.0) : r.s_ok;
    r.c_ok = special ? (x0 == 0.0) : r.c_ok;
    return r;
}

// ---------------------------------------------------------------- atan2f
// glibc s_atanf.c for finite t >= 0, branch-free.  Range reductions:
//   id -1 (t < 7/16):  t                       (t/1, exact)
//   id  0 (< 11/16):   (2t - 1) / (2 + t)
//   id  1 (< 19/16):   (t - 1) / (t + 1)
//   id  2 (< 39/16):   (t - 1.5) / (1 + 1.5t)
//   id  3:             -1 / t                  ((0*t - 1) / (0 + t), exact rewrite for t > 0)
// written as (A*t - Bn) / (Cd + D*t); every product/sum that differs from
// fdlibm's expression is exact (1*t, 0*t, 0+t, t/1), so each id rounds as glibc does.
RTG_HD float crm_atanf_pos(float t)
{
    const int32_t ix = fbits(t);
    const bool huge = ix >= 0x4c000000, tiny = ix < 0x31000000;
    const int id = ix < 0x3ee00000 ? -1 : ix < 0x3f300000 ? 0 : ix < 0x3f980000 ? 1 : ix < 0x401c0000 ? 2 : 3;
    const float A = id == 0 ? 2.0f : (id == 3 ? 0.0f : 1.0f);
    const float Bn = id == 0 ? 1.0f : id == 1 ? 1.0f : id == 2 ? 1.5f : id == 3 ? 1.0f : 0.0f;
    const float Cd = id == 0 ? 2.0f : id == 3 ? 0.0f : 1.0f;
    const float D = id == 2 ? 1.5f : id == -1 ? 0.0f : 1.0f;
    const float hi = id == 0 ? 4.6364760399e-01f : id == 1 ? 7.8539812565e-01f : id == 2 ? 9.8279368877e-01f
                                                                                        : 1.5707962513e+00f;
    const float lo = id == 0 ? 5.0121582440e-09f : id == 1 ? 3.7748947079e-08f : id == 2 ? 3.4473217170e-08f
                                                                                        : 7.5497894159e-08f;
    const float x = (A * t - Bn) / (Cd + D * t);
    const float z = x * x;
    const float w = z * z;
    const float s1 = z * (3.3333334327e-01f + w * (1.4285714924e-01f + w * (9.0908870101e-02f +
                     w * (6.6610731184e-02f + w * (4.9768779427e-02f + w * 1.6285819933e-02f)))));
    const float s2 = w * (-2.0000000298e-01f + w * (-1.1111110449e-01f + w * (-7.6918758452e-02f +
                     w * (-5.8335702866e-02f + w * -3.6531571299e-02f))));
    const float r_small = x - x * (s1 + s2);
    const float r_red = hi - ((x * (s1 + s2) - lo) - x);
    const float r = id < 0 ? r_small : r_red;
    return huge ? 1.5707962513e+00f + 7.5497894159e-08f : (tiny ? t : r);
}

// true when crm_atan2f's select path applies (finite, non-zero x and y, x != 1)
RTG_HD bool crm_atan2f_regular(float y, float x)
{
    const int32_t hx = fbits(x), ix = hx & 0x7fffffff, iy = fbits(y) & 0x7fffffff;
    return (ix != 0) & (iy != 0) & (ix < 0x7f800000) & (iy < 0x7f800000) & (hx != 0x3f800000);
}

// e_atan2f.c, regular case only (see crm_atan2f_regular)
RTG_HD float crm_atan2f_sel(float y, float x)
{
    const float pi_o_2 = 1.5707963705e+00f, pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;
    const int32_t hx = fbits(x), hy = fbits(y);
    const int32_t ix = hx & 0x7fffffff, iy = hy & 0x7fffffff;
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    const int32_t k = (iy - ix) >> 23;
    const float q = y / x;
    const float za = crm_atanf_pos(__builtin_fabsf(q));   // fabsf: an underflowed -0 becomes +0, as in glibc
    const float z = k > 60 ? pi_o_2 + 0.5f * pi_lo : ((hx < 0 && k < -60) ? 0.0f : za);
    return m == 0 ? z : m == 1 ? -z : m == 2 ? pi - (z - pi_lo) : (z - pi_lo) - pi;
}

}  // namespace crm
}  // namespace rtg
