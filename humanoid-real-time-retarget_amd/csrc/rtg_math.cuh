// rtg_math.cuh -- device math for the retargeting hot path (gfx950).
//
// Every float32 operation is rounded on its own, in the association order the
// reference's torch CPU ops use (build flag -ffp-contract=off plus the pragma
// below); the two places torch itself fuses (torch.linalg.norm of a 3-vector
// and torch.cross) use explicit __builtin_fmaf.  Measured op orders: DESIGN.md §3.
//
//  * torch.sqrt/acos/sin/cos run through MKL VML on the CPU (closed source):
//    here they are correctly rounded (evaluated in float64, rounded once).
//  * atan2 on the 30-element DOF tensor runs glibc's scalar atan2f: restated
//    exactly (fdlibm s_atanf/e_atan2f).
//  * torch.linalg.svd (MKL sgesdd) in the Kabsch fit: the proper-rotation polar
//    factor is computed in float64 (cyclic Jacobi on A^T A) and rounded.
//  * scipy Rotation.as_euler / from_euler: float64 restatement.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rtg_crmath.h"

#pragma clang fp contract(off)

namespace rtg {

struct Q { float x, y, z, w; };
struct V { float x, y, z; };

#define RTG_DEV __device__ __forceinline__

// ---------------------------------------------------------------- helpers
RTG_DEV float ieee_sqrtf(float x) { return __builtin_sqrtf(x); }   // IEEE sqrt (correctly rounded build)
#ifndef RTG_FAST_EXACT
#define RTG_FAST_EXACT 1
#endif
// Correctly rounded f32 sqrt in 6 instructions: v_sqrt_f64 (not accurate enough alone: it misses on 4 % of
// inputs) plus one Newton correction gives ~2^-100, and sqrt of an f32 is never within 2^-51 of an f32
// midpoint, so the single rounding is exact.  0 / inf / NaN / negative: the residual is 0 or NaN and the raw
// v_sqrt_f64 value (IEEE for those) is kept.  Proven equal to __builtin_sqrtf on all 2^32 inputs by
// tools/check_fastmath.hip (run by tests/test_gpu_parity.py).
RTG_DEV float cr_sqrt(float x)
{
#if RTG_FAST_EXACT
    const double d = (double)x;
    const double y = __builtin_amdgcn_sqrt(d);
    const double r = __builtin_fma(-y, y, d);
    const double y1 = __builtin_fma(r, 0.5 * __builtin_amdgcn_rcp(y), y);
    return (float)((r == 0.0 || r != r) ? y : y1);
#else
    return __builtin_sqrtf(x);
#endif
}
RTG_DEV float cr_acos(float x) { return (float)::acos((double)x); }
RTG_DEV float cr_sin(float x) { return (float)::sin((double)x); }
RTG_DEV float cr_cos(float x) { return (float)::cos((double)x); }
// sin and cos of one argument, correctly rounded: fast shared-reduction path
// (rtg_crmath.h, exhaustively checked against glibc) with the libm f64 call as
// the exact fallback for the ~1-in-10^7 values the rounding test declines.
struct SC { float s, c; };
RTG_DEV SC cr_sincos(double x)
{
    const crm::SinCos r = crm::crm_sincos(x);
    return SC{r.s_ok ? r.s : (float)::sin(x), r.c_ok ? r.c : (float)::cos(x)};
}
// k float divisions by one denominator n: RN(a/n) == (float)((double)a * RN(1/(double)n))
// for all f32 a, n.  (An f32 quotient is never within 2^-50 relative of an f32
// rounding midpoint, and the f64 product is within 2^-52; checked on 4.3e9
// random pairs incl. subnormals / zeros / infinities, tests/test_oracle_golden.py.)
// One f64 reciprocal replaces k correctly rounded f32 divide sequences.
// 1/n for k divisions by one denominator: v_rcp_f64 + two Newton steps, i.e. RN(1/n) to within an ulp even
// from a 14-bit estimate (the IEEE f64 divide sequence is twice as long).  0 / inf / NaN make the residual NaN;
// the raw v_rcp_f64 value (inf, 0, NaN) is then the IEEE answer.
struct Rcp {
    double r;
    float n;
};
RTG_DEV Rcp rcp64(float n)
{
#if RTG_FAST_EXACT
    const double d = (double)n;
    const double r0 = __builtin_amdgcn_rcp(d);
    const double e0 = __builtin_fma(-d, r0, 1.0);
    const double r1 = __builtin_fma(r0, e0, r0);
    const double e1 = __builtin_fma(-d, r1, 1.0);
    return Rcp{e0 == e0 ? __builtin_fma(r1, e1, r1) : r0, n};
#else
    return Rcp{1.0 / (double)n, n};
#endif
}
// RN(a/n) == (float)((double)a * 1/n) whenever the quotient is a normal f32: an f32 quotient is never within
// 2^-50 (relative) of an f32 midpoint and the f64 product is within 2^-52.  A subnormal quotient (absolute
// grid) takes the IEEE division; that branch is rare and divergent.  tools/check_fastmath.hip: 2^32 random
// pairs + all special-value pairs, 0 mismatches.
RTG_DEV float mulr(float a, const Rcp &r)
{
    const double p = (double)a * r.r;
    float q = (float)p;
    if (__builtin_expect(__builtin_fabs(p) < 0x1p-126 && p != 0.0, 0)) q = a / r.n;
    return q;
}
RTG_DEV float tsign(float v) { return v > 0.0f ? 1.0f : (v < 0.0f ? -1.0f : 0.0f); }
RTG_DEV float clamp_lo(float v, float lo) { return v < lo ? lo : v; }          // NaN passes through
RTG_DEV float clamp_lohi(float v, float lo, float hi) { return v < lo ? lo : (v > hi ? hi : v); }

// glibc 2.35 float atanf (fdlibm s_atanf.c algorithm, decimal constants)
RTG_DEV float g_atanf(float x)
{
    const float atanhi0 = 4.6364760399e-01f, atanhi1 = 7.8539812565e-01f, atanhi2 = 9.8279368877e-01f,
                atanhi3 = 1.5707962513e+00f;
    const float atanlo0 = 5.0121582440e-09f, atanlo1 = 3.7748947079e-08f, atanlo2 = 3.4473217170e-08f,
                atanlo3 = 7.5497894159e-08f;
    const int32_t hx = __float_as_int(x);
    const int32_t ix = hx & 0x7fffffff;
    if (ix >= 0x4c000000) {
        if (ix > 0x7f800000) return x + x;
        return hx > 0 ? atanhi3 + atanlo3 : -atanhi3 - atanlo3;
    }
    int id;
    float hi = 0.0f, lo = 0.0f;
    if (ix < 0x3ee00000) {
        if (ix < 0x31000000) return x;
        id = -1;
    } else {
        x = fabsf(x);
        if (ix < 0x3f980000) {
            if (ix < 0x3f300000) { id = 0; x = (2.0f * x - 1.0f) / (2.0f + x); hi = atanhi0; lo = atanlo0; }
            else { id = 1; x = (x - 1.0f) / (x + 1.0f); hi = atanhi1; lo = atanlo1; }
        } else {
            if (ix < 0x401c0000) { id = 2; x = (x - 1.5f) / (1.0f + 1.5f * x); hi = atanhi2; lo = atanlo2; }
            else { id = 3; x = -1.0f / x; hi = atanhi3; lo = atanlo3; }
        }
    }
    const float z = x * x;
    const float w = z * z;
    const float s1 = z * (3.3333334327e-01f + w * (1.4285714924e-01f + w * (9.0908870101e-02f +
                     w * (6.6610731184e-02f + w * (4.9768779427e-02f + w * 1.6285819933e-02f)))));
    const float s2 = w * (-2.0000000298e-01f + w * (-1.1111110449e-01f + w * (-7.6918758452e-02f +
                     w * (-5.8335702866e-02f + w * -3.6531571299e-02f))));
    if (id < 0) return x - x * (s1 + s2);
    const float r = hi - ((x * (s1 + s2) - lo) - x);
    return hx < 0 ? -r : r;
}

// glibc 2.35 e_atan2f.c (torch.atan2 on <32-element tensors takes the scalar std::atan2 path)
RTG_DEV float g_atan2f(float y, float x)
{
    const float tiny = 1.0e-30f, pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f,
                pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;
    const int32_t hx = __float_as_int(x), hy = __float_as_int(y);
    const int32_t ix = hx & 0x7fffffff, iy = hy & 0x7fffffff;
    if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;
    if (hx == 0x3f800000) return g_atanf(y);
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    if (iy == 0) {
        if (m <= 1) return y;
        return m == 2 ? pi + tiny : -pi - tiny;
    }
    if (ix == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    if (ix == 0x7f800000) {
        if (iy == 0x7f800000) {
            if (m == 0) return pi_o_4 + tiny;
            if (m == 1) return -pi_o_4 - tiny;
            if (m == 2) return 3.0f * pi_o_4 + tiny;
            return -3.0f * pi_o_4 - tiny;
        }
        if (m == 0) return 0.0f;
        if (m == 1) return -0.0f;
        return m == 2 ? pi + tiny : -pi - tiny;
    }
    if (iy == 0x7f800000) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    const int32_t k = (iy - ix) >> 23;
    float z;
    if (k > 60) z = pi_o_2 + 0.5f * pi_lo;
    else if (hx < 0 && k < -60) z = 0.0f;
    else z = g_atanf(fabsf(y / x));
    if (m == 0) return z;
    if (m == 1) return -z;
    if (m == 2) return pi - (z - pi_lo);
    return (z - pi_lo) - pi;
}

// atan2f with the finite non-zero case branch-free (rtg_crmath.h); special
// operands take the branchy restatement above.
RTG_DEV float f_atan2f(float y, float x)
{
    return crm::crm_atan2f_regular(y, x) ? crm::crm_atan2f_sel(y, x) : g_atan2f(y, x);
}
RTG_DEV float normalize_angle(float a)   // rotation3d.py:582-584: atan2(sin a, cos a)
{
    const SC t = cr_sincos((double)a);
    return f_atan2f(t.s, t.c);
}

// ------------------------------------------------ quaternion algebra (rotation3d.py)
RTG_DEV Q qmul(Q a, Q b)   // :14-27, each component a left fold of four products
{
    Q r;
    r.w = ((a.w * b.w - a.x * b.x) - a.y * b.y) - a.z * b.z;
    r.x = ((a.w * b.x + a.x * b.w) + a.y * b.z) - a.z * b.y;
    r.y = ((a.w * b.y + a.y * b.w) + a.z * b.x) - a.x * b.z;
    r.z = ((a.w * b.z + a.z * b.w) + a.x * b.y) - a.y * b.x;
    return r;
}
RTG_DEV Q qconj(Q a) { return Q{-a.x, -a.y, -a.z, a.w}; }
RTG_DEV Q qident() { return Q{0.0f, 0.0f, 0.0f, 1.0f}; }

RTG_DEV Q qnormalize(Q q)  // quat_unit(quat_pos(q)) :30-56,92-98
{
    const float f = 1.0f - 2.0f * (q.w < 0.0f ? 1.0f : 0.0f);
    q.x = f * q.x; q.y = f * q.y; q.z = f * q.z; q.w = f * q.w;
    float n = cr_sqrt(((q.x * q.x + q.y * q.y) + q.z * q.z) + q.w * q.w);
    n = clamp_lo(n, 1e-9f);
    const Rcp r = rcp64(n);
    return Q{mulr(q.x, r), mulr(q.y, r), mulr(q.z, r), mulr(q.w, r)};
}
RTG_DEV Q qmul_norm(Q a, Q b) { return qnormalize(qmul(a, b)); }
RTG_DEV float qabs(Q q) { return cr_sqrt(((q.x * q.x + q.y * q.y) + q.z * q.z) + q.w * q.w); }   // :41-47
RTG_DEV Q qunit(Q q)                                                                                 // :50-56
{
    const float n = clamp_lo(qabs(q), 1e-9f);
    const Rcp r = rcp64(n);
    return Q{mulr(q.x, r), mulr(q.y, r), mulr(q.z, r), mulr(q.w, r)};
}
// quat_angle_axis (:230-240): angle = acos(clamp(2 w^2 - 1)), axis = xyz / max(|xyz|, 1e-9)
RTG_DEV Q qangle_axis_abs(Q q)
{
    const float s = clamp_lohi(2.0f * (q.w * q.w) - 1.0f, -1.0f, 1.0f);
    const float n = clamp_lo(cr_sqrt((q.x * q.x + q.y * q.y) + q.z * q.z), 1e-9f);
    const Rcp r = rcp64(n);
    return Q{cr_acos(s), mulr(q.x, r), mulr(q.y, r), mulr(q.z, r)};
}

RTG_DEV V qrotate(Q q, V v)  // :205-211, two Hamilton products
{
    const Q r = qmul(qmul(q, Q{v.x, v.y, v.z, 0.0f}), qconj(q));
    return V{r.x, r.y, r.z};
}

RTG_DEV Q qfrom_angle_axis(float angle, V axis)  // :122-143
{
    const float theta = angle / 2.0f;
    float n = cr_sqrt((axis.x * axis.x + axis.y * axis.y) + axis.z * axis.z);
    n = clamp_lo(n, 1e-9f);
    const Rcp r = rcp64(n);
    const float ax = mulr(axis.x, r), ay = mulr(axis.y, r), az = mulr(axis.z, r);
    const SC t = cr_sincos((double)theta);
    const float s = t.s, c = t.c;
    return qnormalize(Q{ax * s, ay * s, az * s, c});
}
// quat_from_angle_axis about an exact unit axis (ex / ey / ez): the axis normalisation is the identity
// (sqrt(1) = 1, +0 and 1 times RN(1/1) stay +0 and 1), so it is skipped -- the same bits.
RTG_DEV Q qfrom_angle_unit_axis(float angle, V axis)
{
    const float theta = angle / 2.0f;
    const SC t = cr_sincos((double)theta);
    return qnormalize(Q{axis.x * t.s, axis.y * t.s, axis.z * t.s, t.c});
}

RTG_DEV Q qfrom_rotmat(const float m[9])  // :146-193 (the four overlapping branches, in order)
{
    const float d0 = m[0], d1 = m[4], d2 = m[8];
    float w = cr_sqrt(clamp_lo((((d0 + d1) + d2) + 1.0f) / 4.0f, 0.0f));
    float x = cr_sqrt(clamp_lo((((d0 - d1) - d2) + 1.0f) / 4.0f, 0.0f));
    float y = cr_sqrt(clamp_lo((((-d0 + d1) - d2) + 1.0f) / 4.0f, 0.0f));
    float z = cr_sqrt(clamp_lo((((-d0 - d1) + d2) + 1.0f) / 4.0f, 0.0f));
    if (w >= x && w >= y && w >= z) {
        x *= tsign(m[7] - m[5]);
        y *= tsign(m[2] - m[6]);
        z *= tsign(m[3] - m[1]);
    }
    if (x >= w && x >= y && x >= z) {
        w *= tsign(m[7] - m[5]);
        y *= tsign(m[3] + m[1]);
        z *= tsign(m[2] + m[6]);
    }
    if (y >= w && y >= x && y >= z) {
        w *= tsign(m[2] - m[6]);
        x *= tsign(m[3] + m[1]);
        z *= tsign(m[7] + m[5]);
    }
    if (z >= w && z >= x && z >= y) {
        w *= tsign(m[3] - m[1]);
        x *= tsign(m[6] + m[2]);
        y *= tsign(m[7] + m[5]);
    }
    return qnormalize(Q{x, y, z, w});
}

// quat_to_angle_axis + angle_axis_to_exp_map (:587-627), returns the 3 exp-map components
RTG_DEV V qexp_map(Q q)
{
    const float sin_theta = cr_sqrt(1.0f - q.w * q.w);
    float angle = 2.0f * cr_acos(q.w);
    angle = normalize_angle(angle);   // normalize_angle :582-584
    const bool mask = fabsf(sin_theta) > 1e-5f;
    const float a = mask ? angle : 0.0f;
    const float ax = mask ? q.x / sin_theta : 0.0f;
    const float ay = mask ? q.y / sin_theta : 0.0f;
    const float az = mask ? q.z / sin_theta : 1.0f;
    return V{a * ax, a * ay, a * az};
}
// quat_to_angle_axis (:587-608) as [angle, axis]
RTG_DEV Q qangle_axis(Q q)
{
    const float sin_theta = cr_sqrt(1.0f - q.w * q.w);
    float angle = 2.0f * cr_acos(q.w);
    angle = normalize_angle(angle);
    const bool mask = fabsf(sin_theta) > 1e-5f;
    const Rcp r = rcp64(sin_theta);
    return Q{mask ? angle : 0.0f, mask ? mulr(q.x, r) : 0.0f, mask ? mulr(q.y, r) : 0.0f,
             mask ? mulr(q.z, r) : 1.0f};
}
RTG_DEV float qexp_component(Q q, int k)
{
    const V e = qexp_map(q);
    return k == 0 ? e.x : (k == 1 ? e.y : e.z);
}

// ------------------------------------------------ exp-map angle table
// The angle of quat_to_angle_axis (:595-597) is R(w) = normalize_angle(2 acos w) = atan2f(RN sin A, RN cos A)
// with A = 2 RN(acos w): glibc atan2f is not correctly rounded, so R has no closed form.  For w in [0.25, 1) --
// joint angles below 151 degrees -- R(w) is stored as a short move from a cheap f32 estimate P(w) =
// 4 asin(sqrt((1 - w) / 2)) (v_sqrt_f32 and a degree-6 fma polynomial, within 3 ulps of R): the 3-bit code c in
// 1..7 means R = P + (c - 4) ulps, 0 means "not tabulated" (exact path).  2^24 entries, 10 per 32-bit word, in
// 6.7 MiB (RTG_ANG_TAB_BITS=4 packs 8 per word in 8 MiB; measured no faster), built on the device by the exact path
// itself (ang_tab_code, k_build_ang_tab) with the same P.  qexp_component_tab thus skips acos, sincos and
// atan2f (290 of the 330 instructions of an exp-map); w outside the table or a code-0 entry takes the exact
// path.  tools/check_fastmath.hip checks qexp_component_tab == qexp_component for every f32 w.
#ifndef RTG_EXP_NO_TABLE
#define RTG_EXP_NO_TABLE 0
#endif
constexpr uint32_t kAngTabLo = 0x3e800000u;                     // bits of 0.25f
constexpr uint32_t kAngTabEntries = 0x3f800000u - kAngTabLo;    // up to 1.0f (exclusive): 2^24
#ifndef RTG_ANG_TAB_BITS
#define RTG_ANG_TAB_BITS 3
#endif
constexpr uint32_t kAngTabBits = RTG_ANG_TAB_BITS;              // 3: moves -3..3, 10 codes per word; 4: -7..7, 8
constexpr uint32_t kAngTabPer = kAngTabBits == 3 ? 10u : 8u;
constexpr uint32_t kAngTabWords = (kAngTabEntries + kAngTabPer - 1) / kAngTabPer;
constexpr uint32_t kAngTabBias = 1u << (kAngTabBits - 1);      // code = move + bias; code 0 = not tabulated
RTG_DEV uint32_t ang_tab_word(uint32_t i) { return kAngTabPer == 10u ? __umulhi(i, 0xCCCCCCCDu) >> 3 : i >> 3; }
RTG_DEV float exp_angle_estimate(float w)
{
    const float t2 = (1.0f - w) * 0.5f;
    const float t = __builtin_amdgcn_sqrtf(t2);
    float p = __builtin_fmaf(0.04965998747593211f, t2, -0.005969297163659217f);
    p = __builtin_fmaf(p, t2, 0.029188122223620813f);
    p = __builtin_fmaf(p, t2, 0.02938421651028137f);
    p = __builtin_fmaf(p, t2, 0.0447135443846629f);
    p = __builtin_fmaf(p, t2, 0.07499796602478857f);
    p = __builtin_fmaf(p, t2, 0.1666666806527845f);
    return 4.0f * __builtin_fmaf(t, t2 * p, t);
}
RTG_DEV uint32_t ang_tab_code(float w)
{
    const float R = normalize_angle(2.0f * cr_acos(w));
    const float P = exp_angle_estimate(w);
    if (!(R > 0.0f) || !(P > 0.0f) || !(R < 4.0f) || !(P < 4.0f)) return 0u;
    const int32_t d = (int32_t)__float_as_uint(R) - (int32_t)__float_as_uint(P);
    const int32_t lim = (int32_t)kAngTabBias - 1;
    return (d >= -lim && d <= lim) ? (uint32_t)(d + (int32_t)kAngTabBias) : 0u;
}
// word wd of the table: the codes of entries wd * kAngTabPer ... (k_build_ang_tab, tools/check_fastmath.hip)
RTG_DEV uint32_t ang_tab_build_word(uint32_t wd)
{
    uint32_t word = 0;
    for (uint32_t e = 0; e < kAngTabPer; ++e) {
        const uint32_t i = wd * kAngTabPer + e;
        if (i < kAngTabEntries) word |= ang_tab_code(__uint_as_float(kAngTabLo + i)) << (kAngTabBits * e);
    }
    return word;
}
// quat_to_exp_map(q)[k] given only w = q.w and qk = q[k]: for |sin_theta| <= 1e-5 the reference's product is
// 0 * (0 or 1) = +0 whatever k is, so the component index itself is not needed.
RTG_DEV float exp_dof_tab(float w, float qk, const uint32_t *__restrict__ tab)
{
    const uint32_t i = __float_as_uint(w) - kAngTabLo;
    const bool in = i < kAngTabEntries;
#if RTG_EXP_NO_TABLE   // measurement knob (tools/build_variants.sh): no table traffic, wrong angles
    const uint32_t wd = ang_tab_word(i);
    const uint32_t word = 0x24924924u + 0u * tab[0];
#else
    const uint32_t wd = ang_tab_word(i);
    const uint32_t word = tab[in ? wd : 0u];
#endif
    const float sin_theta = cr_sqrt(1.0f - w * w);
    const bool mask = fabsf(sin_theta) > 1e-5f;
    const float P = exp_angle_estimate(w);
    const uint32_t code = in ? (word >> ((i - wd * kAngTabPer) * kAngTabBits)) & ((1u << kAngTabBits) - 1u) : 0u;
    float angle = __uint_as_float(__float_as_uint(P) + code - kAngTabBias);
    if (__builtin_expect(mask && code == 0u, 0)) angle = normalize_angle(2.0f * cr_acos(w));
    return mask ? angle * (qk / sin_theta) : 0.0f;
}
RTG_DEV float qexp_component_tab(Q q, int k, const uint32_t *__restrict__ tab)
{
    return exp_dof_tab(q.w, k == 0 ? q.x : (k == 1 ? q.y : q.z), tab);
}

// ------------------------------------------------ vectors (transform3d.py)
RTG_DEV float dot3(V a, V b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }          // torch.dot
RTG_DEV float lnorm3(V a)                                                              // torch.linalg.norm
{
    return cr_sqrt(__builtin_fmaf(a.z, a.z, __builtin_fmaf(a.y, a.y, a.x * a.x)));
}
RTG_DEV V cross3(V a, V b)                                                             // torch.cross
{
    return V{__builtin_fmaf(a.y, b.z, -(a.z * b.y)), __builtin_fmaf(a.z, b.x, -(a.x * b.z)),
             __builtin_fmaf(a.x, b.y, -(a.y * b.x))};
}
RTG_DEV V vsub(V a, V b) { return V{a.x - b.x, a.y - b.y, a.z - b.z}; }
RTG_DEV V vdiv(V a, float s)
{
    const Rcp r = rcp64(s);
    return V{mulr(a.x, r), mulr(a.y, r), mulr(a.z, r)};
}
RTG_DEV V vmul(V a, float s) { return V{s * a.x, s * a.y, s * a.z}; }

RTG_DEV V proj_in_plane(V v, V n)  // :61-75
{
    const float nn = lnorm3(n);
    return vsub(v, vmul(n, dot3(v, n) / (nn * nn)));
}

RTG_DEV float radians_between(V v1, V v2, V n)  // :77-100
{
    v1 = vdiv(v1, lnorm3(v1));
    v2 = vdiv(v2, lnorm3(v2));
    const V nrm = vdiv(n, lnorm3(n));
    const float c = clamp_lohi(dot3(v1, v2), -1.0f, 1.0f);
    return cr_acos(c) * tsign(dot3(nrm, cross3(v1, v2)));
}
// radians_between with v1 and n exact unit axes (the arm maps' ex / ey / ez): their normalisation is the
// identity (lnorm3 = sqrt(1) = 1, x * RN(1/1) = x), so only v2 is normalised -- the same bits, 2/3 fewer divides.
RTG_DEV float radians_between_axes(V v1, V v2, V n)
{
    v2 = vdiv(v2, lnorm3(v2));
    const float c = clamp_lohi(dot3(v1, v2), -1.0f, 1.0f);
    return cr_acos(c) * tsign(dot3(n, cross3(v1, v2)));
}

// ------------------------------------------------ Kabsch (float64)
// Proper-rotation polar factor of A: R = u1 v1^T + u2 v2^T + (u1 x u2)(v1 x v2)^T
// where (v_i) are eigenvectors of A^T A for the two largest eigenvalues and
// u_i = A v_i / |A v_i| (u2 re-orthogonalised).  Equals U diag(1,1,det(UV^T)) V^T,
// the reference's det-fixed SVD solution (transform3d.py:40-45).
RTG_DEV void jacobi_eig3(double S[3][3], double Vm[3][3])
{
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) Vm[i][j] = i == j ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 8; ++sweep) {
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            const int p = r == 2 ? 1 : 0;
            const int qq = r == 0 ? 1 : 2;
            const double apq = S[p][qq];
            if (apq == 0.0) continue;
            const double theta = (S[qq][qq] - S[p][p]) / (2.0 * apq);
            double t = 1.0 / (fabs(theta) + sqrt(theta * theta + 1.0));
            if (theta < 0.0) t = -t;
            const double c = 1.0 / sqrt(t * t + 1.0);
            const double s = t * c;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const double skp = S[k][p], skq = S[k][qq];
                S[k][p] = c * skp - s * skq;
                S[k][qq] = s * skp + c * skq;
            }
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const double spk = S[p][k], sqk = S[qq][k];
                S[p][k] = c * spk - s * sqk;
                S[qq][k] = s * spk + c * sqk;
            }
            S[p][qq] = 0.0;
            S[qq][p] = 0.0;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const double vkp = Vm[k][p], vkq = Vm[k][qq];
                Vm[k][p] = c * vkp - s * vkq;
                Vm[k][qq] = s * vkp + c * vkq;
            }
        }
    }
}

RTG_DEV void kabsch_rot_jacobi(const float A[9], float R[9])
{
    double a[3][3], S[3][3], Vm[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) a[i][j] = (double)A[i * 3 + j];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) S[i][j] = a[0][i] * a[0][j] + a[1][i] * a[1][j] + a[2][i] * a[2][j];
    jacobi_eig3(S, Vm);
    // descending order of the eigenvalues (same selection as the oracle's sort),
    // done on values so no array is indexed at run time
    int o0 = 0, o1 = 1, o2 = 2, ti;
    double a0 = S[0][0], a1 = S[1][1], a2 = S[2][2], td;
    if (a1 > a0) { ti = o0; o0 = o1; o1 = ti; td = a0; a0 = a1; a1 = td; }
    if (a2 > a0) { ti = o0; o0 = o2; o2 = ti; td = a0; a0 = a2; a2 = td; }
    if (a2 > a1) { ti = o1; o1 = o2; o2 = ti; td = a1; a1 = a2; a2 = td; }
    double v1[3], v2[3], u1[3], u2[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        v1[i] = o0 == 0 ? Vm[i][0] : (o0 == 1 ? Vm[i][1] : Vm[i][2]);
        v2[i] = o1 == 0 ? Vm[i][0] : (o1 == 1 ? Vm[i][1] : Vm[i][2]);
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        u1[i] = a[i][0] * v1[0] + a[i][1] * v1[1] + a[i][2] * v1[2];
        u2[i] = a[i][0] * v2[0] + a[i][1] * v2[1] + a[i][2] * v2[2];
    }
    const double n1 = sqrt(u1[0] * u1[0] + u1[1] * u1[1] + u1[2] * u1[2]);
#pragma unroll
    for (int i = 0; i < 3; ++i) u1[i] /= n1;
    const double d = u1[0] * u2[0] + u1[1] * u2[1] + u1[2] * u2[2];
#pragma unroll
    for (int i = 0; i < 3; ++i) u2[i] -= d * u1[i];
    const double n2 = sqrt(u2[0] * u2[0] + u2[1] * u2[1] + u2[2] * u2[2]);
#pragma unroll
    for (int i = 0; i < 3; ++i) u2[i] /= n2;
    const double u3[3] = {u1[1] * u2[2] - u1[2] * u2[1], u1[2] * u2[0] - u1[0] * u2[2],
                          u1[0] * u2[1] - u1[1] * u2[0]};
    const double v3[3] = {v1[1] * v2[2] - v1[2] * v2[1], v1[2] * v2[0] - v1[0] * v2[2],
                          v1[0] * v2[1] - v1[1] * v2[0]};
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) R[i * 3 + j] = (float)(u1[i] * v1[j] + u2[i] * v2[j] + u3[i] * v3[j]);
}

// 4x4 adjugate (and determinant) by 2x2 sub-determinants; m row-major
RTG_DEV double adj4(const double m[16], double inv[16], bool want_adj)
{
    const double s0 = m[0] * m[5] - m[4] * m[1], s1 = m[0] * m[6] - m[4] * m[2];
    const double s2 = m[0] * m[7] - m[4] * m[3], s3 = m[1] * m[6] - m[5] * m[2];
    const double s4 = m[1] * m[7] - m[5] * m[3], s5 = m[2] * m[7] - m[6] * m[3];
    const double c5 = m[10] * m[15] - m[14] * m[11], c4 = m[9] * m[15] - m[13] * m[11];
    const double c3 = m[9] * m[14] - m[13] * m[10], c2 = m[8] * m[15] - m[12] * m[11];
    const double c1 = m[8] * m[14] - m[12] * m[10], c0 = m[8] * m[13] - m[12] * m[9];
    if (want_adj) {
        inv[0] = m[5] * c5 - m[6] * c4 + m[7] * c3;
        inv[1] = -m[1] * c5 + m[2] * c4 - m[3] * c3;
        inv[2] = m[13] * s5 - m[14] * s4 + m[15] * s3;
        inv[3] = -m[9] * s5 + m[10] * s4 - m[11] * s3;
        inv[4] = -m[4] * c5 + m[6] * c2 - m[7] * c1;
        inv[5] = m[0] * c5 - m[2] * c2 + m[3] * c1;
        inv[6] = -m[12] * s5 + m[14] * s2 - m[15] * s1;
        inv[7] = m[8] * s5 - m[10] * s2 + m[11] * s1;
        inv[8] = m[4] * c4 - m[5] * c2 + m[7] * c0;
        inv[9] = -m[0] * c4 + m[1] * c2 - m[3] * c0;
        inv[10] = m[12] * s4 - m[13] * s2 + m[15] * s0;
        inv[11] = -m[8] * s4 + m[9] * s2 - m[11] * s0;
        inv[12] = -m[4] * c3 + m[5] * c1 - m[6] * c0;
        inv[13] = m[0] * c3 - m[1] * c1 + m[2] * c0;
        inv[14] = -m[12] * s3 + m[13] * s1 - m[14] * s0;
        inv[15] = m[8] * s3 - m[9] * s1 + m[10] * s0;
    }
    return s0 * c5 - s1 * c4 + s2 * c3 + s3 * c2 - s4 * c1 + s5 * c0;
}

// Kabsch rotation, fast path: Horn's quaternion form of the same problem
// (max tr(R^T A) over proper rotations == the det-fixed SVD solution).  The
// largest eigenvalue of the 4x4 key matrix N of S = A^T comes from Newton on
// its characteristic quartic started above the root at sqrt(3)|S|_F (QCP);
// the quaternion is the largest-diagonal column of adj(N - lambda I).  A
// (nearly) degenerate top eigenvalue -- a reflection fit with sigma2 ~ sigma3,
// ill-posed for any method -- falls back to the Jacobi polar factor.
RTG_DEV void kabsch_rot(const float A[9], float R[9])
{
    const double Sxx = A[0], Sxy = A[3], Sxz = A[6], Syx = A[1], Syy = A[4], Syz = A[7], Szx = A[2], Szy = A[5],
                 Szz = A[8];
    const double F2 = Sxx * Sxx + Sxy * Sxy + Sxz * Sxz + Syx * Syx + Syy * Syy + Syz * Syz + Szx * Szx +
                      Szy * Szy + Szz * Szz;
    if (F2 == 0.0) {   // all-zero fit: the reference's SVD gives U = V = I
#pragma unroll
        for (int i = 0; i < 9; ++i) R[i] = (i % 4 == 0) ? 1.0f : 0.0f;
        return;
    }
    double N[16] = {Sxx + Syy + Szz, Syz - Szy, Szx - Sxz, Sxy - Syx,
                    Syz - Szy, Sxx - Syy - Szz, Sxy + Syx, Szx + Sxz,
                    Szx - Sxz, Sxy + Syx, -Sxx + Syy - Szz, Syz + Szy,
                    Sxy - Syx, Szx + Sxz, Syz + Szy, -Sxx - Syy + Szz};
    const double detS = Sxx * (Syy * Szz - Syz * Szy) - Sxy * (Syx * Szz - Syz * Szx) + Sxz * (Syx * Szy - Syy * Szx);
    double scratch[16];
    const double c0 = adj4(N, scratch, false);
    const double c2 = -2.0 * F2, c1 = -8.0 * detS;
    double lam = sqrt(3.0 * F2);
    int it = 0;
    for (; it < 50; ++it) {
        const double P = ((lam * lam + c2) * lam + c1) * lam + c0;
        const double dP = (4.0 * lam * lam + 2.0 * c2) * lam + c1;
        // the step only has to be near P/dP: v_rcp_f64's estimate keeps Newton's convergence (each step's error
        // shrinks by the estimate's ~2^-26 on top of the quadratic term) at a tenth of the IEEE divide's cost
        const double d = P * __builtin_amdgcn_rcp(dP);
        lam -= d;
        if (fabs(d) <= 1e-13 * fabs(lam)) break;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) N[i * 5] -= lam;
    double adj[16];
    adj4(N, adj, true);
    int k = 0;
    double best = fabs(adj[0]);
    if (fabs(adj[5]) > best) { best = fabs(adj[5]); k = 1; }
    if (fabs(adj[10]) > best) { best = fabs(adj[10]); k = 2; }
    if (fabs(adj[15]) > best) { best = fabs(adj[15]); k = 3; }
    if (it >= 16 || best * best <= 1e-12 * F2 * F2 * F2) {   // best <= 1e-6 |S|_F^3, without the sqrt
        kabsch_rot_jacobi(A, R);
        return;
    }
    double q[4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
        q[r] = k == 0 ? adj[r * 4] : (k == 1 ? adj[r * 4 + 1] : (k == 2 ? adj[r * 4 + 2] : adj[r * 4 + 3]));
    // R(q) of the unnormalised column: R = I + s [..] with s = 2 / |q|^2 (one divide instead of sqrt + 4 divides)
    const double w = q[0], x = q[1], y = q[2], z = q[3];
    const double s = 2.0 / (w * w + x * x + y * y + z * z);
    R[0] = (float)(1.0 - s * (y * y + z * z));
    R[1] = (float)(s * (x * y - w * z));
    R[2] = (float)(s * (x * z + w * y));
    R[3] = (float)(s * (x * y + w * z));
    R[4] = (float)(1.0 - s * (x * x + z * z));
    R[5] = (float)(s * (y * z - w * x));
    R[6] = (float)(s * (x * z - w * y));
    R[7] = (float)(s * (y * z + w * x));
    R[8] = (float)(1.0 - s * (x * x + y * y));
}

// cal_joint_quat (transform3d.py:31-50): A = M^T Z by einsum (sequential in j, no FMA)
template <int N>
RTG_DEV Q cal_joint_quat(const V (&Z)[N], const V (&M)[N])
{
    float A[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            float acc = 0.0f;
#pragma unroll
            for (int j = 0; j < N; ++j) {
                const float mi = i == 0 ? M[j].x : (i == 1 ? M[j].y : M[j].z);
                const float zk = k == 0 ? Z[j].x : (k == 1 ? Z[j].y : Z[j].z);
                const float pr = mi * zk;
                acc = j == 0 ? pr : acc + pr;
            }
            A[i * 3 + k] = acc;
        }
    float R[9];
    kabsch_rot(A, R);
    return qfrom_rotmat(R);
}

// ------------------------------------------------ scipy Rotation (float64)
// from_quat(q).as_euler(seq): quaternion method of Bernardes & Viollet (2022),
// as scipy 1.15 implements it; seq given as axis indices + intrinsic flag.
RTG_DEV void scipy_as_euler(Q qf, int s0, int s1, int s2, bool extrinsic, double ang[3])
{
    double q[4] = {(double)qf.x, (double)qf.y, (double)qf.z, (double)qf.w};
    const double nrm = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    q[0] /= nrm; q[1] /= nrm; q[2] /= nrm; q[3] /= nrm;
    int i = extrinsic ? s0 : s2, j = s1, k = extrinsic ? s2 : s0;
    const bool symmetric = i == k;
    if (symmetric) k = 3 - i - j;
    const int sign = (i - j) * (j - k) * (k - i) / 2;
    const double qi = i == 0 ? q[0] : (i == 1 ? q[1] : q[2]);
    const double qj = j == 0 ? q[0] : (j == 1 ? q[1] : q[2]);
    const double qk = k == 0 ? q[0] : (k == 1 ? q[1] : q[2]);
    double a, b, c, d;
    if (symmetric) {
        a = q[3]; b = qi; c = qj; d = qk * sign;
    } else {
        a = q[3] - qj; b = qi + qk * sign; c = qj + q[3]; d = qk * sign - qi;
    }
    ang[1] = 2.0 * ::atan2(::hypot(c, d), ::hypot(a, b));
    int kase = 0;
    if (fabs(ang[1]) <= 1e-7) kase = 1;
    else if (fabs(ang[1] - M_PI) <= 1e-7) kase = 2;
    const double half_sum = ::atan2(b, a), half_diff = ::atan2(d, c);
    if (kase == 0) {
        ang[0] = half_sum - half_diff;
        ang[2] = half_sum + half_diff;
    } else if (extrinsic) {
        ang[2] = 0.0;
        ang[0] = kase == 1 ? 2.0 * half_sum : -2.0 * half_diff;
    } else {
        ang[0] = 0.0;
        ang[2] = kase == 1 ? 2.0 * half_sum : 2.0 * half_diff;
    }
    if (!symmetric) {
        ang[2] *= sign;
        ang[1] -= M_PI / 2.0;
    }
    if (!extrinsic) { const double tt = ang[0]; ang[0] = ang[2]; ang[2] = tt; }
#pragma unroll
    for (int t = 0; t < 3; ++t) {
        if (ang[t] < -M_PI) ang[t] += 2.0 * M_PI;
        else if (ang[t] > M_PI) ang[t] -= 2.0 * M_PI;
    }
}

// from_euler(axis, angle).as_quat() for one elementary rotation, cast to float32
RTG_DEV Q elementary_quat(int axis, double angle)
{
    const double h = angle / 2.0;
    const SC t = cr_sincos(h);
    const float s = t.s, c = t.c;
    return Q{axis == 0 ? s : 0.0f, axis == 1 ? s : 0.0f, axis == 2 ? s : 0.0f, c};
}

// quat_in_xyz_axis (transform3d.py:52-59)
RTG_DEV void quat_in_xyz_axis(Q q, int s0, int s1, int s2, bool extrinsic, Q out[3])
{
    double ang[3];
    scipy_as_euler(q, s0, s1, s2, extrinsic, ang);
    out[0] = elementary_quat(s0, ang[0]);
    out[1] = elementary_quat(s1, ang[1]);
    out[2] = elementary_quat(s2, ang[2]);
}

// ------------------------------------------------ arm joint maps
// Frame-independent halves of cal_shoulderPR / cal_elbowP_and_shoulderY:
// theta0 / phi0 depend only on the zero-pose vector v0 and are evaluated once.
struct ArmZero { float th0, ph0; };

RTG_DEV ArmZero shoulder_zero(V v0)
{
    const V ex{1.f, 0.f, 0.f}, ey{0.f, 1.f, 0.f};
    const V v0p = proj_in_plane(v0, ey);
    return ArmZero{radians_between(ex, v0p, ey), radians_between(v0p, v0, cross3(v0p, ey))};
}
RTG_DEV ArmZero elbow_zero(V v0)
{
    const V ex{1.f, 0.f, 0.f}, ez{0.f, 0.f, 1.f};
    const V v0p = proj_in_plane(v0, ez);
    return ArmZero{radians_between(ex, v0p, ez), radians_between(v0p, v0, cross3(ez, v0p))};
}

// cal_shoulderPR (full_body_pos_retargeter.py:246-278)
RTG_DEV void shoulder_pr(V v1, ArmZero z0, Q parent, Q &pitch, Q &roll)
{
    const V ex{1.f, 0.f, 0.f}, ey{0.f, 1.f, 0.f};
    const V v1r = qrotate(qconj(parent), v1);
    const V v1p = proj_in_plane(v1r, ey);
    const float th1 = radians_between_axes(ex, v1p, ey);
    pitch = qfrom_angle_unit_axis(th1 - z0.th0, ey);
    const float ph1 = radians_between(v1p, v1r, cross3(v1p, ey));
    roll = qfrom_angle_unit_axis(ph1 - z0.ph0, ex);
}

// cal_elbowP_and_shoulderY (full_body_pos_retargeter.py:220-243)
RTG_DEV void elbow_py(V v1, ArmZero z0, Q parent, Q &yaw, Q &elbow)
{
    const V ex{1.f, 0.f, 0.f}, ey{0.f, 1.f, 0.f}, ez{0.f, 0.f, 1.f};
    const V v1r = qrotate(qconj(parent), v1);
    const V v1p = proj_in_plane(v1r, ez);
    const float th1 = radians_between_axes(ex, v1p, ez);
    yaw = qfrom_angle_unit_axis(th1 - z0.th0, ez);
    const float ph1 = radians_between(v1p, v1r, cross3(ez, v1p));
    elbow = qfrom_angle_unit_axis(ph1 - z0.ph0, ey);
}

// torch sum of 5 elements (cascade reduce order, measured) / 5
RTG_DEV float mean5(float v0, float v1, float v2, float v3, float v4)
{
    return ((((v0 + v4) + v1) + v2) + v3) / 5.0f;
}

// Hu_v5.Hu_DOF_AXIS (retarget/robot_config/Hu_v5.py:12-18), dof k <-> link k+1
__constant__ static const int8_t kHuDofAxis[30] = {2, 0, 1, 1, 1, 2, 0, 1, 1, 1, 2, 1, 0, 2, 1,
                                                   0, 1, 2, 1, 1, 1, 0, 2, 1, 0, 1, 2, 1, 1, 2};
__host__ __device__ constexpr int hu_dof_axis(int k)
{
    // compile-time table for unrolled uses; avoids a constant-memory load
    constexpr int8_t t[30] = {2, 0, 1, 1, 1, 2, 0, 1, 1, 1, 2, 1, 0, 2, 1,
                              0, 1, 2, 1, 1, 1, 0, 2, 1, 0, 1, 2, 1, 1, 2};
    return t[k];
}

}  // namespace rtg
