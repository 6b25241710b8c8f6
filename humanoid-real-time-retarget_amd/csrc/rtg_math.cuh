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
//  * torch.linalg.svd (MKL sgesdd) in the Kabsch fit: oneMKL 2024.2's 3x3 path
//    (SGEBD2 / SBDSQR / SORMBR with MKL's measured FMA placement), restated.
//  * scipy Rotation.as_euler / from_euler: float64 restatement.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rtg_crmath.h"
#include "rtg_knobs.h"

#pragma clang fp contract(off)

namespace rtg {

struct Q { float x, y, z, w; };
struct V { float x, y, z; };

#define RTG_DEV __device__ __forceinline__

// ---------------------------------------------------------------- helpers
RTG_DEV float ieee_sqrtf(float x) { return __builtin_sqrtf(x); }   // IEEE sqrt (correctly rounded build)
// Correctly rounded f32 sqrt in 6 instructions: v_sqrt_f64 (not accurate enough alone: it misses on 4 % of
// inputs) plus one Newton correction gives ~2^-100, and sqrt of an f32 is never within 2^-51 of an f32
// midpoint, so the single rounding is exact.  0 / inf / NaN / negative: the residual is 0 or NaN and the raw
// v_sqrt_f64 value (IEEE for those) is kept.  The rare-input path of cr_sqrt below.
RTG_DEV float cr_sqrt64(float x)
{
    const double d = (double)x;
    const double y = __builtin_amdgcn_sqrt(d);
    const double r = __builtin_fma(-y, y, d);
    const double y1 = __builtin_fma(r, 0.5 * __builtin_amdgcn_rcp(y), y);
    return (float)((r == 0.0 || r != r) ? y : y1);
}
// Correctly rounded f32 sqrt in f32 arithmetic (round 5): v_sqrt_f32 is within 1 ulp for x >= 2^-96, and of the
// candidates s - ulp, s, s + ulp the signs of the exact residuals x - (s - ulp) s and x - (s + ulp) s (one fma each)
// pick the correctly rounded one -- the sequence LLVM emits for a correctly rounded f32 sqrt.  +-0 comes out of the
// same sequence exactly (v_sqrt_f32(+-0) = +-0 and neither residual test moves it: quat_from_rotation_matrix clamps
// negative estimates to 0, so zeros are common there); x below 2^-96 (denormals, negatives) is scaled by 2^64 first
// (below; RTG_EXP_SQRT_CALL keeps the first form, cr_sqrt64 behind one rare-case branch).  No f64 instruction (cr_sqrt64:
// three f64 ops and two quarter-rate f64 transcendentals).  Proven equal to __builtin_sqrtf on all 2^32 inputs by
// tools/check_fastmath.hip [1] (run by tests/test_gpu_parity.py).
__device__ __attribute__((noinline)) float cr_sqrt64_call(float x) { return cr_sqrt64(x); }
RTG_DEV float cr_sqrt(float x)
{
#if RTG_EXP_SQRT64   // A/B knob (same values): round 4's f64 form everywhere
    return cr_sqrt64(x);
#endif
#if RTG_EXP_SQRT_CALL   // A/B knob (same values): the round-5 first form, x < 2^-96 / inf / NaN behind a call
    float s = __builtin_amdgcn_sqrtf(x);
    const float sdn = __uint_as_float(__float_as_uint(s) - 1u), sup = __uint_as_float(__float_as_uint(s) + 1u);
    const float rdn = __builtin_fmaf(-sdn, s, x), rup = __builtin_fmaf(-sup, s, x);
    s = rdn <= 0.0f ? sdn : s;
    s = rup > 0.0f ? sup : s;
    if (!(RTG_EXP_NO_RARE & 1) && __builtin_expect(!((x >= 0x1p-96f && x <= 3.40282347e38f) || x == 0.0f), 0))
        s = cr_sqrt64_call(x);
    return s;
#else
    // branch-free: x < 2^-96 (tiny and denormal positives; negatives and -0, which the scaling keeps negative / -0
    // and the sequence turns into NaN / -0) is scaled by 2^64 into the range where v_sqrt_f32 is within an ulp and
    // the result scaled back by 2^-32 (both exact: sqrt(2^-149 2^64) = 2^-42.5 and the result stays normal).  +-0,
    // inf and NaN come out of the sequence itself (v_sqrt_f32 returns them exactly; every residual test reads
    // false on them).  The branch it replaces was a call (cr_sqrt64) at each of ~150 inlined sites of the side
    // kernel: each site's call set-up and call-clobbered registers cost more than the 4 instructions here.
    const bool tiny = x < 0x1p-96f;
    const float xs = tiny ? x * 0x1p64f : x;
    float s = __builtin_amdgcn_sqrtf(xs);
    const float sdn = __uint_as_float(__float_as_uint(s) - 1u), sup = __uint_as_float(__float_as_uint(s) + 1u);
    const float rdn = __builtin_fmaf(-sdn, s, xs), rup = __builtin_fmaf(-sup, s, xs);
    s = rdn <= 0.0f ? sdn : s;
    s = rup > 0.0f ? sup : s;
    return tiny ? s * 0x1p-32f : s;
#endif
}
// Rounding test for an f64 approximation y of a value whose f32 rounding is wanted: true when the bits f32 rounding
// drops (29 of them, for an f32-normal |y|) are not within D f64 ulps of the midpoint 2^28, i.e. every value within
// D ulps of y rounds to (float)y.  An approximation with relative error <= 2^-k is within 2^(53-k) ulps.  Integer
// work only (v_and, v_sub, v_cmp).  0 and results below the f32 normal range read as not safe.
RTG_DEV bool f32_round_safe(double y, uint32_t D)
{
    const uint64_t b = (uint64_t)__double_as_longlong(y);
    const uint32_t lo = (uint32_t)b & 0x1FFFFFFFu;
    const uint32_t ex = (uint32_t)(b >> 52) & 0x7FFu;
    return ((lo - (0x10000000u - D)) > 2u * D) & (ex >= 1023u - 126u) & (ex <= 1023u + 127u);
}
RTG_DEV float acos_libm(float x) { return (float)::acos((double)x); }
// the rare-case call of cr_acos, out of line: inlined into the hot path, its registers raised the side kernel from
// 127 to 145 VGPRs (3 waves/SIMD instead of 4)
__device__ __attribute__((noinline)) float acos_libm_call(float x) { return acos_libm(x); }
// Correctly rounded f32 acos (round 5): torch.acos's value, rounded once.  acos x = pi/2 - sign(x) asin|x| for
// |x| <= 1/2 and 2 asin s (x > 0) / pi - 2 asin s (x < 0) with s = sqrt((1 - |x|) / 2) otherwise -- one instruction
// stream for both, asin s = s + s t P(t) with t = s^2 in [0, 1/4] (P: degree-9 minimax of (asin sqrt t - sqrt t) /
// t^1.5, error 2^-44 -> 2^-46 relative in asin), all in f64.  s comes from f32 seeds: s_hi = v_sqrt_f32(t), then
// s = s_hi + (t - s_hi^2) / (2 s_hi) with v_rcp_f32 (relative error <= 2^-46).  The result is within 2^-45 of acos
// x, i.e. 2^8 f64 ulps; f32_round_safe with D = 2^12 accepts it, otherwise (about 1 call in 2^16, and |x| > 1, NaN,
// x = +-1) the libm f64 acos runs behind one rare-case branch.  tools/check_fastmath.hip [6] proves it equal to
// (float)acos((double)x) for every f32 x.
RTG_DEV float acos_fast(float x, bool &ok)
{
    const float ax = __builtin_fabsf(x);
    const bool big = ax > 0.5f, neg = x < 0.0f;
    const float t32 = (1.0f - ax) * 0.5f;   // exact for ax in [1/2, 1]
    const float shi = __builtin_amdgcn_sqrtf(t32), rhi = __builtin_amdgcn_rcpf(shi);
    const double ad = (double)ax, sd = (double)shi;
    const double t = big ? (double)t32 : ad * ad;   // ad * ad is exact (24-bit operands)
    const double sb = __builtin_fma(__builtin_fma(-sd, sd, t), 0.5 * (double)rhi, sd);
    const double sv = big ? sb : ad;
    double p = 0.02812845967375316;
    p = __builtin_fma(p, t, -0.0031884549095405512);
    p = __builtin_fma(p, t, 0.0157919883306133);
    p = __builtin_fma(p, t, 0.013158578722490823);
    p = __builtin_fma(p, t, 0.01744580641234927);
    p = __builtin_fma(p, t, 0.02236569402301675);
    p = __builtin_fma(p, t, 0.03038220079156473);
    p = __builtin_fma(p, t, 0.04464285200108894);
    p = __builtin_fma(p, t, 0.07500000003992044);
    p = __builtin_fma(p, t, 0.16666666666661556);
    const double as = __builtin_fma(sv * t, p, sv);
    const double A = big ? (neg ? 3.141592653589793 : 0.0) : 1.5707963267948966;
    const double Bc = big ? (neg ? -2.0 : 2.0) : (neg ? 1.0 : -1.0);
    const double y = __builtin_fma(Bc, as, A);
    // x = +-1 (radians_between clamps its cosine to [-1, 1], so exactly parallel / antiparallel vectors give them):
    // acos is +0 / RN(pi), set here rather than through the rare-case branch
    const bool one = ax == 1.0f;
    ok = (f32_round_safe(y, 1u << 12) & (ax < 1.0f)) | one;
    return one ? (neg ? 3.14159274f : 0.0f) : (float)y;
}
RTG_DEV float cr_acos(float x)
{
#if RTG_EXP_ACOS_LIBM   // A/B knob (same values): round 4's libm f64 acos everywhere
    return acos_libm(x);
#endif
    bool ok;
    float r = acos_fast(x, ok);
    if (!(RTG_EXP_NO_RARE & 2) && __builtin_expect(!ok, 0)) r = acos_libm_call(x);
    return r;
}
RTG_DEV float cr_sin(float x) { return (float)::sin((double)x); }
RTG_DEV float cr_cos(float x) { return (float)::cos((double)x); }
// sin and cos of one argument, correctly rounded: fast shared-reduction path
// (rtg_crmath.h, exhaustively checked against glibc) with the libm f64 call as
// the exact fallback for the ~1-in-10^7 values the rounding test declines.
struct SC { float s, c; };
// the rare-case libm calls of cr_sincos, out of line (registers: see acos_libm_call)
__device__ __attribute__((noinline)) float sin_libm_call(double x) { return (float)::sin(x); }
__device__ __attribute__((noinline)) float cos_libm_call(double x) { return (float)::cos(x); }
RTG_DEV SC cr_sincos(double x)
{
    const crm::SinCos r = crm::crm_sincos(x);
    SC out{r.s, r.c};
    if (!(RTG_EXP_NO_RARE & 4) && __builtin_expect(!(r.s_ok & r.c_ok), 0)) {   // one rare-case branch for the pair
        if (!r.s_ok) out.s = sin_libm_call(x);
        if (!r.c_ok) out.c = cos_libm_call(x);
    }
    return out;
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
    const double d = (double)n;
    const double r0 = __builtin_amdgcn_rcp(d);
    const double e0 = __builtin_fma(-d, r0, 1.0);
    const double r1 = __builtin_fma(r0, e0, r0);
    const double e1 = __builtin_fma(-d, r1, 1.0);
    return Rcp{e0 == e0 ? __builtin_fma(r1, e1, r1) : r0, n};
}
// RN(a/n) == (float)((double)a * 1/n) whenever the quotient is a normal f32: an f32 quotient is never within
// 2^-50 (relative) of an f32 midpoint and the f64 product is within 2^-52.  A subnormal quotient (absolute
// grid) takes the IEEE division; that branch is rare and divergent.  tools/check_fastmath.hip: 2^32 random
// pairs + all special-value pairs, 0 mismatches.
RTG_DEV float mulr(float a, const Rcp &r)
{
    const double p = (double)a * r.r;
    float q = (float)p;
#if !RTG_EXP_MULR_NOBRANCH   // measurement knob: no subnormal-quotient branch (wrong on rare exact subnormal midpoints)
    if (__builtin_expect(__builtin_fabs(p) < 0x1p-126 && p != 0.0, 0)) q = a / r.n;
#endif
    return q;
}
// K quotients by one denominator behind ONE rare-case branch: each is (float)(a_i * 1/n) as in mulr, and if any
// product is a nonzero subnormal, every quotient of the group takes the IEEE division -- identical to separate mulr
// calls (for a normal quotient the IEEE division equals the product, by mulr's argument), one branch instead of K.
template <int K>
RTG_DEV void mulr_k(const float (&a)[K], const Rcp &r, float (&q)[K])
{
    bool sub = false;
#pragma unroll
    for (int i = 0; i < K; ++i) {
        const double p = (double)a[i] * r.r;
        q[i] = (float)p;
        sub |= (__builtin_fabs(p) < 0x1p-126) & (p != 0.0);
    }
#if !RTG_EXP_MULR_NOBRANCH
    if (!(RTG_EXP_NO_RARE & 8) && __builtin_expect(sub, 0)) {
#pragma unroll
        for (int i = 0; i < K; ++i) q[i] = a[i] / r.n;
    }
#endif
}
// the subnormal-quotient path of mulr_q, out of line (registers: see acos_libm_call); returned by value
__device__ __attribute__((noinline)) Q div_q_call(Q v, float n) { return Q{v.x / n, v.y / n, v.z / n, v.w / n}; }
RTG_DEV Q mulr_q(Q v, const Rcp &r)
{
    const double p[4] = {(double)v.x * r.r, (double)v.y * r.r, (double)v.z * r.r, (double)v.w * r.r};
    bool sub = false;
#pragma unroll
    for (int i = 0; i < 4; ++i) sub |= (__builtin_fabs(p[i]) < 0x1p-126) & (p[i] != 0.0);
    Q q{(float)p[0], (float)p[1], (float)p[2], (float)p[3]};
#if !RTG_EXP_MULR_NOBRANCH
    if (!(RTG_EXP_NO_RARE & 8) && __builtin_expect(sub, 0)) q = div_q_call(v, r.n);   // = mulr_k<4>: every quotient by IEEE division
#endif
    return q;
}
RTG_DEV V mulr_v(V v, const Rcp &r)
{
    const float a[3] = {v.x, v.y, v.z};
    float q[3];
    mulr_k<3>(a, r, q);
    return V{q[0], q[1], q[2]};
}
RTG_DEV float clamp_lo(float v, float lo) { return v < lo ? lo : v; }          // NaN passes through
// n = max(RN32(sqrt(s)), lo) and its reciprocal for mulr -- the normalisation step every quat_unit / quat_normalize /
// axis normalisation takes (clamp(norm, 1e-9), then k divisions by it).  cr_sqrt + rcp64 issue three f64
// transcendentals (v_sqrt_f64, v_rcp_f64 in the sqrt correction, v_rcp_f64 for 1/n) on the dependent chain; this
// form issues ONE (v_rsq_f64): two coupled Goldschmidt steps refine sqrt(s) and 1/(2 sqrt(s)) together, the f32
// rounding of the first gives n, and two Newton steps from 2 * the second give 1/n.  s = 0, +inf, NaN, negative
// and a clamped n take the cr_sqrt + rcp64 path (rare, divergent).  tools/check_fastmath.hip [4] checks on the
// device that (n, r) are bitwise those of the cr_sqrt + rcp64 path for every f32 s (both lo used here).
struct NormRcp {
    float n;
    Rcp r;
};
// the fast path of sqrt_clamp_rcp; `ok` false where its value must be replaced by sqrt_clamp_rcp_exact's
RTG_DEV NormRcp sqrt_clamp_rcp_fast(float s, float lo, bool &ok)
{
    const double d = (double)s;
    const double y = __builtin_amdgcn_rsq(d);
    double g = d * y, h = 0.5 * y;
    double e = __builtin_fma(-g, h, 0.5);
    g = __builtin_fma(g, e, g);
    h = __builtin_fma(h, e, h);
    e = __builtin_fma(-g, h, 0.5);
    g = __builtin_fma(g, e, g);
    h = __builtin_fma(h, e, h);
    const float n = (float)g;
    const double dn = (double)n, r0 = h + h;
    const double e0 = __builtin_fma(-dn, r0, 1.0);
    const double r1 = __builtin_fma(r0, e0, r0);
    const double e1 = __builtin_fma(-dn, r1, 1.0);
    ok = (d > 0.0) & (d < __builtin_inf()) & (n >= lo);
    return NormRcp{n, Rcp{__builtin_fma(r1, e1, r1), n}};
}
RTG_DEV NormRcp sqrt_clamp_rcp_exact(float s, float lo)
{
    const float nc = clamp_lo(cr_sqrt(s), lo);
    return NormRcp{nc, rcp64(nc)};
}
RTG_DEV NormRcp sqrt_clamp_rcp(float s, float lo)
{
    // the fast path runs unconditionally (on s <= 0 / inf / NaN its values are discarded) and ONE rare-case branch
    // takes the cr_sqrt + rcp64 path when s is not a positive finite number or n needs the clamp
    bool ok;
    NormRcp out = sqrt_clamp_rcp_fast(s, lo, ok);
    if (!(RTG_EXP_NO_RARE & 16) && __builtin_expect(!ok, 0)) out = sqrt_clamp_rcp_exact(s, lo);
    return out;
}

RTG_DEV float tsign(float v) { return v > 0.0f ? 1.0f : (v < 0.0f ? -1.0f : 0.0f); }
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
    const Rcp r = sqrt_clamp_rcp(((q.x * q.x + q.y * q.y) + q.z * q.z) + q.w * q.w, 1e-9f).r;
    return mulr_q(q, r);
}
RTG_DEV Q qmul_norm(Q a, Q b) { return qnormalize(qmul(a, b)); }
RTG_DEV float qabs(Q q) { return cr_sqrt(((q.x * q.x + q.y * q.y) + q.z * q.z) + q.w * q.w); }   // :41-47
RTG_DEV Q qunit(Q q)                                                                                 // :50-56
{
    const Rcp r = sqrt_clamp_rcp(((q.x * q.x + q.y * q.y) + q.z * q.z) + q.w * q.w, 1e-9f).r;
    return mulr_q(q, r);
}
// quat_angle_axis (:230-240): angle = acos(clamp(2 w^2 - 1)), axis = xyz / max(|xyz|, 1e-9)
RTG_DEV Q qangle_axis_abs(Q q)
{
    const float s = clamp_lohi(2.0f * (q.w * q.w) - 1.0f, -1.0f, 1.0f);
    const Rcp r = sqrt_clamp_rcp((q.x * q.x + q.y * q.y) + q.z * q.z, 1e-9f).r;
    const V ax = mulr_v(V{q.x, q.y, q.z}, r);
    return Q{cr_acos(s), ax.x, ax.y, ax.z};
}

RTG_DEV V qrotate(Q q, V v)  // :205-211, two Hamilton products
{
    const Q r = qmul(qmul(q, Q{v.x, v.y, v.z, 0.0f}), qconj(q));
    return V{r.x, r.y, r.z};
}

RTG_DEV Q qfrom_angle_axis(float angle, V axis)  // :122-143
{
    const float theta = angle / 2.0f;
    // axis.norm(p=2, dim=-1) of a 3-vector: torch's fma chain (measured: 100 % vs 90 % for the plain left fold)
    const Rcp r = sqrt_clamp_rcp(__builtin_fmaf(axis.z, axis.z, __builtin_fmaf(axis.y, axis.y, axis.x * axis.x)),
                                 1e-9f).r;
    const V u = mulr_v(axis, r);
    const float ax = u.x, ay = u.y, az = u.z;
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

// ------------------------------------------------ N-way forms of the leaf math (round 6)
// Element by element the same values as the scalar functions above (each element's fast path, and its exact path
// where that one declines), but the fast paths of all N elements run first and the whole group shares ONE rare-case
// branch.  A rare-case branch ends a basic block, and the scheduler does not move instructions across it: in the
// scalar forms two independent chains (the two arms of a frame) could not interleave, ~17 branches per arm map.
template <int N>
RTG_DEV void sqrt_clamp_rcp_n(const float (&s)[N], float lo, NormRcp (&out)[N])
{
    bool ok[N], all = true;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        out[i] = sqrt_clamp_rcp_fast(s[i], lo, ok[i]);
        all &= ok[i];
    }
    if (!(RTG_EXP_NO_RARE & 16) && __builtin_expect(!all, 0)) {
#pragma unroll
        for (int i = 0; i < N; ++i)
            if (!ok[i]) out[i] = sqrt_clamp_rcp_exact(s[i], lo);
    }
}
// v_i * 1/n_i for N vectors: mulr_v's products; a vector with a nonzero subnormal product takes IEEE divisions
// (the same quotients: mulr_k)
template <int N>
RTG_DEV void mulr_v_n(const V (&v)[N], const NormRcp (&r)[N], V (&out)[N])
{
    bool sub[N], any = false;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const double p[3] = {(double)v[i].x * r[i].r.r, (double)v[i].y * r[i].r.r, (double)v[i].z * r[i].r.r};
        out[i] = V{(float)p[0], (float)p[1], (float)p[2]};
        sub[i] = false;
#pragma unroll
        for (int k = 0; k < 3; ++k) sub[i] |= (__builtin_fabs(p[k]) < 0x1p-126) & (p[k] != 0.0);
        any |= sub[i];
    }
#if !RTG_EXP_MULR_NOBRANCH
    if (!(RTG_EXP_NO_RARE & 8) && __builtin_expect(any, 0)) {
#pragma unroll
        for (int i = 0; i < N; ++i)
            if (sub[i]) out[i] = V{v[i].x / r[i].r.n, v[i].y / r[i].r.n, v[i].z / r[i].r.n};
    }
#endif
}
template <int N>
RTG_DEV void mulr_q_n(const Q (&v)[N], const NormRcp (&r)[N], Q (&out)[N])
{
    bool sub[N], any = false;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const double p[4] = {(double)v[i].x * r[i].r.r, (double)v[i].y * r[i].r.r, (double)v[i].z * r[i].r.r,
                             (double)v[i].w * r[i].r.r};
        out[i] = Q{(float)p[0], (float)p[1], (float)p[2], (float)p[3]};
        sub[i] = false;
#pragma unroll
        for (int k = 0; k < 4; ++k) sub[i] |= (__builtin_fabs(p[k]) < 0x1p-126) & (p[k] != 0.0);
        any |= sub[i];
    }
#if !RTG_EXP_MULR_NOBRANCH
    if (!(RTG_EXP_NO_RARE & 8) && __builtin_expect(any, 0)) {
#pragma unroll
        for (int i = 0; i < N; ++i)
            if (sub[i]) out[i] = div_q_call(v[i], r[i].r.n);
    }
#endif
}
template <int N>
RTG_DEV void cr_acos_n(const float (&x)[N], float (&out)[N])
{
    bool ok[N], all = true;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        out[i] = acos_fast(x[i], ok[i]);
        all &= ok[i];
    }
    if (!(RTG_EXP_NO_RARE & 2) && __builtin_expect(!all, 0)) {
#pragma unroll
        for (int i = 0; i < N; ++i)
            if (!ok[i]) out[i] = acos_libm_call(x[i]);
    }
}
template <int N>
RTG_DEV void cr_sincos_n(const double (&x)[N], SC (&out)[N])
{
    bool sok[N], cok[N], all = true;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const crm::SinCos r = crm::crm_sincos(x[i]);
        out[i] = SC{r.s, r.c};
        sok[i] = r.s_ok;
        cok[i] = r.c_ok;
        all &= r.s_ok & r.c_ok;
    }
    if (!(RTG_EXP_NO_RARE & 4) && __builtin_expect(!all, 0)) {
#pragma unroll
        for (int i = 0; i < N; ++i) {
            if (!sok[i]) out[i].s = sin_libm_call(x[i]);
            if (!cok[i]) out[i].c = cos_libm_call(x[i]);
        }
    }
}
template <int N>
RTG_DEV void vunit_n(const V (&a)[N], V (&u)[N])   // vunit
{
    float s[N];
#pragma unroll
    for (int i = 0; i < N; ++i) s[i] = __builtin_fmaf(a[i].z, a[i].z, __builtin_fmaf(a[i].y, a[i].y, a[i].x * a[i].x));
    NormRcp r[N];
    sqrt_clamp_rcp_n<N>(s, 0.0f, r);
    mulr_v_n<N>(a, r, u);
}
template <int N>
RTG_DEV void qnormalize_n(const Q (&q0)[N], Q (&out)[N])   // qnormalize
{
    Q q[N];
    float s[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const float f = 1.0f - 2.0f * (q0[i].w < 0.0f ? 1.0f : 0.0f);
        q[i] = Q{f * q0[i].x, f * q0[i].y, f * q0[i].z, f * q0[i].w};
        s[i] = ((q[i].x * q[i].x + q[i].y * q[i].y) + q[i].z * q[i].z) + q[i].w * q[i].w;
    }
    NormRcp r[N];
    sqrt_clamp_rcp_n<N>(s, 1e-9f, r);
    mulr_q_n<N>(q, r, out);
}
// ------------------------------------------------ near-unit normalisation (round 6)
// Most quaternions the kinematics normalise are products of unit quaternions, or {e_ax sin, cos} from a correctly
// rounded pair: |q|^2 lands within a few f32 codes of 1.0f.  sqrt_clamp_rcp's (n, 1/n) for the 2K + 1 codes around
// 1.0f are a table, filled by the kernel with sqrt_clamp_rcp_exact itself (unit_tab_fill: one code per lane, while
// its loads are in flight), so a lookup returns exactly that function's values; a |q|^2 outside the table (a
// non-unit input row, NaN) takes the ordinary path.
constexpr int kUnitTabK = RTG_UNIT_TAB_K;
struct UnitEnt {
    double r;
    float n, pad;
};
RTG_DEV void unit_tab_fill(UnitEnt *tab, int t)   // t: the filling thread's index in a wave (0 .. 63)
{
    for (int e = t; e >= 0 && e <= 2 * kUnitTabK; e += 64) {
        const NormRcp n = sqrt_clamp_rcp_exact(__int_as_float(0x3F800000 - kUnitTabK + e), 1e-9f);
        tab[e] = UnitEnt{n.r.r, n.n, 0.0f};
    }
}
RTG_DEV bool unit_tab_index(float s, uint32_t &idx)
{
    idx = (uint32_t)(__float_as_int(s) - (0x3F800000 - kUnitTabK));
    const bool in = idx <= 2u * kUnitTabK;
    idx = in ? idx : 0u;
    return in;
}
// qnormalize for N quaternions through the table: the same sign flip, sum, products and subnormal test, element by
// element; the ones off the table (or with a subnormal product) take qnormalize, one rare-case branch per group
template <int N>
RTG_DEV void qnormalize_tab_n(const Q (&q0)[N], const UnitEnt *tab, Q (&out)[N])
{
    bool ok[N], all = true;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const float f = 1.0f - 2.0f * (q0[i].w < 0.0f ? 1.0f : 0.0f);
        const Q q{f * q0[i].x, f * q0[i].y, f * q0[i].z, f * q0[i].w};
        uint32_t idx;
        const bool in = unit_tab_index(((q.x * q.x + q.y * q.y) + q.z * q.z) + q.w * q.w, idx);
        const double r = tab[idx].r;
        const double p[4] = {(double)q.x * r, (double)q.y * r, (double)q.z * r, (double)q.w * r};
        bool sub = false;
#pragma unroll
        for (int k = 0; k < 4; ++k) sub |= (__builtin_fabs(p[k]) < 0x1p-126) & (p[k] != 0.0);
        out[i] = Q{(float)p[0], (float)p[1], (float)p[2], (float)p[3]};
        ok[i] = in & !sub;
        all &= ok[i];
    }
    if (__builtin_expect(!all, 0)) {
#pragma unroll
        for (int i = 0; i < N; ++i)
            if (!ok[i]) out[i] = qnormalize(q0[i]);
    }
}
// compile-time choice of the normalisation: NoTab = qnormalize itself, a table pointer = the table
struct NoTab {};
template <int N>
RTG_DEV void qnormalize_n_t(const Q (&q)[N], Q (&out)[N], NoTab) { qnormalize_n<N>(q, out); }
template <int N>
RTG_DEV void qnormalize_n_t(const Q (&q)[N], Q (&out)[N], const UnitEnt *tab) { qnormalize_tab_n<N>(q, tab, out); }
RTG_DEV Q qnormalize_t(Q q, NoTab) { return qnormalize(q); }
template <typename Tab>
RTG_DEV Q qfrom_angle_unit_axis_t(float angle, V axis, Tab tab)   // qfrom_angle_unit_axis, normalised per Tab
{
    const float theta = angle / 2.0f;
    const SC t = cr_sincos((double)theta);
    return qnormalize_t(Q{axis.x * t.s, axis.y * t.s, axis.z * t.s, t.c}, tab);
}
template <bool ON> struct TabSel {   // a table pointer where ON, NoTab elsewhere
    static RTG_DEV const UnitEnt *get(const UnitEnt *t) { return t; }
};
template <> struct TabSel<false> {
    static RTG_DEV NoTab get(const UnitEnt *) { return NoTab{}; }
};
RTG_DEV Q qnormalize_t(Q q, const UnitEnt *tab)
{
    const Q a[1] = {q};
    Q o[1];
    qnormalize_tab_n<1>(a, tab, o);
    return o[0];
}

template <int N, typename Tab = NoTab>
RTG_DEV void qfrom_angle_unit_axis_n(const float (&angle)[N], const V (&axis)[N], Q (&out)[N], Tab tab = Tab{})
{
    double th[N];
#pragma unroll
    for (int i = 0; i < N; ++i) th[i] = (double)(angle[i] / 2.0f);
    SC t[N];
    cr_sincos_n<N>(th, t);
    Q q[N];
#pragma unroll
    for (int i = 0; i < N; ++i) q[i] = Q{axis[i].x * t[i].s, axis[i].y * t[i].s, axis[i].z * t[i].s, t[i].c};
    qnormalize_n_t<N>(q, out, tab);
}

template <typename Tab = NoTab>
RTG_DEV Q qfrom_rotmat(const float m[9], Tab tab = Tab{})  // :146-193 (the four overlapping branches, in order)
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
    return qnormalize_t(Q{x, y, z, w}, tab);
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
    const V u = mulr_v(V{q.x, q.y, q.z}, r);
    return Q{mask ? angle : 0.0f, mask ? u.x : 0.0f, mask ? u.y : 0.0f, mask ? u.z : 1.0f};
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
// 6.7 MiB (4-bit codes, 8 per word in 8 MiB, measured no faster), built on the device by the exact path
// itself (ang_tab_code, k_build_ang_tab) with the same P.  qexp_component_tab thus skips acos, sincos and
// atan2f (290 of the 330 instructions of an exp-map); w outside the table or a code-0 entry takes the exact
// path.  tools/check_fastmath.hip checks qexp_component_tab == qexp_component for every f32 w.
constexpr uint32_t kAngTabLo = 0x3e800000u;                     // bits of 0.25f
constexpr uint32_t kAngTabEntries = 0x3f800000u - kAngTabLo;    // up to 1.0f (exclusive): 2^24
constexpr uint32_t kAngTabBits = 3;                             // moves -3..3
constexpr uint32_t kAngTabPer = 10u;                            // codes per 32-bit word
constexpr uint32_t kAngTabWords = (kAngTabEntries + kAngTabPer - 1) / kAngTabPer;
constexpr uint32_t kAngTabBias = 1u << (kAngTabBits - 1);      // code = move + bias; code 0 = not tabulated
RTG_DEV uint32_t ang_tab_word(uint32_t i) { return __umulhi(i, 0xCCCCCCCDu) >> 3; }   // i / 10
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
// exp_dof_tab split for a batch of read-outs that shares ONE rare-case branch (Emit::finalize): the table angle
// and whether this w needs the exact path; then exp_dof_finish.  Same operations, same values as exp_dof_tab.
struct ExpDof {
    float angle, sin_theta;
    bool mask, exact;
};
// the table word a read-out of w needs (word 0 when w is outside the table: its code is not used)
RTG_DEV uint32_t ang_tab_word_of(float w)
{
    const uint32_t i = __float_as_uint(w) - kAngTabLo;
    return i < kAngTabEntries ? ang_tab_word(i) : 0u;
}
RTG_DEV ExpDof exp_dof_word_part(float w, uint32_t word);
RTG_DEV ExpDof exp_dof_table_part(float w, const uint32_t *__restrict__ tab)
{
#if RTG_EXP_NO_TABLE
    const uint32_t word = 0x24924924u + 0u * tab[0];
#else
    const uint32_t word = tab[ang_tab_word_of(w)];
#endif
    return exp_dof_word_part(w, word);
}
// the read-out of w from its table word (loaded by the caller: exp_dof_table_part, or early into LDS, Emit::wd)
RTG_DEV ExpDof exp_dof_word_part(float w, uint32_t word)
{
    const uint32_t i = __float_as_uint(w) - kAngTabLo;
    const bool in = i < kAngTabEntries;
    const uint32_t wd = ang_tab_word(i);
#if RTG_EXP_NO_TABLE
    word = 0x24924924u;
#endif
    const float sin_theta = cr_sqrt(1.0f - w * w);
    const bool mask = fabsf(sin_theta) > 1e-5f;
    const float P = exp_angle_estimate(w);
    const uint32_t code = in ? (word >> ((i - wd * kAngTabPer) * kAngTabBits)) & ((1u << kAngTabBits) - 1u) : 0u;
    return ExpDof{__uint_as_float(__float_as_uint(P) + code - kAngTabBias), sin_theta, mask, mask && code == 0u};
}
RTG_DEV float exp_dof_finish(const ExpDof &e, float qk) { return e.mask ? e.angle * (qk / e.sin_theta) : 0.0f; }
// the exact path of one read-out whose mask holds (w outside the table or a code-0 entry), out of line
__device__ __attribute__((noinline)) float exp_dof_exact(float w, float qk)
{
    const float angle = normalize_angle(2.0f * cr_acos(w));
    return angle * (qk / cr_sqrt(1.0f - w * w));
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
    return mulr_v(a, r);
}
RTG_DEV V vmul(V a, float s) { return V{s * a.x, s * a.y, s * a.z}; }
// v / torch.linalg.norm(v): vdiv(v, lnorm3(v)) through one sqrt_clamp_rcp (lo = 0 clamps nothing)
RTG_DEV V vunit(V a)
{
    const Rcp r = sqrt_clamp_rcp(__builtin_fmaf(a.z, a.z, __builtin_fmaf(a.y, a.y, a.x * a.x)), 0.0f).r;
    return mulr_v(a, r);
}

RTG_DEV V proj_in_plane(V v, V n)  // :61-75
{
    const float nn = lnorm3(n);
    return vsub(v, vmul(n, dot3(v, n) / (nn * nn)));
}

RTG_DEV float radians_between(V v1, V v2, V n);   // :77-100 (after the N-way leaf math below)
// radians_between with v1 and n exact unit axes (the arm maps' ex / ey / ez): their normalisation is the
// identity (lnorm3 = sqrt(1) = 1, x * RN(1/1) = x), so only v2 is normalised -- the same bits, 2/3 fewer divides.
RTG_DEV float radians_between_axes(V v1, V v2, V n)
{
    v2 = vunit(v2);
    const float c = clamp_lohi(dot3(v1, v2), -1.0f, 1.0f);
    return cr_acos(c) * tsign(dot3(n, cross3(v1, v2)));
}

// ------------------------------------------------ the rest of the rotation3d / transform3d surface
// (not on the solver path; the elementwise ops 18-31 of rtg_quat_op_f32).  torch's norm(dim=-1) of a 3-vector is
// the fma chain of lnorm3, torch.sum over 4 a left fold, x**2 = x*x, atan2 on small tensors glibc's atan2f.

// exp_map_to_angle_axis (rotation3d.py:629-646) as [angle, axis]
RTG_DEV Q exp_map_angle_axis(V e)
{
    const NormRcp nr = sqrt_clamp_rcp(__builtin_fmaf(e.z, e.z, __builtin_fmaf(e.y, e.y, e.x * e.x)), 0.0f);
    const float n = nr.n;
    const Rcp r = nr.r;
    const float a = normalize_angle(n);
    const bool mask = fabsf(a) > 1e-5f;
    const V u = mulr_v(e, r);
    return Q{mask ? a : 0.0f, mask ? u.x : 0.0f, mask ? u.y : 0.0f, mask ? u.z : 1.0f};
}
// quat_slerp (transform3d.py:152-174), t per row
RTG_DEV Q qslerp(Q q0, Q q1, float t)
{
    float ch = ((q0.x * q1.x + q0.y * q1.y) + q0.z * q1.z) + q0.w * q1.w;
    if (ch < 0.0f) q1 = Q{-q1.x, -q1.y, -q1.z, -q1.w};
    ch = fabsf(ch);
    const float half = cr_acos(ch);
    const float sh = cr_sqrt(1.0f - ch * ch);
    const float ra = cr_sin((1.0f - t) * half) / sh;
    const float rb = cr_sin(t * half) / sh;
    if (fabsf(ch) >= 1.0f) return q0;
    if (fabsf(sh) < 0.001f)
        return Q{0.5f * q0.x + 0.5f * q1.x, 0.5f * q0.y + 0.5f * q1.y, 0.5f * q0.z + 0.5f * q1.z, 0.5f * q0.w + 0.5f * q1.w};
    return Q{ra * q0.x + rb * q1.x, ra * q0.y + rb * q1.y, ra * q0.z + rb * q1.z, ra * q0.w + rb * q1.w};
}
// rot_matrix_det (rotation3d.py:338-350), m row-major
RTG_DEV float rotmat_det(const float m[9])
{
    const float t1 = m[0] * (m[4] * m[8] - m[5] * m[7]);
    const float t2 = m[1] * (m[3] * m[8] - m[5] * m[6]);
    const float t3 = m[2] * (m[3] * m[7] - m[4] * m[6]);
    return (t1 - t2) + t3;
}
// rot_matrix_from_quaternion (rotation3d.py:398-427): [i, j, k, r] = [x, y, z, w], row-major out
RTG_DEV void rotmat_from_quat(Q q, float o[9])
{
    const float i = q.x, j = q.y, k = q.z, r = q.w;
    const float two_s = 2.0f / (((i * i + j * j) + k * k) + r * r);
    o[0] = 1.0f - two_s * (j * j + k * k);
    o[1] = two_s * (i * j - k * r);
    o[2] = two_s * (i * k + j * r);
    o[3] = two_s * (i * j + k * r);
    o[4] = 1.0f - two_s * (i * i + k * k);
    o[5] = two_s * (j * k - i * r);
    o[6] = two_s * (i * k - j * r);
    o[7] = two_s * (j * k + i * r);
    o[8] = 1.0f - two_s * (i * i + j * j);
}
// extract_rotation_along_axis (rotation3d.py:534-556) / the angles of project_quat_to_axis_* (:479-530)
RTG_DEV float axis_angle_of(Q q, int axis)
{
    if (axis == 0) return g_atan2f(2.0f * (q.w * q.x + q.y * q.z), 1.0f - 2.0f * (q.x * q.x + q.z * q.z));
    if (axis == 1) return g_atan2f(2.0f * (q.w * q.y + q.x * q.z), 1.0f - 2.0f * (q.y * q.y + q.z * q.z));
    return g_atan2f(2.0f * (q.w * q.z + q.x * q.y), 1.0f - 2.0f * (q.z * q.z + q.y * q.y));
}
// [sin(a/2) e_axis, cos(a/2)], unnormalised (the new_q of project_quat_to_axis_*)
RTG_DEV Q axis_half_quat(int axis, float a)
{
    const float h = a / 2.0f;
    const float s = cr_sin(h), c = cr_cos(h);
    return Q{axis == 0 ? s : 0.0f, axis == 1 ? s : 0.0f, axis == 2 ? s : 0.0f, c};
}

// ------------------------------------------------ Kabsch: torch.linalg.svd as MKL sgesdd computes it
// transform3d.py:40-45 runs torch.linalg.svd on one (1,3,3) float32 matrix, i.e. oneMKL 2024.2 SGESDD(JOBZ='A').
// For 3x3 that is SGEBD2 -> SBDSDC('U','I') -> SLASDQ -> SBDSQR -> SORMBR('Q') on U / SORMBR('P') on VT.  Each
// routine follows the published LAPACK algorithm; the FMA placement inside MKL's BLAS kernels was measured stage
// by stage against MKL's own entry points (tools/mkl_sgesdd_probe.py) and matches bit for bit.  The
// oracle (oracle/rtg_oracle.c, la_gesdd3) restates the same routines independently.  All divisions / square
// roots are IEEE-exact (fdiv = the compiler's IEEE f32 division; shared denominators rcp64 + mulr_k; cr_sqrt).  Matrices are column-major: a[r + 3 c].
RTG_DEV float fdiv(float a, float b)
{
    return a / b;   // the compiler's IEEE f32 division sequence (measured 6 % faster here than rcp64 + mulr)
}
RTG_DEV float la_sqrt(float x)
{
    return cr_sqrt(x);
}
RTG_DEV float la_sign(float a, float b) { return __builtin_copysignf(fabsf(a), b); }   // Fortran SIGN
RTG_DEV float la_lapy2(float x, float y)                                                 // SLAPY2
{
    const float xa = fabsf(x), ya = fabsf(y);
    const float w = fmaxf(xa, ya), z = fminf(xa, ya);
    const float r = fdiv(z, w);
    return z == 0.0f ? w : w * la_sqrt(1.0f + r * r);
}
// SLARFG(n, alpha, x): n = 3 (x = x0, x1) or n = 2 (x = x0); returns tau, updates alpha (= beta) and x
template <int NX>
RTG_DEV float la_larfg(float &alpha, float &x0, float &x1)
{
    const float safmin = 1.17549435e-38f / 5.96046448e-08f, rsafmn = 1.0f / safmin;
    float xn = NX == 1 ? fabsf(x0) : la_lapy2(x0, x1);
    float beta = -__builtin_copysignf(la_lapy2(alpha, xn), alpha);   // discarded when xn == 0
    int knt = 0;
    if (__builtin_expect((xn == 0.0f) | (fabsf(beta) < safmin), 0)) {   // ONE rare-case branch for both cases
        if (xn == 0.0f) return 0.0f;
        do {
            ++knt;
            x0 *= rsafmn;
            if (NX == 2) x1 *= rsafmn;
            beta *= rsafmn;
            alpha *= rsafmn;
        } while (fabsf(beta) < safmin && knt < 20);
        xn = NX == 1 ? fabsf(x0) : la_lapy2(x0, x1);
        beta = -__builtin_copysignf(la_lapy2(alpha, xn), alpha);
    }
    const float tau = fdiv(beta - alpha, beta);
    const float sc = fdiv(1.0f, alpha - beta);
    x0 *= sc;
    if (NX == 2) x1 *= sc;
    for (int j = 0; j < knt; ++j) beta *= safmin;
    alpha = beta;
    return tau;
}
RTG_DEV void la_lartg(float f, float g, float &c, float &s, float &r)   // SLARTG (LAPACK >= 3.10)
{
    const float safmin = 1.17549435e-38f, safmax = 1.0f / safmin;
    const float rtmin = 1.08420217e-19f, rtmax = 1.30438176e+19f;   // sqrt(safmin), sqrt(safmax / 2)
    const float f1 = fabsf(f), g1 = fabsf(g);
    // the common case (f, g nonzero and in range) runs unconditionally; the other three cases of SLARTG redo the
    // outputs behind ONE rare-case branch -- the same operations per case as the reference's cascade
    {
        const float d = la_sqrt(f * f + g * g);
#if RTG_EXP_LARTG_RCP64   // A/B knob (round 5): the two quotients through rcp64 + mulr_k<2> (same values)
        const Rcp rd = rcp64(d);
        const float num[2] = {f1, g};
        float quo[2];
        mulr_k<2>(num, rd, quo);
#else
        const float quo[2] = {fdiv(f1, d), fdiv(g, d)};
#endif
        c = quo[0];
        r = __builtin_copysignf(d, f);
        s = f < 0.0f ? -quo[1] : quo[1];   // g / r with r = +-d (RN is sign-symmetric)
    }
    if (__builtin_expect(!((g != 0.0f) & (f != 0.0f) & (f1 > rtmin) & (f1 < rtmax) & (g1 > rtmin) & (g1 < rtmax)), 0)) {
        if (g == 0.0f) { c = 1.0f; s = 0.0f; r = f; }
        else if (f == 0.0f) { c = 0.0f; s = __builtin_copysignf(1.0f, g); r = g1; }
        else {
            const float u = fminf(safmax, fmaxf(safmin, fmaxf(f1, g1)));
            const float fs = fdiv(f, u), gs = fdiv(g, u), d = la_sqrt(fs * fs + gs * gs);
            c = fdiv(fabsf(fs), d);
            r = __builtin_copysignf(d, f);
            s = fdiv(gs, r);
            r *= u;
        }
    }
}
RTG_DEV float la_las2_min(float f, float g, float h)   // SLAS2, SSMIN only (the shift)
{
    const float fa = fabsf(f), ga = fabsf(g), ha = fabsf(h);
    const float fhmn = fminf(fa, ha), fhmx = fmaxf(fa, ha);
    if (fhmn == 0.0f) return 0.0f;
    if (ga < fhmx) {
        const float as = 1.0f + fdiv(fhmn, fhmx), at = fdiv(fhmx - fhmn, fhmx);
        float au = fdiv(ga, fhmx);
        au = au * au;
        const float c = fdiv(2.0f, la_sqrt(as * as + au) + la_sqrt(at * at + au));
        return fhmn * c;
    }
    const float au = fdiv(fhmx, ga);
    if (au == 0.0f) return fdiv(fhmn * fhmx, ga);
    const float as = 1.0f + fdiv(fhmn, fhmx), at = fdiv(fhmx - fhmn, fhmx), p = as * au, q = at * au;
    const float c = fdiv(1.0f, la_sqrt(1.0f + p * p) + la_sqrt(1.0f + q * q));
    const float mn = (fhmn * c) * au;
    return mn + mn;
}
// SLASV2
RTG_DEV void la_lasv2(float f, float g, float h, float &ssmin, float &ssmax, float &snr, float &csr, float &snl,
                      float &csl)
{
    const float eps = 5.96046448e-08f;
    float ft = f, fa = fabsf(ft), ht = h, ha = fabsf(h), gt = g;
    float clt = 1.0f, crt = 1.0f, slt = 0.0f, srt = 0.0f;
    int pmax = 1;
    const bool swap = ha > fa;
    if (swap) { pmax = 3; float t = ft; ft = ht; ht = t; t = fa; fa = ha; ha = t; }
    const float ga = fabsf(gt);
    if (ga == 0.0f) { ssmin = ha; ssmax = fa; }
    else {
        bool gasmal = true;
        if (ga > fa) {
            pmax = 2;
            if (fdiv(fa, ga) < eps) {
                gasmal = false;
                ssmax = ga;
                ssmin = ha > 1.0f ? fdiv(fa, fdiv(ga, ha)) : fdiv(fa, ga) * ha;
                clt = 1.0f; slt = fdiv(ht, gt); srt = 1.0f; crt = fdiv(ft, gt);
            }
        }
        if (gasmal) {
            const float d = fa - ha, l = d == fa ? 1.0f : fdiv(d, fa);
            const float m = fdiv(gt, ft), mm = m * m;
            float t = 2.0f - l;
            const float tt = t * t;
            const float s = la_sqrt(tt + mm);
            const float r = l == 0.0f ? fabsf(m) : la_sqrt(l * l + mm);
            const float a = 0.5f * (s + r);
            ssmin = fdiv(ha, a);
            ssmax = fa * a;
            if (mm == 0.0f) t = l == 0.0f ? la_sign(2.0f, ft) * la_sign(1.0f, gt) : fdiv(gt, la_sign(d, ft)) + fdiv(m, t);
            else t = (fdiv(m, s + t) + fdiv(m, r + l)) * (1.0f + a);
            const float l2 = la_sqrt(t * t + 4.0f);
#if RTG_EXP_LARTG_RCP64
            const Rcp rl = rcp64(l2);
            {
                const float num[2] = {2.0f, t};
                float quo[2];
                mulr_k<2>(num, rl, quo);
                crt = quo[0];
                srt = quo[1];
            }
            const Rcp ra = rcp64(a);
            const float num[2] = {crt + srt * m, fdiv(ht, ft) * srt};
            float quo[2];
            mulr_k<2>(num, ra, quo);
            clt = quo[0];
            slt = quo[1];
#else
            crt = fdiv(2.0f, l2);
            srt = fdiv(t, l2);
            clt = fdiv(crt + srt * m, a);
            slt = fdiv(fdiv(ht, ft) * srt, a);
#endif
        }
    }
    if (swap) { csl = srt; snl = crt; csr = slt; snr = clt; }
    else { csl = clt; snl = slt; csr = crt; snr = srt; }
    const float tsg = pmax == 1 ? la_sign(1.0f, csr) * la_sign(1.0f, csl) * la_sign(1.0f, f)
                    : pmax == 2 ? la_sign(1.0f, snr) * la_sign(1.0f, csl) * la_sign(1.0f, g)
                                : la_sign(1.0f, snr) * la_sign(1.0f, snl) * la_sign(1.0f, h);
    ssmax = la_sign(ssmax, tsg);
    ssmin = la_sign(ssmin, tsg * la_sign(1.0f, f) * la_sign(1.0f, h));
}
RTG_DEV void la_rot(float &x, float &y, float c, float s)   // MKL's SROT / SLASR pair update
{
    const float xv = x, yv = y;
    x = __builtin_fmaf(s, yv, c * xv);
    y = __builtin_fmaf(c, yv, -(s * xv));
}
struct Svd3 { float u[9], vt[9]; };
// rotate VT rows (p, p+1) / U columns (p, p+1), p = p1 ? 1 : 0 chosen per lane by selects (no divergence)
RTG_DEV void vt_rot(Svd3 &z, bool p1, float c, float s)
{
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        float x = p1 ? z.vt[1 + 3 * k] : z.vt[3 * k], y = p1 ? z.vt[2 + 3 * k] : z.vt[1 + 3 * k];
        la_rot(x, y, c, s);
        z.vt[3 * k] = p1 ? z.vt[3 * k] : x;
        z.vt[1 + 3 * k] = p1 ? x : y;
        z.vt[2 + 3 * k] = p1 ? y : z.vt[2 + 3 * k];
    }
}
RTG_DEV void u_rot(Svd3 &z, bool p1, float c, float s)
{
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        float x = p1 ? z.u[k + 3] : z.u[k], y = p1 ? z.u[k + 6] : z.u[k + 3];
        la_rot(x, y, c, s);
        z.u[k] = p1 ? z.u[k] : x;
        z.u[k + 3] = p1 ? x : y;
        z.u[k + 6] = p1 ? y : z.u[k + 6];
    }
}
// SBDSQR('U', 3, ncvt = 3, nru = 3, ncc = 0) from U = VT = I (SBDSDC / SLASDQ), n = 3 specialised: the only
// multi-element block is (ll, m) = (1, 3); every other case ends in one 2x2 SLASV2 block.  A bottom-to-top
// chase (IDIR = 2) is the top-to-bottom chase (IDIR = 1) of the reversed bidiagonal (d3, d2, d1; e2, e1) -- the
// same scalar recurrences, with the rotations applied to the mirrored row / column pairs and negated sines
// (SBDSQR :130/:150 store -SN) -- so both directions run one code path and a wave never executes both.
RTG_DEV void la_bdsqr3(float &d1, float &d2, float &d3, float e1, float e2, Svd3 &z)
{
    const float eps = 5.96046448e-08f, tol = 10.0f * eps, unfl = 1.17549435e-38f;
    float sminoa = fabsf(d1);
    if (sminoa != 0.0f) {
        float mu = fabsf(d2) * fdiv(sminoa, sminoa + fabsf(e1));
        sminoa = fminf(sminoa, mu);
        if (sminoa != 0.0f) {
            mu = fabsf(d3) * fdiv(mu, mu + fabsf(e2));
            sminoa = fminf(sminoa, mu);
        }
    }
    sminoa = fdiv(sminoa, 1.73205078f);   // / sqrt(real(3))
    const float thresh = fmaxf(tol * sminoa, 6.0f * (3.0f * (3.0f * unfl)));
    int m = 3, iter = -1, iterdivn = 0;
    bool mir = false, fresh = true;   // mir: IDIR = 2; fresh: (ll, m) = (1, 3) differs from (oldll, oldm)
    // A lane whose last step is a 2x2 block leaves the loop with blk set, and the block (SLASV2 + its two
    // rotations) runs once after the loop for every such lane: the lanes of a wave finish at different sweeps,
    // and inside the loop the block would execute once per distinct exit sweep.  Same operations, same values.
    bool blk = false, p1 = false;
    for (;;) {
        if (m <= 1) break;
        if (iter >= 3) { iter -= 3; if (++iterdivn >= 18) break; }   // no convergence: INFO > 0 (never seen)
        if (m == 2) {                       // block (1, 2)
            if (fabsf(e1) <= thresh) break;
            blk = true;
            break;
        }
        if (fabsf(e2) <= thresh) { e2 = 0.0f; m = 2; continue; }
        if (fabsf(e1) <= thresh) { e1 = 0.0f; blk = true; p1 = true; break; }   // split at E(1): block (2, 3)
        const float smax = fmaxf(fmaxf(fabsf(d3), fmaxf(fabsf(d2), fabsf(e2))), fmaxf(fabsf(d1), fabsf(e1)));
        if (fresh) { mir = !(fabsf(d1) >= fabsf(d3)); fresh = false; }
        // the IDIR = 1 form on (D1, D2, D3; E1, E2) = mir ? (d3, d2, d1; e2, e1) : (d1, d2, d3; e1, e2)
        float D1 = mir ? d3 : d1, D2 = d2, D3 = mir ? d1 : d3, E1 = mir ? e2 : e1, E2 = mir ? e1 : e2;
        bool zeroed = false;
        float smin;
        if (fabsf(E2) <= fabsf(tol) * fabsf(D3)) { E2 = 0.0f; zeroed = true; }
        else {
            float mu = fabsf(D1);
            smin = mu;
            if (fabsf(E1) <= tol * mu) { E1 = 0.0f; zeroed = true; }
            else {
                mu = fabsf(D2) * fdiv(mu, mu + fabsf(E1));
                smin = fminf(smin, mu);
                if (fabsf(E2) <= tol * mu) { E2 = 0.0f; zeroed = true; }
                else {
                    mu = fabsf(D3) * fdiv(mu, mu + fabsf(E2));
                    smin = fminf(smin, mu);
                }
            }
        }
        if (zeroed) {
            e1 = mir ? E2 : E1;
            e2 = mir ? E1 : E2;
            continue;
        }
        float shift = 0.0f;
        if (!((3.0f * tol) * fdiv(smin, smax) <= fmaxf(eps, 0.01f * tol))) {
            const float sll = fabsf(D1);
            shift = la_las2_min(D2, E2, D3);
            if (sll > 0.0f) { const float q = fdiv(shift, sll); if (q * q < eps) shift = 0.0f; }
        }
        iter += 2;
        // rotations of the two steps: (ac, as) / (bc, bs) at the first, (cc, cs) / (dc, ds) at the second
        float ac, as, bc, bs, cc, cs, dc, ds;
        if (shift == 0.0f) {
            float r, h;
            la_lartg(D1, E1, ac, as, r);                 // cs = 1
            la_lartg(r, D2 * as, bc, bs, D1);            // oldcs = 1
            la_lartg(D2 * ac, E2, cc, cs, r);
            E1 = bs * r;
            la_lartg(bc * r, D3 * cs, dc, ds, D2);
            h = D3 * cc;
            D3 = h * dc;
            E2 = h * ds;
        } else {
            float f = (fabsf(D1) - shift) * (__builtin_copysignf(1.0f, D1) + fdiv(shift, D1)), g = E1, r;
            la_lartg(f, g, ac, as, r);
            f = ac * D1 + as * E1;
            E1 = ac * E1 - as * D1;
            g = as * D2;
            D2 = ac * D2;
            la_lartg(f, g, bc, bs, r);
            D1 = r;
            f = bc * E1 + bs * D2;
            D2 = bc * D2 - bs * E1;
            g = bs * E2;
            E2 = bc * E2;
            la_lartg(f, g, cc, cs, r);
            E1 = r;
            f = cc * D2 + cs * E2;
            E2 = cc * E2 - cs * D2;
            g = cs * D3;
            D3 = cc * D3;
            la_lartg(f, g, dc, ds, r);
            D2 = r;
            f = dc * E2 + ds * D3;
            D3 = dc * D3 - ds * E2;
            E2 = f;
        }
        if (fabsf(E2) <= thresh) E2 = 0.0f;
        d1 = mir ? D3 : D1; d2 = D2; d3 = mir ? D1 : D3;
        e1 = mir ? E2 : E1; e2 = mir ? E1 : E2;
        // IDIR = 1: VT pairs (1,2) then (2,3) by (a, c), U by (b, d).  IDIR = 2: VT (2,3) then (1,2) by (b, d),
        // U by (a, c), sines negated.
        vt_rot(z, mir, mir ? bc : ac, mir ? -bs : as);
        vt_rot(z, !mir, mir ? dc : cc, mir ? -ds : cs);
        u_rot(z, mir, mir ? ac : bc, mir ? -as : bs);
        u_rot(z, !mir, mir ? cc : dc, mir ? -cs : ds);
    }
    if (blk) {   // 2x2 block (p1 ? 2 : 1, +1)
        float sigmn, sigmx, sinr, cosr, sinl, cosl;
        la_lasv2(p1 ? d2 : d1, p1 ? e2 : e1, p1 ? d3 : d2, sigmn, sigmx, sinr, cosr, sinl, cosl);
        d1 = p1 ? d1 : sigmx;
        d2 = p1 ? sigmx : sigmn;
        d3 = p1 ? sigmn : d3;
        vt_rot(z, p1, cosr, sinr);
        u_rot(z, p1, cosl, sinl);
    }
    // singular values made positive (VT rows negated), then sorted decreasing (SBDSQR :160-190)
    if (d1 < 0.0f) { d1 = -d1; z.vt[0] = -z.vt[0]; z.vt[3] = -z.vt[3]; z.vt[6] = -z.vt[6]; }
    if (d2 < 0.0f) { d2 = -d2; z.vt[1] = -z.vt[1]; z.vt[4] = -z.vt[4]; z.vt[7] = -z.vt[7]; }
    if (d3 < 0.0f) { d3 = -d3; z.vt[2] = -z.vt[2]; z.vt[5] = -z.vt[5]; z.vt[8] = -z.vt[8]; }
    // pass 1: smallest of (d1, d2, d3), ties to the later index, moves to position 3
    {
        int isub = 1;
        float mn = d1;
        if (d2 <= mn) { isub = 2; mn = d2; }
        if (d3 <= mn) { isub = 3; mn = d3; }
        const bool s1 = isub == 1, s2 = isub == 2;
        d1 = s1 ? d3 : d1;
        d2 = s2 ? d3 : d2;
        d3 = mn;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float v0 = z.vt[3 * k], v1 = z.vt[1 + 3 * k], v2 = z.vt[2 + 3 * k];
            z.vt[3 * k] = s1 ? v2 : v0;
            z.vt[1 + 3 * k] = s2 ? v2 : v1;
            z.vt[2 + 3 * k] = s1 ? v0 : (s2 ? v1 : v2);
            const float u0 = z.u[k], u1 = z.u[k + 3], u2 = z.u[k + 6];
            z.u[k] = s1 ? u2 : u0;
            z.u[k + 3] = s2 ? u2 : u1;
            z.u[k + 6] = s1 ? u0 : (s2 ? u1 : u2);
        }
    }
    // pass 2: smaller of (d1, d2), ties to d2, moves to position 2
    {
        const bool sw = !(d2 <= d1);
        const float t0 = d1;
        d1 = sw ? d2 : d1;
        d2 = sw ? t0 : d2;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float v0 = z.vt[3 * k], v1 = z.vt[1 + 3 * k];
            z.vt[3 * k] = sw ? v1 : v0;
            z.vt[1 + 3 * k] = sw ? v0 : v1;
            const float u0 = z.u[k], u1 = z.u[k + 3];
            z.u[k] = sw ? u1 : u0;
            z.u[k + 3] = sw ? u0 : u1;
        }
    }
}
// Stage marks for the timestamp measurement builds (RTG_EXP_TIMESTAMPS): hook(k) at a stage boundary, a no-op otherwise.
// cal_joint_quat: 0 A formed, 1 rotation done; la_gesdd3: 10 bidiagonal form (SGEBD2) done, 11 SBDSQR done.
struct NoHook {
    RTG_DEV void operator()(int) const {}
};
// SGESDD(JOBZ='A') of a 3x3 (column-major a, overwritten): U and VT (column-major) in z
template <typename Hook = NoHook>
RTG_DEV void la_gesdd3(float a[9], Svd3 &z, const Hook &hook = Hook{})
{
    const float smlnum = 9.09494702e-13f, bignum = 1.0f / smlnum;   // sqrt(slamch('S')) / slamch('P') = 2^-40
    float anrm = 0.0f;
#pragma unroll
    for (int i = 0; i < 9; ++i) anrm = fmaxf(anrm, fabsf(a[i]));
    if (__builtin_expect((anrm > 0.0f && anrm < smlnum) || anrm > bignum, 0)) {
        const float mul = anrm < smlnum ? fdiv(smlnum, anrm) : fdiv(bignum, anrm);
#pragma unroll
        for (int i = 0; i < 9; ++i) a[i] *= mul;
    }
    // SGEBD2, i = 0: H_0 from the left (v = (1, a1, a2)), G_0 from the right (v = (1, a6))
    const float tq0 = la_larfg<2>(a[0], a[1], a[2]);
    const float d1 = a[0];
    if (tq0 != 0.0f) {
#pragma unroll
        for (int j = 1; j < 3; ++j) {
            const float w = a[3 * j] + (a[1 + 3 * j] * a[1] + a[2 + 3 * j] * a[2]);
            const float tw = -(tq0 * w);
            a[3 * j] = __builtin_fmaf(1.0f, tw, a[3 * j]);
            a[1 + 3 * j] = __builtin_fmaf(a[1], tw, a[1 + 3 * j]);
            a[2 + 3 * j] = __builtin_fmaf(a[2], tw, a[2 + 3 * j]);
        }
    }
    float dum = 0.0f;
    const float tp0 = la_larfg<1>(a[3], a[6], dum);
    const float e1 = a[3];
    if (tp0 != 0.0f) {
        const float tv1 = -(tp0 * 1.0f), tv2 = -(tp0 * a[6]);
#pragma unroll
        for (int r = 1; r < 3; ++r) {
            const float w = __builtin_fmaf(a[r + 6], a[6], a[r + 3]);
            a[r + 3] = __builtin_fmaf(w, tv1, a[r + 3]);
            a[r + 6] = __builtin_fmaf(w, tv2, a[r + 6]);
        }
    }
    // i = 1: H_1 from the left (v = (1, a5)) on column 2; G_1 = I (one-element reflector)
    const float tq1 = la_larfg<1>(a[4], a[5], dum);
    const float d2 = a[4];
    if (tq1 != 0.0f) {
        const float w = a[7] + a[8] * a[5];
        const float tw = -(tq1 * w);
        a[7] = __builtin_fmaf(1.0f, tw, a[7]);
        a[8] = __builtin_fmaf(a[5], tw, a[8]);
    }
    const float e2 = a[7];
    const float d3 = a[8];   // i = 2: H_2 = I
    hook(10);
    // SBDSDC('U','I') -> SLASDQ -> SBDSQR with U = VT = I
#pragma unroll
    for (int i = 0; i < 9; ++i) { z.u[i] = (i % 4 == 0) ? 1.0f : 0.0f; z.vt[i] = z.u[i]; }
    float s1 = d1, s2 = d2, s3 = d3;
    la_bdsqr3(s1, s2, s3, e1, e2, z);
    hook(11);
    // SORMBR('Q','L','N'): U := H_0 H_1 U (H_1 first), the unit row fused as fma(-tau, w, c)
    if (tq1 != 0.0f) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const float w = z.u[1 + 3 * j] + z.u[2 + 3 * j] * a[5];
            const float tw = -(tq1 * w);
            z.u[1 + 3 * j] = __builtin_fmaf(-tq1, w, z.u[1 + 3 * j]);
            z.u[2 + 3 * j] = __builtin_fmaf(a[5], tw, z.u[2 + 3 * j]);
        }
    }
    if (tq0 != 0.0f) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const float w = z.u[3 * j] + (z.u[1 + 3 * j] * a[1] + z.u[2 + 3 * j] * a[2]);
            const float tw = -(tq0 * w);
            z.u[3 * j] = __builtin_fmaf(-tq0, w, z.u[3 * j]);
            z.u[1 + 3 * j] = __builtin_fmaf(a[1], tw, z.u[1 + 3 * j]);
            z.u[2 + 3 * j] = __builtin_fmaf(a[2], tw, z.u[2 + 3 * j]);
        }
    }
    // SORMBR('P','R','T'): VT := VT G_0^T on columns 1..2
    if (tp0 != 0.0f) {
        const float tv1 = -(tp0 * 1.0f), tv2 = -(tp0 * a[6]);
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            const float w = __builtin_fmaf(z.vt[r + 6], a[6], z.vt[r + 3]);
            z.vt[r + 3] = __builtin_fmaf(w, tv1, z.vt[r + 3]);
            z.vt[r + 6] = __builtin_fmaf(w, tv2, z.vt[r + 6]);
        }
    }
}
// transform3d.py:40-45: R = U Vt ((p0 + p1) + p2, torch's bmm order); det(R) < 0 -> Vt[-1,:] *= -1; R = U Vt.
// A and R row-major.  det only decides a sign (|det| = 1 up to rounding), taken in float64.
template <typename Hook = NoHook>
RTG_DEV void kabsch_rot(const float A[9], float R[9], const Hook &hook = Hook{})
{
#if RTG_EXP_STUB_SVD
#pragma unroll
    for (int i = 0; i < 9; ++i) R[i] = (i % 4 == 0) ? 1.0f : A[i] * 1e-3f;
    return;
#endif
    float a[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int k = 0; k < 3; ++k) a[i + 3 * k] = A[i * 3 + k];
    Svd3 z;
    la_gesdd3(a, z, hook);
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int k = 0; k < 3; ++k)
            R[i * 3 + k] = (z.u[i] * z.vt[3 * k] + z.u[i + 3] * z.vt[1 + 3 * k]) + z.u[i + 6] * z.vt[2 + 3 * k];
    // R = U Vt is orthogonal to ~1e-6 (U and Vt are products of plane rotations and reflectors) or all NaN, so
    // |det R| = 1 +- 1e-6 and the sign any f32 evaluation gives is torch.linalg.det's (the oracle keeps f64)
    const float det = R[0] * (R[4] * R[8] - R[5] * R[7]) - R[1] * (R[3] * R[8] - R[5] * R[6]) +
                      R[2] * (R[3] * R[7] - R[4] * R[6]);
    if (det < 0.0f) {
#pragma unroll
        for (int k = 0; k < 3; ++k) z.vt[2 + 3 * k] = -z.vt[2 + 3 * k];
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int k = 0; k < 3; ++k)
                R[i * 3 + k] = (z.u[i] * z.vt[3 * k] + z.u[i + 3] * z.vt[1 + 3 * k]) + z.u[i + 6] * z.vt[2 + 3 * k];
    }
}

// cal_joint_quat (transform3d.py:31-50): A = M^T Z by einsum (sequential in j, no FMA).  `hook(k)` marks the
// stages (NoHook above) for the latency-phase measurement knob; a no-op otherwise.
// `svd_nan` is set when A has a NaN entry: torch.linalg.svd refuses such a matrix (LAPACK sgesdd returns info = -4
// on a NaN norm and torch raises "linalg.svd: ... contained non-finite values", transform3d.py:40), so the reference
// frame raises there (an inf entry alone does not raise).
// A = M^T Z (torch.matmul's summation order, measured) and whether it holds a NaN
template <int N>
RTG_DEV bool form_joint_A(const V (&Z)[N], const V (&M)[N], float (&A)[9])
{
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
    bool nan = false;
#pragma unroll
    for (int i = 0; i < 9; ++i) nan |= A[i] != A[i];
    return nan;
}
// the rotation of a formed A: Kabsch then quat_from_rotation_matrix
template <typename Hook = NoHook, typename Tab = NoTab>
RTG_DEV Q joint_quat_of_A(const float (&A)[9], const Hook &hook = Hook{}, Tab tab = Tab{})
{
    hook(0);
    float R[9];
    kabsch_rot(A, R, hook);
    hook(1);
    return qfrom_rotmat(R, tab);
}
template <int N, typename Hook = NoHook, typename Tab = NoTab>
RTG_DEV Q cal_joint_quat(const V (&Z)[N], const V (&M)[N], bool &svd_nan, const Hook &hook = Hook{}, Tab tab = Tab{})
{
    float A[9];
    svd_nan = form_joint_A<N>(Z, M, A);
    return joint_quat_of_A(A, hook, tab);
}
template <int N, typename Hook = NoHook>
RTG_DEV Q cal_joint_quat(const V (&Z)[N], const V (&M)[N], const Hook &hook = Hook{})
{
    bool unused;
    return cal_joint_quat<N>(Z, M, unused, hook);
}

// ------------------------------------------------ scipy Rotation (float64)
// from_quat(q).as_euler(seq): quaternion method of Bernardes & Viollet (2022),
// as scipy 1.15 implements it; seq given as axis indices + intrinsic flag.  Returns true when from_quat would
// refuse q: its float64 norm is not > 0 (all four components zero, or a NaN) -- scipy raises
// "ValueError: Found zero norm quaternions in `quat`." there (transform3d.py:53).
RTG_DEV bool scipy_as_euler(Q qf, int s0, int s1, int s2, bool extrinsic, double ang[3])
{
    double q[4] = {(double)qf.x, (double)qf.y, (double)qf.z, (double)qf.w};
    const double nrm = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    const bool refused = !(nrm > 0.0);
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
    return refused;
}

// from_euler(axis, angle).as_quat() for one elementary rotation, cast to float32
RTG_DEV Q elementary_quat(int axis, double angle)
{
    const double h = angle / 2.0;
    const SC t = cr_sincos(h);
    const float s = t.s, c = t.c;
    return Q{axis == 0 ? s : 0.0f, axis == 1 ? s : 0.0f, axis == 2 ? s : 0.0f, c};
}

// ---- the 'XYZ' split of the solvers without atan2 (round 5)
// scipy's as_euler('XYZ') (intrinsic; scipy_as_euler with i = 2, j = 1, k = 0, sign -1) of q = (x, y, z, w) gives,
// with a = w - y, b = z - x, c = w + y, d = -(x + z) and hs = atan2(b, a), hd = atan2(d, c):
//   X: -(hs + hd)   Y: 2 atan2(|c + id|, |a + ib|) - pi/2   Z: hs - hd,   each wrapped into [-pi, pi]
// and each elementary quaternion is (sin A/2, cos A/2).  Every A is the principal argument of a complex number whose
// half angle needs no trigonometry:  e^{-i(hs + hd)} ~ conj((a + ib)(c + id)) = (ac - bd) - i(ad + bc);
// e^{i(hs - hd)} ~ (a + ib)(c - id) = (ac + bd) + i(bc - ad);  and e^{i A_Y} ~ m + 2i(yw + xz) with
// m = |a + ib| |c + id| (the modulus of the other two; n2 = |q|^2 is this one's).  For z = re + i im of modulus M,
// u = M + |re| (no cancellation) and t = 1 / sqrt(2 M u):  re >= 0: (sin, cos)(A/2) = (im t, u t);
// re < 0: (sign(im) u t, |im| t).  The products of the exact f64 differences a..d are single-rounded (fma), so every
// output is within 2^-48 of its value; the reference's own f64 pipeline (normalise, hypot, atan2, the angle sums,
// the wrap, sin / cos) is within ~2^-50 (1 + 1/|a + ib| + 1/|c + id|) |q| absolute.  An output is accepted when its
// f32 rounding is the same at +-2^-49 (1 + ...) -- the first version, with a fixed 2^-47, differed from the
// restatement on 5,892 of 2^30 near-gimbal quaternions (check [7]); otherwise -- and for n2 not > 0 (scipy
// refuses), NaN / inf, the gimbal cases (m < 1e-6 n2:
// scipy's 1e-7 tests), the wrap boundary (re < 0 with |im| < 2^-30 M) and im == 0 -- the scipy restatement below runs
// (quat_in_xyz_axis).  tools/check_fastmath.hip [7] compares the two on 2^30 quaternions.
RTG_DEV double rsq_nr(double v)   // 1 / sqrt(v), v > 0 finite: v_rsq_f64 (2^-23) and two Newton steps
{
    double r = __builtin_amdgcn_rsq(v);
    const double h = 0.5 * v;
    r = r * __builtin_fma(-h * r, r, 1.5);
    r = r * __builtin_fma(-h * r, r, 1.5);
    return r;
}
RTG_DEV bool f32_round_abs_safe(double y, double E, float &out)   // every value within E of y rounds alike
{
    out = (float)y;
    return (float)(y - E) == (float)(y + E);
}
// (sin, cos) of half the principal argument of re + i im (modulus M > 0), given t = 1 / sqrt(2 M u) with
// u = M + |re|; false when the rounding test at +-E or the wrap boundary declines
RTG_DEV bool half_arg(double re, double im, double M, double u, double t, double E, float &s, float &c)
{
    const double P = u * t, Qv = im * t;
    const bool pos = re >= 0.0;
    const double sv = pos ? Qv : __builtin_copysign(P, im), cv = pos ? P : __builtin_fabs(Qv);
    bool ok = f32_round_abs_safe(sv, E, s);
    ok = f32_round_abs_safe(cv, E, c) && ok;
    return ok && im != 0.0 && (pos || __builtin_fabs(im) >= 0x1p-30 * M);
}
RTG_DEV bool quat_in_xyz_fast(Q qf, Q out[3])
{
    const double X = qf.x, Y = qf.y, Z = qf.z, W = qf.w;
    const double a = W - Y, b = Z - X, c = W + Y, d = -(X + Z);   // exact: f32 operands
    const double n2 = __builtin_fma(W, W, __builtin_fma(Z, Z, __builtin_fma(Y, Y, X * X)));
    const double rab2 = __builtin_fma(b, b, a * a), rcd2 = __builtin_fma(d, d, c * c);
    const double m2 = rab2 * rcd2;
    const double m = m2 * rsq_nr(m2);
    const double bd = b * d, ad = a * d, bc = b * c;
    // Y: re = m, im = 2 (yw + xz), modulus n2
    const double u1 = n2 + m, t1 = rsq_nr(2.0 * n2 * u1);
    // The reference's a..d carry ~2^-52 |q| of rounding (its normalised q), which its atan2 of (b, a) / (d, c)
    // amplifies by |q| / |a + ib| and |q| / |c + id|: near gimbal lock the margin widens with
    // 1 / |a + ib| + 1 / |c + id| = sqrt(2 n2 u1) / m = 1 / (t1 m)
    const double E = 0x1p-49 * (1.0 + __builtin_amdgcn_rcp(t1 * m));
    float sx, cx, sy, cy, sz, cz;
    bool ok = n2 > 0.0 && n2 < 0x1p1000 && m >= 1e-6 * n2;
    ok = half_arg(m, 2.0 * __builtin_fma(Y, W, X * Z), n2, u1, t1, E, sy, cy) && ok;
    const double re0 = __builtin_fma(a, c, -bd), re2 = __builtin_fma(a, c, bd);
    const double u0 = m + __builtin_fabs(re0), u2 = m + __builtin_fabs(re2);
    ok = half_arg(re0, -__builtin_fma(a, d, bc), m, u0, rsq_nr(2.0 * m * u0), E, sx, cx) && ok;
    ok = half_arg(re2, __builtin_fma(b, c, -ad), m, u2, rsq_nr(2.0 * m * u2), E, sz, cz) && ok;
    out[0] = Q{sx, 0.0f, 0.0f, cx};
    out[1] = Q{0.0f, sy, 0.0f, cy};
    out[2] = Q{0.0f, 0.0f, sz, cz};
    return ok;
}

// quat_in_xyz_axis (transform3d.py:52-59); true where the reference raises (scipy_as_euler)
RTG_DEV bool quat_in_xyz_axis(Q q, int s0, int s1, int s2, bool extrinsic, Q out[3])
{
    double ang[3];
    const bool refused = scipy_as_euler(q, s0, s1, s2, extrinsic, ang);
    out[0] = elementary_quat(s0, ang[0]);
    out[1] = elementary_quat(s1, ang[1]);
    out[2] = elementary_quat(s2, ang[2]);
    return refused;
}
// quat_in_xyz_axis(q, 'XYZ') as the solvers call it (full_body_pos_retargeter.py:142/165, full_body_retargeter.py
// :121/138): the atan2-free form above, the scipy restatement where it declines.  Same values (check [7]).
RTG_DEV bool quat_in_xyz_intrinsic(Q q, Q out[3])
{
#if RTG_EXP_EULER_SCIPY   // A/B knob (same values): the scipy restatement for every frame (round 4)
    return quat_in_xyz_axis(q, 0, 1, 2, false, out);
#endif
    bool refused = false;
    if (__builtin_expect(!quat_in_xyz_fast(q, out), 0)) refused = quat_in_xyz_axis(q, 0, 1, 2, false, out);
    return refused;
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

// the three unit vectors through one vunit_n (one rare-case branch instead of three; the same values)
RTG_DEV float radians_between(V v1, V v2, V n)  // :77-100
{
    const V in[3] = {v1, v2, n};
    V u[3];
    vunit_n<3>(in, u);
    const float c = clamp_lohi(dot3(u[0], u[1]), -1.0f, 1.0f);
    return cr_acos(c) * tsign(dot3(u[2], cross3(u[0], u[1])));
}

// shoulder_pr (SHOULDER) / elbow_py of NA arms at once, on the N-way leaf math: per arm the same operations on the
// same operands as the scalar forms above (vunit(v1p) serves both angles, as CSE made it there), so the same bits
template <bool SHOULDER, int NA, typename Tab = NoTab>
RTG_DEV void arm_pair_n(const V (&v1)[NA], const ArmZero (&z0)[NA], const Q (&parent)[NA], Q (&first)[NA],
                        Q (&second)[NA], Tab tab = Tab{})
{
    const V ex{1.f, 0.f, 0.f}, ey{0.f, 1.f, 0.f}, ez{0.f, 0.f, 1.f};
    const V pn = SHOULDER ? ey : ez;   // the plane of the first angle
    V vec[3 * NA];
#pragma unroll
    for (int a = 0; a < NA; ++a) {
        const V v1r = qrotate(qconj(parent[a]), v1[a]);
        const V v1p = proj_in_plane(v1r, pn);
        vec[3 * a] = v1p;
        vec[3 * a + 1] = v1r;
        vec[3 * a + 2] = SHOULDER ? cross3(v1p, ey) : cross3(ez, v1p);
    }
    V u[3 * NA];
    vunit_n<3 * NA>(vec, u);
    float c[2 * NA];
#pragma unroll
    for (int a = 0; a < NA; ++a) {
        c[2 * a] = clamp_lohi(dot3(ex, u[3 * a]), -1.0f, 1.0f);                  // radians_between_axes(ex, v1p, pn)
        c[2 * a + 1] = clamp_lohi(dot3(u[3 * a], u[3 * a + 1]), -1.0f, 1.0f);    // radians_between(v1p, v1r, n)
    }
    float ac[2 * NA];
    cr_acos_n<2 * NA>(c, ac);
    float ang[2 * NA];
    V ax[2 * NA];
#pragma unroll
    for (int a = 0; a < NA; ++a) {
        ang[2 * a] = ac[2 * a] * tsign(dot3(pn, cross3(ex, u[3 * a]))) - z0[a].th0;
        ax[2 * a] = pn;
        ang[2 * a + 1] = ac[2 * a + 1] * tsign(dot3(u[3 * a + 2], cross3(u[3 * a], u[3 * a + 1]))) - z0[a].ph0;
        ax[2 * a + 1] = SHOULDER ? ex : ey;
    }
    Q q[2 * NA];
    qfrom_angle_unit_axis_n<2 * NA>(ang, ax, q, tab);
#pragma unroll
    for (int a = 0; a < NA; ++a) {
        first[a] = q[2 * a];
        second[a] = q[2 * a + 1];
    }
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
