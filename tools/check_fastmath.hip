// check_fastmath.hip -- exhaustive device proof for the two "fast exact" helpers of csrc/rtg_math.cuh:
//  [1] cr_sqrt (v_sqrt_f64 + Newton) == IEEE f32 sqrt for EVERY f32 bit pattern (NaN == NaN);
//  [2] (float)((double)a * rcp64(n)) == IEEE f32 a / n for 2^32 hashed (a, n) pairs (full bit patterns,
//      clustered exponents, n near 1) plus every pair of 64 special values (0, denormals, inf, NaN, extremes);
//  [3] qexp_component_tab (exp-map angle table) == qexp_component for every f32 w bit pattern;
//  [4] sqrt_clamp_rcp (one v_rsq_f64) == clamp(cr_sqrt) + rcp64, bitwise, for every f32 s;
//  [5] mulr_k (K quotients by one denominator behind one subnormal branch) == K IEEE f32 divisions, on 2^30
//      hashed (a0, a1, a2, n) with a quarter of the groups steered to a subnormal first quotient;
//  [6] cr_acos (f64 asin kernel + rounding test, libm fallback) == (float)acos((double)x) for EVERY f32 x;
//  [7] quat_in_xyz_intrinsic (atan2-free 'XYZ' split, scipy fallback) == quat_in_xyz_axis(q, 'XYZ'), outputs and
//      refusal, on 2^30 hashed quaternions from eight families (unnormalised, unit, near gimbal lock, exact zero
//      components, tiny / huge scales, raw bit patterns, near the +-pi wrap, tiny angles).
// Since round 5 [1] checks the f32-arithmetic cr_sqrt (v_sqrt_f32 + two residual fmas).
// Built with the library's flags by __graft_entry__.build(); run by tests/test_gpu_parity.py.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#include "rtg_math.cuh"

using namespace rtg;

__device__ __forceinline__ bool same(float a, float b)
{
    return __float_as_uint(a) == __float_as_uint(b) || (a != a && b != b);
}

__device__ unsigned long long g_done[8];   // threads that ran each check (a failed launch must not read as a pass)
__device__ __forceinline__ void ran(int k)
{
    if (threadIdx.x == 0) atomicAdd(&g_done[k], (unsigned long long)blockDim.x);
}

__global__ void k_sqrt(uint64_t base, unsigned long long *bad)
{
    const uint32_t u = (uint32_t)(base + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x);
    const float x = __uint_as_float(u);
    ran(0);
    if (!same(cr_sqrt(x), ieee_sqrtf(x))) atomicAdd(bad, 1ull);
}

__device__ __forceinline__ uint64_t mix(uint64_t h)
{
    h *= 0x9E3779B97F4A7C15ull;
    h ^= h >> 29;
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 32;
    return h;
}

__device__ uint32_t g_first[16];

__global__ void k_div(uint64_t base, unsigned long long *bad)
{
    const uint64_t i = base + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t h = mix(i);
    uint32_t ua = (uint32_t)h, un = (uint32_t)(h >> 32);
    if (i & 1) {
        ua = (ua & 0x807FFFFFu) | ((((ua >> 23) % 40u) + 107u) << 23);
        un = (un & 0x807FFFFFu) | ((((un >> 23) % 40u) + 107u) << 23);
    }
    if ((i & 7) == 2) un = (un & 0x80FFFFFFu) | 0x3F000000u;
    const float a = __uint_as_float(ua), n = __uint_as_float(un);
    ran(1);
    if (!same(mulr(a, rcp64(n)), a / n)) {
        const unsigned long long k = atomicAdd(bad + 1, 1ull);
        if (k < 4) {
            g_first[4 * k] = ua;
            g_first[4 * k + 1] = un;
            g_first[4 * k + 2] = __float_as_uint(mulr(a, rcp64(n)));
            g_first[4 * k + 3] = __float_as_uint(a / n);
        }
    }
}

__global__ void k_div_special(unsigned long long *bad)
{
    const uint32_t sp[32] = {0x00000000u, 0x00000001u, 0x00000002u, 0x007FFFFFu, 0x00800000u, 0x00800001u,
                             0x3F800000u, 0x3F800001u, 0x3F7FFFFFu, 0x40000000u, 0x3EAAAAABu, 0x7F7FFFFFu,
                             0x7F000000u, 0x7F800000u, 0x7FC00000u, 0x7FA00000u, 0x0DA24260u, 0x71A3C9F0u,
                             0x00400000u, 0x00000003u, 0x3089705Fu, 0x4E6E6B28u, 0x2F800000u, 0x50000000u,
                             0x1E3CE508u, 0x60AD78ECu, 0x01000000u, 0x7E800000u, 0x3F000001u, 0x3FFFFFFFu,
                             0x4B800000u, 0x33800000u};
    const int i = threadIdx.x, j = blockIdx.x;   // 64 x 64
    const float a = __uint_as_float(sp[i & 31] | ((i & 32) ? 0x80000000u : 0u));
    const float n = __uint_as_float(sp[j & 31] | ((j & 32) ? 0x80000000u : 0u));
    ran(2);
    if (!same(mulr(a, rcp64(n)), a / n)) atomicAdd(bad + 2, 1ull);
}

// [3] qexp_component_tab (exp-map angle table) == qexp_component for every f32 w (all 2^32 bit patterns; x, y, z
// hashed, the component cycling through 0..2).  The table is built here exactly as rtg_solver_create builds it.
__global__ void k_build_tab(uint32_t *tab)
{
    const uint32_t wd = blockIdx.x * 256u + threadIdx.x;
    if (wd >= kAngTabWords) return;
    tab[wd] = ang_tab_build_word(wd);
}

__global__ void k_exptab(uint64_t base, const uint32_t *tab, unsigned long long *bad)
{
    const uint64_t i = base + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t h = mix(i);
    const float x = (float)(int32_t)(h & 0xffff) * 0x1p-15f, y = (float)(int32_t)((h >> 16) & 0xffff) * 0x1p-15f,
                z = (float)(int32_t)((h >> 32) & 0xffff) * 0x1p-15f;
    const Q q{x - 1.0f, y - 1.0f, z - 1.0f, __uint_as_float((uint32_t)i)};
    const int k = (int)(i % 3);
    ran(3);
    if (!same(qexp_component_tab(q, k, tab), qexp_component(q, k))) atomicAdd(bad + 3, 1ull);
}

// [4] sqrt_clamp_rcp (one v_rsq_f64) == (clamp(cr_sqrt(s), lo), rcp64(n)) bitwise, n and the f64 reciprocal, for
// EVERY f32 s and both clamps the library uses (1e-9 and 0)
__global__ void k_normrcp(uint64_t base, unsigned long long *bad)
{
    const uint32_t u = (uint32_t)(base + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x);
    const float s = __uint_as_float(u);
    ran(4);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const float lo = k ? 0.0f : 1e-9f;
        const NormRcp f = sqrt_clamp_rcp(s, lo);
        const float n = clamp_lo(cr_sqrt(s), lo);
        const Rcp r = rcp64(n);
        const bool same_r = __double_as_longlong(f.r.r) == __double_as_longlong(r.r) || (f.r.r != f.r.r && r.r != r.r);
        if (!same(f.n, n) || !same(f.r.n, r.n) || !same_r) atomicAdd(bad + 4, 1ull);
    }
}

// [5] the grouped form: one subnormal quotient in the group sends all three to the IEEE division
__global__ void k_divk(uint64_t base, unsigned long long *bad)
{
    const uint64_t i = base + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t h = mix(i), h2 = mix(i ^ 0x5DEECE66Dull);
    uint32_t un = (uint32_t)(h >> 32);
    const uint32_t ua[3] = {(uint32_t)h, (uint32_t)h2, (uint32_t)(h2 >> 32)};
    if ((i & 3) == 1) {   // exponent of n = exponent of a0 + 126 .. 149: a0 / n subnormal or just normal
        const uint32_t ea = (ua[0] >> 23) & 0xFFu, en = ea + 126u + (uint32_t)((h2 >> 8) % 24u);
        if (ea > 0u && en < 255u) un = (un & 0x807FFFFFu) | (en << 23);
    }
    float a[3], q[3];
    for (int k = 0; k < 3; ++k) a[k] = __uint_as_float(ua[k]);
    const float n = __uint_as_float(un);
    ran(5);
    mulr_k<3>(a, rcp64(n), q);
    if (!same(q[0], a[0] / n) || !same(q[1], a[1] / n) || !same(q[2], a[2] / n)) atomicAdd(bad + 5, 1ull);
}

// [6] cr_acos for every f32 bit pattern; g_acos_slow counts the |x| < 1 inputs the fast path hands to libm
__device__ unsigned long long g_acos_slow;
__global__ void k_acos(uint64_t base, unsigned long long *bad)
{
    const uint32_t u = (uint32_t)(base + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x);
    const float x = __uint_as_float(u);
    ran(6);
    bool ok;
    (void)acos_fast(x, ok);
    if (!ok && __builtin_fabsf(x) < 1.0f) atomicAdd(&g_acos_slow, 1ull);
    if (!same(cr_acos(x), acos_libm(x))) atomicAdd(bad + 6, 1ull);
}

// [7] the 'XYZ' split, fast form vs scipy restatement; g_xyz_slow counts the quaternions the fast form declines
__device__ unsigned long long g_xyz_slow;
__device__ __forceinline__ float hf(uint64_t h, int k) { return (float)((h >> (11 * k)) & 0x3FFFFFu) * 0x1p-21f - 1.0f; }
__global__ void k_xyz(uint64_t base, unsigned long long *bad)
{
    const uint64_t i = base + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t h = mix(i), h2 = mix(i ^ 0x5bd1e995u);
    ran(7);
    const int fam = (int)(h2 & 7u);
    Q q{hf(h, 0), hf(h, 1), hf(h, 2), hf(h, 3)};
    if (fam == 1 || fam >= 6) q = qnormalize(q);
    if (fam == 2) {   // Y near +-90 degrees: x, z tiny against y, w (or an exact gimbal)
        const float e = ldexpf(hf(h2, 1), -(int)((h2 >> 8) % 40u));
        q = Q{e * hf(h2, 2), 0.7071068f + 0.1f * hf(h2, 3) * e, e * hf(h2, 4), 0.7071068f};
    } else if (fam == 3) {   // exact zeros
        const uint32_t mz = (uint32_t)(h2 >> 8) & 15u;
        q = Q{(mz & 1) ? 0.0f : q.x, (mz & 2) ? 0.0f : q.y, (mz & 4) ? -0.0f : q.z, (mz & 8) ? 0.0f : q.w};
    } else if (fam == 4) {
        const float sc = (h2 >> 8) & 1 ? 1e-19f : 1e19f;
        q = Q{q.x * sc, q.y * sc, q.z * sc, q.w * sc};
    } else if (fam == 5) {
        q = Q{__uint_as_float((uint32_t)h), __uint_as_float((uint32_t)(h >> 32)), __uint_as_float((uint32_t)h2),
              __uint_as_float((uint32_t)(h2 >> 32))};
    } else if (fam == 6) {   // X / Z arguments near +-pi: w and y small against x, z
        const float e = ldexpf(1.0f, -(int)((h2 >> 8) % 30u));
        q = Q{q.x, q.y * e, q.z, q.w * e};
    } else if (fam == 7) {   // small rotations
        const float e = ldexpf(1.0f, -(int)((h2 >> 8) % 26u));
        q = Q{q.x * e, q.y * e, q.z * e, 1.0f};
    }
    Q f[3], r[3];
    const bool okf = quat_in_xyz_fast(q, f);
    if (!okf) atomicAdd(&g_xyz_slow, 1ull);
    const bool rf = quat_in_xyz_intrinsic(q, f);
    const bool rr = quat_in_xyz_axis(q, 0, 1, 2, false, r);
    bool eq = rf == rr;
    for (int k = 0; k < 3; ++k)
        eq = eq && same(f[k].x, r[k].x) && same(f[k].y, r[k].y) && same(f[k].z, r[k].z) && same(f[k].w, r[k].w);
    if (!eq) {
        const unsigned long long n = atomicAdd(bad + 7, 1ull);
        if (n < 4) {
            g_first[8 + 2 * n] = __float_as_uint(q.x) ^ __float_as_uint(q.w);
            g_first[9 + 2 * n] = (uint32_t)i;
        }
    }
}

int main()
{
    unsigned long long *bad;
    (void)hipMalloc(&bad, 8 * sizeof(unsigned long long));
    (void)hipMemset(bad, 0, 8 * sizeof(unsigned long long));
    uint32_t *tab;
    (void)hipMalloc(&tab, kAngTabWords * sizeof(uint32_t));
    hipLaunchKernelGGL(k_build_tab, dim3((kAngTabWords + 255u) / 256u), dim3(256), 0, 0, tab);
    const uint64_t chunk = 1ull << 30;
    for (uint64_t base = 0; base < (1ull << 32); base += chunk) {
        hipLaunchKernelGGL(k_sqrt, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, base, bad);
        hipLaunchKernelGGL(k_div, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, base, bad);
        hipLaunchKernelGGL(k_exptab, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, base, tab, bad);
        hipLaunchKernelGGL(k_normrcp, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, base, bad);
        hipLaunchKernelGGL(k_acos, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, base, bad);
    }
    hipLaunchKernelGGL(k_divk, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, 0ull, bad);
    hipLaunchKernelGGL(k_xyz, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, 0ull, bad);
    hipLaunchKernelGGL(k_div_special, dim3(64), dim3(64), 0, 0, bad);
    if (hipDeviceSynchronize() != hipSuccess || hipGetLastError() != hipSuccess) {
        printf("launch/run failure: %s\n", hipGetErrorString(hipGetLastError()));
        return 2;
    }
    unsigned long long h[8] = {0, 0, 0, 0, 0, 0, 0, 0}, d[8] = {0, 0, 0, 0, 0, 0, 0, 0}, slow = 0, xslow = 0;
    (void)hipMemcpy(h, bad, sizeof h, hipMemcpyDeviceToHost);
    (void)hipMemcpyFromSymbol(d, HIP_SYMBOL(g_done), sizeof d);
    (void)hipMemcpyFromSymbol(&slow, HIP_SYMBOL(g_acos_slow), sizeof slow);
    (void)hipMemcpyFromSymbol(&xslow, HIP_SYMBOL(g_xyz_slow), sizeof xslow);
    const unsigned long long want[8] = {1ull << 32, 1ull << 32, 4096ull, 1ull << 32, 1ull << 32, 1ull << 30, 1ull << 32,
                                        1ull << 30};
    for (int k = 0; k < 8; ++k)
        if (d[k] != want[k]) {
            printf("check %d covered %llu of %llu inputs\n", k, d[k], want[k]);
            return 2;
        }
    printf("[1] cr_sqrt: 4294967296 inputs, %llu mismatches\n", h[0]);
    printf("[2] rcp64 division: 4294967296 pairs, %llu mismatches\n", h[1]);
    printf("[2b] rcp64 division, special values: 4096 pairs, %llu mismatches\n", h[2]);
    printf("[3] exp-map angle table: 4294967296 w bit patterns, %llu mismatches\n", h[3]);
    printf("[4] sqrt_clamp_rcp: 4294967296 inputs x 2 clamps, %llu mismatches\n", h[4]);
    printf("[5] grouped mulr_k<3>: 1073741824 groups, %llu mismatches\n", h[5]);
    printf("[6] cr_acos: 4294967296 inputs, %llu mismatches (libm fallback on %llu of the 2130706430 |x| < 1)\n",
           h[6], slow);
    printf("[7] 'XYZ' split, fast vs scipy restatement: 1073741824 quaternions, %llu mismatches (fallback on %llu)\n",
           h[7], xslow);
    uint32_t f[16];
    (void)hipMemcpyFromSymbol(f, HIP_SYMBOL(g_first), sizeof f);
    for (unsigned k = 0; k < (h[1] < 4 ? h[1] : 4); ++k)
        printf("  a=%08x n=%08x fast=%08x ieee=%08x\n", f[4 * k], f[4 * k + 1], f[4 * k + 2], f[4 * k + 3]);
    (void)hipFree(tab);
    for (unsigned k = 0; k < (h[7] < 4 ? h[7] : 4); ++k) printf("  xyz mismatch at i=%u\n", f[9 + 2 * k]);
    return (h[0] || h[1] || h[2] || h[3] || h[4] || h[5] || h[6] || h[7]) ? 1 : 0;
}
