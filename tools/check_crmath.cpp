// check_crmath.cpp -- exhaustive host check of csrc/rtg_crmath.h against glibc.
//
//   g++ -O2 -march=x86-64-v3 -ffp-contract=off -fopenmp -I humanoid-real-time-retarget_amd/csrc \
//       tools/check_crmath.cpp -o /tmp/check_crmath -lm && /tmp/check_crmath [stride]
//
// stride 1 (default) is the exhaustive run (~30 s on 8 cores); tests/ use a larger stride.
//
//  1. crm_sincos on EVERY float in [-4pi, 4pi] (the solver's f32 angles): whenever the fast
//     path accepts, it must equal (float)sin((double)x) / (float)cos((double)x) (glibc).
//  2. crm_sincos on 2^30 random doubles in [-pi/2, pi/2] (scipy from_euler half angles),
//     plus the doubles nearest 0 and +-pi/2.
//  4. shared-reciprocal division (rtg_math.cuh rcp64/mulr): (float)((double)a * (1.0 / n)) == a / n
//     for 2^32 random f32 pairs (full bit patterns, clustered exponents, n near 1).
//  3. crm_atan2f_sel vs the fdlibm restatement (glibc's own atan2f) for (sin a, cos a) of EVERY
//     float a in [0, 2pi] (the exp-map's normalize_angle), and 2^30 random bit patterns.
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>

#include "rtg_crmath.h"

using namespace rtg::crm;

static float bits2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t f2bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

int main(int argc, char **argv)
{
    const int64_t stride = argc > 1 ? atoll(argv[1]) : 1;
    long long bad = 0, fallback_s = 0, fallback_c = 0, n = 0;
    // 1. every float with |x| <= 4pi
    const float lim = 4.0f * 3.14159265f;
    const uint32_t top = f2bits(lim);
#pragma omp parallel for reduction(+ : bad, fallback_s, fallback_c, n) schedule(dynamic, 1 << 16)
    for (int64_t u = 0; u <= (int64_t)top; u += stride) {
        for (int sgn = 0; sgn < 2; ++sgn) {
            const float x = bits2f((uint32_t)u | (sgn ? 0x80000000u : 0u));
            const SinCos r = crm_sincos((double)x);
            const float s = (float)sin((double)x), c = (float)cos((double)x);
            ++n;
            if (!r.s_ok) ++fallback_s;
            else if (f2bits(r.s) != f2bits(s)) { ++bad; if (bad < 10) printf("sin mismatch x=%a %a %a\n", x, r.s, s); }
            if (!r.c_ok) ++fallback_c;
            else if (f2bits(r.c) != f2bits(c)) { ++bad; if (bad < 10) printf("cos mismatch x=%a %a %a\n", x, r.c, c); }
        }
    }
    printf("[1] f32 |x|<=4pi: %lld values, %lld mismatches, fallbacks sin %lld cos %lld\n", n, bad, fallback_s, fallback_c);
    long long bad1 = bad;
    // 2. random doubles in [-pi/2, pi/2] + edges
    bad = 0; n = 0; fallback_s = fallback_c = 0;
#pragma omp parallel for reduction(+ : bad, fallback_s, fallback_c, n)
    for (int64_t i = 0; i < (1ll << 30); i += stride) {
        uint64_t h = (uint64_t)i * 0x9E3779B97F4A7C15ull;
        h ^= h >> 29; h *= 0xBF58476D1CE4E5B9ull; h ^= h >> 32;
        double x = ((double)(h >> 11) * 0x1p-53 * 2.0 - 1.0) * 1.5707963267948966;
        if ((i & 0xFFFF) < 64) x = nextafter(1.5707963267948966, (i & 1) ? 0.0 : 4.0) * ((i & 2) ? -1 : 1);
        if ((i & 0xFFFF) == 100) x = 0x1p-1000 * ((i & 1) ? 1 : -1);
        const SinCos r = crm_sincos(x);
        const float s = (float)sin(x), c = (float)cos(x);
        ++n;
        if (!r.s_ok) ++fallback_s;
        else if (f2bits(r.s) != f2bits(s)) { ++bad; if (bad < 10) printf("sin(d) mismatch x=%a\n", x); }
        if (!r.c_ok) ++fallback_c;
        else if (f2bits(r.c) != f2bits(c)) { ++bad; if (bad < 10) printf("cos(d) mismatch x=%a\n", x); }
    }
    printf("[2] f64 |x|<=pi/2: %lld values, %lld mismatches, fallbacks sin %lld cos %lld\n", n, bad, fallback_s, fallback_c);
    long long bad2 = bad;
    // 3. atan2f on (sin a, cos a) for every float a in [0, 2pi], and random bit patterns
    bad = 0; n = 0;
    const uint32_t top2 = f2bits(6.2831855f);
#pragma omp parallel for reduction(+ : bad, n) schedule(dynamic, 1 << 16)
    for (int64_t u = 0; u <= (int64_t)top2; u += stride) {
        const float a = bits2f((uint32_t)u);
        const float y = (float)sin((double)a), x = (float)cos((double)a);
        const float ref = atan2f(y, x);
        const float got = crm_atan2f_regular(y, x) ? crm_atan2f_sel(y, x) : ref;
        ++n;
        if (f2bits(got) != f2bits(ref)) { ++bad; if (bad < 10) printf("atan2 mismatch a=%a y=%a x=%a %a %a\n", a, y, x, got, ref); }
    }
#pragma omp parallel for reduction(+ : bad, n)
    for (int64_t i = 0; i < (1ll << 30); i += stride) {
        uint64_t h = (uint64_t)i * 0x9E3779B97F4A7C15ull + 12345;
        h ^= h >> 31; h *= 0x94D049BB133111EBull; h ^= h >> 29;
        float y = bits2f((uint32_t)h), x = bits2f((uint32_t)(h >> 32));
        if (i & 1) {   // values of moderate magnitude too
            y = (float)((int32_t)(h & 0xFFFFFF) - 0x800000) * 0x1p-20f;
            x = (float)((int32_t)((h >> 24) & 0xFFFFFF) - 0x800000) * 0x1p-20f;
        }
        if (!crm_atan2f_regular(y, x)) continue;
        const float ref = atan2f(y, x);
        const float got = crm_atan2f_sel(y, x);
        ++n;
        if (f2bits(got) != f2bits(ref)) { ++bad; if (bad < 10) printf("atan2 mismatch y=%a x=%a %a %a\n", y, x, got, ref); }
    }
    printf("[3] atan2f: %lld pairs, %lld mismatches\n", n, bad);
    long long bad3 = bad;
    bad = 0; n = 0;
#pragma omp parallel for reduction(+ : bad, n)
    for (int64_t i = 0; i < (1ll << 32); i += stride) {
        uint64_t h = (uint64_t)i * 0x9E3779B97F4A7C15ull;
        h ^= h >> 29; h *= 0xBF58476D1CE4E5B9ull; h ^= h >> 32;
        uint32_t ua = (uint32_t)h, un = (uint32_t)(h >> 32);
        if (i & 1) {
            ua = (ua & 0x807FFFFFu) | (((ua >> 23) % 40 + 107) << 23);
            un = (un & 0x807FFFFFu) | (((un >> 23) % 40 + 107) << 23);
        }
        if ((i & 7) == 2) un = (un & 0x80FFFFFFu) | 0x3F000000u;
        const float a = bits2f(ua), d = bits2f(un);
        if (isnan(a) || isnan(d)) continue;
        volatile float q = a / d;
        const float p = (float)((double)a * (1.0 / (double)d));
        ++n;
        if (f2bits(p) != f2bits(q)) { ++bad; if (bad < 10) printf("rdiv mismatch a=%a n=%a\n", a, d); }
    }
    printf("[4] reciprocal division: %lld pairs, %lld mismatches\n", n, bad);
    return (bad1 || bad2 || bad3 || bad) ? 1 : 0;
}
