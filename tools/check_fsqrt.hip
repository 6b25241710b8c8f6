// check_fsqrt.hip -- exhaustive proof on the device that the 3-instruction
// sqrt (float)v_sqrt_f64((double)x) equals the correctly rounded f32 sqrt for
// EVERY f32 bit pattern (NaNs compared as "both NaN").
//   hipcc --offload-arch=gfx950 -O3 -fhip-fp32-correctly-rounded-divide-sqrt tools/check_fsqrt.hip -o /tmp/check_fsqrt
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

// bad[0]: fast != CR; bad[1]: of those, subnormal x; bad[2]: negative x; bad[3]: CR f32 != IEEE f64 sqrt rounded
__global__ void k(uint64_t base, unsigned long long *bad, uint32_t *first)
{
    const uint64_t u = base + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const float x = __uint_as_float((uint32_t)u);
    const float a = __builtin_sqrtf(x);                                   // IEEE (correctly rounded build)
    const float b = (float)__builtin_amdgcn_sqrt((double)x);              // v_sqrt_f64 + cvt
    const float c = (float)__builtin_sqrt((double)x);                     // IEEE f64 sqrt, rounded once
    const bool same = (__float_as_uint(a) == __float_as_uint(b)) || (a != a && b != b);
    const bool same_c = (__float_as_uint(a) == __float_as_uint(c)) || (a != a && c != c);
    if (!same_c) atomicAdd(bad + 3, 1ull);
    if (!same) {
        const unsigned long long n = atomicAdd(bad, 1ull);
        const uint32_t ax = (uint32_t)u & 0x7fffffffu;
        if (ax != 0 && ax < 0x00800000u) atomicAdd(bad + 1, 1ull);
        if ((uint32_t)u >> 31) atomicAdd(bad + 2, 1ull);
        if (!((uint32_t)u >> 31) && ax >= 0x00800000u && ax < 0x7f800000u) {
            const unsigned long long m = atomicAdd(bad + 4, 1ull);
            if (m < 8) first[m] = (uint32_t)u;
        }
    }
}

int main()
{
    unsigned long long *bad;
    uint32_t *first;
    (void)hipMalloc(&bad, 5 * sizeof *bad);
    (void)hipMalloc(&first, 8 * sizeof *first);
    (void)hipMemset(bad, 0, 5 * sizeof *bad);
    const uint64_t chunk = 1ull << 30;
    for (uint64_t base = 0; base < (1ull << 32); base += chunk)
        hipLaunchKernelGGL(k, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, base, bad, first);
    unsigned long long hb[5] = {0};
    uint32_t f[8] = {0};
    (void)hipMemcpy(hb, bad, sizeof hb, hipMemcpyDeviceToHost);
    (void)hipMemcpy(f, first, sizeof f, hipMemcpyDeviceToHost);
    const unsigned long long h = hb[0];
    printf("fsqrt: 4294967296 inputs, %llu mismatches (subnormal x %llu, negative x %llu, positive normal x %llu); "
           "CR f32 vs IEEE f64-rounded: %llu mismatches\n", h, hb[1], hb[2], hb[4], hb[3]);
    for (unsigned i = 0; i < (hb[4] < 8 ? hb[4] : 8); ++i) printf("  normal x bits 0x%08x\n", f[i]);
    return h != 0;
}
