// angtab_hist.hip -- histogram of the exp-map angle table's moves R(w) - P(w) (csrc/rtg_math.cuh ang_tab_code) per
// binade of w in [0.25, 1), plus how the codes would fit narrower encodings.  Measurement only.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt
//         -fno-fast-math -I include -I humanoid-real-time-retarget_amd/csrc tools/angtab_hist.hip -o tools/angtab_hist
#include <cstdio>

#include "rtg_math.cuh"

using namespace rtg;

__global__ void k_hist(unsigned long long *h)   // h[binade][code 0..7]
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= kAngTabEntries) return;
    const uint32_t code = ang_tab_code(__uint_as_float(kAngTabLo + i));
    const uint32_t binade = i >> 23;   // 0: [0.25, 0.5), 1: [0.5, 1)
    // finer: the top 3 mantissa bits within the binade
    const uint32_t sub = (i >> 20) & 7u;
    atomicAdd(h + (binade * 8 + sub) * 8 + code, 1ull);
}

int main()
{
    unsigned long long *d;
    (void)hipMalloc(&d, 2 * 8 * 8 * sizeof(unsigned long long));
    (void)hipMemset(d, 0, 2 * 8 * 8 * sizeof(unsigned long long));
    hipLaunchKernelGGL(k_hist, dim3(kAngTabEntries / 256), dim3(256), 0, 0, d);
    unsigned long long h[128];
    (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    printf("w range           code0(exact)   -3    -2    -1     0    +1    +2    +3   (counts per 2^20 entries)\n");
    for (int b = 0; b < 2; ++b)
        for (int s = 0; s < 8; ++s) {
            const double lo = (b ? 0.5 : 0.25) * (1.0 + s / 8.0), hi = (b ? 0.5 : 0.25) * (1.0 + (s + 1) / 8.0);
            printf("[%.4f, %.4f)", lo, hi);
            for (int c = 0; c < 8; ++c) printf(" %7llu", h[(b * 8 + s) * 8 + c]);
            printf("\n");
        }
    return 0;
}
