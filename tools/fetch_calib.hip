// fetch_calib.hip -- known-byte micro-kernels that calibrate rocprofv3's FETCH_SIZE for the solver's access
// shapes (MI355X_MICROARCH.md: FETCH_SIZE is calibrated only for 16 B/lane streaming reads, where it reports 1/2).
// Run under `rocprofv3 --pmc FETCH_SIZE` (and a separate WRITE_SIZE pass); tools/pmc_summary.py divides the
// counter by the byte counts this program prints.  Every input buffer is read once per dispatch from a ring of
// buffers larger than the 256 MiB Infinity Cache, so the bytes come from HBM.
//
//   k_stream16      float4 per lane, fully coalesced: the guide's reference shape
//   k_gather_all    the solver's shape: one frame per lane, 12-byte points (global_load_dwordx3) from 252-byte
//                   AoS rows (B, 21, 3) -- all 21 points, so every byte of the buffer is read exactly once
//   k_gather_used   the same rows, only the 10 body points VtrdynFullBodyPosRetargeter reads (10,11,13..20):
//                   known bytes = the 128-byte lines those points touch (printed) and the points' own bytes
//   k_hand_used     hand rows (B, 20, 3): the 11 points the solver reads (0,2,4,6,8,10,12,14,16,17,19)
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/fetch_calib.hip -o tools/fetch_calib
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <set>
#include <vector>

#define CHECK(x)                                                                         \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                \
        }                                                                                \
    } while (0)

struct P3 { float x, y, z; };

__global__ __launch_bounds__(256) void k_stream16(const float4 *__restrict__ in, int64_t n4, float *__restrict__ out)
{
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n4) return;
    const float4 v = in[i];
    out[i] = v.x + v.y + v.z + v.w;
}

template <int ROW, int NP>
__global__ __launch_bounds__(256) void k_gather(const float *__restrict__ rows, int64_t B, const int *__restrict__ pts,
                                                float *__restrict__ out)
{
    const int64_t f = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (f >= B) return;
    const float *r = rows + f * ROW;
    float s = 0.0f;
#pragma unroll
    for (int k = 0; k < NP; ++k) {
        const P3 p = *reinterpret_cast<const P3 *>(r + 3 * pts[k]);   // 12-byte load, as the solver's ld3
        s += p.x + p.y + p.z;
    }
    out[f] = s;
}

static std::vector<int> g_pts_all, g_pts_body, g_pts_hand;

int main(int argc, char **argv)
{
    const int64_t B = argc > 1 ? std::atoll(argv[1]) : 262144;
    const int ring = 8;
    for (int i = 0; i < 21; ++i) g_pts_all.push_back(i);
    g_pts_body = {10, 11, 13, 14, 15, 16, 17, 18, 19, 20};
    g_pts_hand = {0, 2, 4, 6, 8, 10, 12, 14, 16, 17, 19};
    int *d_all, *d_body, *d_hand;
    CHECK(hipMalloc(&d_all, 21 * sizeof(int)));
    CHECK(hipMalloc(&d_body, 10 * sizeof(int)));
    CHECK(hipMalloc(&d_hand, 11 * sizeof(int)));
    CHECK(hipMemcpy(d_all, g_pts_all.data(), 21 * sizeof(int), hipMemcpyHostToDevice));
    CHECK(hipMemcpy(d_body, g_pts_body.data(), 10 * sizeof(int), hipMemcpyHostToDevice));
    CHECK(hipMemcpy(d_hand, g_pts_hand.data(), 11 * sizeof(int), hipMemcpyHostToDevice));
    const size_t body_bytes = (size_t)B * 63 * 4, hand_bytes = (size_t)B * 60 * 4;
    std::vector<float *> body(ring), hand(ring);
    for (int r = 0; r < ring; ++r) {
        CHECK(hipMalloc(&body[r], body_bytes));
        CHECK(hipMalloc(&hand[r], hand_bytes));
        CHECK(hipMemset(body[r], 0, body_bytes));
        CHECK(hipMemset(hand[r], 0, hand_bytes));
    }
    float *out;
    CHECK(hipMalloc(&out, body_bytes / 4 + 64));
    const dim3 blk(256), grd((unsigned)((B + 255) / 256));
    const int64_t n4 = (int64_t)(body_bytes / 16);
    const dim3 grd4((unsigned)((n4 + 255) / 256));
    const int reps = 4;
    for (int it = 0; it < reps; ++it) {
        for (int r = 0; r < ring; ++r)
            hipLaunchKernelGGL(k_stream16, grd4, blk, 0, 0, reinterpret_cast<const float4 *>(body[r]), n4, out);
        for (int r = 0; r < ring; ++r) hipLaunchKernelGGL((k_gather<63, 21>), grd, blk, 0, 0, body[r], B, d_all, out);
        for (int r = 0; r < ring; ++r) hipLaunchKernelGGL((k_gather<63, 10>), grd, blk, 0, 0, body[r], B, d_body, out);
        for (int r = 0; r < ring; ++r) hipLaunchKernelGGL((k_gather<60, 11>), grd, blk, 0, 0, hand[r], B, d_hand, out);
    }
    CHECK(hipDeviceSynchronize());
    // known bytes per dispatch: points' own bytes and the distinct 128-byte lines they touch
    auto lines = [&](int row_floats, const std::vector<int> &pts) {
        std::set<int64_t> L;
        for (int64_t f = 0; f < B; ++f)
            for (int p : pts) {
                const int64_t a = (f * row_floats + 3 * p) * 4;
                L.insert(a >> 7);
                L.insert((a + 11) >> 7);
            }
        return (double)L.size() * 128.0;
    };
    std::printf("{\"B\": %lld, \"ring\": %d, \"dispatches_per_kernel\": %d,\n", (long long)B, ring, ring * reps);
    std::printf(" \"k_stream16\": {\"bytes\": %.0f, \"write_bytes\": %.0f},\n", (double)body_bytes, (double)n4 * 4);
    std::printf(" \"k_gather<63, 21>\": {\"bytes\": %.0f, \"line_bytes\": %.0f, \"write_bytes\": %.0f},\n",
                (double)body_bytes, lines(63, g_pts_all), (double)B * 4);
    std::printf(" \"k_gather<63, 10>\": {\"bytes\": %.0f, \"line_bytes\": %.0f, \"write_bytes\": %.0f},\n",
                (double)B * 10 * 12, lines(63, g_pts_body), (double)B * 4);
    std::printf(" \"k_gather<60, 11>\": {\"bytes\": %.0f, \"line_bytes\": %.0f, \"write_bytes\": %.0f}}\n",
                (double)B * 11 * 12, lines(60, g_pts_hand), (double)B * 4);
    return 0;
}
