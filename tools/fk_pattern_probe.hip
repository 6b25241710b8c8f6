// fk_pattern_probe.hip -- what the streaming FK kernel's MEMORY PATTERN alone costs, with the chain taken out:
// three copy kernels move exactly the bytes of Hu FK (B frames x J = 31 joints: local rotations in (B,J,4), global
// rotations out (B,J,4), positions out (B,J,3)), differing only in which bytes a wave moves together.
//   win   : today's k_fk_stream windows -- per frame, joints [8k, 8k+8): a 128-B rotation piece at 16-B alignment
//           (straddles two 128-B lines) and a 96-B position piece at 4-B alignment, 8 lanes per frame piece;
//   line  : line-synchronous windows -- at step m every frame moves the records of its m-th 128-B LINE of the
//           tile's rotation rows (a 64-frame tile is 248 whole lines), so rotation pieces are line-aligned and
//           the position piece of rotation line L is bytes [96 L, 96 L + 96) of the tile's position rows (32-B
//           aligned); only a line shared by two frames' rows is touched by both (each its own records);
//   linear: the same bytes as one coalesced stream per tile (the copy roof for this traffic).
// Each kernel is checked to have written every output byte exactly as the copy defines it.
// build: hipcc --offload-arch=gfx950 -O3 -o /tmp/fkp tools/fk_pattern_probe.hip ; run: /tmp/fkp [B]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));           \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

constexpr int J = 31;
constexpr int kTile = 64;

// position record of joint record r: the quaternion's x, y, z (a stand-in for the chain's output)
__device__ inline void put_pos(float *pos, int64_t r, float4 q)
{
    pos[3 * r] = q.x;
    pos[3 * r + 1] = q.y;
    pos[3 * r + 2] = q.z;
}

__global__ __launch_bounds__(64) void k_win(const float4 *__restrict__ in, float4 *__restrict__ rot,
                                            float *__restrict__ pos, int64_t B)
{
    const int64_t f0 = (int64_t)blockIdx.x * kTile;
    for (int c0 = 0; c0 < J; c0 += 8) {
        const int nC = J - c0 < 8 ? J - c0 : 8;
#pragma unroll
        for (int it = 0; it < 8; ++it) {
            const int v = it * 64 + threadIdx.x, fr = v / 8, k = v % 8;
            if (k < nC && f0 + fr < B) {
                const int64_t r = (f0 + fr) * J + c0 + k;
                const float4 q = in[r];
                rot[r] = q;
                put_pos(pos, r, q);
            }
        }
    }
}

__global__ __launch_bounds__(64) void k_line(const float4 *__restrict__ in, float4 *__restrict__ rot,
                                             float *__restrict__ pos, int64_t B)
{
    const int64_t f0 = (int64_t)blockIdx.x * kTile;
    const int64_t R0 = f0 * J;   // the tile's first record (line-aligned: 64 J records = 8 J lines)
    for (int m = 0; m < (J + 7) / 8 + 1; ++m) {
#pragma unroll
        for (int it = 0; it < 8; ++it) {
            const int v = it * 64 + threadIdx.x, fr = v / 8, sub = v % 8;
            const int first = (fr * J) / 8;   // the frame's first line in the tile
            const int g = 8 * (first + m) + sub;   // record in the tile
            if (g >= fr * J && g < fr * J + J && f0 + fr < B) {
                const int64_t r = R0 + g;
                const float4 q = in[r];
                rot[r] = q;
                put_pos(pos, r, q);
            }
        }
    }
}

// line, but each rotation line's 96-B position piece leaves as 6 lanes x 16 B (whole piece; a piece two frames
// share is written whole by both, with the same bytes -- fine for a pattern probe, not for the product)
__global__ __launch_bounds__(64) void k_line_p4(const float4 *__restrict__ in, float4 *__restrict__ rot,
                                                float *__restrict__ pos, int64_t B)
{
    const int64_t f0 = (int64_t)blockIdx.x * kTile;
    const int64_t R0 = f0 * J;
    for (int m = 0; m < (J + 7) / 8 + 1; ++m) {
#pragma unroll
        for (int it = 0; it < 8; ++it) {
            const int v = it * 64 + threadIdx.x, fr = v / 8, sub = v % 8;
            const int first = (fr * J) / 8;
            const int g = 8 * (first + m) + sub;
            if (g >= fr * J && g < fr * J + J && f0 + fr < B) rot[R0 + g] = in[R0 + g];
        }
#pragma unroll
        for (int it = 0; it < 6; ++it) {
            const int v = it * 64 + threadIdx.x, fr = v / 6, c = v % 6;
            const int first = (fr * J) / 8, last = (fr * J + J - 1) / 8;
            const int L = first + m;
            if (L <= last && f0 + fr < B) {
                float o[4];
                for (int e = 0; e < 4; ++e) {
                    const int64_t fl = 24 * (int64_t)L + 4 * c + e;   // float in the tile's position rows
                    o[e] = (float)(R0 + fl / 3 + fl % 3);
                }
                reinterpret_cast<float4 *>(pos + 3 * R0)[6 * (int64_t)L + c] = make_float4(o[0], o[1], o[2], o[3]);
            }
        }
    }
}

__global__ __launch_bounds__(64) void k_linear(const float4 *__restrict__ in, float4 *__restrict__ rot,
                                               float *__restrict__ pos, int64_t B)
{
    const int64_t f0 = (int64_t)blockIdx.x * kTile;
    const int64_t R0 = f0 * J, n = ((B - f0) < kTile ? (B - f0) : kTile) * J;
    for (int64_t g = threadIdx.x; g < n; g += 64) {
        const float4 q = in[R0 + g];
        rot[R0 + g] = q;
        put_pos(pos, R0 + g, q);
    }
}

typedef void (*Kern)(const float4 *, float4 *, float *, int64_t);

int main(int argc, char **argv)
{
    const int64_t B = argc > 1 ? atoll(argv[1]) : 262144;
    const int64_t nr = B * J;
    float4 *in, *rot;
    float *pos;
    CK(hipMalloc(&in, nr * 16));
    CK(hipMalloc(&rot, nr * 16));
    CK(hipMalloc(&pos, nr * 12));
    std::vector<float4> h(nr);
    for (int64_t i = 0; i < nr; ++i) h[i] = make_float4((float)i, (float)(i + 1), (float)(i + 2), (float)(i + 3));
    CK(hipMemcpy(in, h.data(), nr * 16, hipMemcpyHostToDevice));
    const double bytes = (double)nr * (16 + 16 + 12);
    const unsigned grid = (unsigned)((B + kTile - 1) / kTile);
    struct { const char *name; Kern k; } ks[] = {{"win", k_win}, {"line", k_line}, {"line_p4", k_line_p4}, {"linear", k_linear}};
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<float4> hr(nr);
    std::vector<float> hp(nr * 3);
    for (int round = 0; round < 3; ++round)
        for (auto &K : ks) {
            CK(hipMemset(rot, 0, nr * 16));
            CK(hipMemset(pos, 0, nr * 12));
            hipLaunchKernelGGL(K.k, dim3(grid), dim3(64), 0, 0, in, rot, pos, B);
            CK(hipDeviceSynchronize());
            if (round == 0) {   // every output byte as the copy defines it
                CK(hipMemcpy(hr.data(), rot, nr * 16, hipMemcpyDeviceToHost));
                CK(hipMemcpy(hp.data(), pos, nr * 12, hipMemcpyDeviceToHost));
                for (int64_t i = 0; i < nr; ++i)
                    if (hr[i].x != h[i].x || hr[i].w != h[i].w || hp[3 * i] != h[i].x || hp[3 * i + 2] != h[i].z) {
                        fprintf(stderr, "%s: wrong record %lld\n", K.name, (long long)i);
                        return 1;
                    }
            }
            const int reps = 20;
            CK(hipEventRecord(a, 0));
            for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(K.k, dim3(grid), dim3(64), 0, 0, in, rot, pos, B);
            CK(hipEventRecord(b, 0));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            const double us = 1e3 * ms / reps;
            printf("round %d %-7s %8.1f us  %6.2f TB/s (algorithmic %.1f MB)\n", round, K.name, us,
                   bytes / (us * 1e-6) / 1e12, bytes / 1e6);
            fflush(stdout);
        }
    return 0;
}
