// bar_probe.hip -- can the host write device-local memory directly (PCIe large BAR), and what does a frame
// server's hand-over cost when its inbox lives there instead of in pinned host memory?
//
//   hipcc --offload-arch=gfx950 -O2 tools/bar_probe.hip -o tools/bar_probe
//   tools/bar_probe <mode> [sfence]   mode: fg (hipExtMallocWithFlags hipDeviceMallocFinegrained)
//                                    uc (hipExtMallocWithFlags hipDeviceMallocUncached)
//                                    host (hipHostMalloc, the server's current inbox)
//
// Each mode runs in its own process (a host store to memory the CPU cannot map faults: the caller sees the
// signal, not a hang).  The ping-pong: the host writes a 184-float frame and then a sequence word into the
// inbox; one resident workgroup polls the word, reads the frame, writes a 30-float reply and the sequence word
// into pinned host memory; the host spins on that word.  Prints one JSON line.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <algorithm>
#include <immintrin.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("{\"error\": \"%s: %s\"}\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void k_pong(const float *in, volatile uint32_t *in_seq, float *out, uint32_t *out_seq, int frames,
                       uint64_t idle_ticks)
{
    __shared__ float s[184];
    __shared__ uint32_t cmd;
    uint32_t last = 0;
    for (int f = 0; f < frames; ++f) {
        if (threadIdx.x == 0) {
            const uint64_t t0 = wall_clock64();
            uint32_t v;
            for (;;) {
                v = __hip_atomic_load((uint32_t *)in_seq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
                if (v != last) break;
                if (wall_clock64() - t0 > idle_ticks) { v = 0xFFFFFFFFu; break; }
                __builtin_amdgcn_s_sleep(1);
            }
            cmd = v;
        }
        __syncthreads();
        const uint32_t c = cmd;
        if (c == 0xFFFFFFFFu) break;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        if (threadIdx.x < 184) s[threadIdx.x] = in[threadIdx.x];
        __syncthreads();
        if (threadIdx.x < 30) out[threadIdx.x] = s[threadIdx.x] + s[threadIdx.x + 100];
        __syncthreads();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __syncthreads();
        if (threadIdx.x == 0) {
            __hip_atomic_store(out_seq, c, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            last = c;
        }
    }
}

int main(int argc, char **argv)
{
    const char *mode = argc > 1 ? argv[1] : "host";
    const bool fence = argc > 2 && !strcmp(argv[2], "sfence");
    const int frames = 2000;
    int dev = 0;
    CK(hipSetDevice(dev));
    int large_bar = -1, direct_managed = -1, pageable = -1;
    (void)hipDeviceGetAttribute(&large_bar, hipDeviceAttributeIsLargeBar, dev);
    (void)hipDeviceGetAttribute(&direct_managed, hipDeviceAttributeDirectManagedMemAccessFromHost, dev);
    (void)hipDeviceGetAttribute(&pageable, hipDeviceAttributePageableMemoryAccess, dev);
    void *inbox = nullptr;   // 184 floats + the sequence word at float 192 (its own 64-byte piece)
    const size_t inbox_bytes = 256 * sizeof(float);
    if (!strcmp(mode, "fg")) CK(hipExtMallocWithFlags(&inbox, inbox_bytes, hipDeviceMallocFinegrained));
    else if (!strcmp(mode, "uc")) CK(hipExtMallocWithFlags(&inbox, inbox_bytes, hipDeviceMallocUncached));
    else CK(hipHostMalloc(&inbox, inbox_bytes, hipHostMallocMapped));
    float *h_out = nullptr;
    uint32_t *h_oseq = nullptr;
    CK(hipHostMalloc((void **)&h_out, 64 * sizeof(float), hipHostMallocMapped));
    CK(hipHostMalloc((void **)&h_oseq, 64, hipHostMallocMapped));
    *h_oseq = 0;
    {   // what the runtime reports for the inbox (rtg_server_inbox_alloc's mapping test reads the same record)
        hipPointerAttribute_t a;
        const hipError_t e = hipPointerGetAttributes(&a, inbox);
        printf("{\"attributes\": {\"rc\": %d, \"type\": %d, \"ptr\": \"%p\", \"hostPointer\": \"%p\", "
               "\"devicePointer\": \"%p\", \"isManaged\": %d, \"allocationFlags\": %u}}\n",
               (int)e, (int)a.type, inbox, a.hostPointer, a.devicePointer, (int)a.isManaged, a.allocationFlags);
    }
    float *fin = static_cast<float *>(inbox);
    uint32_t *iseq = reinterpret_cast<uint32_t *>(fin + 192);
    // the host store that faults if the CPU cannot reach this memory
    for (int i = 0; i < 184; ++i) fin[i] = (float)i;
    __atomic_store_n(iseq, 0u, __ATOMIC_RELEASE);
    float *d_in = fin;
    uint32_t *d_iseq = iseq;
    float *d_out = nullptr;
    uint32_t *d_oseq = nullptr;
    if (strcmp(mode, "fg") && strcmp(mode, "uc")) {
        CK(hipHostGetDevicePointer((void **)&d_in, fin, 0));
        d_iseq = reinterpret_cast<uint32_t *>(d_in + 192);
    }
    CK(hipHostGetDevicePointer((void **)&d_out, h_out, 0));
    CK(hipHostGetDevicePointer((void **)&d_oseq, h_oseq, 0));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipLaunchKernelGGL(k_pong, dim3(1), dim3(256), 0, st, d_in, d_iseq, d_out, d_oseq, frames, (uint64_t)100000000);
    std::vector<double> us;
    us.reserve(frames);
    bool ok = true;
    for (uint32_t seq = 1; seq <= (uint32_t)frames; ++seq) {
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < 184; ++i) fin[i] = (float)(i + seq);
        if (fence) _mm_sfence();   // device memory is mapped write-combining: drain the frame before the word
        __atomic_store_n(iseq, seq, __ATOMIC_RELEASE);
        if (fence) _mm_sfence();   // ... and the word itself out of the write-combining buffer
        long spins = 0;
        while (__atomic_load_n(h_oseq, __ATOMIC_ACQUIRE) != seq) {
            if (++spins > 2000000000L) { ok = false; break; }
        }
        const auto t1 = std::chrono::steady_clock::now();
        if (!ok) break;
        if (h_out[3] != (float)(3 + seq) + (float)(103 + seq)) ok = false;
        us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    }
    CK(hipStreamSynchronize(st));
    std::sort(us.begin(), us.end());
    const double med = us.empty() ? -1 : us[us.size() / 2], p99 = us.empty() ? -1 : us[us.size() * 99 / 100];
    printf("{\"mode\": \"%s%s\", \"ok\": %s, \"frames\": %zu, \"median_us\": %.2f, \"p99_us\": %.2f, "
           "\"direct_managed_access\": %d, \"pageable_access\": %d, \"large_bar\": %d}\n",
           mode, fence ? "+sfence" : "", ok ? "true" : "false", us.size(), med, p99, direct_managed, pageable, large_bar);
    return ok ? 0 : 2;
}
