// tools/vram_probe.cpp -- can the host write straight into HBM on this box (large BAR)?  For the
// drop-in hash service: if a caller could copy its message into device memory and post the slot
// there, a call would need no PCIe read at all (the GPU polls and reads HBM).
//
// 1. hipExtMallocWithFlags(fine-grained) and (uncached): does the host pointer work on the CPU?
// 2. CPU memcpy bandwidth into it (64 KiB copies), and into pinned host memory for comparison.
// 3. a kernel reads what the host wrote (checksum), and a ping-pong: the host writes a word into
//    HBM, a kernel polling HBM answers into pinned host memory; round-trip latency.
//
// Build: hipcc -O2 -std=c++17 --offload-arch=gfx950 tools/vram_probe.cpp -o build_ab/vram_probe
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <vector>

using clk = std::chrono::steady_clock;

__global__ void k_sum(const uint64_t* p, uint64_t n, uint64_t* out) {
    uint64_t s = 0;
    for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) s += p[i];
    __shared__ uint64_t r[256];
    r[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t t = 0;
        for (int k = 0; k < 256; k++) t += r[k];
        out[0] = t;
    }
}

// ping-pong: wait for *ping == k (HBM, written by the host), answer *pong = k (pinned host memory);
// bounded by `rounds` and a 2 s budget of 100 MHz ticks per round
__global__ void k_pong(const uint32_t* ping, uint32_t* pong, uint32_t rounds) {
    if (threadIdx.x != 0) return;
    for (uint32_t k = 1; k <= rounds; k++) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(ping, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != k) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) return;
            __builtin_amdgcn_s_sleep(1);
        }
        __hip_atomic_store(pong, k, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

static double gbs(size_t bytes, clk::time_point t) {
    return bytes / std::chrono::duration<double>(clk::now() - t).count() / 1e9;
}

int main() {
    hipSetDevice(0);
    const size_t N = 64 << 10, REPS = 4000;
    std::vector<uint8_t> src(N);
    for (size_t i = 0; i < N; i++) src[i] = (uint8_t)(i * 131 + 7);
    uint8_t* pin = nullptr;
    hipHostMalloc((void**)&pin, N, hipHostMallocDefault);
    auto t = clk::now();
    for (size_t r = 0; r < REPS; r++) memcpy(pin, src.data(), N);
    printf("memcpy 64 KiB into pinned host memory: %.2f GB/s\n", gbs(N * REPS, t));
    uint64_t* d_out = nullptr;
    hipMalloc((void**)&d_out, 8);
    for (unsigned flag : {(unsigned)hipDeviceMallocFinegrained, (unsigned)hipDeviceMallocUncached}) {
        uint8_t* v = nullptr;
        hipError_t e = hipExtMallocWithFlags((void**)&v, N + 4096, flag);
        printf("flag %u: hipExtMallocWithFlags -> %s (%p)\n", flag, hipGetErrorString(e), (void*)v);
        if (e != hipSuccess) continue;
        hipPointerAttribute_t a;
        if (hipPointerGetAttributes(&a, v) == hipSuccess)
            printf("  attributes: type %d device %d hostPointer %p devicePointer %p\n", (int)a.type, a.device, a.hostPointer,
                   a.devicePointer);
        fflush(stdout);
        // the CPU touches it (a segfault here means: not host-mapped)
        t = clk::now();
        for (size_t r = 0; r < REPS; r++) memcpy(v, src.data(), N);
        _mm_sfence();
        printf("  memcpy 64 KiB into it from the CPU: %.2f GB/s\n", gbs(N * REPS, t));
        t = clk::now();
        for (size_t r = 0; r < 200; r++) {
            const __m256i* s = (const __m256i*)src.data();
            __m256i* d = (__m256i*)v;
            for (size_t i = 0; i < N / 32; i++) _mm256_stream_si256(d + i, _mm256_loadu_si256(s + i));
        }
        _mm_sfence();
        printf("  non-temporal 32-byte stores: %.2f GB/s\n", gbs(N * 200, t));
        uint64_t want = 0;
        for (size_t i = 0; i < N / 8; i++) want += ((const uint64_t*)src.data())[i];
        hipLaunchKernelGGL(k_sum, dim3(1), dim3(256), 0, 0, (const uint64_t*)v, N / 8, d_out);
        uint64_t got = 0;
        hipMemcpy(&got, d_out, 8, hipMemcpyDeviceToHost);
        printf("  GPU checksum of what the CPU wrote: %s\n", got == want ? "equal" : "DIFFERENT");
        volatile uint32_t* ping = (volatile uint32_t*)(v + N);
        uint32_t* pong = (uint32_t*)pin;
        *ping = 0;
        *(volatile uint32_t*)pong = 0;
        _mm_sfence();
        const uint32_t rounds = 2000;
        hipLaunchKernelGGL(k_pong, dim3(1), dim3(64), 0, 0, (const uint32_t*)(v + N), pong, rounds);
        std::vector<double> lat;
        bool ok = true;
        for (uint32_t k = 1; k <= rounds && ok; k++) {
            auto t1 = clk::now();
            *ping = k;
            _mm_sfence();
            while (__atomic_load_n(pong, __ATOMIC_ACQUIRE) != k)
                if (std::chrono::duration<double>(clk::now() - t1).count() > 1.0) {
                    ok = false;
                    break;
                }
            lat.push_back(std::chrono::duration<double, std::micro>(clk::now() - t1).count());
        }
        hipDeviceSynchronize();
        std::sort(lat.begin(), lat.end());
        printf("  ping (host -> HBM word) / pong (kernel -> pinned host word): %s, p50 %.2f us, p90 %.2f us\n",
               ok ? "ok" : "TIMED OUT", lat[lat.size() / 2], lat[lat.size() * 9 / 10]);
        fflush(stdout);
        hipFree(v);
    }
    return 0;
}
