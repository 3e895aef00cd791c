// tools/fetch_cal.hip -- FETCH_SIZE calibration and read-bandwidth ceilings for the access
// patterns of the hot path (diagnostic only; not the product).  Every kernel reads each byte of
// a 4 GiB buffer exactly once, so the algorithmic byte count is known; run under
//   rocprofv3 --kernel-trace --pmc FETCH_SIZE -- build_ab/fetch_cal
// and compare FETCH_SIZE per dispatch with 4 GiB.
//   rd_coalesced  16 B per lane, consecutive lanes consecutive (the guide's calibrated case)
//   rd_scan64     k_scan's pattern: per instruction 16 strips x 64 B (4 lanes per strip), the
//                 strip's next 64 B one step later
//   rd_scan128    8 lanes per strip: every instruction covers whole 128 B lines
//   rd_leaf       k_b3_groups' pattern: each lane walks its own 4 KiB group, 64 B per step
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                                                   \
    do {                                                                                           \
        hipError_t e = (x);                                                                        \
        if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } \
    } while (0)

constexpr uint64_t STRIP = 2048, TILE = 64 * STRIP;

__global__ __launch_bounds__(512) void rd_coalesced(const uint8_t* __restrict__ d, uint64_t n, uint32_t* out) {
    uint32_t acc = 0;
    const uint4* p = (const uint4*)d;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 16; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// one wave per 128 KiB tile (64 strips of 2 KiB); per step each lane issues 4 loads
template <int LANES_PER_STRIP>
__global__ __launch_bounds__(1024) void rd_scan(const uint8_t* __restrict__ d, uint64_t n, uint32_t* out) {
    constexpr int SPI = 64 / LANES_PER_STRIP;        // strips per instruction
    constexpr int SEG = 16 * LANES_PER_STRIP;        // bytes of a strip per instruction
    constexpr int GROUPS = 64 / SPI;                 // instructions to cover all 64 strips per step
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t acc = 0;
    const uint64_t ntiles = n / TILE, nw = (uint64_t)gridDim.x * 16;
    for (uint64_t t = (uint64_t)blockIdx.x * 16 + wid; t < ntiles; t += nw) {
        const uint8_t* src = d + t * TILE + (uint64_t)(lane / LANES_PER_STRIP) * STRIP + (lane % LANES_PER_STRIP) * 16;
        for (int step = 0; step < (int)(STRIP / SEG); step++) {
#pragma unroll
            for (int g = 0; g < GROUPS; g++) {
                const uint4 v = *(const uint4*)(src + (uint64_t)g * SPI * STRIP + step * SEG);
                acc ^= v.x ^ v.y ^ v.z ^ v.w;
            }
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ __launch_bounds__(256) void rd_leaf(const uint8_t* __restrict__ d, uint64_t n, uint32_t* out) {
    uint32_t acc = 0;
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g * 4096 + 4096 <= n) {
        const uint4* p = (const uint4*)(d + g * 4096);
        for (int b = 0; b < 64; b++) {
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const uint4 v = p[b * 4 + q];
                acc ^= v.x ^ v.y ^ v.z ^ v.w;
            }
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main() {
    const uint64_t n = 4ull << 30;
    uint8_t* d;
    uint32_t* out;
    CHECK(hipMalloc(&d, n));
    CHECK(hipMalloc(&out, 64));
    CHECK(hipMemset(d, 0x5a, n));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    auto timed = [&](const char* name, auto launch) {
        launch();
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(a));
        for (int i = 0; i < 3; i++) launch();
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        printf("%-14s %8.3f ms  %8.1f GB/s\n", name, ms / 3, n / (ms / 3 * 1e-3) / 1e9);
    };
    timed("rd_coalesced", [&] { hipLaunchKernelGGL(rd_coalesced, dim3(4096), dim3(512), 0, 0, d, n, out); });
    timed("rd_scan64", [&] { hipLaunchKernelGGL(rd_scan<4>, dim3(512), dim3(1024), 0, 0, d, n, out); });
    timed("rd_scan128", [&] { hipLaunchKernelGGL(rd_scan<8>, dim3(512), dim3(1024), 0, 0, d, n, out); });
    timed("rd_leaf", [&] { hipLaunchKernelGGL(rd_leaf, dim3((unsigned)(n / 4096 / 256)), dim3(256), 0, 0, d, n, out); });
    return 0;
}
