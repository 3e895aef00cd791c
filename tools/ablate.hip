// tools/ablate.hip -- microbenchmarks that take the gear scan and BLAKE3 leaf kernels apart
// (diagnostic only; not part of the product).  Build: hipcc --offload-arch=gfx950 -O3 -std=c++17
// -I backuwup_amd/csrc tools/ablate.hip -o build_ab/ablate ; run on an MI355X.
//
// `ablate scan|b3|both|noload|nolds|copy|b3reg [seconds]` instead repeats one workload for that long (power sampling,
// tools/gpu_ablate_power.sh).  For a 4 GiB random buffer it times:
//   copy_strided   every lane reads its own 2 KiB strip in 128 B lines (the scan's pattern)
//   copy_coalesced every lane reads 16 B at consecutive addresses (the HBM ceiling)
//   scan_full      bw::k_scan exactly as shipped
//   scan_noload    the scan's arithmetic + LDS lookups on register-resident bytes (no HBM)
//   scan_nolds     the scan with the LDS gear lookup replaced by arithmetic on the byte
//   b3_noload      BLAKE3 compressions on register data (pure VALU rate)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <string>

#include "bw_cdc.hip"
#include "bw_blake3.hip"

using namespace bw;

#define CHECK(x)                                                                          \
    do {                                                                                  \
        hipError_t e = (x);                                                               \
        if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } \
    } while (0)

// 512 threads x 2 KiB strips = 1 MiB per block-tile; every byte read lies inside [0, n)
__global__ __launch_bounds__(512) void copy_strided(const uint8_t* __restrict__ data, uint64_t n, uint32_t* out) {
    uint32_t acc = 0;
    const uint64_t TILE = 512ull * 2048;
    for (uint64_t tile = blockIdx.x; (tile + 1) * TILE <= n; tile += gridDim.x) {
        const uint64_t ss = tile * TILE + (uint64_t)threadIdx.x * 2048;
        for (uint64_t p = ss; p < ss + 2048; p += 128) {
            const uint4* wp = (const uint4*)(data + p);
#pragma unroll
            for (int i = 0; i < 8; i++) { uint4 w = wp[i]; acc ^= w.x ^ w.y ^ w.z ^ w.w; }
        }
    }
    if (acc == 0x12345678) out[0] = acc;
}

__global__ __launch_bounds__(512) void copy_coalesced(const uint8_t* __restrict__ data, uint64_t n, uint32_t* out) {
    uint32_t acc = 0;
    const uint4* wp = (const uint4*)data;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 16; i += (uint64_t)gridDim.x * blockDim.x) {
        uint4 w = wp[i];
        acc ^= w.x ^ w.y ^ w.z ^ w.w;
    }
    if (acc == 0x12345678) out[0] = acc;
}

template <bool LDS>
__global__ __launch_bounds__(512, 4) void scan_noload(uint64_t n, Masks mk, uint32_t* out) {
    __shared__ __attribute__((aligned(16))) uint64_t s_gear[256 * GEAR_REP];
    for (int i = threadIdx.x; i < 256 * GEAR_REP; i += blockDim.x) s_gear[i] = c_gear[i / GEAR_REP];
    __syncthreads();
    const uint32_t lane_off = (threadIdx.x & 31) * 8;
    const uint32_t mlo = (uint32_t)mk.mask_pre, mhi = (uint32_t)(mk.mask_pre >> 32);
    uint32_t hits = 0;
    uint64_t h = 0;
    uint32_t seed = threadIdx.x * 0x9E3779B9u + blockIdx.x;
    const uint64_t lines = n / 128 / ((uint64_t)gridDim.x * blockDim.x);
    for (uint64_t line = 0; line < lines; line++) {
        uint32_t ww[32];
#pragma unroll
        for (int i = 0; i < 32; i++) { seed = seed * 1664525u + 1013904223u; ww[i] = seed; }
        uint32_t acc = 0xffffffffu;
#pragma unroll
        for (int i = 0; i < 32; i += 2) {
            uint64_t g[8];
#pragma unroll
            for (int q = 0; q < 8; q++) {
                const uint32_t word = ww[i + q / 4];
                if (LDS) g[q] = gear_fetch(word, BW_SEL(q % 4), lane_off, s_gear);
                else g[q] = (uint64_t)((word >> (8 * (q % 4))) & 0xff) * 0x9E3779B97F4A7C15ull;
            }
#pragma unroll
            for (int q = 0; q < 8; q += 2) {
                h = (h << 1) + g[q];
                const uint32_t t0 = mask_test(h, mlo, mhi);
                h = (h << 1) + g[q + 1];
                const uint32_t t1 = mask_test(h, mlo, mhi);
                acc = min(acc, min(t0, t1));
            }
        }
        hits += acc == 0;
    }
    if (hits == 0x7fffffff) out[0] = hits + (uint32_t)h;
}

__global__ __launch_bounds__(256) void b3_noload(uint64_t blocks_per_lane, uint32_t* out) {
    uint32_t cv[8];
    b3_iv(cv);
    uint32_t m[16];
#pragma unroll
    for (int i = 0; i < 16; i++) m[i] = threadIdx.x * 16 + i;
    for (uint64_t b = 0; b < blocks_per_lane; b++) {
        m[0] ^= (uint32_t)b;
        b3_compress(cv, m, 64, b, 0);
    }
    if (cv[0] == 0x12345678) out[0] = cv[1];
}

template <typename F>
static float timeit(F f, int reps = 5) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    f();
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    for (int i = 0; i < reps; i++) f();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

// Repeats f for `seconds` (power sampling: tools/gpu_ablate_power.sh runs amd-smi beside it).
template <class F>
static void hold(F f, double seconds, const char* name, double gb_per_call) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    CHECK(hipEventRecord(a, 0));
    int calls = 0;
    float ms = 0;
    while (ms < seconds * 1e3) {
        for (int i = 0; i < 20; i++) f();
        calls += 20;
        CHECK(hipEventRecord(b, 0));
        CHECK(hipEventSynchronize(b));
        CHECK(hipEventElapsedTime(&ms, a, b));
    }
    printf("hold %-8s %d calls in %.3f s: %.3f ms/call, %.1f GB/s\n", name, calls, ms / 1e3, ms / calls,
           gb_per_call * calls / (ms / 1e3));
    fflush(stdout);
}

int main(int argc, char** argv) {
    const char* hold_what = argc > 1 ? argv[1] : nullptr;  // "scan", "b3" or "both": power mode
    const double hold_s = argc > 2 ? atof(argv[2]) : 8.0;
    const uint64_t n = 4ull << 30;
    uint8_t* d;
    uint32_t *out, *tc, *ovf;
    uint64_t *ts, *sctr;
    CHECK(hipMalloc(&d, n));
    CHECK(hipMalloc(&out, 64));
    const uint64_t tiles = n / SCAN_TILE;
    CHECK(hipMalloc(&tc, tiles * 4));
    CHECK(hipMalloc(&ts, tiles * SCAN_CAP * 8));
    CHECK(hipMalloc(&ovf, tiles * 4));
    CHECK(hipMalloc(&sctr, 16 * 8));
    {
        uint32_t* h = (uint32_t*)malloc(1 << 26);
        for (int i = 0; i < (1 << 24); i++) h[i] = (uint32_t)rand() * 2654435761u ^ (uint32_t)rand();
        for (uint64_t o = 0; o < n; o += 1 << 26) CHECK(hipMemcpy(d + o, h, 1 << 26, hipMemcpyHostToDevice));
        free(h);
    }
    Masks mk;
    mk.min = 262144; mk.avg = 1048576; mk.max = 3145728; mk.s0 = 262144;
    mk.mask_s = 0x0000d91767537000ull; mk.mask_l = 0x0000d91707537000ull; mk.mask_pre = mk.mask_l;
    mk.pre_shift = 16; mk.pre_hi = (uint32_t)((mk.mask_pre << 16) >> 32);
    mk.tile_shift = SCAN_TILE_SHIFT;  // launch_scan picks the kernel by tile size
    const double gb = n / 1e9;
    float t;
    t = timeit([&] { hipLaunchKernelGGL(copy_strided, dim3(1024), dim3(512), 0, 0, d, n, out); });
    printf("copy_strided   %8.3f ms %8.1f GB/s\n", t, gb / t * 1e3);
    t = timeit([&] { hipLaunchKernelGGL(copy_coalesced, dim3(4096), dim3(512), 0, 0, d, n, out); });
    printf("copy_coalesced %8.3f ms %8.1f GB/s\n", t, gb / t * 1e3);
    auto scan_all = [&](hipStream_t st) {
        CHECK(hipMemsetAsync(sctr, 0, 16 * 8, st));
        launch_scan(st, d, n, tiles, mk, tc, ts, ovf, sctr, 16);
    };
    if (hold_what && std::string(hold_what) == "noload") {
        hold([&] { hipLaunchKernelGGL(scan_noload<true>, dim3(512), dim3(512), 0, 0, n, mk, out); }, hold_s, "noload", gb);
        return 0;
    }
    if (hold_what && std::string(hold_what) == "nolds") {
        hold([&] { hipLaunchKernelGGL(scan_noload<false>, dim3(512), dim3(512), 0, 0, n, mk, out); }, hold_s, "nolds", gb);
        return 0;
    }
    if (hold_what && std::string(hold_what) == "copy") {
        hold([&] { hipLaunchKernelGGL(copy_strided, dim3(1024), dim3(512), 0, 0, d, n, out); }, hold_s, "copy", gb);
        return 0;
    }
    if (hold_what && std::string(hold_what) == "copyhbm") {
        hold([&] { hipLaunchKernelGGL(copy_coalesced, dim3(4096), dim3(512), 0, 0, d, n, out); }, hold_s, "copyhbm", gb);
        return 0;
    }
    if (hold_what && std::string(hold_what) == "copymall") {  // 128 MiB, re-read: Infinity Cache resident
        const uint64_t m = 128ull << 20;
        hold([&] { for (int r = 0; r < 8; r++) hipLaunchKernelGGL(copy_coalesced, dim3(2048), dim3(512), 0, 0, d, m, out); },
             hold_s, "copymall", 8 * m / 1e9);
        return 0;
    }
    if (hold_what && std::string(hold_what) == "copyl2") {  // 16 MiB, re-read: L2 resident (4 MiB per XCD)
        const uint64_t m = 16ull << 20;
        hold([&] { for (int r = 0; r < 64; r++) hipLaunchKernelGGL(copy_coalesced, dim3(2048), dim3(512), 0, 0, d, m, out); },
             hold_s, "copyl2", 64 * m / 1e9);
        return 0;
    }
    if (hold_what && std::string(hold_what) == "b3reg") {
        const uint64_t lanes = 256ull * 4096, bpl = n / 64 / lanes;
        hold([&] { hipLaunchKernelGGL(b3_noload, dim3(4096), dim3(256), 0, 0, bpl, out); }, hold_s, "b3reg", gb);
        return 0;
    }
    if (!hold_what) {
    t = timeit([&] { scan_all(0); });
    printf("scan_full      %8.3f ms %8.1f GB/s\n", t, gb / t * 1e3);
    t = timeit([&] { launch_scan(0, d, n, tiles, mk, tc, ts, ovf, sctr, 8); });
    printf("scan_b512      %8.3f ms %8.1f GB/s (8-wave blocks: leaves LDS for a co-resident kernel)\n", t, gb / t * 1e3);
    t = timeit([&] { hipLaunchKernelGGL(scan_noload<true>, dim3(512), dim3(512), 0, 0, n, mk, out); });
    printf("scan_noload    %8.3f ms %8.1f GB/s\n", t, gb / t * 1e3);
    t = timeit([&] { hipLaunchKernelGGL(scan_noload<false>, dim3(512), dim3(512), 0, 0, n, mk, out); });
    printf("scan_nolds     %8.3f ms %8.1f GB/s (no LDS, no HBM)\n", t, gb / t * 1e3);
    }
    {  // the shipped BLAKE3 kernels on 4096 blobs of 1 MiB (one unaligned start per blob)
        const uint64_t nb = 4096, blen = (1ull << 20) - 64;
        uint64_t *ctr, *bs, *bl, *bg, *fe, *gh;
        uint32_t *bf, *bk, *cv;
        uint8_t* dig;
        CHECK(hipMalloc(&ctr, 16 * 8)); CHECK(hipMalloc(&bs, nb * 8)); CHECK(hipMalloc(&bl, nb * 8));
        CHECK(hipMalloc(&bg, nb * 8)); CHECK(hipMalloc(&fe, nb * 8)); CHECK(hipMalloc(&gh, nb * 8));
        CHECK(hipMalloc(&bf, nb * 4)); CHECK(hipMalloc(&bk, nb * 4)); CHECK(hipMalloc(&dig, nb * 32));
        const uint64_t groups_per = (blen / 1024 + 1 + 3) / 4;
        CHECK(hipMalloc(&cv, nb * groups_per * 32));
        uint64_t hc[16] = {0};
        hc[C_NBLOBS] = nb; hc[C_NGROUPS] = nb * groups_per;
        CHECK(hipMemcpy(ctr, hc, sizeof hc, hipMemcpyHostToDevice));
        uint64_t* tmp = (uint64_t*)malloc(nb * 8 * 3);
        for (uint64_t i = 0; i < nb; i++) { tmp[i] = i * (1ull << 20) + 17; tmp[nb + i] = blen; tmp[2 * nb + i] = i * groups_per; }
        CHECK(hipMemcpy(bs, tmp, nb * 8, hipMemcpyHostToDevice));
        CHECK(hipMemcpy(bl, tmp + nb, nb * 8, hipMemcpyHostToDevice));
        CHECK(hipMemcpy(bg, tmp + 2 * nb, nb * 8, hipMemcpyHostToDevice));
        free(tmp);
        uint32_t* cv2;
        CHECK(hipMalloc(&cv2, nb * groups_per * 32));
        BlobArrays b{bs, bl, bg, bf, bk, fe, gh, nb, n};
        auto b3_all = [&](hipStream_t st) {
            launch_blake3(st, d, ctr, b, nb, nb * groups_per, cv, cv2, dig, (int)(blen / 1024 + 1), nullptr,
                          B3_LOADS_PAIRS, st);
        };
        if (hold_what) {
            hipStream_t s1, s2;
            CHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
            CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
            const std::string w = hold_what;
            if (w == "scan") hold([&] { scan_all(0); }, hold_s, "scan", gb);
            else if (w == "b3") hold([&] { b3_all(0); }, hold_s, "b3", nb * blen / 1e9);
            else if (w == "b3mall") {  // the same kernels over the first 128 blobs (128 MiB, cache-resident)
                const uint64_t nm = 128;
                uint64_t hc2[16] = {0};
                hc2[C_NBLOBS] = nm;
                hc2[C_NGROUPS] = nm * groups_per;
                uint64_t* ctr2;
                CHECK(hipMalloc(&ctr2, 16 * 8));
                CHECK(hipMemcpy(ctr2, hc2, sizeof hc2, hipMemcpyHostToDevice));
                BlobArrays b2{bs, bl, bg, bf, bk, fe, gh, nm, n};
                hold([&] {
                    for (int r = 0; r < 16; r++)
                        launch_blake3(0, d, ctr2, b2, nm, nm * groups_per, cv, cv2, dig, (int)(blen / 1024 + 1), nullptr,
                                      B3_LOADS_PAIRS, 0);
                }, hold_s, "b3mall", 16 * nm * blen / 1e9);
            }
            else hold([&] {
                scan_all(s1);
                b3_all(s2);
                CHECK(hipStreamSynchronize(s1));
                CHECK(hipStreamSynchronize(s2));
            }, hold_s, "both", gb + nb * blen / 1e9);
            return 0;
        }
        t = timeit([&] { b3_all(0); });
        printf("b3_full        %8.3f ms %8.1f GB/s (k_b3_groups + k_b3_upper, 4096 x 1 MiB blobs)\n", t,
               nb * blen / 1e9 / t * 1e3);
        const unsigned g = (unsigned)((nb * groups_per + 255) / 256);
#define B3V(P, W, name)                                                                                   \
        t = timeit([&] { hipLaunchKernelGGL((k_b3_groups<P, W, false>), dim3(g), dim3(256), 0, 0, d, ctr, b, cv, dig); }); \
        printf("%-14s %8.3f ms %8.1f GB/s (k_b3_groups only)\n", name, t, nb * blen / 1e9 / t * 1e3);
        B3V(true, 1, "b3g_pf")
        B3V(false, 1, "b3g_nopf")
        t = timeit([&] { hipLaunchKernelGGL((k_b3_groups<false, 1, true>), dim3(g), dim3(256), 0, 0, d, ctr, b, cv, dig); });
        printf("%-14s %8.3f ms %8.1f GB/s (k_b3_groups only)\n", "b3g_pairs", t, nb * blen / 1e9 / t * 1e3);
#undef B3V
        hipStream_t s1, s2;
        CHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
        CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
        for (int blk : {1024, 512}) {
            t = timeit([&] {
                CHECK(hipMemsetAsync(sctr, 0, 16 * 8, s1));
                launch_scan(s1, d, n, tiles, mk, tc, ts, ovf, sctr, blk == 1024 ? 16 : 8);
                b3_all(s2);
                CHECK(hipStreamSynchronize(s1));
                CHECK(hipStreamSynchronize(s2));
            });
            printf("scan%-4d||b3   %8.3f ms (scan of 4 GiB concurrently with b3 of 4 GiB on two streams)\n", blk, t);
        }
    }
    const uint64_t lanes = 256ull * 4096;
    const uint64_t bpl = n / 64 / lanes;
    t = timeit([&] { hipLaunchKernelGGL(b3_noload, dim3(4096), dim3(256), 0, 0, bpl, out); });
    printf("b3_noload      %8.3f ms %8.1f GB/s (compressions on registers, %llu blocks/lane)\n", t, gb / t * 1e3,
           (unsigned long long)bpl);
    return 0;
}
