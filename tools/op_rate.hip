// tools/op_rate.hip -- issue cost (SIMD cycles per wave64 instruction) of the integer VALU
// instructions the hot path uses, on gfx950 (diagnostic only; not the product).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/op_rate.hip -o build_ab/op_rate
//
// Every lane keeps 8 independent accumulators and runs the instruction under test on each of
// them (inline asm, so the compiler emits exactly that encoding).  Launched with 1 and 8 waves
// per SIMD; cycles come from s_memtime / s_memrealtime stamps, so DVFS does not skew the result.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                                                   \
    do {                                                                                           \
        hipError_t e = (x);                                                                        \
        if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } \
    } while (0)

#define STAMP0()                                                                                   \
    uint64_t t0 = 0, r0 = 0;                                                                       \
    if (threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
#define STAMP1()                                                                                   \
    if (threadIdx.x == 0) {                                                                        \
        st[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;                                    \
        st[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;                            \
    }

#define OP32(name, text)                                                                           \
    __global__ __launch_bounds__(256) void name(uint32_t iters, uint32_t* out, uint64_t* st) {     \
        uint32_t r[8];                                                                             \
        const uint32_t x = threadIdx.x * 0x9e3779b9u, y = blockIdx.x | 0x10203u;                   \
        for (int i = 0; i < 8; i++) r[i] = x + i;                                                  \
        STAMP0();                                                                                  \
        for (uint32_t k = 0; k < iters; k++) {                                                     \
            _Pragma("unroll") for (int i = 0; i < 8; i++) asm volatile(text : "+v"(r[i]) : "v"(x), "v"(y)); \
        }                                                                                          \
        STAMP1();                                                                                  \
        uint32_t s = 0;                                                                            \
        for (int i = 0; i < 8; i++) s ^= r[i];                                                     \
        if (s == 0x12345678u) out[0] = s;                                                          \
    }

#define OP64(name, text)                                                                           \
    __global__ __launch_bounds__(256) void name(uint32_t iters, uint32_t* out, uint64_t* st) {     \
        uint64_t r[8];                                                                             \
        const uint64_t x = threadIdx.x * 0x9e3779b97f4a7c15ull;                                    \
        for (int i = 0; i < 8; i++) r[i] = x + i;                                                  \
        STAMP0();                                                                                  \
        for (uint32_t k = 0; k < iters; k++) {                                                     \
            _Pragma("unroll") for (int i = 0; i < 8; i++) asm volatile(text : "+v"(r[i]) : "v"(x)); \
        }                                                                                          \
        STAMP1();                                                                                  \
        uint64_t s = 0;                                                                            \
        for (int i = 0; i < 8; i++) s ^= r[i];                                                     \
        if (s == 0x12345678u) out[0] = (uint32_t)s;                                                \
    }

OP32(k_add, "v_add_u32_e32 %0, %1, %0")
OP32(k_add_e64, "v_add_u32_e64 %0, %0, %1")
OP32(k_xor, "v_xor_b32_e32 %0, %1, %0")
OP32(k_xor_e64, "v_xor_b32_e64 %0, %0, %1")
OP32(k_and, "v_and_b32_e32 %0, %1, %0")
OP32(k_add3, "v_add3_u32 %0, %0, %1, %2")
OP32(k_alignbit, "v_alignbit_b32 %0, %0, %0, 12")
OP32(k_alignbyte, "v_alignbyte_b32 %0, %0, %1, 1")
OP32(k_perm, "v_perm_b32 %0, %0, %1, %2")
OP32(k_min3, "v_min3_u32 %0, %0, %1, %2")
OP32(k_xad, "v_xad_u32 %0, %0, %1, %2")
OP32(k_bitop3, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96")
OP32(k_lshl_or, "v_lshl_or_b32 %0, %0, 7, %1")
OP32(k_lshrrev, "v_lshrrev_b32_e32 %0, 7, %0")
OP32(k_pk_add_u16, "v_pk_add_u16 %0, %0, %1")
OP64(k_lshl_add_u64, "v_lshl_add_u64 %0, %0, 1, %1")
OP64(k_lshlrev_b64, "v_lshlrev_b64 %0, 1, %0")

static double clock_ghz(uint64_t* d_st, int nblk) {
    uint64_t* h = (uint64_t*)malloc(nblk * 16);
    CHECK(hipMemcpy(h, d_st, nblk * 16, hipMemcpyDeviceToHost));
    double c = 0, r = 0;
    for (int i = 0; i < nblk; i++) { c += h[2 * i]; r += h[2 * i + 1]; }
    free(h);
    return c / r * 0.1;
}

typedef void (*Kern)(uint32_t, uint32_t*, uint64_t*);

int main() {
    uint32_t* out;
    uint64_t* st;
    CHECK(hipMalloc(&out, 64));
    CHECK(hipMalloc(&st, 256 * 8 * 16));
    struct { const char* name; Kern k; } ks[] = {
        {"v_add_u32_e32", k_add},       {"v_add_u32_e64", k_add_e64},   {"v_xor_b32_e32", k_xor},
        {"v_xor_b32_e64", k_xor_e64},   {"v_and_b32_e32", k_and},       {"v_add3_u32", k_add3},
        {"v_alignbit_b32", k_alignbit}, {"v_alignbyte_b32", k_alignbyte}, {"v_perm_b32", k_perm},
        {"v_min3_u32", k_min3},         {"v_xad_u32", k_xad},           {"v_bitop3_b32", k_bitop3},
        {"v_lshl_or_b32", k_lshl_or},   {"v_lshrrev_b32", k_lshrrev},   {"v_pk_add_u16", k_pk_add_u16},
        {"v_lshl_add_u64", k_lshl_add_u64}, {"v_lshlrev_b64", k_lshlrev_b64},
    };
    const uint32_t iters = 40000;
    printf("%-18s %10s %10s %10s %10s\n", "instruction", "cyc@1w/S", "cyc@8w/S", "wall@1w/S", "wall@8w/S");
    for (auto& e : ks) {
        double cyc[2], wall[2];
        int wi = 0;
        for (int wps : {1, 8}) {
            const int nblk = 256 * wps;
            hipLaunchKernelGGL(e.k, dim3(nblk), dim3(256), 0, 0, iters, out, st);
            CHECK(hipDeviceSynchronize());
            hipEvent_t ea, eb;
            CHECK(hipEventCreate(&ea));
            CHECK(hipEventCreate(&eb));
            CHECK(hipEventRecord(ea));
            hipLaunchKernelGGL(e.k, dim3(nblk), dim3(256), 0, 0, iters, out, st);
            CHECK(hipEventRecord(eb));
            CHECK(hipDeviceSynchronize());
            float ms;
            CHECK(hipEventElapsedTime(&ms, ea, eb));
            const double ghz = clock_ghz(st, nblk);
            // wall-clock view: every SIMD of the chip retired wps * iters * 8 wave-instructions
            wall[wi] = ms * 1e-3 * ghz * 1e9 / ((double)iters * 8 * wps);
            // stamps are per block (one wave per SIMD of it): cycles the block spent / its instructions
            uint64_t* h = (uint64_t*)malloc(nblk * 16);
            CHECK(hipMemcpy(h, st, nblk * 16, hipMemcpyDeviceToHost));
            double c = 0;
            for (int i = 0; i < nblk; i++) c += h[2 * i];
            free(h);
            // each block's wave 0 measured its own duration; with wps waves sharing a SIMD the SIMD
            // retired wps * iters * 8 instructions in that time
            cyc[wi++] = (c / nblk) / ((double)iters * 8 * wps);
        }
        printf("%-18s %10.2f %10.2f %10.2f %10.2f\n", e.name, cyc[0], cyc[1], wall[0], wall[1]);
    }
    return 0;
}
