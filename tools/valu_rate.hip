// tools/valu_rate.hip -- how many wave64 integer VALU instructions one SIMD retires per clock on
// gfx950, and the BLAKE3 compression rate from registers (diagnostic only; not the product).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I backuwup_amd/csrc tools/valu_rate.hip
//        -o build_ab/valu_rate
//
// chain<ILP>: every lane runs ILP independent xor/add/alignbit chains; launched with 1..8 waves
// per SIMD.  The in-kernel clock comes from s_memtime / s_memrealtime (100 MHz) stamps of wave 0
// of every block, so cycles per instruction do not depend on the DVFS state.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "bw_device.h"

#define CHECK(x)                                                                                   \
    do {                                                                                           \
        hipError_t e = (x);                                                                        \
        if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } \
    } while (0)

template <int ILP>
__global__ __launch_bounds__(256) void chain(uint32_t iters, uint32_t* out, uint64_t* stamps) {
    uint32_t a[ILP], b[ILP];
#pragma unroll
    for (int i = 0; i < ILP; i++) { a[i] = threadIdx.x * 7 + i; b[i] = blockIdx.x + i * 13; }
    uint64_t t0 = 0, r0 = 0;
    if (threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    for (uint32_t k = 0; k < iters; k++) {
#pragma unroll
        for (int i = 0; i < ILP; i++) {  // 4 VALU per chain per iteration
            a[i] = a[i] + b[i];
            b[i] = __builtin_amdgcn_alignbit(b[i] ^ a[i], b[i] ^ a[i], 12);
            a[i] ^= k;
        }
    }
    if (threadIdx.x == 0) {
        const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        stamps[2 * blockIdx.x] = t1 - t0;
        stamps[2 * blockIdx.x + 1] = r1 - r0;
    }
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < ILP; i++) s += a[i] ^ b[i];
    if (s == 0x12345678) out[0] = s;
}

__global__ __launch_bounds__(256) void b3_regs(uint32_t blocks_per_lane, uint32_t* out, uint64_t* stamps) {
    uint32_t cv[8];
    b3_iv(cv);
    uint32_t m[16];
#pragma unroll
    for (int i = 0; i < 16; i++) m[i] = threadIdx.x * 16 + i;
    uint64_t t0 = 0, r0 = 0;
    if (threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    for (uint32_t b = 0; b < blocks_per_lane; b++) {
        m[0] ^= b;
        b3_compress(cv, m, 64, b, 0);
    }
    if (threadIdx.x == 0) {
        const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        stamps[2 * blockIdx.x] = t1 - t0;
        stamps[2 * blockIdx.x + 1] = r1 - r0;
    }
    if (cv[0] == 0x12345678) out[0] = cv[1];
}

// The same compression with the G function's 2-operand xor/add forced into VOP3 (e64) encodings
#define X64(a, b) ({ uint32_t r_; asm("v_xor_b32_e64 %0, %1, %2" : "=v"(r_) : "v"(a), "v"(b)); r_; })
#define A64(a, b) ({ uint32_t r_; asm("v_add_u32_e64 %0, %1, %2" : "=v"(r_) : "v"(a), "v"(b)); r_; })
#define G64(a, b, c, d, x, y)                 \
    do {                                      \
        a = a + b + (x);                      \
        d = b3_rotr(X64(d, a), 16);           \
        c = A64(c, d);                        \
        b = b3_rotr(X64(b, c), 12);           \
        a = a + b + (y);                      \
        d = b3_rotr(X64(d, a), 8);            \
        c = A64(c, d);                        \
        b = b3_rotr(X64(b, c), 7);            \
    } while (0)
#define R64(m, s0, s1, s2, s3, s4, s5, s6, s7, s8, s9, s10, s11, s12, s13, s14, s15) \
    do {                                                                           \
        G64(v0, v4, v8, v12, m[s0], m[s1]);                                        \
        G64(v1, v5, v9, v13, m[s2], m[s3]);                                        \
        G64(v2, v6, v10, v14, m[s4], m[s5]);                                       \
        G64(v3, v7, v11, v15, m[s6], m[s7]);                                       \
        G64(v0, v5, v10, v15, m[s8], m[s9]);                                       \
        G64(v1, v6, v11, v12, m[s10], m[s11]);                                     \
        G64(v2, v7, v8, v13, m[s12], m[s13]);                                      \
        G64(v3, v4, v9, v14, m[s14], m[s15]);                                      \
    } while (0)

__device__ __forceinline__ void b3_compress64(uint32_t cv[8], const uint32_t m[16], uint32_t block_len,
                                              uint64_t counter, uint32_t flags) {
    uint32_t v0 = cv[0], v1 = cv[1], v2 = cv[2], v3 = cv[3], v4 = cv[4], v5 = cv[5], v6 = cv[6], v7 = cv[7];
    uint32_t v8 = B3_IV0, v9 = B3_IV1, v10 = B3_IV2, v11 = B3_IV3;
    uint32_t v12 = (uint32_t)counter, v13 = (uint32_t)(counter >> 32), v14 = block_len, v15 = flags;
    R64(m, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
    R64(m, 2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8);
    R64(m, 3, 4, 10, 12, 13, 2, 7, 14, 6, 5, 9, 0, 11, 15, 8, 1);
    R64(m, 10, 7, 12, 9, 14, 3, 13, 15, 4, 0, 11, 2, 5, 8, 1, 6);
    R64(m, 12, 13, 9, 11, 15, 10, 14, 8, 7, 2, 5, 3, 0, 1, 6, 4);
    R64(m, 9, 14, 11, 5, 8, 12, 15, 1, 13, 3, 0, 10, 2, 6, 4, 7);
    R64(m, 11, 15, 5, 0, 1, 9, 8, 6, 14, 10, 2, 12, 3, 4, 7, 13);
    cv[0] = v0 ^ v8; cv[1] = v1 ^ v9; cv[2] = v2 ^ v10; cv[3] = v3 ^ v11;
    cv[4] = v4 ^ v12; cv[5] = v5 ^ v13; cv[6] = v6 ^ v14; cv[7] = v7 ^ v15;
}

__global__ __launch_bounds__(256) void b3_regs64(uint32_t blocks_per_lane, uint32_t* out, uint64_t* stamps) {
    uint32_t cv[8];
    b3_iv(cv);
    uint32_t m[16];
#pragma unroll
    for (int i = 0; i < 16; i++) m[i] = threadIdx.x * 16 + i;
    uint64_t t0 = 0, r0 = 0;
    if (threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    for (uint32_t b = 0; b < blocks_per_lane; b++) {
        m[0] ^= b;
        b3_compress64(cv, m, 64, b, 0);
    }
    if (threadIdx.x == 0) {
        const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        stamps[2 * blockIdx.x] = t1 - t0;
        stamps[2 * blockIdx.x + 1] = r1 - r0;
    }
    if (cv[0] == 0x12345678) out[0] = cv[1];
}

static double clock_ghz(uint64_t* d_st, int nblk) {
    uint64_t* h = (uint64_t*)malloc(nblk * 16);
    CHECK(hipMemcpy(h, d_st, nblk * 16, hipMemcpyDeviceToHost));
    double c = 0, r = 0;
    for (int i = 0; i < nblk; i++) { c += h[2 * i]; r += h[2 * i + 1]; }
    free(h);
    return c / r * 0.1;  // memrealtime ticks at 100 MHz
}

template <typename F>
static float timeit(F f, int reps = 3) {
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

int main() {
    uint32_t* out;
    uint64_t* st;
    CHECK(hipMalloc(&out, 64));
    CHECK(hipMalloc(&st, 256 * 8 * 16 * 16));
    const int ncu = 256, simds = 4 * ncu;
    printf("# chain: wave-instr per SIMD per clock (4 VALU per chain-iteration)\n");
    for (int wps = 1; wps <= 8; wps *= 2) {
        const int nblk = ncu * wps;  // 256-thread blocks = one wave per SIMD each
        const uint32_t iters = 20000;
        auto run = [&](auto kern, int ilp) {
            float ms = timeit([&] { hipLaunchKernelGGL(kern, dim3(nblk), dim3(256), 0, 0, iters, out, st); });
            const double ghz = clock_ghz(st, nblk);
            const double winstr = (double)nblk * 4 * iters * ilp * 4;  // waves * iters * ilp * 4 VALU
            const double per_simd_clk = winstr / simds / (ms * 1e-3 * ghz * 1e9);
            printf("waves/SIMD %d ILP %d: %.3f ms, clock %.2f GHz, %.3f wave-instr/SIMD/clk, %.1f T lane-ops/s\n",
                   wps, ilp, ms, ghz, per_simd_clk, winstr * 64 / (ms * 1e-3) / 1e12);
        };
        run(chain<1>, 1);
        run(chain<4>, 4);
        run(chain<8>, 8);
    }
    for (int variant = 0; variant < 2; variant++) {
        printf("# BLAKE3 compress from registers (64 B per compression per lane)%s\n",
               variant ? ", G's xor/add as VOP3 (e64)" : "");
        for (int wps = 1; wps <= 8; wps *= 2) {
            const int nblk = ncu * wps;
            const uint32_t bpl = 4000;
            float ms = timeit([&] {
                if (variant) hipLaunchKernelGGL(b3_regs64, dim3(nblk), dim3(256), 0, 0, bpl, out, st);
                else hipLaunchKernelGGL(b3_regs, dim3(nblk), dim3(256), 0, 0, bpl, out, st);
            });
            const double ghz = clock_ghz(st, nblk);
            const double bytes = (double)nblk * 256 * bpl * 64;
            printf("waves/SIMD %d: %.3f ms, clock %.2f GHz, %.1f GB/s of message, %.3f B/clk/CU\n", wps, ms, ghz,
                   bytes / (ms * 1e-3) / 1e9, bytes / (ms * 1e-3) / (ghz * 1e9) / ncu);
        }
    }
    return 0;
}
