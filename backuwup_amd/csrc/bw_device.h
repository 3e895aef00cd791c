// bw_device.h -- gfx950 device helpers shared by the backuwup_amd kernels.
//
// Everything here is integer/byte work on 64-wide wavefronts; no MFMA (the path is not a
// contraction).  BLAKE3 follows the spec restated in SURVEY.md A.4 (crate blake3 1.3.3, called
// at client/src/backup/filesystem/dir_packer.rs:286); the gear constants are fastcdc 3.0.3
// v2020 (dir_packer.rs:14,254-259), generated into bw_tables.inc by tools/gen_tables.py.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bw_tables.inc"

#define BW_WAVE 64

// Device bounds checks of the BW_DEBUG build (python backuwup_amd/build.py --debug ->
// libbackuwup_amd_debug.so): a failed check prints its location and traps the kernel.
#ifdef BW_DEBUG
#define BW_ASSERT(c)                                                              \
    do {                                                                          \
        if (!(c)) {                                                               \
            printf("BW_ASSERT failed %s:%d: %s\n", __FILE__, __LINE__, #c);       \
            __builtin_trap();                                                     \
        }                                                                         \
    } while (0)
#else
#define BW_ASSERT(c) \
    do {             \
    } while (0)
#endif

// ---------------------------------------------------------------- candidate records
// A gear candidate is a global byte position with the normalized-chunking test results in the
// two top bits: bit 63 = (g & mask_s) == 0, bit 62 = (g & mask_l) == 0.
#define BW_CAND_S (1ull << 63)
#define BW_CAND_L (1ull << 62)
#define BW_CAND_BLK (1ull << 61)  // scan record: a flagged 64-byte block (k_refine makes it exact)
#define BW_CAND_POS(c) ((c) & ((1ull << 61) - 1))
#define BW_NONE (~0ull)

// ---------------------------------------------------------------- wave primitives
__device__ __forceinline__ int bw_lane() { return __lane_id(); }

__device__ __forceinline__ uint64_t bw_shfl_up64(uint64_t v, int d) {
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    lo = __shfl_up(lo, d, BW_WAVE);
    hi = __shfl_up(hi, d, BW_WAVE);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t bw_shfl64(uint64_t v, int src) {
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    lo = __shfl(lo, src, BW_WAVE);
    hi = __shfl(hi, src, BW_WAVE);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t bw_wave_sum64(uint64_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
        lo = __shfl_xor(lo, d, BW_WAVE);
        hi = __shfl_xor(hi, d, BW_WAVE);
        v += ((uint64_t)hi << 32) | lo;
    }
    return v;
}

// Inclusive "shift-scan" of the gear recurrence h_i = (h_{i-1} << 1) + g_i across lanes:
// lane i returns sum_{j<=i} g_j << (i - j)  (mod 2^64).  Six shuffle steps.
__device__ __forceinline__ uint64_t bw_gear_scan(uint64_t g) {
    const int lane = bw_lane();
#pragma unroll
    for (int d = 1; d < BW_WAVE; d <<= 1) {
        uint64_t up = bw_shfl_up64(g, d);
        if (lane >= d) g += up << d;
    }
    return g;
}

// ---------------------------------------------------------------- BLAKE3
#define B3_CHUNK_START 1u
#define B3_CHUNK_END 2u
#define B3_PARENT 4u
#define B3_ROOT 8u
#define B3_LEAF_BYTES 1024u

__device__ __forceinline__ uint32_t b3_rotr(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }

#define B3_IV0 0x6A09E667u
#define B3_IV1 0xBB67AE85u
#define B3_IV2 0x3C6EF372u
#define B3_IV3 0xA54FF53Au
#define B3_IV4 0x510E527Fu
#define B3_IV5 0x9B05688Cu
#define B3_IV6 0x1F83D9ABu
#define B3_IV7 0x5BE0CD19u

// The two-operand xor / add of G are emitted in their VOP3 (e64) encodings: on gfx950 they issue
// faster than the VOP2 (e32) forms the compiler picks (tools/op_rate.hip: 2.7 vs 3.2-3.6 SIMD
// cycles per wave64 instruction at full occupancy; BLAKE3 from registers 4.05 vs 3.68 TB/s at 4
// waves/SIMD, tools/valu_rate.hip).  Non-volatile asm: the compiler still schedules them.
__device__ __forceinline__ uint32_t b3_xor(uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_xor_b32_e64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ uint32_t b3_add(uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_add_u32_e64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

#define B3_G(a, b, c, d, x, y)            \
    do {                                  \
        a = a + b + (x);                  \
        d = b3_rotr(b3_xor(d, a), 16);    \
        c = b3_add(c, d);                 \
        b = b3_rotr(b3_xor(b, c), 12);    \
        a = a + b + (y);                  \
        d = b3_rotr(b3_xor(d, a), 8);     \
        c = b3_add(c, d);                 \
        b = b3_rotr(b3_xor(b, c), 7);     \
    } while (0)

// One round on state v with the message words in schedule order s0..s15 (compile-time names).
#define B3_ROUND(m, s0, s1, s2, s3, s4, s5, s6, s7, s8, s9, s10, s11, s12, s13, s14, s15) \
    do {                                                                               \
        B3_G(v0, v4, v8, v12, m[s0], m[s1]);                                           \
        B3_G(v1, v5, v9, v13, m[s2], m[s3]);                                           \
        B3_G(v2, v6, v10, v14, m[s4], m[s5]);                                          \
        B3_G(v3, v7, v11, v15, m[s6], m[s7]);                                          \
        B3_G(v0, v5, v10, v15, m[s8], m[s9]);                                          \
        B3_G(v1, v6, v11, v12, m[s10], m[s11]);                                        \
        B3_G(v2, v7, v8, v13, m[s12], m[s13]);                                         \
        B3_G(v3, v4, v9, v14, m[s14], m[s15]);                                         \
    } while (0)

// BLAKE3 compression, chaining-value output (first 8 output words).  The message schedule is
// the spec permutation [2,6,3,10,7,0,4,13,1,11,12,5,9,14,15,8] applied round after round,
// spelled out so every message index is a compile-time register name.
__device__ __forceinline__ void b3_compress(uint32_t cv[8], const uint32_t m[16], uint32_t block_len,
                                            uint64_t counter, uint32_t flags) {
    uint32_t v0 = cv[0], v1 = cv[1], v2 = cv[2], v3 = cv[3], v4 = cv[4], v5 = cv[5], v6 = cv[6], v7 = cv[7];
    uint32_t v8 = B3_IV0, v9 = B3_IV1, v10 = B3_IV2, v11 = B3_IV3;
    uint32_t v12 = (uint32_t)counter, v13 = (uint32_t)(counter >> 32), v14 = block_len, v15 = flags;
    B3_ROUND(m, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
    B3_ROUND(m, 2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8);
    B3_ROUND(m, 3, 4, 10, 12, 13, 2, 7, 14, 6, 5, 9, 0, 11, 15, 8, 1);
    B3_ROUND(m, 10, 7, 12, 9, 14, 3, 13, 15, 4, 0, 11, 2, 5, 8, 1, 6);
    B3_ROUND(m, 12, 13, 9, 11, 15, 10, 14, 8, 7, 2, 5, 3, 0, 1, 6, 4);
    B3_ROUND(m, 9, 14, 11, 5, 8, 12, 15, 1, 13, 3, 0, 10, 2, 6, 4, 7);
    B3_ROUND(m, 11, 15, 5, 0, 1, 9, 8, 6, 14, 10, 2, 12, 3, 4, 7, 13);
    cv[0] = b3_xor(v0, v8); cv[1] = b3_xor(v1, v9); cv[2] = b3_xor(v2, v10); cv[3] = b3_xor(v3, v11);
    cv[4] = b3_xor(v4, v12); cv[5] = b3_xor(v5, v13); cv[6] = b3_xor(v6, v14); cv[7] = b3_xor(v7, v15);
}

__device__ __forceinline__ void b3_iv(uint32_t cv[8]) {
    cv[0] = B3_IV0; cv[1] = B3_IV1; cv[2] = B3_IV2; cv[3] = B3_IV3;
    cv[4] = B3_IV4; cv[5] = B3_IV5; cv[6] = B3_IV6; cv[7] = B3_IV7;
}

// parent node: out = compress(IV, left || right, 64, 0, PARENT | flags)
__device__ __forceinline__ void b3_parent(const uint32_t l[8], const uint32_t r[8], uint32_t flags, uint32_t out[8]) {
    uint32_t m[16];
#pragma unroll
    for (int i = 0; i < 8; i++) { m[i] = l[i]; m[8 + i] = r[i]; }
    b3_iv(out);
    b3_compress(out, m, 64, 0, B3_PARENT | flags);
}

// ---------------------------------------------------------------- clock stamps (diagnostic build)
// BW_CLOCK_STAMPS (libbackuwup_amd_clock.so only, tools/clock_windows.py): lane 0 of a wave stamps
// the 100 MHz real-time counter (s_memrealtime) and the shader clock counter (s_memtime) around a
// unit of work -- a scan tile, a leaf-pass wave -- into a device log, so the clock the chip held
// can be split by what ran beside it (what limits the overlap of the two passes).
#ifndef BW_CLOCK_STAMPS
#define BW_CLOCK_STAMPS 0
#endif
#if BW_CLOCK_STAMPS
struct ClockRec {
    uint32_t kind, pad;  // 0 = k_scan tile, 1 = k_b3_lines wave
    uint64_t t0, t1, c0, c1;
};
struct ClockLog {
    ClockRec* rec;
    unsigned long long cap, n;
    uint32_t on;
};
struct ClockStamp {
    ClockLog* L;
    uint64_t t0, c0;
    uint32_t kind;
    bool on;
    __device__ ClockStamp(ClockLog* l, uint32_t k) : L(l), t0(0), c0(0), kind(k) {
        on = L && L->on && (threadIdx.x & 63) == 0;
        if (on) {
            t0 = __builtin_amdgcn_s_memrealtime();
            c0 = __builtin_amdgcn_s_memtime();
        }
    }
    __device__ ~ClockStamp() {
        if (!on) return;
        const uint64_t t1 = __builtin_amdgcn_s_memrealtime(), c1 = __builtin_amdgcn_s_memtime();
        const unsigned long long i = atomicAdd(&L->n, 1ull);
        if (i < L->cap) L->rec[i] = ClockRec{kind, 0, t0, t1, c0, c1};
    }
};
#endif

