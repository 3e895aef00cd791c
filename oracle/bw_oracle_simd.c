/*
 * bw_oracle_simd.c -- AVX-512 BLAKE3 for the CPU baseline.  TEST INFRASTRUCTURE ONLY.
 *
 * The reference's blake3 1.3.3 crate (Cargo.lock:149-159) hashes a large input with its SIMD
 * `hash_many` backends (SSE4.1 / AVX2 / AVX-512, picked at run time): 16 chunks (or 16 parent
 * nodes) compressed at once, one per 32-bit vector lane.  This file restates that strategy so the
 * CPU baseline runs at the reference's own speed on the GPU box's host cores (AMD EPYC 9575F,
 * AVX-512), instead of the scalar restatement's.  Same tree as orc_blake3 (bw_oracle.c §3):
 *   - full 1024-byte chunks 16 at a time, lanes = consecutive chunks (counter = chunk index);
 *   - the ragged last chunk and any chunks left over from the 16-groups, scalar;
 *   - parents level by level (pairs of adjacent nodes, an odd last node carried up -- the spec's
 *     "left subtree = largest power of two" tree), 16 parents at a time, the root parent scalar
 *     with the ROOT flag.
 * Bit-exactness against the scalar orc_blake3 is a test (tests/test_oracle.py).  Without
 * AVX-512 on the host, orc_blake3_fast falls back to orc_blake3.
 */
#include <immintrin.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "bw_oracle.h"

#define T512 __attribute__((target("avx512f")))

enum { CHUNK_START = 1, CHUNK_END = 2, PARENT = 4, ROOT = 8 };
static const uint32_t IV[8] = {0x6A09E667, 0xBB67AE85, 0x3C6EF372, 0xA54FF53A,
                               0x510E527F, 0x9B05688C, 0x1F83D9AB, 0x5BE0CD19};
/* message word order of each of the 7 rounds (the permutation applied round after round) */
static const uint8_t SCHED[7][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8},
    {3, 4, 10, 12, 13, 2, 7, 14, 6, 5, 9, 0, 11, 15, 8, 1}, {10, 7, 12, 9, 14, 3, 13, 15, 4, 0, 11, 2, 5, 8, 1, 6},
    {12, 13, 9, 11, 15, 10, 14, 8, 7, 2, 5, 3, 0, 1, 6, 4}, {9, 14, 11, 5, 8, 12, 15, 1, 13, 3, 0, 10, 2, 6, 4, 7},
    {11, 15, 5, 0, 1, 9, 8, 6, 14, 10, 2, 12, 3, 4, 7, 13}};

#define ADD(a, b) _mm512_add_epi32(a, b)
#define XOR(a, b) _mm512_xor_si512(a, b)
#define G(a, b, c, d, x, y)                     \
    do {                                        \
        a = ADD(ADD(a, b), x);                  \
        d = _mm512_ror_epi32(XOR(d, a), 16);    \
        c = ADD(c, d);                          \
        b = _mm512_ror_epi32(XOR(b, c), 12);    \
        a = ADD(ADD(a, b), y);                  \
        d = _mm512_ror_epi32(XOR(d, a), 8);     \
        c = ADD(c, d);                          \
        b = _mm512_ror_epi32(XOR(b, c), 7);     \
    } while (0)

/* 16 x 16 transpose of u32: row r = lane r's 16 words in -> vector w = word w of every lane. */
T512 static void transpose16(__m512i r[16]) {
    __m512i a[16], b[16];
    for (int i = 0; i < 8; i++) {
        a[2 * i] = _mm512_unpacklo_epi32(r[2 * i], r[2 * i + 1]);
        a[2 * i + 1] = _mm512_unpackhi_epi32(r[2 * i], r[2 * i + 1]);
    }
    for (int j = 0; j < 4; j++) {  /* b[4j + w], 128-bit lane q = word 4q + w of rows 4j..4j+3 */
        b[4 * j + 0] = _mm512_unpacklo_epi64(a[4 * j], a[4 * j + 2]);
        b[4 * j + 1] = _mm512_unpackhi_epi64(a[4 * j], a[4 * j + 2]);
        b[4 * j + 2] = _mm512_unpacklo_epi64(a[4 * j + 1], a[4 * j + 3]);
        b[4 * j + 3] = _mm512_unpackhi_epi64(a[4 * j + 1], a[4 * j + 3]);
    }
    for (int w = 0; w < 4; w++) {  /* 4 x 4 transpose of 128-bit lanes */
        const __m512i p0 = _mm512_shuffle_i32x4(b[w], b[4 + w], 0x44), p1 = _mm512_shuffle_i32x4(b[w], b[4 + w], 0xEE);
        const __m512i p2 = _mm512_shuffle_i32x4(b[8 + w], b[12 + w], 0x44),
                      p3 = _mm512_shuffle_i32x4(b[8 + w], b[12 + w], 0xEE);
        r[0 + w] = _mm512_shuffle_i32x4(p0, p2, 0x88);
        r[4 + w] = _mm512_shuffle_i32x4(p0, p2, 0xDD);
        r[8 + w] = _mm512_shuffle_i32x4(p1, p3, 0x88);
        r[12 + w] = _mm512_shuffle_i32x4(p1, p3, 0xDD);
    }
}

/* hash_many: 16 inputs at base + i * stride, `blocks` 64-byte blocks each, all full.  Chunk
 * mode: counter0 + i per lane, CHUNK_START / CHUNK_END on the first / last block.  Parent mode:
 * counter 0, PARENT on the single block.  out[i][8] = lane i's chaining value. */
T512 static void hash16(const uint8_t* base, size_t stride, size_t blocks, uint64_t counter0, int parent,
                        uint32_t out[16][8]) {
    __m512i cv[8];
    for (int i = 0; i < 8; i++) cv[i] = _mm512_set1_epi32((int)IV[i]);
    const __m512i lane = _mm512_set_epi32(15, 14, 13, 12, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2, 1, 0);
    __m512i ctr_lo, ctr_hi;
    if (parent) {
        ctr_lo = ctr_hi = _mm512_setzero_si512();
    } else {
        const uint64_t c = counter0;
        ctr_lo = ADD(_mm512_set1_epi32((int)(uint32_t)c), lane);
        /* carry into the high word where the low word wrapped */
        const __mmask16 wrap = _mm512_cmplt_epu32_mask(ctr_lo, _mm512_set1_epi32((int)(uint32_t)c));
        ctr_hi = _mm512_mask_add_epi32(_mm512_set1_epi32((int)(uint32_t)(c >> 32)), wrap,
                                       _mm512_set1_epi32((int)(uint32_t)(c >> 32)), _mm512_set1_epi32(1));
    }
    for (size_t blk = 0; blk < blocks; blk++) {
        __m512i m[16];
        for (int i = 0; i < 16; i++) m[i] = _mm512_loadu_si512((const void*)(base + (size_t)i * stride + blk * 64));
        transpose16(m);
        uint32_t flags = parent ? PARENT : 0;
        if (!parent && blk == 0) flags |= CHUNK_START;
        if (!parent && blk + 1 == blocks) flags |= CHUNK_END;
        __m512i v0 = cv[0], v1 = cv[1], v2 = cv[2], v3 = cv[3], v4 = cv[4], v5 = cv[5], v6 = cv[6], v7 = cv[7];
        __m512i v8 = _mm512_set1_epi32((int)IV[0]), v9 = _mm512_set1_epi32((int)IV[1]);
        __m512i v10 = _mm512_set1_epi32((int)IV[2]), v11 = _mm512_set1_epi32((int)IV[3]);
        __m512i v12 = ctr_lo, v13 = ctr_hi, v14 = _mm512_set1_epi32(64), v15 = _mm512_set1_epi32((int)flags);
        for (int r = 0; r < 7; r++) {
            const uint8_t* s = SCHED[r];
            G(v0, v4, v8, v12, m[s[0]], m[s[1]]);
            G(v1, v5, v9, v13, m[s[2]], m[s[3]]);
            G(v2, v6, v10, v14, m[s[4]], m[s[5]]);
            G(v3, v7, v11, v15, m[s[6]], m[s[7]]);
            G(v0, v5, v10, v15, m[s[8]], m[s[9]]);
            G(v1, v6, v11, v12, m[s[10]], m[s[11]]);
            G(v2, v7, v8, v13, m[s[12]], m[s[13]]);
            G(v3, v4, v9, v14, m[s[14]], m[s[15]]);
        }
        cv[0] = XOR(v0, v8); cv[1] = XOR(v1, v9); cv[2] = XOR(v2, v10); cv[3] = XOR(v3, v11);
        cv[4] = XOR(v4, v12); cv[5] = XOR(v5, v13); cv[6] = XOR(v6, v14); cv[7] = XOR(v7, v15);
    }
    uint32_t t[8][16];
    for (int w = 0; w < 8; w++) _mm512_storeu_si512((void*)t[w], cv[w]);
    for (int i = 0; i < 16; i++)
        for (int w = 0; w < 8; w++) out[i][w] = t[w][i];
}

static int have_avx512(void) {
    static int v = -1;
    if (v < 0) {
        __builtin_cpu_init();
        v = __builtin_cpu_supports("avx512f") ? 1 : 0;
    }
    return v;
}

int orc_blake3_simd_available(void) { return have_avx512(); }

static void cv_bytes(const uint32_t cv[8], uint8_t out[32]) {
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 4; j++) out[4 * i + j] = (uint8_t)(cv[i] >> (8 * j));
}

/* blake3::hash(data) with the 16-way backend; bit-identical to orc_blake3. */
void orc_blake3_fast(const uint8_t* data, size_t len, uint8_t out[32]) {
    if (len <= 1024 || !have_avx512()) {
        orc_blake3(data, len, out);
        return;
    }
    const size_t n = (len + 1023) / 1024;  /* >= 2 chunks */
    uint32_t stack_cvs[64][8];
    uint32_t(*cvs)[8] = n <= 64 ? stack_cvs : (uint32_t(*)[8])malloc(n * 32);
    size_t full = len / 1024, c = 0;
    if (full == n) full--;  /* the last chunk (even if full) is hashed scalar below */
    for (; c + 16 <= full; c += 16) hash16(data + c * 1024, 1024, 16, c, 0, (uint32_t(*)[8])cvs[c]);
    for (; c < n; c++) orc_blake3_chunk_cv(data + c * 1024, c + 1 < n ? 1024 : len - c * 1024, c, cvs[c]);
    /* parents level by level until two nodes remain; the last merge is the root */
    size_t m = n;
    while (m > 2) {
        const size_t pairs = m / 2;
        size_t p = 0;
        for (; p + 16 <= pairs; p += 16) hash16((const uint8_t*)cvs[2 * p], 64, 1, 0, 1, (uint32_t(*)[8])cvs[p]);
        for (; p < pairs; p++) orc_blake3_parent_cv(cvs[2 * p], cvs[2 * p + 1], 0, cvs[p]);
        if (m & 1) memcpy(cvs[pairs], cvs[m - 1], 32);
        m = pairs + (m & 1);
    }
    uint32_t root[8];
    orc_blake3_parent_cv(cvs[0], cvs[1], ROOT, root);
    cv_bytes(root, out);
    if (cvs != stack_cvs) free(cvs);
}
