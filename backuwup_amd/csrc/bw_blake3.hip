// bw_blake3.hip -- BLAKE3 chunk IDs on gfx950.
//
// Replaces `blake3::hash(data).into()` of add_file_blob (client/src/backup/filesystem/
// dir_packer.rs:286; crate blake3 1.3.3, Cargo.lock:149-159).  Spec restated in SURVEY.md A.4.
//
// A blob of n BLAKE3 leaves (1 KiB each) hashes as: complete binary subtrees over every aligned
// run of 2^l leaves that fits in n, plus a right spine that merges, from the right, the last
// complete node of every level l whose bit is set in n; the final merge (or the single node when
// n is a power of two, or the leaf when n == 1) carries ROOT.
//
//   k_b3_groups  one lane per aligned 4-leaf group (4 KiB of input, 64 compressions + <=3
//                parents, all lanes busy).  Blobs of <= 4 leaves finish here (ROOT in-lane);
//                otherwise the lane stores the level-2 node, or for a blob's ragged last group
//                the merged tail of the spine (bits 0..1 of n).
//   k_b3_upper   the levels above the groups, one launch: one lane per blob with 4 < n <= 64 (an
//                in-place stack), one wave per blob with n > 64 (global level passes down to 64
//                nodes, then one compression pass per level from registers, spine folded alongside).
#include "bw_device.h"
#include "bw_internal.h"

namespace bw {
#if BW_CLOCK_STAMPS
__device__ ClockLog* g_clk_b3 = nullptr;
void clock_log_register_b3(void* log) { hipMemcpyToSymbol(HIP_SYMBOL(g_clk_b3), &log, sizeof(log)); }
#endif


typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));

// Chaining value of one leaf (<= 1024 bytes at global position `ls`), chunk counter `t`.
// `bend` is the end of the blob: loads never touch bytes at or beyond it except through the
// byte-exact tail path, so a blob at the very end of the caller's buffer is safe.
__device__ uint32_t g_b3_dummy[36];  // target of clamped (never consumed) prefetches

__device__ __forceinline__ void load_words(const uint32_t* src, uint32_t w[17]) {
    const u32x4_a4* q = (const u32x4_a4*)src;
    const u32x4_a4 a = q[0], b = q[1], c = q[2], d = q[3];
    w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w; w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
    w[8] = c.x; w[9] = c.y; w[10] = c.z; w[11] = c.w; w[12] = d.x; w[13] = d.y; w[14] = d.z; w[15] = d.w;
    w[16] = src[16];
}

// Chaining value of one leaf (<= 1024 bytes at global position `ls`), chunk counter `t`.
// `bend` is the end of the blob: the 16-byte loads never touch bytes at or beyond it (a block
// within 68 bytes of the end goes through the byte-exact path), so a blob at the very end of
// the caller's buffer is safe.  Block b+1 is loaded before block b is compressed; the loads are
// unconditional (a block that will take the byte path prefetches a dummy line instead) so the
// compiler's vmcnt waits stay exact.
template <bool PREFETCH>
__device__ __forceinline__ void b3_leaf(const uint8_t* __restrict__ data, uint64_t ls, uint32_t ll, uint64_t bend,
                                        uint64_t t, uint32_t root, uint32_t cv[8]) {
    b3_iv(cv);
    const uint32_t nblk = ll == 0 ? 1 : (ll + 63) / 64;
    const uint8_t* base = data + ls;
    const uint32_t sh = (uint32_t)((uintptr_t)base & 3);
    const uint32_t* wb = (const uint32_t*)(base - sh);
    uint32_t w[17];
    if (PREFETCH) load_words(ls + 68 <= bend ? wb : g_b3_dummy, w);
    for (uint32_t blk = 0; blk < nblk; blk++) {
        if (!PREFETCH) load_words(ls + blk * 64 + 68 <= bend ? wb + blk * 16 : g_b3_dummy, w);
        uint32_t m[16];
        const uint32_t left = ll - blk * 64;
        const uint32_t blen = ll == 0 ? 0 : (left < 64 ? left : 64);
        if (ls + blk * 64 + 68 <= bend) {
#pragma unroll
            for (int i = 0; i < 16; i++) m[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], sh);
        } else {
            const uint8_t* p = base + blk * 64;
#pragma unroll
            for (int i = 0; i < 16; i++) {
                uint32_t v = 0;
#pragma unroll
                for (int j = 0; j < 4; j++)
                    if ((uint32_t)(4 * i + j) < blen) v |= (uint32_t)p[4 * i + j] << (8 * j);
                m[i] = v;
            }
        }
        if (PREFETCH) {
            const bool nfast = blk + 1 < nblk && ls + (blk + 1) * 64 + 68 <= bend;
            load_words(nfast ? wb + (blk + 1) * 16 : g_b3_dummy, w);
        }
        uint32_t flags = 0;
        if (blk == 0) flags |= B3_CHUNK_START;
        if (blk == nblk - 1) flags |= B3_CHUNK_END | root;
        b3_compress(cv, m, blen, t, flags);
    }
}

// The same leaf with blocks taken in pairs: one 132-byte load (both 64-byte halves of the
// 128-byte lines it covers, requested back to back) feeds two compressions.  The per-block loop
// above requests the second half of a line one compression (~3k cycles) after the first, by
// which time L2 has often evicted the line (k_b3_groups fetched 1.30x its bytes).  No prefetch:
// at 5 waves per SIMD the other waves' ~1.5k VALU instructions per pair cover the load.  Pairs
// within 132 bytes of the blob end (and an odd last block) take the per-block path.
__device__ __forceinline__ void load_pair_words(const uint32_t* src, uint32_t w[33]) {
    const u32x4_a4* q = (const u32x4_a4*)src;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const u32x4_a4 v = q[k];
        w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
    }
    w[32] = src[32];
}

__device__ __forceinline__ void b3_leaf_pairs(const uint8_t* __restrict__ data, uint64_t ls, uint32_t ll, uint64_t bend,
                                              uint64_t t, uint32_t root, uint32_t cv[8]) {
    b3_iv(cv);
    const uint32_t nblk = ll == 0 ? 1 : (ll + 63) / 64;
    const uint8_t* base = data + ls;
    const uint32_t sh = (uint32_t)((uintptr_t)base & 3);
    const uint32_t* wb = (const uint32_t*)(base - sh);
    uint32_t blk = 0;
#pragma unroll 1
    for (; blk + 1 < nblk && ls + blk * 64 + 132 <= bend; blk += 2) {
        uint32_t w[33];
        load_pair_words(wb + blk * 16, w);
#pragma unroll
        for (int h = 0; h < 2; h++) {
            uint32_t m[16];
            if (h == 1) {
                // keep the second block's message words unformed until the first compression is done
                // (the scheduler would otherwise build both message sets up front: +20 VGPRs)
#pragma unroll
                for (int i = 16; i < 33; i++) asm volatile("" : "+v"(w[i]) : "v"(cv[0]));
            }
#pragma unroll
            for (int i = 0; i < 16; i++) m[i] = __builtin_amdgcn_alignbyte(w[16 * h + i + 1], w[16 * h + i], sh);
            const uint32_t b = blk + h;
            uint32_t flags = 0;
            if (b == 0) flags |= B3_CHUNK_START;
            if (b == nblk - 1) flags |= B3_CHUNK_END | root;
            b3_compress(cv, m, 64, t, flags);
        }
    }
    for (; blk < nblk; blk++) {  // the leaf's last one or two blocks near the blob end
        uint32_t w[17], m[16];
        const uint32_t left = ll - blk * 64;
        const uint32_t blen = ll == 0 ? 0 : (left < 64 ? left : 64);
        if (ls + blk * 64 + 68 <= bend) {
            load_words(wb + blk * 16, w);
#pragma unroll
            for (int i = 0; i < 16; i++) m[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], sh);
        } else {
            const uint8_t* p = base + blk * 64;
#pragma unroll
            for (int i = 0; i < 16; i++) {
                uint32_t v = 0;
#pragma unroll
                for (int j = 0; j < 4; j++)
                    if ((uint32_t)(4 * i + j) < blen) v |= (uint32_t)p[4 * i + j] << (8 * j);
                m[i] = v;
            }
        }
        uint32_t flags = 0;
        if (blk == 0) flags |= B3_CHUNK_START;
        if (blk == nblk - 1) flags |= B3_CHUNK_END | root;
        b3_compress(cv, m, blen, t, flags);
    }
}

__device__ __forceinline__ void store_digest(uint8_t* out, const uint32_t cv[8]) {
    uint32_t* o = (uint32_t*)out;
#pragma unroll
    for (int i = 0; i < 8; i++) o[i] = cv[i];  // little-endian words = the digest bytes
}

// PREFETCH: block b+1's words are loaded before block b is compressed (17 more VGPRs).
// PAIRS: blocks are loaded two at a time instead (b3_leaf_pairs; PREFETCH is then unused).
template <bool PREFETCH, int MINW, bool PAIRS>
__global__ __launch_bounds__(256, MINW) void k_b3_groups(const uint8_t* __restrict__ data, const uint64_t* ctr,
                                                   BlobArrays b, uint32_t* __restrict__ cv_buf,
                                                   uint8_t* __restrict__ digests) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= ctr[C_NGROUPS]) return;
    const uint64_t nb = ctr[C_NBLOBS];
    uint64_t lo = 0, hi = nb;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (b.goff[mid] <= g) lo = mid + 1;
        else hi = mid;
    }
    const uint64_t blob = lo - 1;
    BW_ASSERT(lo >= 1 && blob < b.cap);
    const uint64_t start = b.start[blob], len = b.len[blob], gi = g - b.goff[blob];
    const uint64_t bend = start + len;
    BW_ASSERT(bend <= b.data_len && gi * 4 * B3_LEAF_BYTES <= (len ? len - 1 : 0));
    const uint64_t n = len == 0 ? 1 : (len + B3_LEAF_BYTES - 1) / B3_LEAF_BYTES;
    const uint64_t first = gi * 4;
    const uint32_t k = (uint32_t)(n - first < 4 ? n - first : 4);
    // Pending subtree nodes wait in LDS (word-major, conflict-free) instead of registers, so the
    // leaf loop keeps its VGPRs for the prefetched block.
    __shared__ uint32_t s_acc[8][256], s_sv[8][256];
    const int me = threadIdx.x;
    uint32_t cv[8];
    for (uint32_t t = 0; t < k; t++) {
        const uint64_t li = first + t, ls = start + li * B3_LEAF_BYTES;
        const uint64_t rest = len - li * B3_LEAF_BYTES;
        const uint32_t ll = len == 0 ? 0 : (uint32_t)(rest < B3_LEAF_BYTES ? rest : B3_LEAF_BYTES);
        if (PAIRS) b3_leaf_pairs(data, ls, ll, bend, li, n == 1 ? B3_ROOT : 0, cv);
        else b3_leaf<PREFETCH>(data, ls, ll, bend, li, n == 1 ? B3_ROOT : 0, cv);
        if (t == 0 || t == 2) {
            uint32_t (*dst)[256] = t == 0 ? s_acc : s_sv;
#pragma unroll
            for (int i = 0; i < 8; i++) dst[i][me] = cv[i];
        } else {
            uint32_t l[8];
            if (t == 3) {
#pragma unroll
                for (int i = 0; i < 8; i++) l[i] = s_sv[i][me];
                b3_parent(l, cv, 0, cv);  // P(leaf2, leaf3)
            }
#pragma unroll
            for (int i = 0; i < 8; i++) l[i] = s_acc[i][me];
            b3_parent(l, cv, (n == 2 && t == 1) || (n == 4 && t == 3) ? B3_ROOT : 0, cv);
#pragma unroll
            for (int i = 0; i < 8; i++) s_acc[i][me] = cv[i];
        }
    }
    uint32_t acc[8];
#pragma unroll
    for (int i = 0; i < 8; i++) acc[i] = s_acc[i][me];
    if (k == 3) {
        uint32_t r[8];
#pragma unroll
        for (int i = 0; i < 8; i++) r[i] = s_sv[i][me];
        b3_parent(acc, r, n == 3 ? B3_ROOT : 0, acc);
    }
    if (n <= 4) store_digest(digests + blob * 32, acc);
    else {
        uint32_t* o = cv_buf + g * 8;
#pragma unroll
        for (int i = 0; i < 8; i++) o[i] = acc[i];
    }
}

// ---------------------------------------------------------------- aligned-line leaf pass
// k_b3_lines: the same work as k_b3_groups (one lane per aligned 4-leaf group), fed from whole
// aligned 128-byte lines.  A group's bytes start at an arbitrary offset o of their first line, so
// the 132-byte pair loads of b3_leaf_pairs touch every line twice, one compression pair apart,
// and L2 has often evicted it in between (k_b3_groups fetched 1.41x its bytes).  Here every line
// is loaded once (8 x 16-byte aligned loads per lane): lines p and p + 1 sit in registers (a, c)
// and block b's 16 message words are cut at dword offset Q = o / 4 + 16 (b mod 2) of a || c with
// the byte shift o mod 4.  Q must be a compile-time register index, so it is dispatched through a
// switch on its wave-uniform value: every group of a blob has the blob's start offset mod 128
// (4096 is a multiple of 128), so a wave whose lanes all lie in one blob shares one Q; a wave
// across blobs takes the per-lane path of k_b3_groups instead.  The leaves' chaining values wait
// in LDS and the group's parents are merged after the loop, so the loop holds no parent
// compression.  A group's last line may extend past its blob's end: an aligned 128-byte line never
// crosses a page, so the load is safe, and bytes at or past the end are masked out.

// The alignbytes are volatile asm: as builtins, the optimizer either merges the cases into one
// block fed by a ring indexed with the case number (scratch memory) or hoists every possible
// word pair out of the switch (64 alignbytes and 224 VGPRs per block instead of 16).
template <int Q>
__device__ __forceinline__ void b3_cut16(const uint32_t a[32], const uint32_t c[32], uint32_t sh, uint32_t m[16]) {
#pragma unroll
    for (int i = 0; i < 16; i++) {
        const uint32_t lo = Q + i < 32 ? a[Q + i] : c[Q + i - 32];
        const uint32_t hi = Q + i + 1 < 32 ? a[Q + i + 1] : c[Q + i + 1 - 32];
        asm volatile("v_alignbyte_b32 %0, %1, %2, %3" : "=v"(m[i]) : "v"(hi), "v"(lo), "v"(sh));
    }
}

#define B3_CUT_CASE(q) \
    case q: b3_cut16<q>(a, c, sh, m); break;
#define B3_CUT_CASE8(q) \
    B3_CUT_CASE(q) B3_CUT_CASE(q + 1) B3_CUT_CASE(q + 2) B3_CUT_CASE(q + 3) B3_CUT_CASE(q + 4) \
    B3_CUT_CASE(q + 5) B3_CUT_CASE(q + 6) B3_CUT_CASE(q + 7)

// m = the 16 words at dword offset u + 16 * H (u wave-uniform, 0..31) of a || c, shifted by sh bytes
template <int H>
__device__ __forceinline__ void b3_cut(const uint32_t a[32], const uint32_t c[32], uint32_t u, uint32_t sh,
                                       uint32_t m[16]) {
    if (H == 0) {
        switch (u) { B3_CUT_CASE8(0) B3_CUT_CASE8(8) B3_CUT_CASE8(16) B3_CUT_CASE8(24) default: break; }
    } else {
        switch (u + 16) { B3_CUT_CASE8(16) B3_CUT_CASE8(24) B3_CUT_CASE8(32) B3_CUT_CASE8(40) default: break; }
    }
}

// An aligned line of zeros: the target of the loads past a group's last line, so every load is
// unconditional
__device__ __attribute__((aligned(128))) uint4 g_b3_zero_line[8];

__device__ __forceinline__ void b3_line_load(const uint4* __restrict__ src, uint32_t w[32]) {
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const uint4 v = src[k];
        w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
    }
}

// One block of a group in k_b3_lines: mask past the blob's end, compress, and at a leaf's end
// park its chaining value in LDS.
__device__ __forceinline__ void b3_line_block(uint32_t m[16], uint32_t blk, uint32_t glen, uint32_t nblk, uint64_t n,
                                              uint64_t first, uint32_t cv[8], uint32_t (*s_leaf)[8][256], int me) {
    const uint32_t left = glen - 64 * blk;
    const uint32_t blen = glen == 0 ? 0 : (left < 64 ? left : 64);
    if (blen < 64) {  // the blob's last block: bytes at or past its end are zero
        const uint32_t whole = blen >> 2, rem = blen & 3;
        const uint32_t pmask = rem ? 0xffffffffu >> (32 - 8 * rem) : 0;
#pragma unroll
        for (uint32_t i = 0; i < 16; i++) m[i] = i < whole ? m[i] : (i == whole ? m[i] & pmask : 0);
    }
    const uint32_t bil = blk & 15, leaf = blk >> 4;
    const bool last = bil == 15 || blk + 1 == nblk;
    if (bil == 0) b3_iv(cv);
    uint32_t flags = bil == 0 ? B3_CHUNK_START : 0;
    if (last) flags |= B3_CHUNK_END | (n == 1 ? B3_ROOT : 0);
    b3_compress(cv, m, blen, first + leaf, flags);
    if (last) {
#pragma unroll
        for (int i = 0; i < 8; i++) s_leaf[leaf][i][me] = cv[i];
    }
}

constexpr uint64_t B3_SMALL_LEAVES = 64;

// Chaining values handed between waves inside one launch (the fused upper levels): agent-scope
// relaxed atomics, i.e. stores written through past the XCD's L2 and loads that miss it, so no
// L2-wide writeback/invalidate fence is needed (a __threadfence per wave made the leaf pass 1.5x
// slower: every wave wrote back and invalidated its XCD's L2, whose lines the neighbouring waves'
// loads were still reusing).  COH = false: plain accesses (the separate k_b3_upper launch, ordered
// by the kernel boundary).
template <bool COH>
__device__ __forceinline__ uint32_t cv_ld(const uint32_t* p) {
    if constexpr (COH) return __hip_atomic_load(const_cast<uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return *p;
}
template <bool COH>
__device__ __forceinline__ void cv_st(uint32_t* p, uint32_t v) {
    if constexpr (COH) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *p = v;
}
// every memory operation this wave issued has completed (coherent stores: at the agent's
// coherence point)
__device__ __forceinline__ void wave_mem_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

template <bool COH>
__device__ __forceinline__ void b3_small_blob(uint64_t blob, const uint64_t* ctr, const BlobArrays& b,
                                              uint32_t* __restrict__ cv_buf, uint8_t* __restrict__ digests);
template <bool COH, int NT = 64>
__device__ __forceinline__ void b3_upper_wave(uint64_t blob, uint64_t len, const BlobArrays& b, uint32_t* __restrict__ cv_buf,
                              uint32_t* __restrict__ cv_tmp, uint8_t* __restrict__ digests);

// FUSED: the upper levels run inside the leaf pass.  Each wave adds the groups it finished to its
// blobs' counters (b.gdone, one atomic per blob per wave); the wave that completes a blob builds its
// upper levels at once -- the whole wave for a blob of > 64 leaves (b3_upper_wave), one lane per blob
// of 5..64 leaves (b3_small_blob) -- and sets the counter back to zero for the next batch.  The
// upper levels then fill the CUs the leaf pass's last round leaves idle instead of running as a
// launch of their own after it.  Measured (profiles/r03/s04_fused): the leaf pass gets 15-21 %
// slower on C1, C2 and C4 (C2 5.71 -> 6.92 ms with the upper levels, against 5.71 + 0.25 ms
// apart), so it is an option (BW_OPT_B3_UPPER), off by default.  With a __threadfence per wave
// instead of the coherent accessors it was 1.5x slower (profiles/r03/s03_fused_fence).
template <int MINW, bool FUSED>
__global__ __launch_bounds__(256, MINW) void k_b3_lines(const uint8_t* __restrict__ data, const uint64_t* ctr,
                                                        BlobArrays b, uint32_t* __restrict__ cv_buf,
                                                        uint32_t* __restrict__ cv_tmp, uint8_t* __restrict__ digests) {
    const uint64_t ng = ctr[C_NGROUPS];
    const uint64_t g0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    // FUSED needs whole waves (the completing wave's shuffles and lane 63's digest store): lanes past
    // the last group repeat the last group's work (identical values to identical addresses) and
    // are not counted; only whole waves past it leave
    const bool live = g0 < ng;
    if (FUSED ? (ng == 0 || g0 - (threadIdx.x & 63) >= ng) : !live) return;
#if BW_CLOCK_STAMPS
    ClockStamp clk((blockIdx.x & 3) == 0 ? g_clk_b3 : nullptr, 1);  // the waves of one block in 4
#endif
    const uint64_t g = live ? g0 : ng - 1;
    // (a group -> blob map written beside Chunk.hash instead of this search measured 5 % slower on
    // C1 and C2: the 30k-instruction kernel's main loop compiled worse around it, profiles/r03/s13_*)
    const uint64_t nb = ctr[C_NBLOBS];
    uint64_t lo = 0, hi = nb;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (b.goff[mid] <= g) lo = mid + 1;
        else hi = mid;
    }
    const uint64_t blob = lo - 1;
    BW_ASSERT(lo >= 1 && blob < b.cap);
    const uint64_t start = b.start[blob], len = b.len[blob], gi = g - b.goff[blob];
    const uint32_t gs = b.gshift, G = 1u << gs;  // leaves per group (1, 2 or 4)
    BW_ASSERT(gs <= 2 && start + len <= b.data_len && (gi << gs) * B3_LEAF_BYTES <= (len ? len - 1 : 0));
    const uint64_t n = len == 0 ? 1 : (len + B3_LEAF_BYTES - 1) / B3_LEAF_BYTES;
    const uint64_t first = gi << gs;
    const uint32_t k = (uint32_t)(n - first < G ? n - first : G);
    __shared__ uint32_t s_leaf[4][8][256];  // the group's leaf chaining values, word-major
    const int me = threadIdx.x;
    const uint8_t* gp = data + start + first * B3_LEAF_BYTES;
    const uint32_t o = (uint32_t)((uintptr_t)gp & 127);
    const uint32_t q = o >> 2, sh = o & 3;
    const uint32_t uq = __builtin_amdgcn_readfirstlane(q);
    uint32_t cv[8];
    if (__builtin_amdgcn_ballot_w64(q != uq) == 0) {
        // the whole wave at one line offset: whole aligned lines, each loaded once
        const uint64_t rest = len - first * B3_LEAF_BYTES;
        const uint32_t glen = len == 0 ? 0 : (uint32_t)(rest < G * B3_LEAF_BYTES ? rest : G * B3_LEAF_BYTES);
        const uint32_t nblk = glen == 0 ? 1 : (glen + 63) / 64;
        const uint4* lp = (const uint4*)(gp - o);
        const uint32_t nlines = glen == 0 ? 0 : (o + glen + 127) / 128;
        uint32_t a[32], c[32];
        b3_line_load(nlines > 0 ? lp : g_b3_zero_line, a);
        b3_line_load(nlines > 1 ? lp + 8 : g_b3_zero_line, c);
        // two pairs per turn, the lines' roles alternating (a = line p, c = line p + 1, then the
        // other way round), so the loop carries the two lines without copies
#pragma unroll 1
        for (uint32_t p = 0;; p += 2) {
            uint32_t m[16];
            b3_cut<0>(a, c, uq, sh, m);
            b3_line_block(m, 2 * p, glen, nblk, n, first, cv, s_leaf, me);
            if (2 * p + 1 >= nblk) break;
            b3_cut<1>(a, c, uq, sh, m);
            b3_line_load(p + 2 < nlines ? lp + 8 * (p + 2) : g_b3_zero_line, a);
            b3_line_block(m, 2 * p + 1, glen, nblk, n, first, cv, s_leaf, me);
            if (2 * p + 2 >= nblk) break;
            b3_cut<0>(c, a, uq, sh, m);
            b3_line_block(m, 2 * p + 2, glen, nblk, n, first, cv, s_leaf, me);
            if (2 * p + 3 >= nblk) break;
            b3_cut<1>(c, a, uq, sh, m);
            b3_line_load(p + 3 < nlines ? lp + 8 * (p + 3) : g_b3_zero_line, c);
            b3_line_block(m, 2 * p + 3, glen, nblk, n, first, cv, s_leaf, me);
            if (2 * p + 4 >= nblk) break;
        }
    } else {
        // a wave across blobs: each lane streams its own leaves with the 132-byte pair loads
        for (uint32_t t = 0; t < k; t++) {
            const uint64_t li = first + t, ls = start + li * B3_LEAF_BYTES;
            const uint64_t lrest = len - li * B3_LEAF_BYTES;
            const uint32_t ll = len == 0 ? 0 : (uint32_t)(lrest < B3_LEAF_BYTES ? lrest : B3_LEAF_BYTES);
            b3_leaf_pairs(data, ls, ll, start + len, li, n == 1 ? B3_ROOT : 0, cv);
#pragma unroll
            for (int i = 0; i < 8; i++) s_leaf[t][i][me] = cv[i];
        }
    }
    // the group's subtree: P(P(l0, l1), P(l2, l3)), or the ragged tail's merge of 2 or 3 leaves
    uint32_t acc[8], r[8];
#pragma unroll
    for (int i = 0; i < 8; i++) acc[i] = s_leaf[0][i][me];
    if (k >= 2) {
#pragma unroll
        for (int i = 0; i < 8; i++) r[i] = s_leaf[1][i][me];
        b3_parent(acc, r, (n == 2 || (n == 4 && false)) ? B3_ROOT : 0, acc);
    }
    if (k == 4) {
        uint32_t l2[8], l3[8];
#pragma unroll
        for (int i = 0; i < 8; i++) { l2[i] = s_leaf[2][i][me]; l3[i] = s_leaf[3][i][me]; }
        b3_parent(l2, l3, 0, r);
        b3_parent(acc, r, n == 4 ? B3_ROOT : 0, acc);
    } else if (k == 3) {
#pragma unroll
        for (int i = 0; i < 8; i++) r[i] = s_leaf[2][i][me];
        b3_parent(acc, r, n == 3 ? B3_ROOT : 0, acc);
    }
    if (n <= G) store_digest(digests + blob * 32, acc);
    else {
        uint32_t* o8 = cv_buf + g * 8;
#pragma unroll
        for (int i = 0; i < 8; i++) cv_st<FUSED>(o8 + i, acc[i]);
    }
    if constexpr (FUSED) {
        const uint32_t lane = threadIdx.x & 63;
        // the wave's lanes hold consecutive groups, so each blob is one run of lanes (live lanes
        // are a prefix of the wave)
        const bool upper = live && n > G;
        const uint64_t pb = bw_shfl_up64(blob, 1);
        const bool head = upper && (lane == 0 || pb != blob);
        const uint64_t H = __ballot(head), U = __ballot(upper);
        if (H == 0) return;  // wave-uniform
        wave_mem_drain();    // this wave's level-2 nodes are written through before any counter moves
        bool complete = false;
        if (head) {
            const uint64_t above = H & ~((2ull << lane) - 1);  // heads after this lane
            const uint32_t end = above ? (uint32_t)__builtin_ctzll(above) : 64u;
            const uint64_t run = (end == 64 ? ~0ull : ((1ull << end) - 1)) & ~((1ull << lane) - 1);
            const uint32_t cnt = (uint32_t)__popcll(U & run);
            const uint32_t total = (uint32_t)((n + G - 1) >> gs);
            const uint32_t old = __hip_atomic_fetch_add(b.gdone + blob, cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            BW_ASSERT(old + cnt <= total);
            complete = old + cnt == total;
            if (complete) b.gdone[blob] = 0;  // nothing else touches it in this pass
        }
        const uint64_t C = __ballot(complete);
        if (C == 0) return;  // (the completing counters were read above: every level-2 node they
                             // count was written through before its counter moved)
        for (uint64_t m = C; m; m &= m - 1) {  // blobs of > 64 leaves: the whole wave, one by one
            const int h = __builtin_ctzll(m);
            const uint64_t cb = bw_shfl64(blob, h), cl = bw_shfl64(len, h);
            if (cl > (uint64_t)B3_SMALL_LEAVES * B3_LEAF_BYTES) b3_upper_wave<true>(cb, cl, b, cv_buf, cv_tmp, digests);
        }
        if (complete) b3_small_blob<true>(blob, ctr, b, cv_buf, digests);  // 5..64 leaves; returns otherwise
    }
}

// Upper levels of a small blob (4 < n <= B3_SMALL_LEAVES leaves), one lane per blob: a batch of
// many small files (C4) keeps every lane busy instead of one wave per blob with <= 8 lanes
// active.  The level-2 nodes are merged left to right on a stack of complete subtrees that lives
// in the blob's own cv_buf slots (slot d < node i, so it only overwrites consumed nodes); the
// stack is then folded from the right onto the ragged tail (bits 0..1 of n).  The merge that
// completes a power-of-two blob, or the last fold, carries ROOT.

template <bool COH>
__device__ __forceinline__ void b3_small_blob(uint64_t blob, const uint64_t* ctr, const BlobArrays& b,
                                              uint32_t* __restrict__ cv_buf, uint8_t* __restrict__ digests) {
    if (blob >= ctr[C_NBLOBS]) return;
    const uint64_t len = b.len[blob];
    const uint64_t n = len == 0 ? 1 : (len + B3_LEAF_BYTES - 1) / B3_LEAF_BYTES;
    const uint32_t gs = b.gshift;
    if (n <= (1u << gs) || n > B3_SMALL_LEAVES) return;
    uint32_t* g = cv_buf + b.goff[blob] * 8;
    const uint32_t m2 = (uint32_t)(n >> gs);                 // complete group nodes
    const bool tail = (n & ((1u << gs) - 1)) != 0;           // the ragged last group's merged node
    uint32_t depth = 0;
    for (uint32_t i = 0; i < m2; i++) {
        uint32_t carry[8];
#pragma unroll
        for (int w = 0; w < 8; w++) carry[w] = cv_ld<COH>(g + i * 8 + w);
        for (uint32_t c = i + 1; (c & 1) == 0; c >>= 1) {
            uint32_t l[8];
            depth--;
#pragma unroll
            for (int w = 0; w < 8; w++) l[w] = cv_ld<COH>(g + depth * 8 + w);
            b3_parent(l, carry, (!tail && i + 1 == m2 && depth == 0) ? B3_ROOT : 0, carry);
        }
#pragma unroll
        for (int w = 0; w < 8; w++) cv_st<COH>(g + depth * 8 + w, carry[w]);
        depth++;
    }
    uint32_t acc[8];
    bool have = false;
    if (tail) {
#pragma unroll
        for (int w = 0; w < 8; w++) acc[w] = cv_ld<COH>(g + m2 * 8 + w);
        have = true;
    }
    while (depth > 0) {
        depth--;
        uint32_t t[8];
#pragma unroll
        for (int w = 0; w < 8; w++) t[w] = cv_ld<COH>(g + depth * 8 + w);
        if (!have) {
#pragma unroll
            for (int w = 0; w < 8; w++) acc[w] = t[w];
            have = true;
        } else {
            b3_parent(t, acc, depth == 0 ? B3_ROOT : 0, acc);
        }
    }
    store_digest(digests + blob * 32, acc);
}

// Upper levels of a larger blob (n > B3_SMALL_LEAVES leaves), one wave per blob.  While a level
// has more than 64 nodes, lanes 0..62 build the next level's parents in passes over global memory
// (ping-ponging between cv_buf, which holds level 2 from k_b3_groups, and cv_tmp at the blob's own
// group offsets) and lane 63 folds the right spine in the same pass (the last node of every level
// whose bit is set in n, merged from the right); from 64 nodes down, node i lives in lane i's
// registers and each level is one compression pass: lanes < cnt/2 build parents from their two
// children (ds_bpermute), lane 63 takes the spine step.  A 3 MiB chunk (768 level-2 nodes) is 20
// compression passes deep; 32 lanes per blob with every level in global memory took 29 plus a
// separate spine compression per level.  C1 (939 blobs): upper levels 0.119 -> 0.051 ms per batch,
// C2 unchanged (0.27 ms, throughput-bound).
__device__ __forceinline__ void b3_shfl8(const uint32_t x[8], int src, uint32_t out[8]) {
#pragma unroll
    for (int w = 0; w < 8; w++) out[w] = __shfl(x[w], src, 64);
}

// NT = 256: the whole workgroup builds the levels that pass through global memory (255 parents per
// round instead of 63, synchronized by the workgroup barrier), and its last wave takes the levels
// from 64 nodes down.  Every thread of the workgroup calls it for the same blobs in the same order.
template <bool COH, int NT>
__device__ __forceinline__ void b3_upper_wave(uint64_t blob, uint64_t len, const BlobArrays& b, uint32_t* __restrict__ cv_buf,
                              uint32_t* __restrict__ cv_tmp, uint8_t* __restrict__ digests) {
    static_assert(NT == 64 || NT == 256, "a wave or a 4-wave workgroup per blob");
    const uint32_t lane = threadIdx.x & 63, t = threadIdx.x & (NT - 1);
    const uint64_t n = (len + B3_LEAF_BYTES - 1) / B3_LEAF_BYTES;  // > B3_SMALL_LEAVES
    uint32_t* src = cv_buf + b.goff[blob] * 8;
    uint32_t* dst = cv_tmp + b.goff[blob] * 8;
    const uint32_t gs = b.gshift;
    uint64_t cnt = n >> gs;  // complete group nodes (level gs); the ragged tail's merged node follows them
    bool have = (n & ((1u << gs) - 1)) != 0;
    uint32_t acc[8];
#pragma unroll
    for (int w = 0; w < 8; w++) acc[w] = 0;
    if (have && t == NT - 1) {
#pragma unroll
        for (int w = 0; w < 8; w++) acc[w] = cv_ld<COH>(src + cnt * 8 + w);
    }
    int l = (int)gs;
    while (cnt > 64) {  // never a root here: at least 65 nodes remain
        const bool spine = cnt & 1;
        const uint64_t next = cnt / 2;
        for (uint64_t base = 0; base < next; base += NT - 1) {
            const uint64_t i = base + t;
            const bool pair = t < NT - 1 && i < next;
            const bool fold = t == NT - 1 && base == 0 && spine && have;
            if (pair || fold) {
                uint32_t L[8], R[8], P[8];
                const uint64_t li = pair ? 2 * i : cnt - 1;
#pragma unroll
                for (int w = 0; w < 8; w++) L[w] = cv_ld<COH>(src + li * 8 + w);
#pragma unroll
                for (int w = 0; w < 8; w++) R[w] = pair ? cv_ld<COH>(src + (li + 1) * 8 + w) : acc[w];
                b3_parent(L, R, 0, P);
                if (pair) {
#pragma unroll
                    for (int w = 0; w < 8; w++) cv_st<COH>(dst + i * 8 + w, P[w]);
                } else {
#pragma unroll
                    for (int w = 0; w < 8; w++) acc[w] = P[w];
                }
            }
        }
        if (spine && !have && t == NT - 1) {
#pragma unroll
            for (int w = 0; w < 8; w++) acc[w] = cv_ld<COH>(src + (cnt - 1) * 8 + w);
        }
        have |= spine;
        // the wave (workgroup) reads the level it just wrote (same CU)
        if constexpr (COH) wave_mem_drain();
        if constexpr (NT == 64) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        } else {
            __syncthreads();
        }
        uint32_t* t = src;
        src = dst;
        dst = t;
        cnt = next;
        l++;
    }
    // from 64 nodes down: the wave that holds the spine (thread NT - 1 = its lane 63)
    if (NT > 64 && t / 64 != (NT - 1) / 64) return;
    uint32_t x[8];
#pragma unroll
    for (int w = 0; w < 8; w++) x[w] = lane < cnt ? cv_ld<COH>(src + lane * 8 + w) : 0;
    for (;;) {
        const bool spine = cnt & 1;
        const uint32_t next = (uint32_t)(cnt / 2);
        uint32_t L[8], R[8], T[8], P[8];
        b3_shfl8(x, (int)(2 * lane) & 63, L);
        b3_shfl8(x, (int)(2 * lane + 1) & 63, R);
        b3_shfl8(x, (int)(cnt - 1), T);
        const bool pair = lane < next;
        const bool fold = lane == 63 && spine && have;
        if (pair || fold) {
            const uint32_t root = pair ? (n == (2ull << l) ? B3_ROOT : 0) : ((n >> (l + 1)) == 0 ? B3_ROOT : 0);
            uint32_t A[8], B[8];
#pragma unroll
            for (int w = 0; w < 8; w++) { A[w] = pair ? L[w] : T[w]; B[w] = pair ? R[w] : acc[w]; }
            b3_parent(A, B, root, P);
        }
        if (lane == 63 && spine) {
#pragma unroll
            for (int w = 0; w < 8; w++) acc[w] = have ? P[w] : T[w];
        }
        have |= spine;
        if (next == 0) break;
        if (pair) {
#pragma unroll
            for (int w = 0; w < 8; w++) x[w] = P[w];
        }
        cnt = next;
        l++;
    }
    if (lane == 63) store_digest(digests + blob * 32, acc);
}

// The upper levels of every blob with more than 4 leaves in one launch: blocks [0, small_blocks)
// run k_b3_small's lane-per-blob stacks, the rest run b3_upper_wave over the blobs with more than
// B3_SMALL_LEAVES leaves, so the two latency-bound passes overlap instead of running back to back.
//
// Blobs of > 64 leaves get a wave each, or with `per_block` (batches of few blobs, where the upper
// levels are latency on the critical path rather than throughput) every blob above one group gets a
// 4-wave workgroup: a 3 MiB chunk at 2 leaves per group is 1,536 nodes, 26 rounds of 63 parents
// through global memory for a wave and 9 of 255 for the workgroup, and a 64-leaf blob's 32 nodes
// take 5 register levels instead of a lane's 31 serial merges (C1: the longest chain of the pass,
// ~75 us of 2.3 us compressions).
__global__ __launch_bounds__(256) void k_b3_upper(const uint64_t* ctr, BlobArrays b, uint32_t* __restrict__ cv_buf,
                                                  uint32_t* __restrict__ cv_tmp, uint8_t* __restrict__ digests,
                                                  uint32_t small_blocks, uint32_t per_block) {
    if (blockIdx.x < small_blocks) {
        b3_small_blob<false>((uint64_t)blockIdx.x * blockDim.x + threadIdx.x, ctr, b, cv_buf, digests);
        return;
    }
    const uint64_t nblobs = ctr[C_NBLOBS];
    if (per_block) {  // every blob above one group, small ones included (no lane-per-blob stacks)
        const uint64_t one_group = (uint64_t)B3_LEAF_BYTES << b.gshift;
        for (uint64_t blob = blockIdx.x - small_blocks; blob < nblobs; blob += gridDim.x - small_blocks) {
            const uint64_t len = b.len[blob];  // workgroup-uniform
            if (len <= one_group) continue;   // rooted in the leaf pass
            b3_upper_wave<false, 256>(blob, len, b, cv_buf, cv_tmp, digests);
        }
        return;
    }
    const uint64_t waves = (uint64_t)(gridDim.x - small_blocks) * (blockDim.x / 64);
    for (uint64_t blob = (uint64_t)(blockIdx.x - small_blocks) * (blockDim.x / 64) + threadIdx.x / 64; blob < nblobs;
         blob += waves) {
        const uint64_t len = b.len[blob];
        if (len <= (uint64_t)B3_SMALL_LEAVES * B3_LEAF_BYTES) continue;  // k_b3_groups / the small path
        b3_upper_wave<false, 64>(blob, len, b, cv_buf, cv_tmp, digests);
    }
}

#ifndef BW_B3_LINES_MINW
#define BW_B3_LINES_MINW 3  // blocks of 256 per CU: 3 = 3 waves per SIMD (168 VGPRs; at 4 the ring spills)
#endif
#ifndef B3_UPPER_BLOCK_BLOBS
#define B3_UPPER_BLOCK_BLOBS 8192  // k_b3_upper: a workgroup per large blob up to this many blobs (bound)
#endif

// Roofline calibration: the leaf pass's compression (b3_compress, the same instruction forms)
// from registers, no memory traffic, at the leaf pass's occupancy.  Wave 0 of every block stamps
// shader cycles (s_memtime) and 100 MHz real time (s_memrealtime), so the bytes per shader clock
// do not depend on the DVFS state the run happens to meet.
__global__ __launch_bounds__(256, BW_B3_LINES_MINW) void k_b3_calib(uint32_t blocks_per_lane, uint32_t* sink,
                                                                    uint64_t* stamps) {
    uint32_t cv[8], m[16];
    b3_iv(cv);
#pragma unroll
    for (int i = 0; i < 16; i++) m[i] = threadIdx.x * 16 + i + blockIdx.x;
    uint64_t t0 = 0, r0 = 0;
    if (threadIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    for (uint32_t k = 0; k < blocks_per_lane; k++) {
        m[0] ^= k;
        b3_compress(cv, m, 64, k, 0);
    }
    if (threadIdx.x == 0) {
        stamps[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;
        stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
    if (cv[0] == 0x9e3779b9u && cv[1] == 0x7f4a7c15u) sink[0] = cv[2];  // keeps the chain live
}

void launch_b3_calib(hipStream_t st, uint32_t n_blocks, uint32_t blocks_per_lane, uint32_t* sink, uint64_t* stamps) {
    hipLaunchKernelGGL(k_b3_calib, dim3(n_blocks), dim3(256), 0, st, blocks_per_lane, sink, stamps);
}

uint32_t b3_calib_blocks_per_cu() { return BW_B3_LINES_MINW; }

void launch_blake3(hipStream_t st, const uint8_t* data, const uint64_t* ctr, BlobArrays b, uint64_t max_blobs,
                   uint64_t max_groups, uint32_t* cv_buf, uint32_t* cv_tmp, uint8_t* digests, int max_leaves,
                   hipEvent_t between, int loads, hipStream_t upper, hipEvent_t leaf_done, hipEvent_t mark) {
    if (!max_blobs) {
        if (leaf_done) hipEventRecord(leaf_done, st);
        return;
    }
#ifndef BW_B3_DYN_LDS
#define BW_B3_DYN_LDS 0  // A/B: extra LDS per block caps the blocks per CU (occupancy experiments)
#endif
#if BW_DIAG
    const bool fused = loads == B3_LOADS_LINES && b.gdone;
    if (fused)
        hipLaunchKernelGGL((k_b3_lines<BW_B3_LINES_MINW, true>), dim3((unsigned)((max_groups + 255) / 256)), dim3(256), 0, st,
                           data, ctr, b, cv_buf, cv_tmp, digests);
    else if (loads == B3_LOADS_PAIRS)
        hipLaunchKernelGGL((k_b3_groups<false, 1, true>), dim3((unsigned)((max_groups + 255) / 256)), dim3(256), BW_B3_DYN_LDS, st,
                           data, ctr, b, cv_buf, digests);
    else if (loads == B3_LOADS_PREFETCH)
        hipLaunchKernelGGL((k_b3_groups<true, 1, false>), dim3((unsigned)((max_groups + 255) / 256)), dim3(256), 0, st,
                           data, ctr, b, cv_buf, digests);
    else
#else
    // the product library: aligned 128-byte lines, upper levels in their own launch
    const bool fused = false;
    (void)loads;
#endif
        hipLaunchKernelGGL((k_b3_lines<BW_B3_LINES_MINW, false>), dim3((unsigned)((max_groups + 255) / 256)), dim3(256), 0, st,
                           data, ctr, b, cv_buf, cv_tmp, digests);
    if (leaf_done) hipEventRecord(leaf_done, st);
    if (mark) hipEventRecord(mark, st);
    if (between) hipEventRecord(between, st);
    if (upper != st) hipStreamWaitEvent(upper, between, 0);
    st = upper;
    if (max_leaves > (1 << b.gshift) && !fused) {
        // few blobs (bound <= B3_UPPER_BLOCK_BLOBS): a workgroup per blob; many: a lane per small
        // blob and a wave per large one
        const bool per_block = max_blobs <= B3_UPPER_BLOCK_BLOBS;
        const uint64_t small = per_block ? 0 : (max_blobs + 255) / 256;
        uint64_t big = per_block ? max_blobs : (max_leaves > (int)B3_SMALL_LEAVES ? (max_blobs + 3) / 4 : 0);
        if (big > 4096) big = 4096;
        hipLaunchKernelGGL(k_b3_upper, dim3((unsigned)(small + big)), dim3(256), 0, st, ctr, b, cv_buf, cv_tmp, digests,
                           (uint32_t)small, (uint32_t)per_block);
    }
}

}  // namespace bw
