// bw_zstd.hip -- per-blob zstd level 3 on the GPU.
//
// Replaces Manager::compress_encrypt_blob's compression (client/src/backup/filesystem/packfile/
// pack.rs:58-64: zstd::bulk::Compressor::new(3), no checksum, no content size, no magic bytes;
// one fresh compressor per blob).  Output: the magicless frame libzstd writes for the blob, byte
// for byte (pinned against the system libzstd through the CPU oracle, tests/test_zstd.py).
//
// A frame is a chain of 128 KiB blocks whose only serial dependencies are the dfast match
// state (hash tables, repeat offsets) and the Huffman table that a block may reuse from the
// previous one.  The work is split along those lines:
//   k_zs_parse   one wave per blob: the dfast match finder (ZSTD_compressBlock_doubleFast) over
//                all of the blob's blocks.  Each step tests the next 64 positions of the skip
//                sequence at once (one per lane: both hash probes, the repeat-offset probe and
//                the candidate bytes), forwards table writes between the lanes, and resumes
//                serially at the first lane that finds a match; match extension compares 512
//                bytes per wave step.  Repeat offsets only carry over blocks that end up
//                compressed, which is not known yet: the parse assumes every block is, and the
//                decision pass flags blobs where that guess changed an offset (rerun with the
//                decisions known, rarely needed).
//   k_zs_stats   one workgroup per block: literal gather, the four Huffman segment histograms,
//                the LL/OF/ML code histograms, the RLE test, and the whole sequences section
//                (encoding types, FSE tables, table descriptions and the backward FSE bitstream)
//                -- nothing in it depends on other blocks at this level.
//   k_zs_decide  one wave per blob, serial over its blocks: the Huffman literal decisions with
//                the table-repeat state, the raw / RLE / compressed decision per block, the
//                frame layout, and the repeat-offset check.
//   k_zs_emit    one workgroup per block: block headers, raw copies, and the Huffman streams
//                (bit offsets by a workgroup suffix scan, symbols OR-ed into LDS words).
// Hash tables live in a pool of per-blob slots that are never cleared between uses: each use
// numbers its positions above every index the slot held before (an "index base"), so stale
// entries fall below the window and read as empty, exactly like libzstd's zeroed tables.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <string>
#include <vector>

#include "bw_device.h"
#include "bw_internal.h"

namespace bw {
namespace zs {

constexpr uint32_t BLOCK = 131072;  // ZSTD_BLOCKSIZE_MAX
constexpr uint32_t HL_MAX = 17, HS_MAX = 16;
// A table entry holds a position AND the bytes the match test compares at it (src is immutable,
// so they are exactly what a load at that position would return): a probe answers the candidate
// test by itself, one memory round per step fewer than libzstd's position-only tables.  Long
// table: 16 B {pos, 0, 8 bytes}; short table: 8 B {pos, 4 bytes}.  2.5 MiB per slot.  The narrow
// layout (libzstd's u32 positions) takes 768 KiB per slot; each layout has a pool of its own.
constexpr uint64_t SLOT_WORDS = (1ull << HL_MAX) * 4 + (1ull << HS_MAX) * 2;
constexpr uint64_t NARROW_WORDS = (1ull << HL_MAX) + (1ull << HS_MAX);
constexpr uint32_t SEC_HDR = 256;  // sequence-section scratch: header bytes, then the bitstream
constexpr uint32_t HUF_HDR_CAP = 256;  // table descriptions libzstd keeps are < 129 bytes
constexpr uint32_t MAXLL = 35, MAXML = 52, MAXOFF = 31, DEFAULT_MAXOFF = 28;
constexpr uint32_t LLFSELOG = 9, MLFSELOG = 9, OFFFSELOG = 8;
constexpr uint32_t FSE_MIN_LOG = 5, FSE_MAX_LOG = 12;
constexpr uint32_t HUF_MAX_LOG = 12, HUF_DEFAULT_LOG = 11;
enum { REP_NONE = 0, REP_CHECK = 1, REP_VALID = 2 };
enum { SET_BASIC = 0, SET_RLE = 1, SET_COMPRESSED = 2, SET_REPEAT = 3 };
enum { BT_RAW = 0, BT_RLE = 1, BT_COMPRESSED = 2 };
enum { LIT_RAW = 0, LIT_RLE = 1, LIT_HUF = 2, LIT_HUF_REPEAT = 3 };

__constant__ uint8_t c_LL_bits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1,
                                      1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
__constant__ int16_t c_LL_norm[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                      2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
__constant__ uint8_t c_ML_bits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                      0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1,
                                      2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
__constant__ int16_t c_ML_norm[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                      1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                      1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
__constant__ int16_t c_OF_norm[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1,
                                      1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};

// ------------------------------------------------------------------ small helpers
__device__ __forceinline__ uint32_t hb32(uint32_t v) { return 31u - (uint32_t)__clz(v); }
typedef uint64_t __attribute__((aligned(1))) u64u;
typedef uint32_t __attribute__((aligned(1))) u32u;
__device__ __forceinline__ uint64_t ld64(const uint8_t* p) { return *(const u64u*)p; }
__device__ __forceinline__ uint32_t ld32(const uint8_t* p) { return *(const u32u*)p; }

__device__ __forceinline__ uint32_t hash_long(uint64_t v, uint32_t bits) {
    return (uint32_t)((v * 0xCF1BBCDCB7A56463ull) >> (64 - bits));
}
__device__ __forceinline__ uint32_t hash_small(uint64_t v, uint32_t bits, uint32_t mls) {
    switch (mls) {
    case 5: return (uint32_t)(((v << 24) * 889523592379ull) >> (64 - bits));
    case 6: return (uint32_t)(((v << 16) * 227718039650203ull) >> (64 - bits));
    case 7: return (uint32_t)(((v << 8) * 58295818150454627ull) >> (64 - bits));
    case 8: return hash_long(v, bits);
    default: return ((uint32_t)v * 2654435761u) >> (32 - bits);
    }
}

__device__ __forceinline__ uint32_t ll_code(uint32_t ll) {
    if (ll > 63) return hb32(ll) + 19;
    if (ll < 16) return ll;
    // codes 16..24 cover 16-17,18-19,20-21,22-23,24-27,28-31,32-39,40-47,48-63
    if (ll < 24) return 16 + ((ll - 16) >> 1);
    if (ll < 32) return 20 + ((ll - 24) >> 2);
    if (ll < 48) return 22 + ((ll - 32) >> 3);
    return 24;
}
__device__ __forceinline__ uint32_t ml_code(uint32_t mb) {
    if (mb > 127) return hb32(mb) + 36;
    if (mb < 32) return mb;
    if (mb < 40) return 32 + ((mb - 32) >> 1);
    if (mb < 48) return 36 + ((mb - 40) >> 2);
    if (mb < 64) return 38 + ((mb - 48) >> 3);
    if (mb < 96) return 40 + ((mb - 64) >> 4);
    return 42;
}

// sequence record: litLength (18 bits) | matchLength - 3 (18 bits) << 18 | offset value << 36
__device__ __forceinline__ uint64_t seq_pack(uint32_t ll, uint32_t mb, uint32_t ov) {
    return (uint64_t)ll | ((uint64_t)mb << 18) | ((uint64_t)ov << 36);
}
__device__ __forceinline__ uint32_t seq_ll(uint64_t q) { return (uint32_t)(q & 0x3FFFF); }
__device__ __forceinline__ uint32_t seq_mb(uint64_t q) { return (uint32_t)((q >> 18) & 0x3FFFF); }
__device__ __forceinline__ uint32_t seq_ov(uint64_t q) { return (uint32_t)(q >> 36); }

__device__ __forceinline__ uint32_t rdlane(uint32_t v, uint32_t l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}

// ------------------------------------------------------------------ FSE (serial, one lane)
struct FseTT {
    int32_t dfs;   // deltaFindState
    uint32_t dnb;  // deltaNbBits
};

__device__ uint32_t fse_optimal_log(uint32_t maxLog, uint32_t srcSize, uint32_t maxSV, uint32_t minus) {
    uint32_t maxBitsSrc = hb32(srcSize - 1) - minus;
    uint32_t a = hb32(srcSize) + 1, b = hb32(maxSV) + 2;
    uint32_t minBits = a < b ? a : b;
    uint32_t t = maxLog;
    if (maxBitsSrc < t) t = maxBitsSrc;
    if (minBits > t) t = minBits;
    if (t < FSE_MIN_LOG) t = FSE_MIN_LOG;
    if (t > FSE_MAX_LOG) t = FSE_MAX_LOG;
    return t;
}

// FSE_normalizeCount (with the low-probability option); returns false on libzstd's error exit.
__device__ bool fse_normalize(int16_t* norm, uint32_t tableLog, const uint32_t* count, uint32_t total,
                              uint32_t maxSV, bool lowProb) {
    const int16_t lowCount = lowProb ? -1 : 1;
    const uint32_t rtb[8] = {0, 473195, 504333, 520860, 550000, 700000, 750000, 830000};
    const uint64_t scale = 62 - tableLog, step = (1ull << 62) / total, vStep = 1ull << (scale - 20);
    int still = 1 << tableLog;
    uint32_t largest = 0;
    int16_t largestP = 0;
    const uint32_t lowThreshold = total >> tableLog;
    for (uint32_t s = 0; s <= maxSV; s++) {
        if (count[s] == total) return true;  // rle: not reached (callers handle it)
        if (count[s] == 0) { norm[s] = 0; continue; }
        if (count[s] <= lowThreshold) { norm[s] = lowCount; still--; continue; }
        int16_t p = (int16_t)(((uint64_t)count[s] * step) >> scale);
        if (p < 8) {
            uint64_t restToBeat = vStep * rtb[p];
            p += ((uint64_t)count[s] * step) - ((uint64_t)p << scale) > restToBeat;
        }
        if (p > largestP) { largestP = p; largest = s; }
        norm[s] = p;
        still -= p;
    }
    if (-still >= (norm[largest] >> 1)) {
        // FSE_normalizeM2
        const int16_t NOT_YET = -2;
        uint32_t distributed = 0, tot = total;
        uint32_t lowOne = (uint32_t)(((uint64_t)tot * 3) >> (tableLog + 1));
        for (uint32_t s = 0; s <= maxSV; s++) {
            if (count[s] == 0) { norm[s] = 0; continue; }
            if (count[s] <= lowThreshold) { norm[s] = lowCount; distributed++; tot -= count[s]; continue; }
            if (count[s] <= lowOne) { norm[s] = 1; distributed++; tot -= count[s]; continue; }
            norm[s] = NOT_YET;
        }
        uint32_t toDist = (1u << tableLog) - distributed;
        if (toDist == 0) return true;
        if ((tot / toDist) > lowOne) {
            lowOne = (uint32_t)(((uint64_t)tot * 3) / ((uint64_t)toDist * 2));
            for (uint32_t s = 0; s <= maxSV; s++)
                if (norm[s] == NOT_YET && count[s] <= lowOne) { norm[s] = 1; distributed++; tot -= count[s]; }
            toDist = (1u << tableLog) - distributed;
        }
        if (distributed == maxSV + 1) {
            uint32_t maxV = 0, maxC = 0;
            for (uint32_t s = 0; s <= maxSV; s++) if (count[s] > maxC) { maxV = s; maxC = count[s]; }
            norm[maxV] += (int16_t)toDist;
            return true;
        }
        if (tot == 0) {
            for (uint32_t s = 0; toDist > 0; s = (s + 1) % (maxSV + 1))
                if (norm[s] > 0) { toDist--; norm[s]++; }
            return true;
        }
        const uint64_t vStepLog = 62 - tableLog, mid = (1ull << (vStepLog - 1)) - 1;
        const uint64_t rStep = (((1ull << vStepLog) * toDist) + mid) / tot;
        uint64_t tmpTotal = mid;
        for (uint32_t s = 0; s <= maxSV; s++) {
            if (norm[s] != NOT_YET) continue;
            uint64_t end = tmpTotal + (uint64_t)count[s] * rStep;
            uint32_t w = (uint32_t)(end >> vStepLog) - (uint32_t)(tmpTotal >> vStepLog);
            if (w < 1) return false;
            norm[s] = (int16_t)w;
            tmpTotal = end;
        }
        return true;
    }
    norm[largest] += (int16_t)still;
    return true;
}

// FSE_writeNCount into out (global or LDS bytes); returns its size.
__device__ uint32_t fse_write_ncount(uint8_t* out, const int16_t* norm, uint32_t maxSV, uint32_t tableLog) {
    uint32_t o = 0;
    const int tableSize = 1 << tableLog;
    int nbBits = (int)tableLog + 1, remaining = tableSize + 1, threshold = tableSize, bitCount = 4;
    uint32_t bits = tableLog - FSE_MIN_LOG, sym = 0;
    bool prev0 = false;
    while (sym <= maxSV && remaining > 1) {
        if (prev0) {
            uint32_t start = sym;
            while (sym <= maxSV && !norm[sym]) sym++;
            if (sym > maxSV) break;
            while (sym >= start + 24) {
                start += 24;
                bits += 0xFFFFu << bitCount;
                out[o] = (uint8_t)bits; out[o + 1] = (uint8_t)(bits >> 8);
                o += 2;
                bits >>= 16;
            }
            while (sym >= start + 3) { start += 3; bits += 3u << bitCount; bitCount += 2; }
            bits += (sym - start) << bitCount;
            bitCount += 2;
            if (bitCount > 16) {
                out[o] = (uint8_t)bits; out[o + 1] = (uint8_t)(bits >> 8);
                o += 2; bits >>= 16; bitCount -= 16;
            }
        }
        int c = norm[sym++];
        const int mx = (2 * threshold - 1) - remaining;
        remaining -= c < 0 ? -c : c;
        c++;
        if (c >= threshold) c += mx;
        bits += (uint32_t)c << bitCount;
        bitCount += nbBits;
        bitCount -= (c < mx);
        prev0 = (c == 1);
        while (remaining < threshold) { nbBits--; threshold >>= 1; }
        if (bitCount > 16) {
            out[o] = (uint8_t)bits; out[o + 1] = (uint8_t)(bits >> 8);
            o += 2; bits >>= 16; bitCount -= 16;
        }
    }
    out[o] = (uint8_t)bits;
    if ((bitCount + 7) / 8 > 1) out[o + 1] = (uint8_t)(bits >> 8);
    return o + (uint32_t)(bitCount + 7) / 8;
}

// FSE_buildCTable_wksp into (state[1 << tableLog], tt[maxSV + 1]); spread = scratch of 1 << tableLog.
__device__ void fse_build(uint16_t* state, FseTT* tt, uint8_t* spread, const int16_t* norm, uint32_t maxSV,
                          uint32_t tableLog) {
    const uint32_t size = 1u << tableLog, mask = size - 1, step = (size >> 1) + (size >> 3) + 3;
    uint32_t cumul[54];
    uint32_t high = size - 1;
    cumul[0] = 0;
    for (uint32_t u = 1; u <= maxSV + 1; u++) {
        if (norm[u - 1] == -1) { cumul[u] = cumul[u - 1] + 1; spread[high--] = (uint8_t)(u - 1); }
        else cumul[u] = cumul[u - 1] + (uint32_t)norm[u - 1];
    }
    uint32_t pos = 0;
    for (uint32_t s = 0; s <= maxSV; s++)
        for (int k = 0; k < norm[s]; k++) {
            spread[pos] = (uint8_t)s;
            pos = (pos + step) & mask;
            while (pos > high) pos = (pos + step) & mask;
        }
    for (uint32_t u = 0; u < size; u++) state[cumul[spread[u]]++] = (uint16_t)(size + u);
    int total = 0;
    for (uint32_t s = 0; s <= maxSV; s++) {
        const int n = norm[s];
        if (n == 0) {
            tt[s].dnb = ((tableLog + 1) << 16) - (1u << tableLog);
            tt[s].dfs = 0;
        } else if (n == -1 || n == 1) {
            tt[s].dnb = (tableLog << 16) - (1u << tableLog);
            tt[s].dfs = total - 1;
            total++;
        } else {
            const uint32_t maxBitsOut = tableLog - hb32((uint32_t)n - 1);
            tt[s].dnb = (maxBitsOut << 16) - ((uint32_t)n << maxBitsOut);
            tt[s].dfs = total - n;
            total += n;
        }
    }
}

// little-endian bit writer into global memory (one lane)
struct BitW {
    uint8_t* p;
    uint32_t n;   // bytes written
    uint32_t cap; // bytes allowed (further bytes are counted, not written)
    uint64_t acc;
    uint32_t nb;
    __device__ void init(uint8_t* dst, uint32_t c) { p = dst; n = 0; cap = c; acc = 0; nb = 0; }
    __device__ __forceinline__ void add(uint64_t v, uint32_t bits) {
        if (!bits) return;
        acc |= (v & ((1ull << bits) - 1)) << nb;
        nb += bits;
        while (nb >= 8) {
            if (n < cap) p[n] = (uint8_t)acc;
            n++;
            acc >>= 8;
            nb -= 8;
        }
    }
    __device__ uint32_t close() {
        add(1, 1);
        if (nb) { if (n < cap) p[n] = (uint8_t)acc; n++; }
        return n;
    }
};

struct FseState {
    uint32_t v;
    const uint16_t* st;
    const FseTT* tt;
    uint32_t log;
    __device__ void init2(const uint16_t* state, const FseTT* t, uint32_t tableLog, uint32_t sym) {
        st = state; tt = t; log = tableLog;
        const FseTT x = t[sym];
        const uint32_t nbOut = (x.dnb + (1u << 15)) >> 16;
        const uint32_t v0 = (nbOut << 16) - x.dnb;
        v = state[(v0 >> nbOut) + x.dfs];
    }
    __device__ __forceinline__ void enc(BitW& b, uint32_t sym) {
        const FseTT x = tt[sym];
        const uint32_t nbOut = (v + x.dnb) >> 16;
        b.add(v, nbOut);
        v = st[(v >> nbOut) + x.dfs];
    }
    __device__ void flush(BitW& b) { b.add(v, log); }
};

}  // namespace zs

// ======================================================================= device tables
struct ZBlob {
    uint64_t src, dst, len;     // byte offsets into the source / frame buffers, blob length
    uint32_t first_block, nblocks;
    uint32_t wlog, hlog, clog, mls;
    uint32_t slot, base;        // hash-table slot and its index base for this use
    uint32_t raw_mask;          // blocks the parse treats as not compressed (repeat offsets kept)
    uint32_t flags;             // 1: the decisions contradicted raw_mask where it mattered (rerun)
    uint64_t frame_len;
#ifdef BW_ZSTD_TIMING
    uint64_t tm[8];             // parse section cycles: probe, length, catch-up, inserts; steps, sequences
#endif
};

struct ZBlock {
    uint64_t off;               // block offset in its blob
    uint64_t seq0, lit0, sec0;  // scratch: first sequence slot, literal bytes, section bytes
    uint64_t out;               // frame buffer offset of the block header (k_zs_decide)
    uint64_t lit_hdr;           // literal section header value (lh_size bytes, little endian)
    uint32_t blob, bs;
    uint32_t nseq, nlit, last_ll;  // sequences, literals, literals after the last sequence
    uint32_t rep_in[3], rep_out[3];
    uint32_t is_rle;            // the block is one repeated byte (only tested when it can matter)
    uint32_t sec_len, sec_hdr;  // sequence section: header bytes at sec0, bitstream at sec0 + SEC_HDR
    uint32_t sec_bad;           // libzstd emits the block raw (old-decoder NCount rule, or oversized)
    uint32_t type, body, last;  // BT_*, body bytes after the 3-byte header, last-block bit
    uint32_t lit_kind, lh_size, huf_hdr_len, streams;
    uint32_t stream_len[4];
};

namespace zs {

// ======================================================================= k_zs_parse
// count of equal bytes at a and b (b < a), up to limit (offsets in s): the wave compares 512 bytes
// per step (ZSTD_count).
__device__ uint32_t wave_count(const uint8_t* s, uint32_t a, uint32_t b, uint32_t limit, uint32_t lane) {
    uint32_t n = 0;
    while (a + n < limit) {
        const uint32_t o = a + n + 8 * lane, m = b + n + 8 * lane;
        uint32_t fd = 8;
        if (o + 8 <= limit) {
            const uint64_t x = ld64(s + o) ^ ld64(s + m);
            if (x) fd = (uint32_t)__builtin_ctzll(x) >> 3;
        } else if (o < limit) {
            const uint32_t rem = limit - o;
            fd = rem;
            for (uint32_t i = 0; i < rem; i++)
                if (s[o + i] != s[m + i]) { fd = i; break; }
        } else {
            fd = 0;
        }
        const uint64_t mm = __ballot(fd < 8);
        if (mm) {
            const uint32_t L = (uint32_t)__builtin_ctzll(mm);
            n += 8 * L + rdlane(fd, L);
            break;
        }
        n += 512;
    }
    return (a + n > limit) ? limit - a : n;
}

// A match's forward length beyond a (vs b, up to limit) and its backward extension before pb (vs mb, up
// to lim byte pairs), with the first 512 forward bytes and the first 64 backward pairs loaded in one
// round (wave_count and the catch-up loop continue when those are all equal).
__device__ void wave_extend(const uint8_t* s, uint32_t a, uint32_t b, uint32_t limit, uint32_t pb, uint32_t mb,
                            uint32_t lim, uint32_t lane, uint32_t& fwd, uint32_t& back) {
    const bool bin = lane < lim;
    uint8_t bp = 0, bm = 1;
    if (bin) {
        bp = s[pb - 1 - lane];
        bm = s[mb - 1 - lane];
    }
    uint32_t fd = 8;
    const uint32_t o = a + 8 * lane, m = b + 8 * lane;
    if (o + 8 <= limit) {
        const uint64_t x = ld64(s + o) ^ ld64(s + m);
        if (x) fd = (uint32_t)__builtin_ctzll(x) >> 3;
    } else if (o < limit) {
        const uint32_t rem = limit - o;
        fd = rem;
        for (uint32_t i = 0; i < rem; i++)
            if (s[o + i] != s[m + i]) { fd = i; break; }
    } else {
        fd = 0;
    }
    const bool beq = bin && bp == bm;
    const uint64_t mm = __ballot(fd < 8), ne = __ballot(!beq);
    if (mm) {
        const uint32_t L = (uint32_t)__builtin_ctzll(mm);
        const uint32_t n = 8 * L + rdlane(fd, L);
        fwd = (a + n > limit) ? limit - a : n;
    } else {
        fwd = 512 + wave_count(s, a + 512, b + 512, limit, lane);
    }
    back = ne ? (uint32_t)__builtin_ctzll(ne) : 64u;
    if (back == 64) {
        while (back < lim) {
            const uint32_t kk = back + lane;
            const bool eq = kk < lim && s[pb - 1 - kk] == s[mb - 1 - kk];
            const uint64_t nn = __ballot(!eq);
            const uint32_t f = nn ? (uint32_t)__builtin_ctzll(nn) : 64u;
            back += f;
            if (f < 64) break;
        }
    }
}

// The step's table writes reach the next probes of other lanes through a workgroup fence (a wait
// for the wave's outstanding stores).  BW_ZS_NOFENCE (diagnostic measurement only, not exact by
// the memory model) drops the two in the step loop to size what those waits cost.
#ifdef BW_ZS_NOFENCE
#define BW_ZS_FENCE() ((void)0)
#else
#define BW_ZS_FENCE() __threadfence_block()
#endif
#ifndef BW_ZS_WMIN
#define BW_ZS_WMIN 2  // probe window after a match at lane 0 (text: the mean first-match lane is 0.2-0.3)
#endif

constexpr uint32_t DUP_SLOTS = 128;  // 2 KiB of LDS: up to 8 waves per SIMD (one blob per wave)
constexpr uint32_t SMALL_W = 8;      // windows of up to this many positions find bucket-mates in registers
constexpr uint32_t ZS_WIDE_MAX_BLOBS = 2048;  // sub-batches of at most this many blobs use wide tables (~2 per SIMD)

// A slot's two tables in one of two layouts (host: zstd_compress picks one per sub-batch):
//   wide    entries carry the bytes at their position (long 16 B, short 8 B): a probe answers the
//           match test itself -- one dependent round fewer, for calls of few blobs, where one
//           wave per SIMD waits out every round;
//   narrow  libzstd's u32 positions (768 KiB of the slot) and a round of candidate loads -- for
//           many blobs, where the 3.3x smaller tables keep more of the caches and TLBs.
template <bool WIDE>
struct ZTab;
template <>
struct ZTab<true> {
    uint4* hl;
    uint2* hs;
    __device__ explicit ZTab(uint32_t* slot) : hl((uint4*)slot), hs((uint2*)(slot + (4u << HL_MAX))) {}
    __device__ void probe(uint32_t h2, uint32_t h, uint32_t h3, uint32_t& mil, uint64_t& xL, uint32_t& mis,
                          uint32_t& xS, uint32_t& m3, uint64_t& x3) const {
        const uint4 eL = hl[h2], e3 = hl[h3];
        const uint2 eS = hs[h];
        mil = eL.x;
        xL = (uint64_t)eL.w << 32 | eL.z;
        mis = eS.x;
        xS = eS.y;
        m3 = e3.x;
        x3 = (uint64_t)e3.w << 32 | e3.z;
    }
    __device__ void put_long(uint32_t k, uint32_t pos, uint64_t v) const {
        hl[k] = make_uint4(pos, 0u, (uint32_t)v, (uint32_t)(v >> 32));
    }
    __device__ void put_short(uint32_t k, uint32_t pos, uint64_t v) const { hs[k] = make_uint2(pos, (uint32_t)v); }
};
template <>
struct ZTab<false> {
    uint32_t* hl;
    uint32_t* hs;
    __device__ explicit ZTab(uint32_t* slot) : hl(slot), hs(slot + (1u << HL_MAX)) {}
    __device__ void probe(uint32_t h2, uint32_t h, uint32_t h3, uint32_t& mil, uint64_t&, uint32_t& mis, uint32_t&,
                          uint32_t& m3, uint64_t&) const {
        mil = hl[h2];
        mis = hs[h];
        m3 = hl[h3];
    }
    __device__ void put_long(uint32_t k, uint32_t pos, uint64_t) const { hl[k] = pos; }
    __device__ void put_short(uint32_t k, uint32_t pos, uint64_t) const { hs[k] = pos; }
};

// The parse of one blob, with the short table's hash length MLS fixed at compile time (level 3
// uses 4 or 5, by blob size; a runtime switch cost ~15 instructions a hash, several a step).
template <uint32_t MLS, bool WIDE>
__device__ void parse_blob(const uint8_t* __restrict__ src, ZBlob* __restrict__ blobs, ZBlock* __restrict__ blocks,
                           uint32_t* tables, uint64_t* __restrict__ seqs, const uint32_t bi, const ZBlob& B,
                           unsigned long long* s_mL, unsigned long long* s_mS, uint32_t* s_h2, uint32_t* s_h,
                           uint32_t* s_cu, unsigned long long* s_v8) {
    const uint32_t lane = threadIdx.x;
    const uint8_t* s = src + B.src;
    const ZTab<WIDE> T(tables + (uint64_t)B.slot * (WIDE ? SLOT_WORDS : NARROW_WORDS));
    const uint32_t ib = B.base + 1;  // index of s[0] (libzstd: dictLimit)
    const uint32_t hlog = B.hlog, clog = B.clog, maxD = 1u << B.wlog;
    const uint32_t mls = MLS ? MLS : B.mls;  // MLS 0: any length, switched at run time
    uint32_t rep0 = 1, rep1 = 4, rep2 = 8;
    // Probe window: a step tests the next W positions of the skip sequence (W <= 64 lanes).  Every
    // probe is a random 16-byte read from a 2.5 MiB table (a cache line from HBM), and on
    // compressible data the first match is usually a few positions ahead, so probing all 64
    // positions fetched ~20x the lines the step consumes.  W follows the data: it doubles after a
    // step without a match and shrinks to ~2x the matched lane after one.  Any W is exact (the
    // lanes past the window are simply tested by a later step).
    uint32_t W = 64;
#ifdef BW_ZSTD_TIMING
    uint64_t tm[8] = {0, 0, 0, 0, 0, 0, 0, 0}, zlast = 0;
#define ZT_START() (zlast = __builtin_amdgcn_s_memtime())
#define ZT_LAP(i)                                              \
    do {                                                       \
        const uint64_t zn_ = __builtin_amdgcn_s_memtime();     \
        tm[i] += zn_ - zlast;                                  \
        zlast = zn_;                                           \
    } while (0)
#define ZT_COUNT(i) (tm[i]++)
#else
#define ZT_START() ((void)0)
#define ZT_LAP(i) ((void)0)
#define ZT_COUNT(i) ((void)0)
#endif
    for (uint32_t k = 0; k < B.nblocks; k++) {
        ZBlock* blk = blocks + B.first_block + k;
        const uint32_t bs = blk->bs, off = (uint32_t)blk->off;
        uint64_t* sq = seqs + blk->seq0;
        uint32_t nseq = 0, r0 = rep0, r1 = rep1;
        if (bs >= 7) {
            const uint32_t iend = off + bs, ilimit = iend >= 8 ? iend - 8 : 0;  // libzstd: iend - 8 (below istart: no search)
            const uint32_t endIndex = ib + iend;
            const uint32_t pli = (endIndex - ib > maxD) ? endIndex - maxD : ib;  // prefixLowestIndex
            const uint32_t plo = pli - ib;
            uint32_t ip = off, anchor = off, o1 = rep0, o2 = rep1, saved = 0;
            if (ip == plo) ip++;
            {
                const uint32_t curr = ib + ip;
                const uint32_t wl = (curr - ib > maxD) ? curr - maxD : ib;
                const uint32_t maxRep = curr - wl;
                if (o2 > maxRep) { saved = o2; o2 = 0; }
                if (o1 > maxRep) { saved = o1; o1 = 0; }
            }
            // the next step's probe data (pos = ip + lane), loaded in the same round as the previous
            // match's insert keys and repeat check
            bool pre = false;
            uint64_t pv8 = 0, pv8n = 0;
            uint32_t pvrep = 0;
            while (ip < ilimit) {
                BW_ZS_FENCE();
                ZT_START();
                ZT_COUNT(4);
                // this lane's position in the skip sequence ip += ((ip - anchor) >> 8) + 1
                uint32_t d = ip - anchor;
                if (d + 63 < 256) {
                    d += lane;  // step 1 for every lane
                } else {
                    // the skip sequence is uniform: walk it once in scalar registers and hand
                    // position i to lane i (per-lane walks with a division per step change cost
                    // ~2k VALU instructions a step on incompressible data, where the step grows
                    // every position)
                    uint32_t dd = __builtin_amdgcn_readfirstlane(d), pd = 0;
                    const uint32_t w = __builtin_amdgcn_readfirstlane(W);
                    for (uint32_t i = 0; i < w; i++) {
                        pd = lane == i ? dd : pd;
                        dd += (dd >> 8) + 1;
                    }
                    d = pd;
                }
                const uint32_t pos = anchor + d;
                const bool valid = pos < ilimit && lane < W;
                // Loads are issued unconditionally (lanes without a use read a safe address) so that
                // each round of a step is one trip to memory: a load under a divergent branch makes
                // the compiler wait for it inside the branch.
                uint64_t v8 = 0, v8n = 0;
                uint32_t vrep = 0;
                if (pre) {  // set only after a match: anchor == ip, so pos == ip + lane
                    v8 = pv8; v8n = pv8n; vrep = pvrep;
                } else if (valid) {
                    v8 = ld64(s + pos);
                    v8n = ld64(s + pos + 1);
                    vrep = ld32(s + pos + 1 - o1);
                }
                pre = false;
                // Round of table probes: the long and short tables at pos, and -- speculatively, for the
                // small-match path -- the long table at pos + 1 (libzstd's search_next_long)
                const uint32_t h2 = hash_long(v8, hlog), h = hash_small(v8, clog, mls), h3 = hash_long(v8n, hlog);
                uint32_t mil = 0, mis = 0, m3 = 0;
                uint64_t xL = 0, x3 = 0;  // the bytes at each candidate (wide: from its table entry)
                uint32_t xS = 0;
                if (valid) T.probe(h2, h, h3, mil, xL, mis, xS, m3, x3);
                const uint32_t curr = ib + pos;
                const uint64_t vmask = __ballot(valid);
                const uint32_t nvalid = (uint32_t)__popcll(vmask);
                // writes of earlier lanes to the same slots reach this lane's probes (the serial
                // loop writes every visited position before it moves on).  Only lanes whose hash
                // shares a bucket of a small LDS map with another lane can be involved: each lane
                // ORs its bit into its two buckets, then walks only its own bucket-mates (usually
                // none), nearest first: the latest earlier lane with the same hash supplies the probe
                // value, the nearest later one decides whether this lane's table write survives the
                // step.  The pos + 1 probe sees the long-table writes up to and including its own lane.
                uint32_t nextL = 64, nextS = 64;
                if (nvalid <= SMALL_W) {
                    // a short window (the usual case after a match: W = 2): each valid lane (a
                    // prefix of the wave) reads the others' keys from their registers, in lane
                    // order; lanes outside the window keep their empty probes
                    for (uint32_t i = 0; i < nvalid; i++) {
                        const uint32_t hi2 = rdlane(h2, i), hi = rdlane(h, i), ci = rdlane(curr, i);
                        const uint64_t vi = (uint64_t)rdlane((uint32_t)(v8 >> 32), i) << 32 | rdlane((uint32_t)v8, i);
                        if (!valid) continue;
                        if (hi2 == h2) {
                            if (i < lane) { mil = ci; xL = vi; }
                            else if (i > lane && nextL == 64) nextL = i;
                        }
                        if (hi == h) {
                            if (i < lane) { mis = ci; xS = (uint32_t)vi; }
                            else if (i > lane && nextS == 64) nextS = i;
                        }
                        if (i <= lane && hi2 == h3) { m3 = ci; x3 = vi; }
                    }
                } else {
                uint64_t mL = 0, mS = 0, m3L = 0;
                if (valid) {
                    atomicOr(&s_mL[h2 & (DUP_SLOTS - 1)], 1ull << lane);
                    atomicOr(&s_mS[h & (DUP_SLOTS - 1)], 1ull << lane);
                    s_h2[lane] = h2;
                    s_h[lane] = h;
                    s_cu[lane] = curr;
                    s_v8[lane] = v8;
                }
                __builtin_amdgcn_wave_barrier();
                if (valid) { mL = s_mL[h2 & (DUP_SLOTS - 1)]; mS = s_mS[h & (DUP_SLOTS - 1)]; m3L = s_mL[h3 & (DUP_SLOTS - 1)]; }
                __builtin_amdgcn_wave_barrier();
                if (valid) { s_mL[h2 & (DUP_SLOTS - 1)] = 0; s_mS[h & (DUP_SLOTS - 1)] = 0; }
                __builtin_amdgcn_wave_barrier();
                if (valid) {
                    const uint64_t below = (1ull << lane) - 1, above = ~below & ~(1ull << lane);
                    for (uint64_t c = mL & below; c; c &= ~(1ull << (63 - __builtin_clzll(c)))) {
                        const uint32_t i = 63 - (uint32_t)__builtin_clzll(c);
                        if (s_h2[i] == h2) { mil = s_cu[i]; xL = s_v8[i]; break; }
                    }
                    for (uint64_t c = mL & above; c; c &= c - 1) {
                        const uint32_t i = (uint32_t)__builtin_ctzll(c);
                        if (s_h2[i] == h2) { nextL = i; break; }
                    }
                    for (uint64_t c = mS & below; c; c &= ~(1ull << (63 - __builtin_clzll(c)))) {
                        const uint32_t i = 63 - (uint32_t)__builtin_clzll(c);
                        if (s_h[i] == h) { mis = s_cu[i]; xS = (uint32_t)s_v8[i]; break; }
                    }
                    for (uint64_t c = mS & above; c; c &= c - 1) {
                        const uint32_t i = (uint32_t)__builtin_ctzll(c);
                        if (s_h[i] == h) { nextS = i; break; }
                    }
                    for (uint64_t c = m3L & (below | (1ull << lane)); c; c &= ~(1ull << (63 - __builtin_clzll(c)))) {
                        const uint32_t i = 63 - (uint32_t)__builtin_clzll(c);
                        if (s_h2[i] == h3) { m3 = s_cu[i]; x3 = s_v8[i]; break; }
                    }
                }
                __builtin_amdgcn_wave_barrier();
                }
                // the evidence of every path at once (the candidates' bytes came with the probes)
                const bool cL = mil > pli, cS = mis > pli, c3 = m3 > pli;  // (invalid lanes: 0, never > pli)
                if constexpr (!WIDE) {  // narrow tables: a round of candidate loads
                    if (cL) xL = ld64(s + (mil - ib));
                    if (c3) x3 = ld64(s + (m3 - ib));
                    if (cS) xS = ld32(s + (mis - ib));
                }
                const bool evR = valid && o1 && vrep == (uint32_t)v8n;
                const bool evL = cL && xL == v8, evS = cS && xS == (uint32_t)v8, ev3 = c3 && x3 == v8n;
                const uint64_t emask = __ballot(evR || evL || evS);
                ZT_LAP(0);
                const uint32_t lastw = emask ? (uint32_t)__builtin_ctzll(emask) : nvalid - 1;
                if (valid && lane <= lastw) {
                    if (nextL > lastw) T.put_long(h2, curr, v8);
                    if (nextS > lastw) T.put_short(h, curr, v8);
                }
                if (!emask) {
                    const uint32_t pl = rdlane(pos, nvalid - 1);
                    ip = pl + ((pl - anchor) >> 8) + 1;
                    W = W < 32 ? 2 * W : 64;
                    continue;
                }
                BW_ZS_FENCE();
                const uint32_t e = lastw;
                W = e < BW_ZS_WMIN / 2 ? BW_ZS_WMIN : (e < 4 ? 8 : (e < 8 ? 16 : (e < 16 ? 32 : 64)));
                uint32_t p = rdlane(pos, e);
                const uint32_t cu = ib + p;
                const bool eR = rdlane(evR, e), eL = rdlane(evL, e);
                ZT_COUNT(5);
#ifdef BW_ZSTD_TIMING
                tm[2] += e;
                if (!eR && !eL) tm[7]++;
#endif
                // the match: start p, candidate m (offsets in s), bytes already known equal, and the
                // backward (catch-up) limit; then one round of loads extends it both ways
                uint32_t m, known, lim = 0;
                if (eR) {
                    p++;
                    m = p - o1;
                    known = 4;
                } else if (eL) {
                    m = rdlane(mil, e) - ib;
                    known = 8;
                } else {
                    const uint32_t n3lo = rdlane((uint32_t)v8n, e), n3hi = rdlane((uint32_t)(v8n >> 32), e);
                    if (lane == 0) T.put_long(rdlane(h3, e), cu + 1, (uint64_t)n3hi << 32 | n3lo);
                    if (rdlane(ev3, e)) {
                        m = rdlane(m3, e) - ib;
                        p++;
                        known = 8;
                    } else {
                        m = rdlane(mis, e) - ib;
                        known = 4;
                    }
                }
                if (!eR) lim = (p - anchor) < (m - plo) ? p - anchor : m - plo;
                uint32_t fwd, back;
                wave_extend(s, p + known, m + known, iend, p, m, lim, lane, fwd, back);
                uint32_t mLength = fwd + known;
                if (eR) {
                    if (lane == 0) sq[nseq] = seq_pack(p - anchor, mLength - 3, 1);
                    nseq++;
                } else {
                    const uint32_t offset = p - m;
                    p -= back;
                    mLength += back;
                    o2 = o1;
                    o1 = offset;
                    if (lane == 0) sq[nseq] = seq_pack(p - anchor, mLength - 3, offset + 3);
                    nseq++;
                }
                ZT_LAP(1);
                p += mLength;
                anchor = p;
                if (p <= ilimit) {
                    // one round of loads: the four insert keys, the repeat check and the next step's data
                    const uint32_t iti = cu + 2, pti = iti - ib;
                    const uint64_t a8 = ld64(s + pti), b8 = ld64(s + p - 2), c8 = ld64(s + p - 1);
                    uint32_t rA = ld32(s + p), rB = ld32(s + p - o2);
                    // lanes past ilimit read at p - 1 (p <= ilimit: bytes up to iend, never past the block)
                    if (p + lane < ilimit) {
                        pv8 = ld64(s + p + lane);
                        pv8n = ld64(s + p + lane + 1);
                        pvrep = ld32(s + p + lane + 1 - o1);
                    }
                    if (!o2) rB = ~rA;
                    pre = true;
                    if (lane == 0) {
                        T.put_long(hash_long(a8, hlog), iti, a8);
                        T.put_long(hash_long(b8, hlog), ib + p - 2, b8);
                        T.put_short(hash_small(a8, clog, mls), iti, a8);
                        T.put_short(hash_small(c8, clog, mls), ib + p - 1, c8);
                    }
                    while (o2 > 0 && rA == rB) {
                        const uint32_t rL = wave_count(s, p + 4, p + 4 - o2, iend, lane) + 4;
                        const uint32_t t = o2;
                        o2 = o1;
                        o1 = t;
                        const uint64_t v = ld64(s + p);
                        if (lane == 0) {
                            T.put_short(hash_small(v, clog, mls), ib + p, v);
                            T.put_long(hash_long(v, hlog), ib + p, v);
                            sq[nseq] = seq_pack(0, rL - 3, 1);
                        }
                        nseq++;
                        p += rL;
                        anchor = p;
                        pre = false;
                        ZT_COUNT(6);
                        if (p > ilimit) break;
                        rA = ld32(s + p);
                        rB = o2 ? ld32(s + p - o2) : ~rA;
                    }
                }
                ZT_LAP(3);
                ip = p;
            }
            r0 = o1 ? o1 : saved;
            r1 = o2 ? o2 : saved;
            if (lane == 0) blk->last_ll = iend - anchor;
        }
        if (lane == 0) {
            blk->nseq = nseq;
            blk->rep_in[0] = rep0; blk->rep_in[1] = rep1; blk->rep_in[2] = rep2;
            blk->rep_out[0] = r0; blk->rep_out[1] = r1; blk->rep_out[2] = rep2;
        }
        if (!((B.raw_mask >> k) & 1)) { rep0 = r0; rep1 = r1; }
        __threadfence_block();
    }
#ifdef BW_ZSTD_TIMING
    if (lane == 0)
        for (int i = 0; i < 8; i++) blobs[bi].tm[i] += tm[i];
#endif
}

__global__ __launch_bounds__(64) void k_zs_parse(const uint8_t* __restrict__ src, ZBlob* __restrict__ blobs,
                                                 ZBlock* __restrict__ blocks, uint32_t* tables,
                                                 uint64_t* __restrict__ seqs, const uint32_t* __restrict__ active,
                                                 int wide) {
    const uint32_t bi = active ? active[blockIdx.x] : blockIdx.x;
    __shared__ unsigned long long s_mL[DUP_SLOTS], s_mS[DUP_SLOTS];
    __shared__ uint32_t s_h2[64], s_h[64], s_cu[64];
    __shared__ unsigned long long s_v8[64];
    for (uint32_t i = threadIdx.x; i < DUP_SLOTS; i += 64) { s_mL[i] = 0; s_mS[i] = 0; }
    __builtin_amdgcn_wave_barrier();
    const ZBlob B = blobs[bi];
#define BW_ZS_PARSE(M, W) parse_blob<M, W>(src, blobs, blocks, tables, seqs, bi, B, s_mL, s_mS, s_h2, s_h, s_cu, s_v8)
    if (wide) {
        if (B.mls == 5) BW_ZS_PARSE(5, true);
        else if (B.mls == 4) BW_ZS_PARSE(4, true);
        else BW_ZS_PARSE(0, true);  // (not at level 3)
    } else {
        if (B.mls == 5) BW_ZS_PARSE(5, false);
        else if (B.mls == 4) BW_ZS_PARSE(4, false);
        else BW_ZS_PARSE(0, false);
    }
#undef BW_ZS_PARSE
}

// ======================================================================= k_zs_stats
constexpr int ST_THREADS = 256;
constexpr int ST_CHUNK = 1024;  // sequences staged in LDS per step of the backward FSE pass

constexpr int ST_BITW = (ST_CHUNK * 80 + 63) / 32 + 2;  // LDS words of one chunk's bitstream (<= 80 bits a sequence)

struct StatsLds {
    union {
        uint32_t hist[4][4][256];  // [wave][segment][byte] (literal statistics)
        struct {                   // then the sequences bitstream, one chunk at a time
            uint32_t code[ST_CHUNK];      // ll code | of code << 8 | ml code << 16, in stream order
            uint32_t sbits[3][ST_CHUNK];  // FSE state output of the OF / ML / LL chains: nbits << 16 | bits
            uint32_t bitbuf[ST_BITW];
        } bs;
    };
    uint32_t cll[36], cof[32], cml[53];
    uint32_t scanA[ST_THREADS], scanB[ST_THREADS];
    uint32_t nlong;
    uint32_t longs[256][3];        // long literal runs: src offset, literal index, length
    uint64_t chunk[ST_CHUNK];
    uint16_t stLL[512], stOF[256], stML[512];
    FseTT ttLL[36], ttOF[32], ttML[53];
    uint8_t spread[512];
    int16_t norm[53];
    uint32_t flag;
};

__device__ void section_tables(StatsLds& L, uint32_t* count, uint32_t maxSym, uint32_t nseq, uint32_t defLog,
                               uint32_t fseLog, const int16_t* defNorm, uint32_t defMax, bool defAllowed,
                               uint32_t lastCode, uint16_t* state, FseTT* tt, uint8_t* out, uint32_t& o,
                               uint32_t& type, uint32_t& tlog, int32_t& lastNC) {
    uint32_t maxSV = maxSym, mf = 0;
    while (maxSV > 0 && !count[maxSV]) maxSV--;
    for (uint32_t s = 0; s <= maxSV; s++) mf = count[s] > mf ? count[s] : mf;
    // ZSTD_selectEncodingType for strategies below lazy (dfast: mult = 8)
    if (mf == nseq) type = (defAllowed && nseq <= 2) ? SET_BASIC : SET_RLE;
    else if (defAllowed && (nseq < ((1u << defLog) * 8u) >> 3 || mf < (nseq >> (defLog - 1)))) type = SET_BASIC;
    else type = SET_COMPRESSED;
    if (type == SET_RLE) {
        tlog = 0;
        state[0] = 0; state[1] = 0;
        tt[maxSV].dfs = 0; tt[maxSV].dnb = 0;
        out[o++] = (uint8_t)maxSV;
    } else if (type == SET_BASIC) {
        tlog = defLog;
        fse_build(state, tt, L.spread, defNorm, defMax, defLog);
    } else {
        tlog = fse_optimal_log(fseLog, nseq, maxSV, 2);
        uint32_t n1 = nseq;
        if (count[lastCode] > 1) { count[lastCode]--; n1--; }
        fse_normalize(L.norm, tlog, count, n1, maxSV, n1 >= 2048);
        lastNC = (int32_t)o;
        o += fse_write_ncount(out + o, L.norm, maxSV, tlog);
        fse_build(state, tt, L.spread, L.norm, maxSV, tlog);
    }
}

__global__ __launch_bounds__(ST_THREADS) void k_zs_stats(const uint8_t* __restrict__ src, const ZBlob* __restrict__ blobs,
                                                         ZBlock* __restrict__ blocks, const uint64_t* __restrict__ seqs,
                                                         uint8_t* __restrict__ lits, uint8_t* __restrict__ sec,
                                                         uint32_t* __restrict__ hist_out, const uint32_t* __restrict__ active) {
    __shared__ StatsLds L;
    const uint32_t b = active ? active[blockIdx.x] : blockIdx.x;
    const uint32_t t = threadIdx.x, wave = t >> 6;
    ZBlock* blk = blocks + b;
    const uint32_t bs = blk->bs;
    uint32_t* hout = hist_out + (uint64_t)b * 1024;
    if (bs < 7) {
        if (t == 0) { blk->is_rle = 0; blk->sec_len = 0; blk->sec_hdr = 0; blk->sec_bad = 1; blk->nlit = 0; }
        return;
    }
    const uint8_t* s = src + blobs[blk->blob].src + blk->off;  // the block's bytes
    const uint64_t* sq = seqs + blk->seq0;
    const uint32_t nseq = blk->nseq, lastLL = blk->last_ll;
    for (uint32_t i = t; i < 4 * 4 * 256; i += ST_THREADS) (&L.hist[0][0][0])[i] = 0;
    for (uint32_t i = t; i < 36; i += ST_THREADS) L.cll[i] = 0;
    for (uint32_t i = t; i < 32; i += ST_THREADS) L.cof[i] = 0;
    for (uint32_t i = t; i < 53; i += ST_THREADS) L.cml[i] = 0;
    if (t == 0) { L.nlong = 0; L.flag = 0; }
    // per-thread chunk of sequences: literal and source totals, then a workgroup scan
    const uint32_t per = (nseq + ST_THREADS - 1) / ST_THREADS;
    const uint32_t q0 = t * per < nseq ? t * per : nseq, q1 = q0 + per < nseq ? q0 + per : nseq;
    uint32_t sl = 0, ss = 0;
    for (uint32_t i = q0; i < q1; i++) {
        const uint64_t q = sq[i];
        sl += seq_ll(q);
        ss += seq_ll(q) + seq_mb(q) + 3;
    }
    L.scanA[t] = sl;
    L.scanB[t] = ss;
    __syncthreads();
    for (uint32_t d = 1; d < ST_THREADS; d <<= 1) {
        const uint32_t a = t >= d ? L.scanA[t - d] : 0, c = t >= d ? L.scanB[t - d] : 0;
        __syncthreads();
        L.scanA[t] += a;
        L.scanB[t] += c;
        __syncthreads();
    }
    const uint32_t litTotal = L.scanA[ST_THREADS - 1] + lastLL;
    const uint32_t srcTotal = L.scanB[ST_THREADS - 1];
    const uint32_t seg = (litTotal + 3) / 4, seg2 = 2 * seg, seg3 = 3 * seg;
    // Huffman segment of literal i (i < litTotal <= 4 * seg): compares, not a division per byte
    auto seg_of = [&](uint32_t i) -> uint32_t { return (uint32_t)(i >= seg) + (i >= seg2) + (i >= seg3); };
    uint8_t* lo = lits + blk->lit0;
    // literal gather + segment histograms + code histograms
    {
        uint32_t li = L.scanA[t] - sl, si = L.scanB[t] - ss;
        for (uint32_t i = q0; i < q1; i++) {
            const uint64_t q = sq[i];
            const uint32_t ll = seq_ll(q), mb = seq_mb(q), ov = seq_ov(q);
            if (ll > 32) {
                const uint32_t k = atomicAdd(&L.nlong, 1u);
                if (k < 256) { L.longs[k][0] = si; L.longs[k][1] = li; L.longs[k][2] = ll; }
                else
                    for (uint32_t x = 0; x < ll; x++) {
                        const uint8_t c = s[si + x];
                        lo[li + x] = c;
                        atomicAdd(&L.hist[wave][seg_of(li + x)][c], 1u);
                    }
            } else {
                for (uint32_t x = 0; x < ll; x++) {
                    const uint8_t c = s[si + x];
                    lo[li + x] = c;
                    atomicAdd(&L.hist[wave][seg_of(li + x)][c], 1u);
                }
            }
            atomicAdd(&L.cll[ll_code(ll)], 1u);
            atomicAdd(&L.cof[hb32(ov)], 1u);
            atomicAdd(&L.cml[ml_code(mb)], 1u);
            li += ll;
            si += ll + mb + 3;
        }
    }
    // the last literals
    {
        // four bytes per thread and step (a random block is one 128 KiB run of last literals)
        const uint32_t li0 = litTotal - lastLL, si0 = srcTotal, n4 = lastLL & ~3u;
        for (uint32_t x = 4 * t; x < n4; x += 4 * ST_THREADS) {
            const uint32_t w = ld32(s + si0 + x);
            *(u32u*)(lo + li0 + x) = w;
#pragma unroll
            for (int j = 0; j < 4; j++) atomicAdd(&L.hist[wave][seg_of(li0 + x + j)][(w >> (8 * j)) & 255u], 1u);
        }
        for (uint32_t x = n4 + t; x < lastLL; x += ST_THREADS) {
            const uint8_t c = s[si0 + x];
            lo[li0 + x] = c;
            atomicAdd(&L.hist[wave][seg_of(li0 + x)][c], 1u);
        }
    }
    __syncthreads();
    {
        const uint32_t nl = L.nlong < 256 ? L.nlong : 256;
        for (uint32_t k = 0; k < nl; k++) {
            const uint32_t si = L.longs[k][0], li = L.longs[k][1], ll = L.longs[k][2];
            for (uint32_t x = t; x < ll; x += ST_THREADS) {
                const uint8_t c = s[si + x];
                lo[li + x] = c;
                atomicAdd(&L.hist[wave][seg_of(li + x)][c], 1u);
            }
        }
    }
    // RLE block test (only where libzstd's decision can depend on it: an RLE block parses into
    // a couple of sequences and literals)
    if (nseq <= 16 && litTotal <= 64) {
        const uint8_t c0 = s[0];
        bool diff = false;
        for (uint32_t x = t; x < bs; x += ST_THREADS) diff |= s[x] != c0;
        if (diff) atomicOr(&L.flag, 1u);
    } else if (t == 0) {
        L.flag = 1;
    }
    __syncthreads();
    for (uint32_t i = t; i < 1024; i += ST_THREADS) {
        const uint32_t k = i >> 8, c = i & 255;
        hout[i] = L.hist[0][k][c] + L.hist[1][k][c] + L.hist[2][k][c] + L.hist[3][k][c];
    }
    // the sequences section
    uint8_t* so = sec + blk->sec0;
    uint8_t* bo = so + SEC_HDR;
    if (nseq == 0) {
        if (t == 0) {
            so[0] = 0;
            blk->sec_hdr = 1; blk->sec_len = 1; blk->sec_bad = 0;
            blk->nlit = litTotal;
            blk->is_rle = L.flag ? 0 : 1;
        }
        return;
    }
    __shared__ uint32_t s_hdr, s_logs, s_lastNC;
    if (t == 0) {
        uint32_t o = 0;
        if (nseq < 128) so[o++] = (uint8_t)nseq;
        else if (nseq < 0x7F00) { so[o++] = (uint8_t)((nseq >> 8) + 0x80); so[o++] = (uint8_t)nseq; }
        else { so[o++] = 0xFF; so[o++] = (uint8_t)(nseq - 0x7F00); so[o++] = (uint8_t)((nseq - 0x7F00) >> 8); }
        const uint32_t headAt = o++;
        const uint64_t ql = sq[nseq - 1];
        int32_t lastNC = -1;
        uint32_t tLL, tOF, tML, gLL, gOF, gML;
        section_tables(L, L.cll, MAXLL, nseq, 6, LLFSELOG, c_LL_norm, MAXLL, true, ll_code(seq_ll(ql)), L.stLL,
                       L.ttLL, so, o, tLL, gLL, lastNC);
        uint32_t mo = MAXOFF;
        while (mo > 0 && !L.cof[mo]) mo--;
        section_tables(L, L.cof, MAXOFF, nseq, 5, OFFFSELOG, c_OF_norm, DEFAULT_MAXOFF, mo <= DEFAULT_MAXOFF,
                       hb32(seq_ov(ql)), L.stOF, L.ttOF, so, o, tOF, gOF, lastNC);
        section_tables(L, L.cml, MAXML, nseq, 6, MLFSELOG, c_ML_norm, MAXML, true, ml_code(seq_mb(ql)), L.stML,
                       L.ttML, so, o, tML, gML, lastNC);
        so[headAt] = (uint8_t)((tLL << 6) + (tOF << 4) + (tML << 2));
        s_hdr = o;
        s_logs = gLL | (gOF << 8) | (gML << 16);
        s_lastNC = (uint32_t)lastNC;
    }
    __syncthreads();
    // The backward sequences bitstream, in the order libzstd's bit writer produces it (sequence
    // nseq - 1 first), one chunk of ST_CHUNK sequences at a time: every thread computes codes; lanes
    // 0..2 of wave 0 run the three FSE state chains (OF, ML, LL) side by side over the chunk; every
    // thread then places the six fields of its sequences at their bit offsets (a workgroup scan of
    // the field lengths) in an LDS word buffer, which is stored as whole words.  The partially
    // filled last word carries into the next chunk.  (One lane writing bytes serially took ~1/3 of
    // the whole compressor's time.)
    const uint32_t capB = bs + 64, capW = capB / 4;  // libzstd's limit: longer sections go raw
    uint32_t* bo32 = (uint32_t*)bo;
    const uint32_t gLL = s_logs & 255, gOF = (s_logs >> 8) & 255, gML = s_logs >> 16;
    const uint16_t* stAll = L.stLL;  // stLL[512] | stOF[256] | stML[512]
    const FseTT* ttAll = L.ttLL;     // ttLL[36] | ttOF[32] | ttML[53]
    const uint32_t stb = t == 0 ? 512 : (t == 1 ? 768 : 0), ttb = t == 0 ? 36 : (t == 1 ? 68 : 0);
    const uint32_t csh = t == 0 ? 8 : (t == 1 ? 16 : 0);
    uint32_t fv = 0;  // the chain's FSE state (lanes 0..2)
    uint64_t bitpos = 0;
    uint32_t carry = 0;
    for (uint32_t hi = nseq; hi > 0;) {
        const uint32_t lo_i = hi > (uint32_t)ST_CHUNK ? hi - ST_CHUNK : 0, m = hi - lo_i;
        __syncthreads();
        for (uint32_t j = t; j < m; j += ST_THREADS) {
            const uint64_t q = sq[hi - 1 - j];
            L.chunk[j] = q;
            L.bs.code[j] = ll_code(seq_ll(q)) | (hb32(seq_ov(q)) << 8) | (ml_code(seq_mb(q)) << 16);
        }
        const uint32_t nw = (m * 80 + 63) / 32 + 2;
        for (uint32_t i = t; i < nw; i += ST_THREADS) L.bs.bitbuf[i] = 0;
        __syncthreads();
        if (t < 3) {
            for (uint32_t j = 0; j < m; j++) {
                const uint32_t sym = (L.bs.code[j] >> csh) & 255;
                const FseTT x = ttAll[ttb + sym];
                uint32_t out = 0;
                if (hi == nseq && j == 0) {  // the last sequence initialises the states (no bits)
                    const uint32_t nbOut = (x.dnb + (1u << 15)) >> 16;
                    const uint32_t v0 = (nbOut << 16) - x.dnb;
                    fv = stAll[stb + (v0 >> nbOut) + (uint32_t)x.dfs];
                } else {
                    const uint32_t nbOut = (fv + x.dnb) >> 16;
                    out = (nbOut << 16) | (fv & ((1u << nbOut) - 1));
                    fv = stAll[stb + (fv >> nbOut) + (uint32_t)x.dfs];
                }
                L.bs.sbits[t][j] = out;
            }
        }
        __syncthreads();
        // field lengths of this thread's run of sequences, then the workgroup scan
        const uint32_t per = (m + ST_THREADS - 1) / ST_THREADS;
        const uint32_t j0 = t * per < m ? t * per : m, j1 = j0 + per < m ? j0 + per : m;
        uint32_t mine = 0;
        for (uint32_t j = j0; j < j1; j++) {
            const uint32_t cd = L.bs.code[j];
            mine += (L.bs.sbits[0][j] >> 16) + (L.bs.sbits[1][j] >> 16) + (L.bs.sbits[2][j] >> 16) +
                    c_LL_bits[cd & 255] + c_ML_bits[cd >> 16] + ((cd >> 8) & 255);
        }
        L.scanA[t] = mine;
        __syncthreads();
        for (uint32_t d = 1; d < ST_THREADS; d <<= 1) {
            const uint32_t a = t >= d ? L.scanA[t - d] : 0;
            __syncthreads();
            L.scanA[t] += a;
            __syncthreads();
        }
        const uint32_t chunkBits = L.scanA[ST_THREADS - 1];
        const uint32_t r0 = (uint32_t)(bitpos & 31);
        uint32_t r = r0 + L.scanA[t] - mine;  // this run's first bit, relative to word bitpos >> 5
        auto put = [&](uint32_t v, uint32_t nb) {
            if (!nb) return;
            const uint64_t x = (uint64_t)(v & (0xFFFFFFFFu >> (32 - nb))) << (r & 31);
            atomicOr(&L.bs.bitbuf[r >> 5], (uint32_t)x);
            if (x >> 32) atomicOr(&L.bs.bitbuf[(r >> 5) + 1], (uint32_t)(x >> 32));
            r += nb;
        };
        if (t == 0 && r0) atomicOr(&L.bs.bitbuf[0], carry);
        for (uint32_t j = j0; j < j1; j++) {
            const uint32_t cd = L.bs.code[j];
            const uint64_t q = L.chunk[j];
            const uint32_t cl = cd & 255, co = (cd >> 8) & 255, cm = cd >> 16;
            put(L.bs.sbits[0][j] & 0xFFFF, L.bs.sbits[0][j] >> 16);
            put(L.bs.sbits[1][j] & 0xFFFF, L.bs.sbits[1][j] >> 16);
            put(L.bs.sbits[2][j] & 0xFFFF, L.bs.sbits[2][j] >> 16);
            put(seq_ll(q), c_LL_bits[cl]);
            put(seq_mb(q), c_ML_bits[cm]);
            put(seq_ov(q), co);
        }
        __syncthreads();
        const uint32_t endR = r0 + chunkBits, full = endR >> 5;
        const uint64_t w0 = bitpos >> 5;
        for (uint32_t i = t; i < full; i += ST_THREADS)
            if (w0 + i < capW) bo32[w0 + i] = L.bs.bitbuf[i];
        carry = L.bs.bitbuf[full];  // bits [0, endR & 31) of the next word
        bitpos += chunkBits;
        hi = lo_i;
    }
    // the state flushes (ML, OF, LL) and the end mark, by one lane
    const uint32_t fOF = __shfl(fv, 0, 64), fML = __shfl(fv, 1, 64), fLL = __shfl(fv, 2, 64);
    if (t == 0) {
        uint64_t acc = carry;
        uint32_t nb = (uint32_t)(bitpos & 31);
        uint64_t wi = bitpos >> 5;
        auto put1 = [&](uint32_t v, uint32_t bits) {
            if (!bits) return;
            acc |= (uint64_t)(v & (0xFFFFFFFFu >> (32 - bits))) << nb;
            nb += bits;
            while (nb >= 32) {
                if (wi < capW) bo32[wi] = (uint32_t)acc;
                wi++;
                acc >>= 32;
                nb -= 32;
            }
        };
        put1(fML, gML);
        put1(fOF, gOF);
        put1(fLL, gLL);
        put1(1, 1);
        if (nb && wi < capW) bo32[wi] = (uint32_t)acc;
        const uint64_t totalBits = bitpos + gML + gOF + gLL + 1;
        const uint32_t nbytes = (uint32_t)((totalBits + 7) / 8);
        const uint32_t hdr = s_hdr;
        uint32_t bad = nbytes > capB;
        // zstd <= 1.3.4 decoders misread an NCount shorter than 4 bytes before the end
        if (s_lastNC != 0xFFFFFFFFu && (hdr - s_lastNC) + nbytes < 4) bad = 1;
        blk->sec_hdr = hdr;
        blk->sec_len = hdr + nbytes;
        blk->sec_bad = bad;
        blk->nlit = litTotal;
        blk->is_rle = L.flag ? 0 : 1;
    }
}

// ======================================================================= k_zs_decide
struct HufNode {
    uint32_t count;
    uint16_t parent;
    uint8_t byte, nbBits;
};

struct DecideLds {
    uint32_t prev[256], next[256], ct[256];  // Huffman tables: nbBits << 16 | val
    uint32_t count[256];
    HufNode node[2 * 256 + 2];
    uint8_t w[256];
    uint16_t fst[64];
    FseTT ftt[13];
    uint8_t spread[64];
    int16_t norm[13];
    uint32_t cnt13[13];
    uint32_t red[64];
};

__device__ uint32_t huf_build(DecideLds& L, uint32_t maxSV, uint32_t maxNbBits) {
    HufNode* node = L.node + 1;
    for (uint32_t i = 0; i < 2 * 256 + 2; i++) { L.node[i].count = 0; L.node[i].parent = 0; L.node[i].byte = 0; L.node[i].nbBits = 0; }
    // HUF_sort
    {
        uint32_t base[32], cur[32];
        for (int i = 0; i < 32; i++) base[i] = 0;
        for (uint32_t n = 0; n <= maxSV; n++) base[hb32(L.count[n] + 1)]++;
        for (int n = 30; n > 0; n--) base[n - 1] += base[n];
        for (int n = 0; n < 32; n++) cur[n] = base[n];
        for (uint32_t n = 0; n <= maxSV; n++) {
            const uint32_t c = L.count[n], r = hb32(c + 1) + 1;
            uint32_t pos = cur[r]++;
            while (pos > base[r] && c > node[pos - 1].count) { node[pos] = node[pos - 1]; pos--; }
            node[pos].count = c;
            node[pos].byte = (uint8_t)n;
        }
    }
    int nonNull = (int)maxSV;
    while (node[nonNull].count == 0) nonNull--;
    int lowS = nonNull, nodeNb = 256;
    const int nodeRoot = nodeNb + lowS - 1;
    int lowN = nodeNb;
    node[nodeNb].count = node[lowS].count + node[lowS - 1].count;
    node[lowS].parent = node[lowS - 1].parent = (uint16_t)nodeNb;
    nodeNb++;
    lowS -= 2;
    for (int n = nodeNb; n <= nodeRoot; n++) node[n].count = 1u << 30;
    L.node[0].count = 1u << 31;
    while (nodeNb <= nodeRoot) {
        const int n1 = (node[lowS].count < node[lowN].count) ? lowS-- : lowN++;
        const int n2 = (node[lowS].count < node[lowN].count) ? lowS-- : lowN++;
        node[nodeNb].count = node[n1].count + node[n2].count;
        node[n1].parent = node[n2].parent = (uint16_t)nodeNb;
        nodeNb++;
    }
    node[nodeRoot].nbBits = 0;
    for (int n = nodeRoot - 1; n >= 256; n--) node[n].nbBits = node[node[n].parent].nbBits + 1;
    for (int n = 0; n <= nonNull; n++) node[n].nbBits = node[node[n].parent].nbBits + 1;
    // HUF_setMaxHeight
    const uint32_t largestBits = node[nonNull].nbBits;
    if (largestBits > maxNbBits) {
        int totalCost = 0;
        const uint32_t baseCost = 1u << (largestBits - maxNbBits);
        int n = nonNull;
        while (node[n].nbBits > maxNbBits) {
            totalCost += (int)(baseCost - (1u << (largestBits - node[n].nbBits)));
            node[n].nbBits = (uint8_t)maxNbBits;
            n--;
        }
        while (node[n].nbBits == maxNbBits) n--;
        totalCost >>= (largestBits - maxNbBits);
        const uint32_t noSym = 0xF0F0F0F0u;
        uint32_t rankLast[HUF_MAX_LOG + 2];
        for (int i = 0; i < (int)HUF_MAX_LOG + 2; i++) rankLast[i] = noSym;
        {
            uint32_t curNb = maxNbBits;
            for (int pos = n; pos >= 0; pos--) {
                if (node[pos].nbBits >= curNb) continue;
                curNb = node[pos].nbBits;
                rankLast[maxNbBits - curNb] = (uint32_t)pos;
            }
        }
        while (totalCost > 0) {
            uint32_t nBits = hb32((uint32_t)totalCost) + 1;
            for (; nBits > 1; nBits--) {
                const uint32_t highPos = rankLast[nBits], lowPos = rankLast[nBits - 1];
                if (highPos == noSym) continue;
                if (lowPos == noSym) break;
                if (node[highPos].count <= 2 * node[lowPos].count) break;
            }
            while (nBits <= HUF_MAX_LOG && rankLast[nBits] == noSym) nBits++;
            totalCost -= 1 << (nBits - 1);
            if (rankLast[nBits - 1] == noSym) rankLast[nBits - 1] = rankLast[nBits];
            node[rankLast[nBits]].nbBits++;
            if (rankLast[nBits] == 0) rankLast[nBits] = noSym;
            else {
                rankLast[nBits]--;
                if (node[rankLast[nBits]].nbBits != maxNbBits - nBits) rankLast[nBits] = noSym;
            }
        }
        while (totalCost < 0) {
            if (rankLast[1] == noSym) {
                while (node[n].nbBits == maxNbBits) n--;
                node[n + 1].nbBits--;
                rankLast[1] = (uint32_t)(n + 1);
                totalCost++;
                continue;
            }
            node[rankLast[1] + 1].nbBits--;
            rankLast[1]++;
            totalCost++;
        }
    } else {
        maxNbBits = largestBits;
    }
    // canonical values: per rank, in symbol order
    uint16_t nbPerRank[HUF_MAX_LOG + 1], valPerRank[HUF_MAX_LOG + 1];
    for (int i = 0; i <= (int)HUF_MAX_LOG; i++) { nbPerRank[i] = 0; valPerRank[i] = 0; }
    for (int n = 0; n <= nonNull; n++) nbPerRank[node[n].nbBits]++;
    {
        uint16_t mn = 0;
        for (int n = (int)maxNbBits; n > 0; n--) { valPerRank[n] = mn; mn += nbPerRank[n]; mn >>= 1; }
    }
    for (uint32_t i = 0; i < 256; i++) L.ct[i] = 0;
    for (uint32_t n = 0; n <= maxSV; n++) L.ct[node[n].byte] = (uint32_t)node[n].nbBits << 16;
    for (uint32_t n = 0; n <= maxSV; n++) {
        const uint32_t nb = L.ct[n] >> 16;
        L.ct[n] |= valPerRank[nb]++;
    }
    return maxNbBits;
}

// HUF_writeCTable into out; 0 = libzstd's error exit (the literals then go raw)
__device__ uint32_t huf_write(DecideLds& L, uint8_t* out, uint32_t maxSV, uint32_t huffLog) {
    uint8_t b2w[HUF_MAX_LOG + 1];
    b2w[0] = 0;
    for (uint32_t n = 1; n < huffLog + 1; n++) b2w[n] = (uint8_t)(huffLog + 1 - n);
    for (uint32_t n = 0; n < maxSV; n++) L.w[n] = b2w[L.ct[n] >> 16];
    // HUF_compressWeights
    uint32_t hSize = 0;
    const uint32_t wt = maxSV;
    if (wt > 2) {
        uint32_t mx = HUF_MAX_LOG, maxCount = 0;
        for (uint32_t i = 0; i <= HUF_MAX_LOG; i++) L.cnt13[i] = 0;
        for (uint32_t i = 0; i < wt; i++) L.cnt13[L.w[i]]++;
        while (!L.cnt13[mx]) mx--;
        for (uint32_t i = 0; i <= mx; i++) maxCount = L.cnt13[i] > maxCount ? L.cnt13[i] : maxCount;
        if (maxCount == wt) hSize = 1;
        else if (maxCount > 1) {
            const uint32_t tl = fse_optimal_log(6, wt, mx, 2);
            if (fse_normalize(L.norm, tl, L.cnt13, wt, mx, false)) {
                uint32_t o = fse_write_ncount(out + 1, L.norm, mx, tl);
                fse_build(L.fst, L.ftt, L.spread, L.norm, mx, tl);
                // FSE_compress_usingCTable, two interleaved states from the end
                BitW bw;
                bw.init(out + 1 + o, HUF_HDR_CAP - 1 - o);  // longer ones are counted, not kept
                FseState s1, s2;
                int ip = (int)wt;
                if (wt & 1) {
                    s1.init2(L.fst, L.ftt, tl, L.w[--ip]);
                    s2.init2(L.fst, L.ftt, tl, L.w[--ip]);
                    s1.enc(bw, L.w[--ip]);
                } else {
                    s2.init2(L.fst, L.ftt, tl, L.w[--ip]);
                    s1.init2(L.fst, L.ftt, tl, L.w[--ip]);
                }
                if ((wt - 2) & 2) { s2.enc(bw, L.w[--ip]); s1.enc(bw, L.w[--ip]); }
                while (ip > 0) {
                    s2.enc(bw, L.w[--ip]);
                    s1.enc(bw, L.w[--ip]);
                    s2.enc(bw, L.w[--ip]);
                    s1.enc(bw, L.w[--ip]);
                }
                s2.flush(bw);
                s1.flush(bw);
                hSize = o + bw.close();
            }
        }
    }
    if (hSize > 1 && hSize < maxSV / 2) {
        out[0] = (uint8_t)hSize;
        return hSize + 1;
    }
    if (maxSV > 128) return 0;
    out[0] = (uint8_t)(128 + (maxSV - 1));
    L.w[maxSV] = 0;
    for (uint32_t n = 0; n < maxSV; n += 2) out[(n / 2) + 1] = (uint8_t)((L.w[n] << 4) + L.w[n + 1]);
    return ((maxSV + 1) / 2) + 1;
}

// exact compressed size of the literals with table tab (1 or 4 streams; 0 = "not compressible")
__device__ uint32_t huf_streams(const uint32_t* hist, const uint32_t* tab, uint32_t n, bool single,
                                uint32_t* slen) {
    if (single) {
        uint64_t bits = 0;
        for (uint32_t s = 0; s < 256; s++)
            bits += (uint64_t)(hist[s] + hist[256 + s] + hist[512 + s] + hist[768 + s]) * (tab[s] >> 16);
        slen[0] = (uint32_t)((bits + 1 + 7) / 8);
        return slen[0];
    }
    if (n < 12) return 0;
    uint32_t tot = 6;
    for (int k = 0; k < 4; k++) {
        uint64_t bits = 0;
        for (uint32_t s = 0; s < 256; s++) bits += (uint64_t)hist[256 * k + s] * (tab[s] >> 16);
        slen[k] = (uint32_t)((bits + 1 + 7) / 8);
        tot += slen[k];
    }
    return tot;
}

__global__ __launch_bounds__(64) void k_zs_decide(const uint8_t* __restrict__ src, ZBlob* __restrict__ blobs,
                                                  ZBlock* __restrict__ blocks, const uint32_t* __restrict__ hist_in,
                                                  uint32_t* __restrict__ huf_use, uint8_t* __restrict__ huf_hdr,
                                                  uint8_t* __restrict__ dst, const uint32_t* __restrict__ active,
                                                  uint32_t* __restrict__ rerun /* [0] = count, then blob ids */) {
    __shared__ DecideLds L;
    const uint32_t bi = active ? active[blockIdx.x] : blockIdx.x;
    const uint32_t lane = threadIdx.x;
    ZBlob* B = blobs + bi;
    const uint32_t nb = B->nblocks;
    uint8_t* fo = dst + B->dst;
    if (lane == 0) {
        fo[0] = 0;
        fo[1] = (uint8_t)((B->wlog - 10) << 3);
    }
    if (nb == 0) {  // empty blob: one empty last raw block
        if (lane == 0) {
            fo[2] = 1; fo[3] = 0; fo[4] = 0;
            B->frame_len = 5;
            B->flags = 0;
        }
        return;
    }
    for (uint32_t i = lane; i < 256; i += 64) L.prev[i] = 0;
    uint32_t prevRepeat = REP_NONE;
    uint64_t out = B->dst + 2;
    uint32_t newMask = 0;
    bool mis = false;
    for (uint32_t k = 0; k < nb; k++) {
        const uint32_t b = B->first_block + k;
        ZBlock* blk = blocks + b;
        const uint32_t bs = blk->bs;
        uint32_t cSize = 0, litKind = LIT_RAW, lhSize = 0, hufLen = 0, streams = 0, slen[4] = {0, 0, 0, 0};
        uint64_t litHdr = 0;
        uint32_t nextRepeat = prevRepeat;
        if (bs >= 7 && !blk->sec_bad) {
            const uint32_t n = blk->nlit;
            const uint32_t* hist = hist_in + (uint64_t)b * 1024;
            for (uint32_t i = lane; i < 256; i += 64) L.next[i] = L.prev[i];
            // ZSTD_compressLiterals
            const uint32_t minGain = (n >> 6) + 2;
            uint32_t lh = 3 + (n >= 1024) + (n >= 16384);
            bool single = n < 256;
            uint32_t hType = LIT_HUF;
            uint32_t cLit = 0;  // 0 = raw literals, 1 = rle, else compressed size
            const uint32_t minLit = prevRepeat == REP_VALID ? 6 : 63;
            if (n > minLit) {
                for (uint32_t s = lane; s < 256; s += 64)
                    L.count[s] = hist[s] + hist[256 + s] + hist[512 + s] + hist[768 + s];
                __syncthreads();
                uint32_t repeat = prevRepeat;
                const bool preferRepeat = n <= 1024;
                if (repeat == REP_VALID && lh == 3) single = true;
                uint32_t res = 0;  // HUF_compress_internal's result
                bool useOld = false, useNew = false;
                if (lane == 0) {
                    if (preferRepeat && repeat == REP_VALID) useOld = true;
                    else {
                        uint32_t maxSV = 255, largest = 0;
                        while (!L.count[maxSV]) maxSV--;
                        for (uint32_t s = 0; s <= maxSV; s++) largest = L.count[s] > largest ? L.count[s] : largest;
                        if (largest == n) res = 1;
                        else if (largest <= (n >> 7) + 4) res = 0;
                        else {
                            if (repeat == REP_CHECK) {
                                bool bad = false;
                                for (uint32_t s = 0; s <= maxSV; s++) bad |= L.count[s] != 0 && (L.prev[s] >> 16) == 0;
                                if (bad) repeat = REP_NONE;
                            }
                            if (preferRepeat && repeat != REP_NONE) useOld = true;
                            else {
                                uint32_t huffLog = fse_optimal_log(HUF_DEFAULT_LOG, n, maxSV, 1);
                                huffLog = huf_build(L, maxSV, huffLog);
                                uint8_t* hh = huf_hdr + (uint64_t)b * HUF_HDR_CAP;
                                const uint32_t hSize = huf_write(L, hh, maxSV, huffLog);
                                if (hSize == 0) res = 0xFFFFFFFFu;
                                else {
                                    bool old = false;
                                    if (repeat != REP_NONE) {
                                        uint64_t oldS = 0, newS = 0;
                                        for (uint32_t s = 0; s <= maxSV; s++) {
                                            oldS += (uint64_t)(L.prev[s] >> 16) * L.count[s];
                                            newS += (uint64_t)(L.ct[s] >> 16) * L.count[s];
                                        }
                                        oldS >>= 3;
                                        newS >>= 3;
                                        if (oldS <= hSize + newS || hSize + 12 >= n) old = true;
                                    }
                                    if (old) useOld = true;
                                    else if (hSize + 12 >= n) res = 0;
                                    else {
                                        repeat = REP_NONE;
                                        useNew = true;
                                        hufLen = hSize;
                                        for (uint32_t s = 0; s < 256; s++) L.next[s] = L.ct[s];
                                    }
                                }
                            }
                        }
                    }
                    if (useOld || useNew) {
                        const uint32_t* tab = useOld ? L.prev : L.ct;
                        const uint32_t pre = useNew ? hufLen : 0;
                        const uint32_t c = huf_streams(hist, tab, n, single, slen);
                        if (c == 0 || pre + c >= n - 1) res = 0;
                        else res = pre + c;
                        if (useOld) hufLen = 0;
                    }
                    if (repeat != REP_NONE) hType = LIT_HUF_REPEAT;
                    L.red[0] = res;
                    L.red[1] = hType | (useOld ? 4u : 0u) | (useNew ? 8u : 0u) | (single ? 16u : 0u);
                    L.red[2] = hufLen;
                    L.red[3] = slen[0]; L.red[4] = slen[1]; L.red[5] = slen[2]; L.red[6] = slen[3];
                }
                __syncthreads();
                res = L.red[0];
                const uint32_t fl = L.red[1];
                hType = fl & 3;
                useOld = fl & 4;
                useNew = fl & 8;
                single = fl & 16;
                hufLen = L.red[2];
                slen[0] = L.red[3]; slen[1] = L.red[4]; slen[2] = L.red[5]; slen[3] = L.red[6];
                cLit = res;
                if (res == 0xFFFFFFFFu || res == 0 || res >= n - minGain) cLit = 0;
                // table used by the emitter
                if (cLit > 1) {
                    const uint32_t* tab = useOld ? L.prev : L.ct;
                    uint32_t* dstTab = huf_use + (uint64_t)b * 256;
                    for (uint32_t s = lane; s < 256; s += 64) dstTab[s] = tab[s];
                }
            }
            uint32_t litSize;
            if (cLit == 0) {  // raw literals; next table = prev
                for (uint32_t i = lane; i < 256; i += 64) L.next[i] = L.prev[i];
                nextRepeat = prevRepeat;
                lh = 1 + (n > 31) + (n > 4095);
                litKind = LIT_RAW;
                litHdr = lh == 1 ? (uint64_t)(n << 3) : lh == 2 ? (uint64_t)((1u << 2) + (n << 4)) : (uint64_t)((3u << 2) + (n << 4));
                litSize = lh + n;
                hufLen = 0;
                streams = 0;
            } else if (cLit == 1) {
                for (uint32_t i = lane; i < 256; i += 64) L.next[i] = L.prev[i];
                nextRepeat = prevRepeat;
                lh = 1 + (n > 31) + (n > 4095);
                litKind = LIT_RLE;
                litHdr = 1 + (lh == 1 ? (uint64_t)(n << 3) : lh == 2 ? (uint64_t)((1u << 2) + (n << 4)) : (uint64_t)((3u << 2) + (n << 4)));
                litSize = lh + 1;
                hufLen = 0;
                streams = 0;
            } else {
                nextRepeat = hType == LIT_HUF ? REP_CHECK : prevRepeat;
                litKind = hType;
                if (lh == 3) litHdr = (uint64_t)hType + ((uint64_t)(!single) << 2) + ((uint64_t)n << 4) + ((uint64_t)cLit << 14);
                else if (lh == 4) litHdr = (uint64_t)hType + (2ull << 2) + ((uint64_t)n << 4) + ((uint64_t)cLit << 18);
                else litHdr = (uint64_t)hType + (3ull << 2) + ((uint64_t)n << 4) + ((uint64_t)cLit << 22);
                litSize = lh + cLit;
                streams = single ? 1 : 4;
            }
            lhSize = lh;
            cSize = litSize + blk->sec_len;
            if (cSize >= bs - ((bs >> 6) + 2)) cSize = 0;
        }
        if (bs >= 7 && k > 0 && cSize < 25 && blk->is_rle) cSize = 1;
        const uint32_t type = cSize == 0 ? BT_RAW : cSize == 1 ? BT_RLE : BT_COMPRESSED;
        const uint32_t body = type == BT_RAW ? bs : type == BT_RLE ? 1 : cSize;
        if (type == BT_COMPRESSED) {
            for (uint32_t i = lane; i < 256; i += 64) L.prev[i] = L.next[i];
            prevRepeat = nextRepeat;
        }
        __syncthreads();
        if (lane == 0) {
            blk->type = type;
            blk->body = body;
            blk->last = k + 1 == nb;
            blk->out = out;
            blk->lit_kind = litKind;
            blk->lit_hdr = litHdr;
            blk->lh_size = lhSize;
            blk->huf_hdr_len = hufLen;
            blk->streams = streams;
            for (int i = 0; i < 4; i++) blk->stream_len[i] = slen[i];
        }
        out += 3 + body;
        if (k + 1 < nb) {
            const bool pred = !((B->raw_mask >> k) & 1), act = cSize > 1;
            const bool changed = blk->rep_in[0] != blk->rep_out[0] || blk->rep_in[1] != blk->rep_out[1] ||
                                 blk->rep_in[2] != blk->rep_out[2];
            if (pred != act && changed) mis = true;
            if (!act) newMask |= 1u << k;
        }
    }
    if (lane == 0) {
        B->frame_len = out - B->dst;
        if (mis) {
            B->flags = 1;
            B->raw_mask = newMask;
            B->base += (uint32_t)B->len + 2;  // a fresh index range: the slot's entries read as empty
            const uint32_t k = atomicAdd(rerun, 1u);
            rerun[1 + k] = bi;
        } else {
            B->flags = 0;
        }
    }
}

// ======================================================================= k_zs_emit
constexpr int EM_THREADS = 256;
constexpr uint32_t EM_WORDS = 11264 + 8;  // one Huffman stream of <= 32768 literals x 11 bits

__device__ void copy_bytes(uint8_t* d, const uint8_t* s, uint32_t n, uint32_t t) {
    for (uint32_t i = t; i < n; i += EM_THREADS) d[i] = s[i];
}

__global__ __launch_bounds__(EM_THREADS) void k_zs_emit(const uint8_t* __restrict__ src, const ZBlob* __restrict__ blobs,
                                                        const ZBlock* __restrict__ blocks, const uint8_t* __restrict__ lits,
                                                        const uint8_t* __restrict__ sec, const uint32_t* __restrict__ huf_use,
                                                        const uint8_t* __restrict__ huf_hdr, uint8_t* __restrict__ dst) {
    __shared__ uint32_t buf[EM_WORDS];
    __shared__ uint32_t tab[256];
    __shared__ uint32_t scan[EM_THREADS];
    const uint32_t b = blockIdx.x, t = threadIdx.x;
    const ZBlock blk = blocks[b];
    const uint8_t* s = src + blobs[blk.blob].src + blk.off;
    uint8_t* o = dst + blk.out;
    if (t == 0) {
        const uint32_t h = blk.last + (blk.type << 1) + ((blk.type == BT_COMPRESSED ? blk.body : blk.bs) << 3);
        o[0] = (uint8_t)h; o[1] = (uint8_t)(h >> 8); o[2] = (uint8_t)(h >> 16);
    }
    o += 3;
    if (blk.type == BT_RAW) { copy_bytes(o, s, blk.bs, t); return; }
    if (blk.type == BT_RLE) { if (t == 0) o[0] = s[0]; return; }
    // literals section
    const uint8_t* L = lits + blk.lit0;
    const uint32_t n = blk.nlit;
    if (t < blk.lh_size) o[t] = (uint8_t)(blk.lit_hdr >> (8 * t));
    o += blk.lh_size;
    if (blk.lit_kind == LIT_RAW) {
        copy_bytes(o, L, n, t);
        o += n;
    } else if (blk.lit_kind == LIT_RLE) {
        if (t == 0) o[0] = L[0];
        o += 1;
    } else {
        if (blk.huf_hdr_len) {
            copy_bytes(o, huf_hdr + (uint64_t)b * HUF_HDR_CAP, blk.huf_hdr_len, t);
            o += blk.huf_hdr_len;
        }
        for (uint32_t i = t; i < 256; i += EM_THREADS) tab[i] = huf_use[(uint64_t)b * 256 + i];
        const uint32_t ns = blk.streams;
        if (ns == 4) {
            if (t < 6) o[t] = (uint8_t)(blk.stream_len[t >> 1] >> (8 * (t & 1)));
            o += 6;
        }
        const uint32_t seg = ns == 1 ? n : (n + 3) / 4;
        for (uint32_t k = 0; k < ns; k++) {
            const uint32_t a = k * seg, m = (k + 1 < ns) ? seg : n - a;
            const uint32_t words = ((m * 11u + 1) >> 5) + 2;
            __syncthreads();
            for (uint32_t i = t; i < words; i += EM_THREADS) buf[i] = 0;
            // each thread: a contiguous run of literals; bit offsets grow from the last literal
            const uint32_t per = (m + EM_THREADS - 1) / EM_THREADS;
            const uint32_t i0 = t * per < m ? t * per : m, i1 = i0 + per < m ? i0 + per : m;
            uint32_t bits = 0;
            for (uint32_t i = i0; i < i1; i++) bits += tab[L[a + i]] >> 16;
            scan[t] = bits;
            __syncthreads();
            // suffix scan: bit offset of this run = bits of every later run
            for (uint32_t d = 1; d < EM_THREADS; d <<= 1) {
                const uint32_t v = t + d < EM_THREADS ? scan[t + d] : 0;
                __syncthreads();
                scan[t] += v;
                __syncthreads();
            }
            const uint32_t total = scan[0];
            uint32_t pos = scan[t] - bits;
            for (uint32_t i = i1; i-- > i0;) {
                const uint32_t e = tab[L[a + i]], nbits = e >> 16, v = e & 0xFFFF;
                if (nbits) {
                    const uint32_t w = pos >> 5, sh = pos & 31;
                    atomicOr(&buf[w], v << sh);
                    if (sh + nbits > 32) atomicOr(&buf[w + 1], v >> (32 - sh));
                }
                pos += nbits;
            }
            __syncthreads();
            if (t == 0) atomicOr(&buf[total >> 5], 1u << (total & 31));
            __syncthreads();
            const uint32_t len = (total + 1 + 7) >> 3;
            BW_ASSERT(len == blk.stream_len[k]);
            const uint8_t* bb = (const uint8_t*)buf;
            for (uint32_t i = t; i < len; i += EM_THREADS) o[i] = bb[i];
            o += len;
        }
    }
    // sequences section
    const uint8_t* sh = sec + blk.sec0;
    copy_bytes(o, sh, blk.sec_hdr, t);
    o += blk.sec_hdr;
    copy_bytes(o, sh + SEC_HDR, blk.sec_len - blk.sec_hdr, t);
}

}  // namespace zs

// ======================================================================= host driver
namespace {

struct DBuf {
    void* p = nullptr;
    size_t cap = 0;
};

bool dgrow(DBuf& b, size_t bytes, hipStream_t st, std::string& err) {
    if (bytes == 0) bytes = 16;
    if (b.cap >= bytes) return true;
    if (b.p) {
        hipStreamSynchronize(st);
        hipFree(b.p);
        b.p = nullptr;
        b.cap = 0;
    }
    const size_t want = bytes + bytes / 8 + 256;
    if (hipMalloc(&b.p, want) != hipSuccess) {
        err = "hipMalloc(" + std::to_string(want) + ") failed (zstd workspace)";
        return false;
    }
    b.cap = want;
    return true;
}

}  // namespace

struct ZstdWork {
    DBuf blobs, blocks, hist, huf_use, huf_hdr, seqs, lits, sec, active, rerun;
    // hash-table slot pools, one per layout (a pool at the wide stride cost 3.3x the memory
    // of the narrow tables that many-blob sub-batches use): [0] narrow, 768 KiB per slot, up to
    // max_slots; [1] wide, 2.5 MiB per slot, up to ZS_WIDE_MAX_BLOBS
    DBuf tables[2];
    std::vector<uint32_t> next_base[2];  // per slot: the index base its next use starts from
    uint32_t n_slots[2] = {0, 0};
    uint64_t max_slots = 16384;        // blobs parsed at once
    uint64_t max_bytes = 8ull << 30;   // input bytes per sub-batch (scratch ~4.2 x this)
    uint32_t* h_rerun = nullptr;       // pinned
    ~ZstdWork() {
        for (DBuf* b : {&blobs, &blocks, &hist, &huf_use, &huf_hdr, &seqs, &lits, &sec, &tables[0], &tables[1], &active,
                        &rerun})
            if (b->p) hipFree(b->p);
        if (h_rerun) hipHostFree(h_rerun);
    }
};

void zstd_work_free(ZstdWork* w) { delete w; }

void zstd_work_copy_limits(ZstdWork*& dst, const ZstdWork* src) {
    if (!dst) dst = new ZstdWork();
    if (src) {
        dst->max_slots = src->max_slots;
        dst->max_bytes = src->max_bytes;
    }
}

void zstd_work_limits(ZstdWork*& w, uint64_t max_slots, uint64_t max_bytes) {
    if (!w) w = new ZstdWork();
    if (max_slots) w->max_slots = max_slots;
    if (max_bytes) w->max_bytes = max_bytes;
}

// level-3 parameters for a blob of n bytes (ZSTD_getCParams(3, n, 0) after ZSTD_adjustCParams)
static void zstd_params(uint64_t n, uint32_t& wlog, uint32_t& clog, uint32_t& hlog, uint32_t& mls) {
    if (n <= 16384) { wlog = 14; clog = 14; hlog = 15; mls = 4; }
    else if (n <= 131072) { wlog = 17; clog = 15; hlog = 16; mls = 5; }
    else if (n <= 262144) { wlog = 18; clog = 16; hlog = 16; mls = 4; }
    else { wlog = 21; clog = 16; hlog = 17; mls = 5; }
    const uint32_t srcLog = n < 64 ? 6 : 64 - (uint32_t)__builtin_clzll(n - 1);
    if (wlog > srcLog) wlog = srcLog;
    if (hlog > wlog + 1) hlog = wlog + 1;
    if (clog > wlog) clog = wlog;
    if (wlog < 10) wlog = 10;
}

uint64_t zstd_scratch_estimate(uint64_t bytes) { return bytes * 4 + (bytes >> 5) * 45 + (64ull << 20); }

int zstd_compress(hipStream_t st, ZstdWork*& w, const uint8_t* d_src, const uint64_t* src_off, const uint64_t* src_len,
                  uint64_t n, uint8_t* d_dst, const uint64_t* dst_off, uint64_t* frame_len, std::string& err) {
    using namespace zs;
    if (!w) w = new ZstdWork();
    for (uint64_t i = 0; i < n; i++)
        if (src_len[i] > 3ull * 1024 * 1024) {
            err = "zstd: blob larger than BLOB_MAX_UNCOMPRESSED_SIZE (3 MiB)";
            return BW_EINVAL;
        }
    if (!w->h_rerun && hipHostMalloc((void**)&w->h_rerun, sizeof(uint32_t) * (1 + 65536), hipHostMallocDefault) != hipSuccess) {
        err = "hipHostMalloc failed (zstd)";
        return BW_ENOMEM;
    }
    uint64_t i0 = 0;
    std::vector<ZBlob> hb;
    std::vector<ZBlock> hk;
    std::vector<uint32_t> act;
    while (i0 < n) {
        // sub-batch: up to max_slots blobs and max_bytes input bytes
        uint64_t i1 = i0, bytes = 0;
        while (i1 < n && i1 - i0 < w->max_slots && (i1 == i0 || bytes + src_len[i1] <= w->max_bytes)) bytes += src_len[i1++];
        const uint32_t nb = (uint32_t)(i1 - i0);
        // wide table entries for sub-batches of few blobs (one wave per SIMD: latency-bound), narrow
        // ones when the blobs fill the SIMDs several times over (measured: wide +3 % on 836 blobs of
        // 1 GiB of text, -1..-9 % on 6,808 blobs of 8 GiB; profiles/r04/s10_zsfat, s13_zsab8)
        const bool wide = nb <= ZS_WIDE_MAX_BLOBS;
        const int L = wide ? 1 : 0;
        const uint64_t stride = (wide ? SLOT_WORDS : NARROW_WORDS) * 4;
        if (nb > w->n_slots[L]) {
            // grow the layout's slot pool (fresh slots are zero: every entry reads as empty)
            DBuf nt;
            if (!dgrow(nt, (size_t)nb * stride, st, err)) return BW_ENOMEM;
            if (hipMemsetAsync(nt.p, 0, nt.cap, st) != hipSuccess) { err = "hipMemsetAsync failed"; return BW_EHIP; }
            if (w->tables[L].p) { hipStreamSynchronize(st); hipFree(w->tables[L].p); }
            w->tables[L] = nt;
            w->n_slots[L] = (uint32_t)(nt.cap / stride);
            w->next_base[L].assign(w->n_slots[L], 0);
        }
        hb.resize(nb);
        hk.clear();
        uint64_t seqCap = 0, litCap = 0, secCap = 0;
        for (uint32_t j = 0; j < nb; j++) {
            const uint64_t len = src_len[i0 + j];
            ZBlob& B = hb[j];
            B = ZBlob{};
            B.src = src_off[i0 + j];
            B.dst = dst_off[i0 + j];
            B.len = len;
            zstd_params(len, B.wlog, B.clog, B.hlog, B.mls);
            B.first_block = (uint32_t)hk.size();
            B.nblocks = (uint32_t)((len + BLOCK - 1) / BLOCK);
            B.slot = j;
            // index range of this use, with room for every rerun (one block flips per rerun)
            uint32_t& nbase = w->next_base[L][j];
            const uint64_t need = (uint64_t)(B.nblocks + 2) * (len + 2);
            if ((uint64_t)nbase + need >= 0xFFFFFF00ull) {  // the index space of the slot is used up: clear it
                if (hipMemsetAsync((uint8_t*)w->tables[L].p + (uint64_t)j * stride, 0, stride, st) != hipSuccess) {
                    err = "hipMemsetAsync failed";
                    return BW_EHIP;
                }
                nbase = 0;
            }
            B.base = nbase;
            nbase += (uint32_t)need;
            for (uint32_t k = 0; k < B.nblocks; k++) {
                ZBlock K{};
                K.off = (uint64_t)k * BLOCK;
                K.bs = (uint32_t)std::min<uint64_t>(BLOCK, len - K.off);
                K.blob = j;
                K.seq0 = seqCap;
                K.lit0 = litCap;
                K.sec0 = secCap;
                seqCap += K.bs / 4 + 2;
                litCap += (K.bs + 15) & ~15u;
                secCap += (SEC_HDR + K.bs + 128 + 15) & ~15u;  // 16-byte aligned: the bitstream is stored in words
                hk.push_back(K);
            }
        }
        const uint64_t nk = hk.size();
        if (!dgrow(w->blobs, nb * sizeof(ZBlob), st, err) || !dgrow(w->blocks, nk * sizeof(ZBlock), st, err) ||
            !dgrow(w->hist, nk * 4096, st, err) || !dgrow(w->huf_use, nk * 1024, st, err) ||
            !dgrow(w->huf_hdr, nk * HUF_HDR_CAP, st, err) || !dgrow(w->seqs, seqCap * 8, st, err) ||
            !dgrow(w->lits, litCap, st, err) || !dgrow(w->sec, secCap, st, err) ||
            !dgrow(w->active, std::max<uint64_t>(nk, nb) * 4, st, err) || !dgrow(w->rerun, (1 + nb) * 4, st, err))
            return BW_ENOMEM;
        ZBlob* dB = (ZBlob*)w->blobs.p;
        ZBlock* dK = (ZBlock*)w->blocks.p;
        uint32_t* dR = (uint32_t*)w->rerun.p;
        uint32_t* dA = (uint32_t*)w->active.p;
        if (hipMemcpyAsync(dB, hb.data(), nb * sizeof(ZBlob), hipMemcpyHostToDevice, st) != hipSuccess ||
            (nk && hipMemcpyAsync(dK, hk.data(), nk * sizeof(ZBlock), hipMemcpyHostToDevice, st) != hipSuccess)) {
            err = "hipMemcpyAsync failed (zstd tables)";
            return BW_EHIP;
        }
        // parse -> stats -> decide, then reruns of the blobs whose repeat-offset guess failed
        const uint32_t* blobList = nullptr;
        const uint32_t* blockList = nullptr;
        uint32_t nBlobs = nb;
        uint64_t nBlocks = nk;
        for (int pass = 0;; pass++) {
            if (pass > 32) { err = "zstd: decisions did not converge"; return BW_ESTATE; }
            hipMemsetAsync(dR, 0, 4, st);
            if (nBlocks) {
                hipLaunchKernelGGL(k_zs_parse, dim3(nBlobs), dim3(64), 0, st, d_src, dB, dK, (uint32_t*)w->tables[L].p,
                                   (uint64_t*)w->seqs.p, blobList, (int)wide);
                hipLaunchKernelGGL(k_zs_stats, dim3((uint32_t)nBlocks), dim3(ST_THREADS), 0, st, d_src, dB, dK,
                                   (const uint64_t*)w->seqs.p, (uint8_t*)w->lits.p, (uint8_t*)w->sec.p,
                                   (uint32_t*)w->hist.p, blockList);
            }
            hipLaunchKernelGGL(k_zs_decide, dim3(nBlobs), dim3(64), 0, st, d_src, dB, dK, (const uint32_t*)w->hist.p,
                               (uint32_t*)w->huf_use.p, (uint8_t*)w->huf_hdr.p, d_dst, blobList, dR);
            if (hipMemcpyAsync(w->h_rerun, dR, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipStreamSynchronize(st) != hipSuccess) {
                err = "zstd: kernel failure";
                return BW_EHIP;
            }
            const uint32_t nr = w->h_rerun[0];
            if (nr == 0) break;
            std::vector<uint32_t> ids(nr);
            if (hipMemcpy(ids.data(), dR + 1, nr * 4, hipMemcpyDeviceToHost) != hipSuccess) { err = "hipMemcpy failed"; return BW_EHIP; }
            act.clear();
            for (uint32_t id : ids) {
                for (uint32_t k = 0; k < hb[id].nblocks; k++) act.push_back(hb[id].first_block + k);
            }
            // blob ids first, then the block ids, in the active buffer
            if (!dgrow(w->active, (ids.size() + act.size()) * 4, st, err)) return BW_ENOMEM;
            dA = (uint32_t*)w->active.p;
            hipMemcpyAsync(dA, ids.data(), ids.size() * 4, hipMemcpyHostToDevice, st);
            hipMemcpyAsync(dA + ids.size(), act.data(), act.size() * 4, hipMemcpyHostToDevice, st);
            hipStreamSynchronize(st);
            blobList = dA;
            blockList = dA + ids.size();
            nBlobs = nr;
            nBlocks = act.size();
        }
        if (nk)
            hipLaunchKernelGGL(k_zs_emit, dim3((uint32_t)nk), dim3(EM_THREADS), 0, st, d_src, dB, dK,
                               (const uint8_t*)w->lits.p, (const uint8_t*)w->sec.p, (const uint32_t*)w->huf_use.p,
                               (const uint8_t*)w->huf_hdr.p, d_dst);
        std::vector<ZBlob> back(nb);
        if (hipMemcpyAsync(back.data(), dB, nb * sizeof(ZBlob), hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess) {
            err = "zstd: kernel failure";
            return BW_EHIP;
        }
        for (uint32_t j = 0; j < nb; j++) frame_len[i0 + j] = back[j].frame_len;
#ifdef BW_ZSTD_TIMING
        {
            double sum[8] = {0};
            for (uint32_t j = 0; j < nb; j++)
                for (int i = 0; i < 8; i++) sum[i] += (double)back[j].tm[i];
            fprintf(stderr, "zstd parse timing over %u blobs: cycles/blob probe %.4g length %.4g catchup %.4g insert+rep %.4g; "
                    "steps/blob %.4g sequences/blob %.4g rep-loop/blob %.4g; mean first-match lane %.3f, small-path share %.3f\n", nb,
                    sum[0] / nb, sum[1] / nb, 0.0, sum[3] / nb, sum[4] / nb, sum[5] / nb, sum[6] / nb,
                    sum[2] / (sum[5] - sum[6] + 1e-9), sum[7] / (sum[5] - sum[6] + 1e-9));
        }
#endif
        i0 = i1;
    }
    return BW_OK;
}

}  // namespace bw
