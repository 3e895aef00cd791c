// bw_cdc.hip -- FastCDC v2020 content-defined chunking on gfx950.
//
// Replaces `FastCDC::new(&mmap, 262144, 1048576, 3145728)` + its iterator as called by
// process_file (client/src/backup/filesystem/dir_packer.rs:254-266); crate fastcdc 3.0.3
// (Cargo.lock:557-560), semantics restated in SURVEY.md A.1 and oracle/bw_oracle.c.
//
// The crate's cut() is a serial two-bytes-per-step loop; the equivalent per-byte form is
//   h_p = (h_{p-1} << 1) + GEAR[src[p]],  hash reset to 0 at chunk_start + 2*(min/2),
// and position p cuts iff (h_p & mask) == 0 (mask_s before `center`, mask_l after).  Because
// every mask bit is <= 47, (h_p & mask) depends only on src[p-47 ..= p]; so the candidate test
// can run at EVERY byte of the stream in parallel, and only the first 47 positions after each
// chunk's start+min need the truncated (chunk-local) hash.
//
// Pipeline (all on the stream, no host round trip):
//   k_scan      gear hash at every byte, LDS lane-replicated table, one-v_and prefilter per
//               byte; flagged 64-byte blocks made exact by the wave at the end of each tile
//   k_tile_partial  exclusive scan of per-tile counts -> candidate array offsets (block scans; the
//               grid's last block scans the block totals)
//               (it first rescans its overflowed tiles for exact counts: candidate-dense data)
//   k_compact   copy slots; overflowed tiles are rescanned by their block and written in place
//   k_chains    one wave per segment: speculative boundary chain from the segment start
//   k_extend    continue each chain until it merges with the next segment's chain (CDC resync)
//   k_resolve   prefix-max of merge points -> true chain entry of every segment, validity
//   k_fallback  serial wave walker for files whose chains did not merge (exact, slower)
//   k_unit_*    canonical-order blob table + BLAKE3 group offsets (count + scan, emit)
//   k_cut_hash  Chunk.hash (the crate's returned gear state) for every CDC chunk
#include "bw_device.h"
#include "bw_internal.h"

namespace bw {
#if BW_CLOCK_STAMPS
__device__ ClockLog* g_clk_cdc = nullptr;
void clock_log_register_cdc(void* log) { hipMemcpyToSymbol(HIP_SYMBOL(g_clk_cdc), &log, sizeof(log)); }
#endif


__constant__ uint64_t c_gear[256] = BW_GEAR_INIT;

// ======================================================================== gear scan

__device__ __forceinline__ uint64_t gear_fetch(uint32_t word, uint32_t sel, uint32_t lane_off, const uint64_t* lds) {
    // v_perm_b32 builds the LDS byte address (byte << 8) | lane_off in one instruction:
    // result byte0 = lane_off, byte1 = byte k of `word`, bytes 2..3 = 0.  The table holds 32
    // lane-replicated copies of each entry, so a half-wave's ds_read_b64 is bank-conflict free.
    const uint32_t addr = __builtin_amdgcn_perm(word, lane_off, sel);
    return *(const uint64_t*)((const uint8_t*)lds + addr);
}

__device__ __forceinline__ void gear_step(uint64_t& h, uint32_t word, uint32_t sel, uint32_t lane_off,
                                          const uint64_t* lds) {
    h = (h << 1) + gear_fetch(word, sel, lane_off, lds);
}

#define BW_SEL(k) (0x0c0c0000u | ((4u + (k)) << 8))

__device__ __forceinline__ uint32_t mask_test(uint64_t h, uint32_t mlo, uint32_t mhi) {
    // (lo & mlo) | (hi & mhi): zero iff (h & mask) == 0 -- one v_and + one v_and_or
    uint32_t r;
    const uint32_t t = (uint32_t)h & mlo;
    asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"((uint32_t)(h >> 32)), "s"(mhi), "v"(t));
    return r;
}

// Exact normalized-chunking test of the plain gear state h at `pos`; a hit is appended to the
// wave's LDS slots as pos | S | L.
__device__ __forceinline__ void record_hit(uint64_t pos, uint64_t h, const Masks& mk, uint32_t* s_cnt,
                                           uint64_t* s_slots) {
    const bool S = (h & mk.mask_s) == 0, L = (h & mk.mask_l) == 0;
    if (S || L) {
        uint32_t i = atomicAdd(s_cnt, 1u);
        if (i < (uint32_t)SCAN_CAP) s_slots[i] = pos | (S ? BW_CAND_S : 0) | (L ? BW_CAND_L : 0);
    }
}

// Gear scan.  The lanes carry the SHIFTED state h' = h << pre_shift (the LDS table holds
// GEAR[b] << pre_shift; pre_shift = 63 - top mask bit, 16 at backuwup's parameters), so the
// high dword of h' is the 32-bit window of h that holds the top mask bits, and the per-byte
// prefilter is ONE v_and on it: (hi(h') & pre_hi) == 0 is implied by a real candidate (pre_hi =
// the intersection mask's bits inside the window: 16 of mask_l's 19 at backuwup's parameters).
// 128 positions fold into one min() per step; a step whose fold hits records only its 64-byte
// block (rate ~64 * 2^-16 per lane-step), and at the end of the tile the wave makes each flagged
// block exact with every lane busy (refine_block), instead of replaying it inside the hot loop.
//
// Each wavefront owns a 128 KiB sub-tile = 64 strips of 2 KiB, one per lane.  The gear state
// is warmed up on the 64 bytes before the strip (after 64 steps it IS the windowed hash), then
// every byte is tested.  Bytes reach the lanes coalesced: per 64-byte step, four
// global_load_dwordx4 fetch 16 strips x 64 B each (4 lanes per half line), the wave stages them
// in its own padded LDS rows and every lane reads back its strip's 64 bytes (16 B per
// ds_read_b128, conflict-free with 80-byte rows).  Loads run one double step (128 B per strip)
// ahead, both halves of each 128-byte line back to back (two register sets, unconditional loads
// so the vmcnt waits are exact).  No block barrier after the table fill: records are collected
// per wave in LDS and published by lane 0.
__device__ __forceinline__ void hash_words(uint64_t& h, uint32_t& acc, const uint32_t (&ww)[16], uint32_t lane_off,
                                           const uint64_t* s_gear, uint32_t phi) {
#pragma unroll
    for (int i = 0; i < 16; i += 2) {
        uint64_t g[8];  // 8 independent LDS reads ahead of the serial recurrence
#pragma unroll
        for (int q = 0; q < 8; q++) g[q] = gear_fetch(ww[i + q / 4], BW_SEL(q % 4), lane_off, s_gear);
#pragma unroll
        for (int q = 0; q < 8; q += 2) {
            h = (h << 1) + g[q];
            const uint32_t t0 = (uint32_t)(h >> 32) & phi;
            h = (h << 1) + g[q + 1];
            const uint32_t t1 = (uint32_t)(h >> 32) & phi;
            // one v_min3 per two positions (left to itself the compiler builds a v_min tree)
            asm("v_min3_u32 %0, %1, %2, %3" : "=v"(acc) : "v"(acc), "v"(t0), "v"(t1));
        }
    }
}

// One 64-byte step of one lane: stage the wave's four coalesced loads, read back this lane's
// strip bytes, hash them; a prefilter hit records the block at `at`.
__device__ __forceinline__ void stage_hash_step(uint4 r0, uint4 r1, uint4 r2, uint4 r3, uint8_t* wr,
                                                const uint8_t* rd, uint64_t& h, uint64_t at, uint32_t lane_off,
                                                const uint64_t* s_gear, uint32_t phi, uint32_t* cnt,
                                                uint64_t* slots) {
    *(uint4*)(wr) = r0;
    *(uint4*)(wr + 16 * STAGE_ROW) = r1;
    *(uint4*)(wr + 32 * STAGE_ROW) = r2;
    *(uint4*)(wr + 48 * STAGE_ROW) = r3;
    __builtin_amdgcn_wave_barrier();
    const uint4 v0 = *(const uint4*)(rd), v1 = *(const uint4*)(rd + 16), v2 = *(const uint4*)(rd + 32),
                v3 = *(const uint4*)(rd + 48);
    __builtin_amdgcn_wave_barrier();
    const uint32_t ww[16] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w,
                             v2.x, v2.y, v2.z, v2.w, v3.x, v3.y, v3.z, v3.w};
    uint32_t acc = 0xffffffffu;
    hash_words(h, acc, ww, lane_off, s_gear, phi);
    if (__builtin_expect(acc == 0, 0)) {
        const uint32_t i = atomicAdd(cnt, 1u);
        if (i < (uint32_t)SCAN_CAP) slots[i] = at | BW_CAND_BLK;
    }
}

constexpr uint32_t TILE_OVF = 0x80000000u;  // tile_count flag: candidates come from k_rescan

__device__ __forceinline__ void ovf_push(uint64_t t, uint32_t* ovf, uint64_t* ctr) {
    const uint64_t k = atomicAdd((unsigned long long*)&ctr[C_NOVF], 1ull);
    ovf[k] = (uint32_t)t;
}

// Exact candidates of one flagged 64-byte block at b, by the whole wave: lane j takes position
// b + j.  Two wave shift-scans of the (shifted) gear recurrence give h'_{b-1} from the 64 bytes
// before the block (from 0 at the buffer start, where b == 0: the history the scan's lane had)
// and then h'_{b+j} = scan_j + (h'_{b-1} << (j + 1)).  ~2 flagged blocks per 128 KiB tile on
// random data at backuwup's parameters; the bytes were just streamed by this wave (L2 hits).
__device__ __forceinline__ void refine_block(const uint8_t* __restrict__ data, uint64_t b, const uint64_t* s_gear,
                                             uint32_t lane, const Masks& mk, uint32_t* cnt, uint64_t* slots) {
    const uint32_t rep = (lane & 31) * 8;
    const uint64_t g0 = b >= 64 ? *(const uint64_t*)((const uint8_t*)s_gear + ((uint32_t)data[b - 64 + lane] << 8) + rep) : 0;
    const uint64_t g1 = *(const uint64_t*)((const uint8_t*)s_gear + ((uint32_t)data[b + lane] << 8) + rep);
    const uint64_t pre = bw_shfl64(bw_gear_scan(g0), 63);
    const uint64_t h = bw_gear_scan(g1) + ((pre << lane) << 1);
    record_hit(b + lane, h >> mk.pre_shift, mk, cnt, slots);
}


template <int BLOCK, int STRIP>
__global__ __launch_bounds__(BLOCK, 4) void k_scan(const uint8_t* __restrict__ data, uint64_t n_bytes,
                                                       uint64_t n_tiles, Masks mk,
                                                       uint32_t* __restrict__ tile_count,
                                                       uint64_t* __restrict__ tile_slots, uint32_t* __restrict__ ovf,
                                                       uint64_t* ctr) {
    constexpr int WAVES = BLOCK / 64;
    // one LDS object so the gear table sits at LDS address 0 and every lookup address is the
    // v_perm result itself (a table at a non-zero base costs one v_add per byte)
    struct ScanLds {
        uint64_t gear[256 * GEAR_REP];        // 64 KiB, 32 lane replicas
        uint8_t stage[WAVES][64 * STAGE_ROW]; // per-wave staging rows
        uint64_t slots[WAVES][SCAN_CAP];  // exact candidates pos | S | L
        uint64_t flags[WAVES][SCAN_CAP];  // flagged 64-byte blocks
        uint32_t cnt[WAVES], nflag[WAVES];
    };
    __shared__ __attribute__((aligned(16))) ScanLds lds;
    uint64_t* s_gear = lds.gear;
    uint8_t (*s_stage)[64 * STAGE_ROW] = lds.stage;
    uint64_t (*s_slots)[SCAN_CAP] = lds.slots;
    uint32_t* s_cnt = lds.cnt;
    for (int i = threadIdx.x; i < 256 * GEAR_REP; i += blockDim.x) s_gear[i] = c_gear[i / GEAR_REP] << mk.pre_shift;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t lane_off = (lane & 31) * 8;
    const uint32_t phi = mk.pre_hi;
    uint8_t* stage = s_stage[wid];
    uint32_t* cnt = &s_cnt[wid];
    uint64_t* slots = s_slots[wid];
    uint32_t* fcnt = &lds.nflag[wid];
    uint64_t* fslots = lds.flags[wid];
    const uint64_t nw = (uint64_t)gridDim.x * WAVES;

    for (uint64_t tile = (uint64_t)blockIdx.x * WAVES + wid; tile < n_tiles; tile += nw) {
#if BW_CLOCK_STAMPS
        ClockStamp clk((tile & 15) == 0 ? g_clk_cdc : nullptr, 0);  // one tile in 16: the stamps' atomics
                                                                    // must not slow what they time
#endif
        if (lane == 0) { *cnt = 0; *fcnt = 0; }
        const uint64_t base = tile * (64ull * STRIP);
        const uint64_t ss = base + (uint64_t)lane * STRIP;
        uint64_t h = 0;
        if (base + (64ull * STRIP) <= n_bytes) {
            if (ss >= 64) {  // warm-up on the 64 bytes before the strip
                const uint4* wp = (const uint4*)(data + ss - 64);
                uint4 w[4];
#pragma unroll
                for (int i = 0; i < 4; i++) w[i] = wp[i];
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const uint32_t ww[4] = {w[i].x, w[i].y, w[i].z, w[i].w};
#pragma unroll
                    for (int j = 0; j < 4; j++)
#pragma unroll
                        for (int k = 0; k < 4; k++) gear_step(h, ww[j], BW_SEL(k), lane_off, s_gear);
                }
            }
            {
                // Both 64-byte halves of every 128-byte line are requested back to back: the
                // loads run one double step (two 64-byte steps) ahead, so the second half of a
                // line meets the first half's miss in L2 instead of arriving one step later,
                // after ~4 MiB of other waves' half-open lines per XCD have evicted it.
                const uint8_t* src = data + base + (uint64_t)(lane >> 2) * STRIP + (lane & 3) * 16;
                uint8_t* wr = stage + (lane >> 2) * STAGE_ROW + (lane & 3) * 16;
                const uint8_t* rd = stage + lane * STAGE_ROW;
                constexpr int STEPS = STRIP / SCAN_STEP;
                constexpr uint64_t JS = 16ull * STRIP;
#define BW_LOAD8(r, ds)                                                                          \
    do {                                                                                         \
        const uint8_t* s_ = src + (uint64_t)(ds) * (2 * SCAN_STEP);                              \
        _Pragma("unroll") for (int j = 0; j < 4; j++) {                                          \
            r[j] = *(const uint4*)(s_ + j * JS);                                                 \
            r[4 + j] = *(const uint4*)(s_ + SCAN_STEP + j * JS);                                 \
        }                                                                                        \
    } while (0)
                uint4 a[8], b[8];
                BW_LOAD8(a, 0);
#pragma unroll 1
                for (int ds = 0; ds < STEPS / 2; ds += 2) {
                    BW_LOAD8(b, ds + 1);
                    stage_hash_step(a[0], a[1], a[2], a[3], wr, rd, h, ss + (uint64_t)(2 * ds) * SCAN_STEP, lane_off,
                                    s_gear, phi, fcnt, fslots);
                    stage_hash_step(a[4], a[5], a[6], a[7], wr, rd, h, ss + (uint64_t)(2 * ds + 1) * SCAN_STEP,
                                    lane_off, s_gear, phi, fcnt, fslots);
                    BW_LOAD8(a, ds + 2 < STEPS / 2 ? ds + 2 : STEPS / 2 - 1);  // clamped, unused at the end
                    stage_hash_step(b[0], b[1], b[2], b[3], wr, rd, h, ss + (uint64_t)(2 * ds + 2) * SCAN_STEP,
                                    lane_off, s_gear, phi, fcnt, fslots);
                    stage_hash_step(b[4], b[5], b[6], b[7], wr, rd, h, ss + (uint64_t)(2 * ds + 3) * SCAN_STEP,
                                    lane_off, s_gear, phi, fcnt, fslots);
                }
#undef BW_LOAD8
            }
        } else if (ss < n_bytes) {  // ragged last sub-tile: exact byte path (h' >> pre_shift is h
                                    // modulo 2^(64 - pre_shift), which holds every mask bit)
            const uint64_t se = ss + STRIP < n_bytes ? ss + STRIP : n_bytes;
            for (uint64_t p = ss >= 64 ? ss - 64 : 0; p < se; p++) {
                h = (h << 1) + s_gear[(uint32_t)data[p] * GEAR_REP];
                if (p >= ss) record_hit(p, h >> mk.pre_shift, mk, cnt, slots);
            }
        }
        __builtin_amdgcn_wave_barrier();
        const uint32_t nf = __builtin_amdgcn_readfirstlane(*fcnt);
        if (nf <= (uint32_t)SCAN_CAP)
            for (uint32_t f = 0; f < nf; f++) refine_block(data, BW_CAND_POS(fslots[f]), s_gear, lane, mk, cnt, slots);
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) {
            const uint32_t c = *cnt, n = c < (uint32_t)SCAN_CAP ? c : (uint32_t)SCAN_CAP;
            if (nf > (uint32_t)SCAN_CAP || c > (uint32_t)SCAN_CAP) ovf_push(tile, ovf, ctr);  // exact list from k_rescan
            for (uint32_t i = 1; i < n; i++) {  // insertion sort by position (n is ~0.25)
                uint64_t v = slots[i];
                int k = (int)i - 1;
                while (k >= 0 && BW_CAND_POS(slots[k]) > BW_CAND_POS(v)) {
                    slots[k + 1] = slots[k];
                    k--;
                }
                slots[k + 1] = v;
            }
            tile_count[tile] = c;
            for (uint32_t i = 0; i < n; i++) tile_slots[tile * SCAN_CAP + i] = slots[i];
        }
        __builtin_amdgcn_wave_barrier();
    }
}

template <int BLOCK, int STRIP>
static void launch_scan_t(hipStream_t st, const uint8_t* data, uint64_t n_bytes, uint64_t n_tiles, const Masks& mk,
                          uint32_t* tile_count, uint64_t* tile_slots, uint32_t* ovf, uint64_t* ctr) {
    uint64_t grid = (n_tiles + BLOCK / 64 - 1) / (BLOCK / 64);
    // Every CU holds one block (LDS).  Large batches: 512 persistent blocks (two rounds, each wave
    // streams many tiles).  Small batches (half-size tiles): 1024 blocks, four rounds of about one
    // tile per wave -- C1's scan 0.32 -> 0.27 ms; 512 or an uncapped grid (one tile per wave, a
    // ragged fifth round) measured 0.32 / 0.43 ms, and 1024 on C2 changed nothing (profiles/r02/s15_grid).
    const uint64_t cap = STRIP == SCAN_STRIP ? 512 : 1024;
    if (grid > cap) grid = cap;
    hipLaunchKernelGGL((k_scan<BLOCK, STRIP>), dim3((unsigned)grid), dim3(BLOCK), 0, st, data, n_bytes,
                       n_tiles, mk, tile_count, tile_slots, ovf, ctr);
}

bool launch_scan(hipStream_t st, const uint8_t* data, uint64_t n_bytes, uint64_t n_tiles, const Masks& mk,
                 uint32_t* tile_count, uint64_t* tile_slots, uint32_t* ovf, uint64_t* ctr, int waves) {
    if (!n_tiles) return true;
    const bool big = 64ull * SCAN_STRIP == 1ull << mk.tile_shift, small = 64ull * SCAN_STRIP_SMALL == 1ull << mk.tile_shift;
    if (!big && !small) return false;  // a tile size no kernel was built for: the caller reports BW_EINVAL
    // 16-wave blocks hold 148 KiB of LDS (one per CU); 8-wave blocks hold 106 KiB and leave room
    // for two k_b3_groups blocks of another batch on the same CU
#if BW_DIAG
    if (waves == 8) {
        if (big) launch_scan_t<512, SCAN_STRIP>(st, data, n_bytes, n_tiles, mk, tile_count, tile_slots, ovf, ctr);
        else launch_scan_t<512, SCAN_STRIP_SMALL>(st, data, n_bytes, n_tiles, mk, tile_count, tile_slots, ovf, ctr);
        return true;
    }
#endif
    (void)waves;
    if (big) launch_scan_t<SCAN_BLOCK, SCAN_STRIP>(st, data, n_bytes, n_tiles, mk, tile_count, tile_slots, ovf, ctr);
    else launch_scan_t<SCAN_BLOCK, SCAN_STRIP_SMALL>(st, data, n_bytes, n_tiles, mk, tile_count, tile_slots, ovf, ctr);
    return true;
}

// ======================================================================== block scan helpers

template <int T>
__device__ __forceinline__ uint64_t block_excl_sum(uint64_t v, uint64_t* s, uint64_t* total) {
    s[threadIdx.x] = v;
    __syncthreads();
    for (int d = 1; d < T; d <<= 1) {
        uint64_t a = threadIdx.x >= (unsigned)d ? s[threadIdx.x - d] : 0;
        __syncthreads();
        s[threadIdx.x] += a;
        __syncthreads();
    }
    const uint64_t incl = s[threadIdx.x];
    if (total) *total = s[T - 1];
    __syncthreads();
    return incl - v;
}

// (flag, max) segmented exclusive scan; flag = this element starts a new segment
template <int T>
__device__ __forceinline__ uint64_t block_excl_segmax(uint32_t f, uint64_t v, uint64_t* s, uint32_t* sf) {
    s[threadIdx.x] = v;
    sf[threadIdx.x] = f;
    __syncthreads();
    for (int d = 1; d < T; d <<= 1) {
        uint64_t a = 0;
        uint32_t af = 0;
        const bool has = threadIdx.x >= (unsigned)d;
        if (has) { a = s[threadIdx.x - d]; af = sf[threadIdx.x - d]; }
        __syncthreads();
        if (has && !sf[threadIdx.x]) { s[threadIdx.x] = a > s[threadIdx.x] ? a : s[threadIdx.x]; sf[threadIdx.x] = af; }
        __syncthreads();
    }
    // exclusive: value of previous element's inclusive result unless this starts a segment
    uint64_t r = (threadIdx.x > 0) ? s[threadIdx.x - 1] : 0;
    __syncthreads();
    return r;
}

// The "last block done" pattern: every block of a grid counts itself in *done once its results
// are written; the block that completes the count returns true, with every other block's writes
// visible, and resets the counter.  Folds a one-block follow-up kernel into the grid before it.
__device__ __forceinline__ bool last_block_done(uint64_t* done) {
    __shared__ bool last;
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        last = atomicAdd((unsigned long long*)done, 1ull) == gridDim.x - 1;
    }
    __syncthreads();
    if (last) {
        __threadfence();  // acquire: the other blocks' results
        if (threadIdx.x == 0) *done = 0;
    }
    return last;
}

// Exclusive scan, in place, of n block totals by one block of T threads; returns the grand total.
template <int T>
__device__ __forceinline__ uint64_t scan_totals(uint64_t* tot, uint64_t n, uint64_t* s) {
    const uint64_t per = (n + T - 1) / T, lo = threadIdx.x * per;
    const uint64_t hi = lo + per < n ? lo + per : n;
    uint64_t sum = 0;
    for (uint64_t i = lo; i < hi; i++) sum += tot[i];
    uint64_t total;
    uint64_t run = block_excl_sum<T>(sum, s, &total);
    for (uint64_t i = lo; i < hi; i++) {
        const uint64_t t = tot[i];
        tot[i] = run;
        run += t;
    }
    return total;
}

// ======================================================================== candidate compaction

constexpr int BLK = 1024;

// Exact ordered re-scan of a tile on the overflow list (candidate-dense data or small parameters)
// by a whole block of RESCAN_THREADS: WRITE = false returns the tile's candidate count (before the
// offset scan), WRITE = true also stores its candidates from cand[base] on (after it).  s_gear is
// the plain 256-entry table in LDS.
constexpr int RESCAN_THREADS = 256;

template <bool WRITE>
__device__ uint64_t rescan_tile(const uint8_t* __restrict__ data, uint64_t n_bytes, const Masks& mk, uint64_t tile,
                                uint64_t base, uint64_t* __restrict__ cand, uint64_t cap, const uint64_t* s_gear,
                                uint64_t* s_scan) {
    const uint64_t rs = (1ull << mk.tile_shift) / RESCAN_THREADS;  // bytes per thread
    const uint64_t ss = (tile << mk.tile_shift) + (uint64_t)threadIdx.x * rs;
    const uint64_t se = ss + rs < n_bytes ? ss + rs : n_bytes;
    uint64_t mine = 0, total = 0;
    for (int pass = 0; pass < (WRITE ? 2 : 1); pass++) {
        uint64_t h = 0, w = 0;
        if (pass == 1) w = base + block_excl_sum<RESCAN_THREADS>(mine, s_scan, nullptr);
        if (ss < n_bytes) {
            for (uint64_t p = ss >= 64 ? ss - 64 : 0; p < se; p++) {
                h = (h << 1) + s_gear[data[p]];
                if (p < ss) continue;
                const bool S = (h & mk.mask_s) == 0, L = (h & mk.mask_l) == 0;
                if (S || L) {
                    if (pass == 0) mine++;
                    else if (w < cap) cand[w++] = p | (S ? BW_CAND_S : 0) | (L ? BW_CAND_L : 0);
                }
            }
        }
    }
    if (!WRITE) block_excl_sum<RESCAN_THREADS>(mine, s_scan, &total);
    __syncthreads();
    return total;
}

// The overflowed tiles in [t0, t1), each by the whole block (WRITE as in rescan_tile).  The list
// is short (empty on random data at backuwup's parameters): every block reads all of it.
template <bool WRITE>
__device__ void rescan_range(const uint8_t* __restrict__ data, uint64_t n_bytes, const Masks& mk,
                             const uint32_t* __restrict__ ovf, uint64_t novf, uint64_t t0, uint64_t t1,
                             uint32_t* __restrict__ tile_count, const uint64_t* __restrict__ off,
                             uint64_t* __restrict__ cand, uint64_t cap, uint64_t* s_gear, uint64_t* s_scan) {
    bool loaded = false;
    for (uint64_t k = 0; k < novf; k++) {
        const uint64_t tile = ovf[k];
        if (tile < t0 || tile >= t1) continue;
        if (!loaded) {
            for (int i = threadIdx.x; i < 256; i += blockDim.x) s_gear[i] = c_gear[i];
            __syncthreads();
            loaded = true;
        }
        const uint64_t total = rescan_tile<WRITE>(data, n_bytes, mk, tile, WRITE ? off[tile] : 0, cand, cap, s_gear,
                                                  s_scan);
        if (!WRITE && threadIdx.x == 0) tile_count[tile] = (uint32_t)total | TILE_OVF;
    }
    __syncthreads();
}

// Candidate offsets: a scan over the per-tile counts (tiles are 128 KiB, so a 16 GiB batch has
// 131072 of them): block-local scans of 1024 counts, the last block over the block totals, then
// compaction adds the block base and copies the slots.
constexpr int TS_BLOCK = 256;  // threads per block, 4 counts each

// Candidate-dense batches (small parameters: most tiles overflow) rescan their overflowed tiles
// in a kernel of their own, the list spread over the whole grid (inside k_tile_partial a
// block owns 1,024 tiles, so a 64 MiB batch of 64 KiB tiles rescanned all of them on one block);
// sparse ones (backuwup's parameters: no overflow on random data) keep the rescan inside
// k_tile_partial / k_compact and save the two launches.
template <bool WRITE>
__global__ __launch_bounds__(RESCAN_THREADS) void k_rescan(const uint8_t* __restrict__ data, uint64_t n_bytes, Masks mk,
                                                            const uint32_t* __restrict__ ovf, uint32_t* __restrict__ cnt,
                                                            const uint64_t* __restrict__ off, uint64_t* __restrict__ cand,
                                                            uint64_t cap, const uint64_t* ctr) {
    __shared__ uint64_t s_gear[256], s_scan[RESCAN_THREADS];
    const uint64_t novf = ctr[C_NOVF];
    if (blockIdx.x >= novf) return;  // uniform per block
    for (int i = threadIdx.x; i < 256; i += blockDim.x) s_gear[i] = c_gear[i];
    __syncthreads();
    for (uint64_t k = blockIdx.x; k < novf; k += gridDim.x) {
        const uint64_t tile = ovf[k];
        const uint64_t total = rescan_tile<WRITE>(data, n_bytes, mk, tile, WRITE ? off[tile] : 0, cand, cap, s_gear, s_scan);
        if (!WRITE && threadIdx.x == 0) cnt[tile] = (uint32_t)total | TILE_OVF;
    }
}

__global__ __launch_bounds__(TS_BLOCK) void k_tile_partial(const uint8_t* __restrict__ data, uint64_t n_bytes, Masks mk,
                                                           const uint32_t* __restrict__ ovf, uint32_t* __restrict__ cnt,
                                                           uint64_t n, uint64_t* __restrict__ off,
                                                           uint64_t* __restrict__ btot, uint64_t cap, uint64_t* ctr,
                                                           bool spread) {
    __shared__ uint64_t s[TS_BLOCK];
    __shared__ uint64_t s_gear[256];
    // exact counts of this block's overflowed tiles first (what a separate k_rescan<false> did)
    const uint64_t novf = spread ? 0 : ctr[C_NOVF];
    if (novf) {
        const uint64_t t0 = (uint64_t)blockIdx.x * 4 * TS_BLOCK, t1 = t0 + 4 * TS_BLOCK;
        rescan_range<false>(data, n_bytes, mk, ovf, novf, t0, t1 < n ? t1 : n, cnt, nullptr, nullptr, 0, s_gear, s);
    }
    const uint64_t i0 = ((uint64_t)blockIdx.x * TS_BLOCK + threadIdx.x) * 4;
    uint32_t c[4] = {0, 0, 0, 0};
    if (i0 + 4 <= n) {
        const uint4 v = *(const uint4*)(cnt + i0);
        c[0] = v.x; c[1] = v.y; c[2] = v.z; c[3] = v.w;
    } else {
        for (int k = 0; k < 4; k++) c[k] = i0 + k < n ? cnt[i0 + k] : 0;
    }
    for (int k = 0; k < 4; k++) c[k] &= ~TILE_OVF;
    const uint64_t sum = (uint64_t)c[0] + c[1] + c[2] + c[3];
    uint64_t total;
    uint64_t run = block_excl_sum<TS_BLOCK>(sum, s, &total);
    for (int k = 0; k < 4; k++)
        if (i0 + k < n) { off[i0 + k] = run; run += c[k]; }
    if (threadIdx.x == 0) btot[blockIdx.x] = total;
    // the last block scans the block totals (what a separate one-block kernel did)
    if (!last_block_done(&ctr[C_DONE_TILES])) return;
    const uint64_t all = scan_totals<TS_BLOCK>(btot, gridDim.x, s);
    if (threadIdx.x == 0) {
        off[n] = all;
        ctr[C_NCAND] = all < cap ? all : cap;
        ctr[C_CANDTOTAL] = all;
        ctr[C_TRUNC] = BW_NONE;  // lowered by k_compact when the array cannot hold every candidate
    }
}

// A tile whose candidates do not all fit below `cap` marks the candidate array as incomplete from
// its first byte on (C_TRUNC = the lowest such tile start); the boundary walkers then test the
// bytes at and beyond that position themselves (walk_next), so an undersized array never changes
// a boundary and a batch never has to be re-run (which would break the dedup order of a shared
// index).
__global__ __launch_bounds__(256) void k_compact(const uint8_t* __restrict__ data, uint64_t n_bytes, Masks mk,
                                                 const uint32_t* __restrict__ ovf, const uint32_t* __restrict__ cnt,
                                                 const uint64_t* __restrict__ slots, uint64_t* __restrict__ off,
                                                 const uint64_t* __restrict__ bbase, uint64_t n_tiles,
                                                 uint64_t* __restrict__ cand, uint64_t cap, uint64_t* ctr, bool spread) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n_tiles) {
        const uint64_t o = off[t] + bbase[t / (4 * TS_BLOCK)];
        off[t] = o;  // final offset: the walkers start their candidate cursor here
        const uint32_t c = cnt[t];
        if (o + (c & ~TILE_OVF) > cap)
            atomicMin((unsigned long long*)&ctr[C_TRUNC], (unsigned long long)(t << mk.tile_shift));
        if (!(c & TILE_OVF)) {  // overflowed tiles are written by the block below
            for (uint32_t i = 0; i < c; i++)
                if (o + i < cap) cand[o + i] = slots[t * SCAN_CAP + i];
        }
    }
    // this block's overflowed tiles, at their final offsets (what a separate k_rescan<true> did)
    const uint64_t novf = spread ? 0 : ctr[C_NOVF];
    if (novf) {
        __shared__ uint64_t s_gear[256], s_scan[RESCAN_THREADS];
        __syncthreads();  // the block's final offsets are written
        const uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x, t1 = t0 + blockDim.x;
        rescan_range<true>(data, n_bytes, mk, ovf, novf, t0, t1 < n_tiles ? t1 : n_tiles, nullptr, off, cand, cap,
                           s_gear, s_scan);
    }
}

void launch_compact(hipStream_t st, const uint8_t* data, uint64_t n_bytes, uint64_t n_tiles, const Masks& mk,
                    uint32_t* tile_count, uint64_t* tile_slots, uint64_t* tile_off, uint64_t* cand,
                    uint64_t cand_cap, uint32_t* ovf_list, uint64_t* ctr, uint64_t* btot) {
    if (!n_tiles) return;
    const uint64_t nb = (n_tiles + 4 * TS_BLOCK - 1) / (4 * TS_BLOCK);
    // candidate-dense parameters: expected flagged 64-byte blocks per tile (the scan's prefilter
    // keeps 2^-popcount(pre_hi) of the bytes) above half of the SCAN_CAP slots a tile holds
    const double flagged = (double)(1ull << mk.tile_shift) / 64.0 *
                           (1.0 - pow(1.0 - ldexp(1.0, -__builtin_popcount(mk.pre_hi)), 64.0));
    const bool spread = flagged > SCAN_CAP / 2;
    const unsigned rb = (unsigned)std::min<uint64_t>(n_tiles, 2048);
    if (spread)
        hipLaunchKernelGGL(k_rescan<false>, dim3(rb), dim3(RESCAN_THREADS), 0, st, data, n_bytes, mk, ovf_list, tile_count,
                           nullptr, nullptr, 0, ctr);
    hipLaunchKernelGGL(k_tile_partial, dim3((unsigned)nb), dim3(TS_BLOCK), 0, st, data, n_bytes, mk, ovf_list,
                       tile_count, n_tiles, tile_off, btot, cand_cap, ctr, spread);
    hipLaunchKernelGGL(k_compact, dim3((unsigned)((n_tiles + 255) / 256)), dim3(256), 0, st, data, n_bytes, mk, ovf_list,
                       tile_count, tile_slots, tile_off, btot, n_tiles, cand, cand_cap, ctr, spread);
    if (spread)
        hipLaunchKernelGGL(k_rescan<true>, dim3(rb), dim3(RESCAN_THREADS), 0, st, data, n_bytes, mk, ovf_list, tile_count,
                           tile_off, cand, cand_cap, ctr);
}

// ======================================================================== the boundary walker

struct Walker {
    const uint8_t* data;
    const uint64_t* cand;
    uint64_t ncand;
    const uint64_t* lgear;  // plain 256-entry table in LDS
    Masks mk;
    uint64_t trunc;         // ctr[C_TRUNC]: candidates are complete only below this position
    uint64_t data_len;      // bytes of the batch buffer (BW_DEBUG checks)
};

// First position p in [a, hi) whose windowed gear hash passes its region's mask (mask_s below
// c2a, mask_l from c2a on), or BW_NONE; the whole wave tests 64 positions per step.  Used where
// the candidate array is incomplete (p >= trunc).  Requires a >= chunk start + s0 + 47 (so the
// 64-byte window is inside the hashed range) and a >= 64.
__device__ uint64_t direct_scan(const Walker& W, uint64_t a, uint64_t hi, uint64_t c2a) {
    const int lane = bw_lane();
    BW_ASSERT(a >= 64 && a <= hi && hi <= W.data_len);
    // h_{a-1} from the 64 bytes before a (only its low 48 bits matter)
    uint64_t carry = bw_shfl64(bw_gear_scan(W.lgear[W.data[a - 64 + lane]]), 63);
    for (uint64_t b = a; b < hi; b += 64) {
        const uint64_t p = b + (uint64_t)lane;
        const bool valid = p < hi;
        const uint64_t g = valid ? W.lgear[W.data[p]] : 0;
        const uint64_t h = bw_gear_scan(g) + ((carry << lane) << 1);
        const uint64_t mask = p < c2a ? W.mk.mask_s : W.mk.mask_l;
        const uint64_t hb = __ballot(valid && (h & mask) == 0);
        if (hb) return b + (uint64_t)__builtin_ctzll(hb);
        carry = bw_shfl64(h, 63);
    }
    return BW_NONE;
}

// One step of fastcdc::v2020::cut for the chunk starting at s in a file ending at fe, executed by a
// whole wavefront (all 64 lanes, wave-uniform control flow).  Returns the next chunk start.
// `cptr` is the wave's running index into the sorted candidate array; it only moves forward.
__device__ uint64_t walk_next(const Walker& W, uint64_t s, uint64_t fe, uint64_t& cptr) {
    const int lane = bw_lane();
    BW_ASSERT(s < fe && fe <= W.data_len);
    const uint64_t rem = fe - s;
    if (rem <= W.mk.min) return fe;  // cut(): remaining <= min_size -> (0, remaining)
    uint64_t center = W.mk.avg, remaining = rem;
    if (rem > W.mk.max) remaining = W.mk.max;
    else if (rem < center) center = rem;
    const uint64_t s0 = W.mk.s0, c2 = center & ~1ull, r2 = remaining & ~1ull;

    // Head: the first 47 tested positions see a hash truncated at s + s0; recompute them with a
    // wave-wide shift-scan of the gear recurrence.
    const uint64_t p = s0 + (uint64_t)lane;
    const bool valid = lane < 47 && p < r2;
    const uint64_t g = valid ? W.lgear[W.data[s + p]] : 0;
    const uint64_t h = bw_gear_scan(g);
    const uint64_t mask = p < c2 ? W.mk.mask_s : W.mk.mask_l;
    const uint64_t hb = __ballot(valid && (h & mask) == 0);
    if (hb) return s + s0 + (uint64_t)__builtin_ctzll(hb);

    // Body: first candidate in [s+s0+47, s+r2) that passes its region's mask.  The candidate array
    // answers for positions below W.trunc; from there on the bytes are tested directly.
    const uint64_t lo = s + s0 + 47, hi = s + r2, c2a = s + c2;
    const uint64_t hc = hi < W.trunc ? hi : W.trunc;
    for (;;) {
        const uint64_t idx = cptr + (uint64_t)lane;
        const uint64_t c = idx < W.ncand ? W.cand[idx] : BW_NONE;
        const uint64_t pos = c == BW_NONE ? BW_NONE : BW_CAND_POS(c);
        const uint64_t below = __ballot(pos < lo);
        const bool match = pos >= lo && pos < hc && ((pos < c2a) ? (c & BW_CAND_S) != 0 : (c & BW_CAND_L) != 0);
        const uint64_t mb = __ballot(match);
        if (mb) {
            const uint64_t cut = bw_shfl64(pos, __builtin_ctzll(mb));
            cptr += (uint64_t)__popcll(below);
            BW_ASSERT(cut > s && cut < s + remaining && cptr <= W.ncand + 64);
            return cut;
        }
        if (__ballot(pos >= hc) != 0) {  // window exhausted (also covers the array end)
            cptr += (uint64_t)__popcll(below);
            break;
        }
        cptr += 64;
    }
    if (hc < hi) {
        const uint64_t cut = direct_scan(W, lo > hc ? lo : hc, hi, c2a);
        if (cut != BW_NONE) return cut;
    }
    return s + remaining;
}

__device__ __forceinline__ void load_lgear(uint64_t* lg) {
    for (int i = threadIdx.x; i < 256; i += blockDim.x) lg[i] = c_gear[i];
    __syncthreads();
}

// ======================================================================== speculative chains

constexpr int WAVES_PER_BLOCK = 4;

__global__ __launch_bounds__(64 * WAVES_PER_BLOCK) void k_chains(Walker W, const uint64_t* __restrict__ tile_off,
                                                                 const uint64_t* ctr, const SegDesc* __restrict__ segs,
                                                                 uint64_t nseg, uint64_t* __restrict__ chains,
                                                                 uint32_t* __restrict__ chain_n,
                                                                 uint64_t* __restrict__ chain_cptr) {
    __shared__ uint64_t lg[256];
    load_lgear(lg);
    W.lgear = lg;
    W.ncand = ctr[C_NCAND];
    W.trunc = ctr[C_TRUNC];
    const uint64_t j = (uint64_t)blockIdx.x * WAVES_PER_BLOCK + threadIdx.x / 64;
    if (j >= nseg) return;
    const SegDesc sd = segs[j];
    uint64_t s = sd.start, cptr = tile_off[s >> W.mk.tile_shift];
    uint32_t n = 0;
    for (;;) {
        const uint64_t c = walk_next(W, s, sd.file_end, cptr);
        if (n < (uint32_t)CHAIN_CAP && bw_lane() == 0) chains[j * CHAIN_CAP + n] = c;
        n++;
        if (c >= sd.end || n > (uint32_t)CHAIN_CAP) break;
        s = c;
    }
    if (bw_lane() == 0) { chain_n[j] = n; chain_cptr[j] = cptr; }
}

// Continue chain j past the next segment's start until one of its cuts is also a cut of chain
// j+1 (CDC resynchronises: from a shared cut on, both chains are identical).  merge[j] = that
// cut, or BW_NONE when chain j+1's coverage is exhausted first (-> serial walker).
__global__ __launch_bounds__(64 * WAVES_PER_BLOCK) void k_extend(Walker W, const uint64_t* ctr,
                                                                 const SegDesc* __restrict__ segs, uint64_t nseg,
                                                                 uint64_t* __restrict__ chains,
                                                                 uint32_t* __restrict__ chain_n,
                                                                 const uint64_t* __restrict__ chain_cptr,
                                                                 uint64_t* __restrict__ merge) {
    __shared__ uint64_t lg[256];
    load_lgear(lg);
    W.lgear = lg;
    W.ncand = ctr[C_NCAND];
    W.trunc = ctr[C_TRUNC];
    const uint64_t j = (uint64_t)blockIdx.x * WAVES_PER_BLOCK + threadIdx.x / 64;
    if (j >= nseg) return;
    const int lane = bw_lane();
    const SegDesc sd = segs[j];
    if (sd.last) { if (lane == 0) merge[j] = sd.file_end; return; }
    uint32_t n = chain_n[j];
    const uint32_t n1r = chain_n[j + 1];
    if (n > (uint32_t)CHAIN_CAP || n1r == 0) { if (lane == 0) merge[j] = BW_NONE; return; }
    const uint32_t n1 = n1r < (uint32_t)CHAIN_CAP ? n1r : (uint32_t)CHAIN_CAP;
    const uint64_t* c1 = chains + (j + 1) * CHAIN_CAP;
    const uint64_t v0 = (uint32_t)lane < n1 ? c1[lane] : BW_NONE;
    const uint64_t v1 = (uint32_t)lane + 64 < n1 ? c1[lane + 64] : BW_NONE;
    const uint64_t last1 = c1[n1 - 1];
    const uint64_t b1 = segs[j + 1].start;
    uint64_t e = chains[j * CHAIN_CAP + n - 1], cptr = chain_cptr[j], m = BW_NONE;
    for (;;) {
        if (e == b1 || __ballot(v0 == e || v1 == e) != 0) { m = e; break; }
        if (e >= last1 || n >= (uint32_t)CHAIN_CAP) break;
        e = walk_next(W, e, sd.file_end, cptr);
        if (lane == 0) chains[j * CHAIN_CAP + n] = e;
        n++;
    }
    if (lane == 0) { chain_n[j] = n; merge[j] = m; }
}

void launch_chains(hipStream_t st, const uint8_t* data, uint64_t data_len, const Masks& mk, const uint64_t* cand,
                   const uint64_t* tile_off, uint64_t* ctr, const SegDesc* segs, uint64_t nseg, uint64_t* chains,
                   uint32_t* chain_n, uint64_t* chain_cptr, uint64_t* merge, int force_serial) {
    if (!nseg || force_serial) return;
    Walker W{data, cand, 0, nullptr, mk, 0, data_len};
    const unsigned grid = (unsigned)((nseg + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK);
    hipLaunchKernelGGL(k_chains, dim3(grid), dim3(64 * WAVES_PER_BLOCK), 0, st, W, tile_off, ctr, segs, nseg,
                       chains, chain_n, chain_cptr);
    hipLaunchKernelGGL(k_extend, dim3(grid), dim3(64 * WAVES_PER_BLOCK), 0, st, W, ctr, segs, nseg, chains,
                       chain_n, chain_cptr, merge);
}

// ======================================================================== resolution

// M_j (first true chunk start inside chain j) = file start for a file's first segment, else
// max(merge[first .. j-1]).  Segment j contributes its chain entries in [M_j, M_{j+1}).
__global__ __launch_bounds__(BLK) void k_resolve(const SegDesc* __restrict__ segs, uint64_t nseg,
                                                 const CFileDesc* __restrict__ cfiles, uint64_t ncf,
                                                 const uint64_t* __restrict__ chains,
                                                 const uint32_t* __restrict__ chain_n,
                                                 const uint64_t* __restrict__ merge, uint64_t* __restrict__ seg_M,
                                                 uint32_t* __restrict__ seg_cnt, uint32_t* __restrict__ cf_invalid,
                                                 int force_serial) {
    __shared__ uint64_t s_v[BLK];
    __shared__ uint32_t s_f[BLK];
    for (uint64_t f = threadIdx.x; f < ncf; f += BLK) cf_invalid[f] = 0;  // (was a memset before the launch)
    __syncthreads();
    const uint64_t per = (nseg + BLK - 1) / BLK, lo = threadIdx.x * per;
    const uint64_t hi = lo + per < nseg ? lo + per : nseg;
    // local aggregate of (starts-new-file, max merge)
    uint32_t af = 0;
    uint64_t av = 0;
    for (uint64_t j = lo; j < hi; j++) {
        const bool head = cfiles[segs[j].cfile].first_seg == j;
        const uint64_t m = merge[j];
        if (head) { af = 1; av = m; } else { av = m > av ? m : av; }
    }
    uint64_t run = block_excl_segmax<BLK>(af, av, s_v, s_f);
    for (uint64_t j = lo; j < hi; j++) {
        const SegDesc sd = segs[j];
        const bool head = cfiles[sd.cfile].first_seg == j;
        if (head) run = 0;
        const uint64_t M = head ? sd.start : run;
        seg_M[j] = M;
        const uint64_t m = merge[j];
        run = m > run ? m : run;
        if (force_serial) { cf_invalid[sd.cfile] = 1; continue; }
    }
    __syncthreads();
    if (force_serial) return;
    // membership + counts (needs every seg_M)
    for (uint64_t j = lo; j < hi; j++) {
        const SegDesc sd = segs[j];
        const uint32_t nr = chain_n[j];
        const uint64_t M = seg_M[j];
        const uint64_t R = sd.last ? sd.file_end : seg_M[j + 1];
        bool ok = nr <= (uint32_t)CHAIN_CAP && M != BW_NONE && R != BW_NONE;
        uint32_t cnt = 0;
        if (ok) {
            bool found = (M == sd.start);
            cnt = (M == sd.start && sd.start < R) ? 1 : 0;
            for (uint32_t k = 0; k < nr; k++) {
                const uint64_t e = chains[j * CHAIN_CAP + k];
                if (e == M) found = true;
                if (e >= M && e < R && e != sd.start) cnt++;
            }
            if (!sd.last && R > M) {  // the chain must reach R (R is one of its cuts)
                bool reach = false;
                for (uint32_t k = 0; k < nr; k++) reach |= chains[j * CHAIN_CAP + k] == R;
                ok = reach;
            }
            ok = ok && found;
        }
        seg_cnt[j] = cnt;
        if (!ok) cf_invalid[sd.cfile] = 1;
    }
}

// Serial walker for files whose speculative chains did not resolve: one wave walks the whole
// file, exactly like the crate's iterator, and records every chunk start.
__global__ __launch_bounds__(64 * WAVES_PER_BLOCK) void k_fallback(Walker W, const uint64_t* __restrict__ tile_off,
                                                                   uint64_t* ctr, const CFileDesc* __restrict__ cfiles,
                                                                   uint64_t ncf, const uint32_t* __restrict__ cf_invalid,
                                                                   uint64_t* __restrict__ fb_starts,
                                                                   uint64_t* __restrict__ fb_count) {
    __shared__ uint64_t lg[256];
    load_lgear(lg);
    W.lgear = lg;
    W.ncand = ctr[C_NCAND];
    W.trunc = ctr[C_TRUNC];
    const uint64_t f = (uint64_t)blockIdx.x * WAVES_PER_BLOCK + threadIdx.x / 64;
    if (f >= ncf || !cf_invalid[f]) return;
    const CFileDesc cf = cfiles[f];
    uint64_t s = cf.start, cptr = tile_off[s >> W.mk.tile_shift], n = 0;
    while (s < cf.end) {
        if (bw_lane() == 0) fb_starts[cf.fb_off + n] = s;
        n++;
        s = walk_next(W, s, cf.end, cptr);
    }
    if (bw_lane() == 0) {
        fb_count[f] = n;
        atomicAdd((unsigned long long*)&ctr[C_NINVALID], 1ull);
    }
}

void launch_resolve(hipStream_t st, const uint8_t* data, uint64_t data_len, const Masks& mk, const uint64_t* cand,
                    const uint64_t* tile_off, uint64_t* ctr, const SegDesc* segs, uint64_t nseg,
                    const CFileDesc* cfiles, uint64_t ncf, const uint64_t* chains, const uint32_t* chain_n,
                    const uint64_t* merge, uint64_t* seg_M, uint32_t* seg_cnt, uint32_t* cf_invalid,
                    uint64_t* fb_starts, uint64_t* fb_count, int force_serial) {
    if (!nseg) return;
    hipLaunchKernelGGL(k_resolve, dim3(1), dim3(BLK), 0, st, segs, nseg, cfiles, ncf, chains, chain_n, merge, seg_M,
                       seg_cnt, cf_invalid, force_serial);
    Walker W{data, cand, 0, nullptr, mk, 0, data_len};
    const unsigned grid = (unsigned)((ncf + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK);
    hipLaunchKernelGGL(k_fallback, dim3(grid), dim3(64 * WAVES_PER_BLOCK), 0, st, W, tile_off, ctr, cfiles, ncf,
                       cf_invalid, fb_starts, fb_count);
}

// ======================================================================== assembly

__device__ __forceinline__ uint64_t groups_of(uint64_t len, uint32_t gshift) {
    const uint64_t leaves = len == 0 ? 1 : (len + B3_LEAF_BYTES - 1) / B3_LEAF_BYTES;
    return (leaves + (1u << gshift) - 1) >> gshift;
}

// Emit (or just count) the blobs of unit u.  Returns blob and group counts.
template <bool WRITE>
__device__ void unit_blobs(const UnitDesc& u, const SegDesc* segs, const CFileDesc* cfiles, const uint64_t* chains,
                           const uint32_t* chain_n, const uint64_t* seg_M, const uint32_t* cf_invalid,
                           const uint64_t* fb_starts, const uint64_t* fb_count, BlobArrays b, uint64_t bbase,
                           uint64_t gbase, uint64_t& nb, uint64_t& ng) {
    nb = 0;
    ng = 0;
    auto emit = [&](uint64_t start, uint64_t end, uint32_t kind, uint64_t fend) {
        const uint64_t len = end - start;
        BW_ASSERT(start <= end && end <= fend && fend <= b.data_len);
        if (WRITE) {
            const uint64_t k = bbase + nb;
            BW_ASSERT(k < b.cap);
            b.start[k] = start;
            b.len[k] = len;
            b.goff[k] = gbase + ng;
            b.file[k] = u.file;
            b.kind[k] = kind;
            b.fend[k] = fend;
        }
        nb++;
        ng += groups_of(len, b.gshift);
    };
    if (u.kind == 0) { emit(u.start, u.start + u.len, 0, u.start + u.len); return; }
    const SegDesc sd = segs[u.seg];
    if (cf_invalid[u.cfile]) {
        const CFileDesc cf = cfiles[u.cfile];
        if (cf.first_seg != u.seg) return;
        const uint64_t n = fb_count[u.cfile];
        for (uint64_t i = 0; i < n; i++) {
            const uint64_t s = fb_starts[cf.fb_off + i];
            const uint64_t e = i + 1 < n ? fb_starts[cf.fb_off + i + 1] : cf.end;
            emit(s, e, 1, cf.end);
        }
        return;
    }
    const uint64_t M = seg_M[u.seg];
    const uint64_t R = sd.last ? sd.file_end : seg_M[u.seg + 1];
    if (M >= R) return;
    const uint32_t nr = chain_n[u.seg];
    uint64_t prev = BW_NONE;
    if (M == sd.start) prev = sd.start;
    for (uint32_t k = 0; k < nr; k++) {
        const uint64_t e = chains[u.seg * CHAIN_CAP + k];
        if (e < M || e == sd.start) continue;
        if (e >= R) break;
        if (prev != BW_NONE) emit(prev, e, 1, sd.file_end);
        prev = e;
    }
    if (prev != BW_NONE) emit(prev, R, 1, sd.file_end);
}

// Canonical blob table over all units, in three passes so a batch of a million small files
// (C4) spreads over the chip: per-unit blob/group counts (one thread per unit), a two-level
// exclusive scan of the counts (1024 units per block, then one block over the block totals),
// and the emit pass writing each unit's blobs at its offsets.
constexpr int AS_BLOCK = 256;                      // threads per block, one unit each
constexpr uint64_t AS_UNITS = AS_BLOCK;            // units per partial-scan block

// Per-unit blob/group counts (one unit per thread: a CDC segment's count walks up to 128 chain
// entries, so four per thread made C1's pass 4x longer), their exclusive scan inside the block,
// and in the grid's last block the scan of the block totals (the batch's blob and group counts).
__global__ __launch_bounds__(AS_BLOCK) void k_unit_count(const UnitDesc* __restrict__ units, uint64_t nunits,
                                                         const SegDesc* __restrict__ segs,
                                                         const CFileDesc* __restrict__ cfiles,
                                                         const uint64_t* __restrict__ chains,
                                                         const uint32_t* __restrict__ chain_n,
                                                         const uint64_t* __restrict__ seg_M,
                                                         const uint32_t* __restrict__ cf_invalid,
                                                         const uint64_t* __restrict__ fb_starts,
                                                         const uint64_t* __restrict__ fb_count, BlobArrays b,
                                                         uint64_t* __restrict__ ucb, uint64_t* __restrict__ ucg,
                                                         uint64_t* __restrict__ bt_b, uint64_t* __restrict__ bt_g,
                                                         uint64_t* ctr) {
    __shared__ uint64_t s[AS_BLOCK];
    const uint64_t u = (uint64_t)blockIdx.x * AS_BLOCK + threadIdx.x;
    uint64_t nb = 0, ng = 0;
    if (u < nunits)
        unit_blobs<false>(units[u], segs, cfiles, chains, chain_n, seg_M, cf_invalid, fb_starts, fb_count, b, 0, 0, nb,
                          ng);
    uint64_t tb, tg;
    const uint64_t rb = block_excl_sum<AS_BLOCK>(nb, s, &tb);
    const uint64_t rg = block_excl_sum<AS_BLOCK>(ng, s, &tg);
    if (u < nunits) {
        ucb[u] = rb;
        ucg[u] = rg;
    }
    if (threadIdx.x == 0) {
        bt_b[blockIdx.x] = tb;
        bt_g[blockIdx.x] = tg;
    }
    if (!last_block_done(&ctr[C_DONE_UNITS])) return;
    const uint64_t totb = scan_totals<AS_BLOCK>(bt_b, gridDim.x, s);
    const uint64_t totg = scan_totals<AS_BLOCK>(bt_g, gridDim.x, s);
    if (threadIdx.x == 0) {
        ctr[C_NBLOBS] = totb;
        ctr[C_NGROUPS] = totg;
        ctr[C_DEDUPN] = totb;
    }
}

__global__ __launch_bounds__(256) void k_unit_emit(const UnitDesc* __restrict__ units, uint64_t nunits,
                                                   const SegDesc* __restrict__ segs,
                                                   const CFileDesc* __restrict__ cfiles,
                                                   const uint64_t* __restrict__ chains,
                                                   const uint32_t* __restrict__ chain_n,
                                                   const uint64_t* __restrict__ seg_M,
                                                   const uint32_t* __restrict__ cf_invalid,
                                                   const uint64_t* __restrict__ fb_starts,
                                                   const uint64_t* __restrict__ fb_count, BlobArrays b,
                                                   const uint64_t* __restrict__ ucb, const uint64_t* __restrict__ ucg,
                                                   const uint64_t* __restrict__ bt_b,
                                                   const uint64_t* __restrict__ bt_g) {
    const uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= nunits) return;
    const uint64_t bb = ucb[u] + bt_b[u / AS_UNITS], gb = ucg[u] + bt_g[u / AS_UNITS];
    uint64_t nb, ng;
    unit_blobs<true>(units[u], segs, cfiles, chains, chain_n, seg_M, cf_invalid, fb_starts, fb_count, b, bb, gb, nb,
                     ng);
}

void launch_assemble(hipStream_t st, uint64_t* ctr, const UnitDesc* units, uint64_t nunits, const SegDesc* segs,
                     const CFileDesc* cfiles, const uint64_t* chains, const uint32_t* chain_n, const uint64_t* seg_M,
                     const uint32_t* cf_invalid, const uint64_t* fb_starts, const uint64_t* fb_count, BlobArrays b,
                     uint64_t* ucnt, uint64_t* ubtot) {
    const uint64_t nblk = (nunits + AS_UNITS - 1) / AS_UNITS;
    uint64_t *ucb = ucnt, *ucg = ucnt + nunits, *bt_b = ubtot, *bt_g = ubtot + nblk + 1;
    if (!nunits) return;  // ctr's blob and group counts stay 0 (zeroed at submit)
    hipLaunchKernelGGL(k_unit_count, dim3((unsigned)nblk), dim3(AS_BLOCK), 0, st, units, nunits, segs, cfiles, chains,
                       chain_n, seg_M, cf_invalid, fb_starts, fb_count, b, ucb, ucg, bt_b, bt_g, ctr);
    hipLaunchKernelGGL(k_unit_emit, dim3((unsigned)((nunits + 255) / 256)), dim3(256), 0, st, units, nunits, segs,
                       cfiles, chains, chain_n, seg_M, cf_invalid, fb_starts, fb_count, b, ucb, ucg, bt_b, bt_g);
}

// ======================================================================== batch tables upload

// The batch's tables from the slot's pinned staging into HBM, read over PCIe by the kernel itself.
// A hipMemcpyAsync of the same ~17 KB (C1) ran as a blit kernel below ~16 KB but as an SDMA copy
// above, and the compute stream then waited ~22 us for the copy engine after the scan
// (profiles/r03/s11_*); a kernel on the stream costs a few us and no cross-engine sync.
__global__ __launch_bounds__(256) void k_upload(const uint4* __restrict__ src, uint4* __restrict__ dst, uint64_t n16) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

__global__ __launch_bounds__(64) void k_zero(uint64_t* __restrict__ p, uint32_t n) {
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) p[i] = 0;
}

void launch_zero(hipStream_t st, uint64_t* p, uint32_t n) {
    hipLaunchKernelGGL(k_zero, dim3(1), dim3(64), 0, st, p, n);
}

void launch_upload(hipStream_t st, const void* host_src, void* dst, uint64_t bytes) {
    const uint64_t n16 = (bytes + 15) / 16;
    if (!n16) return;
    uint64_t grid = (n16 + 255) / 256;
    if (grid > 1024) grid = 1024;
    hipLaunchKernelGGL(k_upload, dim3((unsigned)grid), dim3(256), 0, st, (const uint4*)host_src, (uint4*)dst, n16);
}

// ======================================================================== Chunk.hash

// The crate returns its running gear state with the cut: h_p (odd p) or h_p << 1 (even p, the
// two-byte loop keeps the even half-step shifted), h of the last tested position when no
// position cut, and 0 for a tail of <= min bytes.  One wave per CDC chunk, <= 64 terms.
__global__ __launch_bounds__(256) void k_cut_hash(const uint8_t* __restrict__ data, Masks mk,
                                                  const uint64_t* ctr, BlobArrays b) {
    const uint64_t k = (uint64_t)blockIdx.x * 4 + threadIdx.x / 64;
    if (k >= ctr[C_NBLOBS]) return;
    const int lane = bw_lane();
    if (b.kind[k] == 0) { if (lane == 0) b.ghash[k] = 0; return; }
    const uint64_t s = b.start[k], len = b.len[k], fe = b.fend[k];
    const uint64_t rem = fe - s;
    uint64_t out = 0;
    if (rem > mk.min) {
        const uint64_t remaining = rem > mk.max ? mk.max : rem;
        const uint64_t r2 = remaining & ~1ull;
        uint64_t p = BW_NONE;
        if (len == remaining) { if (r2 > mk.s0) p = r2 - 1; }
        else p = len;
        if (p != BW_NONE) {
            const uint64_t q = p - (uint64_t)lane;
            uint64_t term = 0;
            if ((uint64_t)lane <= p && q >= mk.s0) term = c_gear[data[s + q]] << lane;
            out = bw_wave_sum64(term);
            if ((p & 1) == 0) out <<= 1;
        }
    }
    if (lane == 0) b.ghash[k] = out;
}

void launch_cut_hash(hipStream_t st, const uint8_t* data, const Masks& mk, const uint64_t* ctr, BlobArrays b,
                     uint64_t max_blobs) {
    if (!max_blobs) return;
    hipLaunchKernelGGL(k_cut_hash, dim3((unsigned)((max_blobs + 3) / 4)), dim3(256), 0, st, data, mk, ctr, b);
}

}  // namespace bw
