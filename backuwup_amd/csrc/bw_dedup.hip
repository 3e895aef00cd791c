// bw_dedup.hip -- seen-chunk index in HBM.
//
// Replaces the dedup gate of Manager::add_blob (client/src/backup/filesystem/packfile/pack.rs:
// 37-39) -> BlobIndex::is_blob_duplicate (blob_index.rs:130-148: `blobs_queued` HashSet OR
// binary search of the sorted prior `items`), with the insert of BlobIndex::add_to_packfile
// (blob_index.rs:109).  The reference decides duplicates in a racy task order;
// here the decision is defined on the canonical order (files in batch order, chunks by offset),
// which reproduces the reference's final stored set exactly: blob i is a duplicate iff its
// digest was seeded (prior backups) or appeared at an earlier canonical position.
//
// Layout: a digest log (32 B per blob ever submitted, position = canonical sequence number)
// and an open-addressing table with one 64-bit word per distinct digest: tag << 40 | seq, where
// seq is the first (minimum) log position holding that digest and tag is 24 bits of the slot hash
// (the slot index takes the low bits).  Slots are compared by the FULL 32-byte digest (the
// reference's HashSet<BlobHash> and binary search compare whole digests, blob_index.rs:109,
// 130-148): two distinct digests that share their first 8 bytes, or the whole slot hash, simply
// occupy two slots.  A slot never changes its digest once claimed, so every word of one slot
// carries the same tag and atomicMin on the word is atomicMin on the position.
//   k_append_claim  per digest: its log entry, then the probe: an empty slot is CAS'd with this
//              position, a slot whose tag matches is compared with the digest it names -- from the
//              batch's own digest array when it names a position of this batch (the log entries of
//              this launch are not read), from the log otherwise (earlier launches) -- equal ->
//              atomicMin, different -> keep probing
//   k_verdict  dup iff the slot holding this digest names an earlier position; the last block
//              advances the log length.
#include "bw_device.h"
#include "bw_internal.h"

namespace bw {

constexpr uint64_t SLOT_EMPTY = ~0ull;
constexpr int SEQ_BITS = 40;
constexpr uint64_t SEQ_MASK = (1ull << SEQ_BITS) - 1;

__device__ __forceinline__ uint64_t fmix64(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}

struct Dig {
    uint4 a, b;
};

__device__ __forceinline__ Dig load_dig(const uint8_t* p) {
    const uint4* q = (const uint4*)p;
    return Dig{q[0], q[1]};
}

__device__ __forceinline__ bool dig_eq(const Dig& x, const Dig& y) {
    return ((x.a.x ^ y.a.x) | (x.a.y ^ y.a.y) | (x.a.z ^ y.a.z) | (x.a.w ^ y.a.w) | (x.b.x ^ y.b.x) |
            (x.b.y ^ y.b.y) | (x.b.z ^ y.b.z) | (x.b.w ^ y.b.w)) == 0;
}

// slot hash of a digest: fmix64 of its first 8 bytes (the digest is uniformly random already;
// the mix keeps crafted keys that differ in a few bits apart)
__device__ __forceinline__ uint64_t dig_hash(const Dig& d) { return fmix64(((uint64_t)d.a.y << 32) | d.a.x); }

__global__ void k_table_clear(uint64_t* __restrict__ table, uint64_t cap) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < cap) table[i] = SLOT_EMPTY;
}

void launch_table_clear(hipStream_t st, uint64_t* table, uint64_t cap) {
    hipLaunchKernelGGL(k_table_clear, dim3((unsigned)((cap + 255) / 256)), dim3(256), 0, st, table, cap);
}

__device__ __forceinline__ uint64_t batch_n(const uint64_t* n_dev, uint64_t n_host) {
    return n_dev ? *n_dev : n_host;
}

// The digest at log position w: positions of the running batch (>= base) from its own digest array,
// earlier ones from the log (written by earlier launches, so visible).
__device__ __forceinline__ Dig digest_at(uint64_t w, const uint8_t* __restrict__ log, uint64_t base,
                                         const uint8_t* __restrict__ batch) {
    return w >= base ? load_dig(batch + (w - base) * 32) : load_dig(log + w * 32);
}

// Claim log position seq (digest d) into the table: the first occurrence of each distinct digest
// wins.
__device__ __forceinline__ void claim(uint64_t* table, uint64_t cap, const uint8_t* __restrict__ log, const Dig& d,
                                      uint64_t seq, uint64_t base, const uint8_t* __restrict__ batch) {
    const uint64_t mask = cap - 1, h = dig_hash(d), tag = h >> SEQ_BITS;
    const uint64_t mine = (tag << SEQ_BITS) | seq;
    uint64_t s = h & mask;
    for (uint64_t probes = 0; probes <= mask; probes++, s = (s + 1) & mask) {
        unsigned long long* p = (unsigned long long*)&table[s];
        uint64_t v = *p;  // possibly stale: an empty read is settled by the CAS, a slot never changes digest
        if (v == SLOT_EMPTY) {
            v = atomicCAS(p, (unsigned long long)SLOT_EMPTY, (unsigned long long)mine);
            if (v == SLOT_EMPTY) return;
        }
        if ((v >> SEQ_BITS) == tag && dig_eq(digest_at(v & SEQ_MASK, log, base, batch), d)) {
            atomicMin(p, (unsigned long long)mine);
            return;
        }
    }
}

// The batch's digests to the log tail, each claimed at its position as it is written.
__global__ void k_append_claim(uint64_t* __restrict__ table, uint64_t cap, uint8_t* __restrict__ log,
                               const uint64_t* dstate, const uint8_t* __restrict__ digests, const uint64_t* n_dev,
                               uint64_t n_host) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= batch_n(n_dev, n_host)) return;
    const uint64_t base = dstate[D_LOGLEN], seq = base + i;
    const Dig d = load_dig(digests + i * 32);
    uint4* l = (uint4*)(log + seq * 32);
    l[0] = d.a;
    l[1] = d.b;
    claim(table, cap, log, d, seq, base, digests);
}

// Verdicts of the batch (after every claim); the last block to finish advances the log length,
// which every block read first (no separate launch).
__global__ void k_verdict(const uint64_t* __restrict__ table, uint64_t cap, const uint8_t* __restrict__ log,
                          uint64_t* dstate, const uint8_t* __restrict__ digests, const uint64_t* n_dev, uint64_t n_host,
                          uint8_t* __restrict__ is_dup) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t n = batch_n(n_dev, n_host);
    const uint64_t base = dstate[D_LOGLEN];
    if (i < n) {
        const uint64_t seq = base + i;
        const Dig d = load_dig(digests + i * 32);
        const uint64_t mask = cap - 1, h = dig_hash(d), tag = h >> SEQ_BITS;
        uint64_t s = h & mask, w = SLOT_EMPTY;
        for (uint64_t probes = 0; probes <= mask; probes++, s = (s + 1) & mask) {
            const uint64_t v = table[s];
            if (v == SLOT_EMPTY) break;  // unreachable: this position's own claim is in the table
            if ((v >> SEQ_BITS) == tag && ((v & SEQ_MASK) == seq || dig_eq(digest_at(v & SEQ_MASK, log, base, digests), d))) {
                w = v & SEQ_MASK;
                break;
            }
        }
        uint8_t v;
        if (w == seq) {
            v = 0;
            atomicAdd((unsigned long long*)&dstate[D_NUNIQUE], 1ull);
        } else {
            v = 1;
            if (w == SLOT_EMPTY) atomicOr((unsigned long long*)&dstate[D_LOST], 1ull);
        }
        if (is_dup) is_dup[i] = v;
    }
    __shared__ bool last;
    __syncthreads();  // every thread of the block has read D_LOGLEN
    if (threadIdx.x == 0) {
        __threadfence();
        last = atomicAdd((unsigned long long*)&dstate[D_DONE], 1ull) == gridDim.x - 1;
    }
    __syncthreads();
    if (last && threadIdx.x == 0) {  // every block has read D_LOGLEN: advance it for the next gate
        dstate[D_LOGLEN] = base + n;
        dstate[D_DONE] = 0;
    }
}

void launch_dedup(hipStream_t st, uint64_t* table, uint64_t cap, uint8_t* log, uint64_t* dstate,
                  const uint8_t* digests, const uint64_t* n_dev, uint64_t n_host, uint64_t max_n, uint8_t* is_dup) {
    if (!max_n) return;
    const dim3 g((unsigned)((max_n + 255) / 256)), b(256);
    hipLaunchKernelGGL(k_append_claim, g, b, 0, st, table, cap, log, dstate, digests, n_dev, n_host);
    hipLaunchKernelGGL(k_verdict, g, b, 0, st, table, cap, log, dstate, digests, n_dev, n_host, is_dup);
}

__global__ void k_rehash(uint64_t* __restrict__ table, uint64_t cap, const uint8_t* __restrict__ log,
                         const uint64_t* dstate) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= dstate[D_LOGLEN]) return;
    claim(table, cap, log, load_dig(log + i * 32), i, ~0ull, nullptr);  // every entry from the log
}

void launch_rehash(hipStream_t st, uint64_t* table, uint64_t cap, const uint8_t* log, const uint64_t* dstate,
                   uint64_t max_n) {
    if (!max_n) return;
    hipLaunchKernelGGL(k_rehash, dim3((unsigned)((max_n + 255) / 256)), dim3(256), 0, st, table, cap, log, dstate);
}

// ------------------------------------------------------------------ multi-GPU exchange helpers

constexpr int PBLK = 1024;

__global__ __launch_bounds__(PBLK) void k_partition(const uint8_t* __restrict__ digests, uint64_t n, uint32_t n_owners,
                                                    uint8_t* __restrict__ out, uint64_t* __restrict__ perm,
                                                    uint64_t* __restrict__ counts) {
    __shared__ uint64_t s[PBLK];
    const uint32_t bits = 31 - __builtin_clz(n_owners | 1);
    const uint32_t shift = 8 - bits;
    const uint64_t per = (n + PBLK - 1) / PBLK, lo = threadIdx.x * per;
    const uint64_t hi = lo + per < n ? lo + per : n;
    uint64_t base = 0;
    for (uint32_t o = 0; o < n_owners; o++) {
        uint64_t c = 0;
        for (uint64_t i = lo; i < hi; i++) c += (n_owners == 1 || (uint32_t)(digests[i * 32] >> shift) == o);
        __syncthreads();
        uint64_t total;
        uint64_t pos = base + [&] {
            s[threadIdx.x] = c;
            __syncthreads();
            for (int d = 1; d < PBLK; d <<= 1) {
                uint64_t a = threadIdx.x >= (unsigned)d ? s[threadIdx.x - d] : 0;
                __syncthreads();
                s[threadIdx.x] += a;
                __syncthreads();
            }
            uint64_t incl = s[threadIdx.x];
            total = s[PBLK - 1];
            __syncthreads();
            return incl - c;
        }();
        for (uint64_t i = lo; i < hi; i++) {
            if (n_owners == 1 || (uint32_t)(digests[i * 32] >> shift) == o) {
                const uint4* a = (const uint4*)(digests + i * 32);
                uint4* d = (uint4*)(out + pos * 32);
                d[0] = a[0];
                d[1] = a[1];
                perm[pos] = i;
                pos++;
            }
        }
        if (threadIdx.x == 0) counts[o] = total;
        base += total;
    }
}

void launch_partition(hipStream_t st, const uint8_t* digests, uint64_t n, uint32_t n_owners, uint8_t* out,
                      uint64_t* perm, uint64_t* counts_dev) {
    hipLaunchKernelGGL(k_partition, dim3(1), dim3(PBLK), 0, st, digests, n, n_owners, out, perm, counts_dev);
}

__global__ void k_scatter(const uint8_t* __restrict__ verdict, const uint64_t* __restrict__ perm, uint64_t n,
                          uint8_t* __restrict__ is_dup) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) is_dup[perm[i]] = verdict[i];
}

void launch_scatter(hipStream_t st, const uint8_t* verdict, const uint64_t* perm, uint64_t n, uint8_t* is_dup) {
    if (!n) return;
    hipLaunchKernelGGL(k_scatter, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, verdict, perm, n, is_dup);
}

// ------------------------------------------------------------------ fixed-capacity owner buckets
// The exchange without host round trips: every rank sends every owner a bucket of `cap` slots
// (an upper bound of its batch's blob count agreed once per session), so the all-to-alls have
// equal splits and the counts travel on the device.  Bucket o holds the digests owned by o in
// canonical order; perm maps each slot back to its blob.
constexpr int BP_THREADS = 256, BP_ITEMS = 16, BP_CHUNK = BP_THREADS * BP_ITEMS;

template <int T>
__device__ __forceinline__ uint64_t block_excl_sum_u64(uint64_t v, uint64_t* s, uint64_t* total) {
    s[threadIdx.x] = v;
    __syncthreads();
    for (int d = 1; d < T; d <<= 1) {
        const uint64_t a = threadIdx.x >= (unsigned)d ? s[threadIdx.x - d] : 0;
        __syncthreads();
        s[threadIdx.x] += a;
        __syncthreads();
    }
    const uint64_t incl = s[threadIdx.x];
    *total = s[T - 1];
    __syncthreads();
    return incl - v;
}

__device__ __forceinline__ uint32_t owner_of(const uint8_t* d, uint32_t shift) { return shift >= 8 ? 0 : d[0] >> shift; }

// Per block: for owner o, each thread's count of its 16 items, block-scanned.  WRITE: place them
// (bucket o at o * cap, or, with cap == FLAT, at the owner's base that k_owner_top added to blk).
constexpr uint64_t FLAT = ~0ull;
template <bool WRITE>
__global__ __launch_bounds__(BP_THREADS) void k_bucket_pass(const uint8_t* __restrict__ digests, const uint64_t* n_dev,
                                                            uint32_t n_owners, uint32_t shift, uint64_t cap,
                                                            uint64_t* __restrict__ blk /* [blocks][n_owners] */,
                                                            uint8_t* __restrict__ out, uint64_t* __restrict__ perm) {
    __shared__ uint64_t s[BP_THREADS];
    const uint64_t n = *n_dev;
    const uint64_t i0 = (uint64_t)blockIdx.x * BP_CHUNK + (uint64_t)threadIdx.x * BP_ITEMS;
    if ((uint64_t)blockIdx.x * BP_CHUNK >= n) return;  // whole block past the end (uniform)
    uint32_t own[BP_ITEMS];
#pragma unroll
    for (int k = 0; k < BP_ITEMS; k++) own[k] = i0 + k < n ? owner_of(digests + (i0 + k) * 32, shift) : ~0u;
    for (uint32_t o = 0; o < n_owners; o++) {
        uint64_t c = 0;
#pragma unroll
        for (int k = 0; k < BP_ITEMS; k++) c += own[k] == o;
        uint64_t total;
        uint64_t pos = block_excl_sum_u64<BP_THREADS>(c, s, &total);
        if (!WRITE) {
            if (threadIdx.x == 0) blk[(uint64_t)blockIdx.x * n_owners + o] = total;
        } else {
            pos += blk[(uint64_t)blockIdx.x * n_owners + o];
#pragma unroll
            for (int k = 0; k < BP_ITEMS; k++)
                if (own[k] == o) {
                    if (pos < cap) {
                        const uint64_t at = cap == FLAT ? pos : (uint64_t)o * cap + pos;
                        const uint4* a = (const uint4*)(digests + (i0 + k) * 32);
                        uint4* d = (uint4*)(out + at * 32);
                        d[0] = a[0];
                        d[1] = a[1];
                        perm[at] = i0 + k;
                    }
                    pos++;
                }
        }
    }
}

// Per owner: exclusive scan of the block totals (in place) and the bucket count.
__global__ void k_bucket_top(uint64_t* __restrict__ blk, uint64_t nblk, uint32_t n_owners, const uint64_t* n_dev,
                             uint64_t cap, uint64_t* __restrict__ counts, uint64_t* err) {
    const uint32_t o = blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= n_owners) return;
    const uint64_t used = (*n_dev + BP_CHUNK - 1) / BP_CHUNK;
    uint64_t run = 0;
    for (uint64_t b = 0; b < used && b < nblk; b++) {
        const uint64_t t = blk[b * n_owners + o];
        blk[b * n_owners + o] = run;
        run += t;
    }
    counts[o] = run < cap ? run : cap;
    if (run > cap) atomicOr((unsigned long long*)err, 1ull);
}

void launch_bucket_partition(hipStream_t st, const uint8_t* digests, const uint64_t* n_dev, uint64_t max_n,
                             uint32_t n_owners, uint64_t cap, uint8_t* out, uint64_t* perm, uint64_t* counts,
                             uint64_t* blk, uint64_t* err) {
    const uint32_t bits = 31 - __builtin_clz(n_owners | 1);
    const uint32_t shift = 8 - bits;
    const uint64_t nblk = (max_n + BP_CHUNK - 1) / BP_CHUNK;
    if (nblk)
        hipLaunchKernelGGL(k_bucket_pass<false>, dim3((unsigned)nblk), dim3(BP_THREADS), 0, st, digests, n_dev,
                           n_owners, shift, cap, blk, out, perm);
    hipLaunchKernelGGL(k_bucket_top, dim3((n_owners + 255) / 256), dim3(256), 0, st, blk, nblk, n_owners, n_dev, cap,
                       counts, err);
    if (nblk)
        hipLaunchKernelGGL(k_bucket_pass<true>, dim3((unsigned)nblk), dim3(BP_THREADS), 0, st, digests, n_dev,
                           n_owners, shift, cap, blk, out, perm);
}

// ------------------------------------------------------------------ exactly sized owner sections
// bw_exchange_dedup since round 5: the digests grouped by owner back to back (owner o's section
// starts at the sum of the counts of the owners before it), so every transfer carries exactly its
// digests.  One block: per owner the exclusive scan over the count pass's blocks, then the owners'
// bases added in; msg[2o] = digests for owner o, msg[2o + 1] = the largest of them (every rank
// learns the global largest section from the counts all-to-all: the host transport pads to it).
__global__ __launch_bounds__(256) void k_owner_top(uint64_t* __restrict__ blk, uint64_t nblk, uint32_t n_owners,
                                                   const uint64_t* n_dev, uint64_t* __restrict__ msg) {
    __shared__ uint64_t s[256];
    __shared__ uint64_t mx;
    const uint32_t o = threadIdx.x;
    const uint64_t used = (*n_dev + BP_CHUNK - 1) / BP_CHUNK;
    uint64_t run = 0;
    if (o < n_owners)
        for (uint64_t b = 0; b < used && b < nblk; b++) {
            const uint64_t t = blk[b * n_owners + o];
            blk[b * n_owners + o] = run;
            run += t;
        }
    if (o == 0) mx = 0;
    __syncthreads();
    if (o < n_owners) atomicMax((unsigned long long*)&mx, (unsigned long long)run);
    uint64_t total;
    const uint64_t base = block_excl_sum_u64<256>(o < n_owners ? run : 0, s, &total);
    if (o < n_owners) {
        for (uint64_t b = 0; b < used && b < nblk; b++) blk[b * n_owners + o] += base;
        msg[2 * o] = run;
        msg[2 * o + 1] = mx;
    }
}

void launch_owner_partition(hipStream_t st, const uint8_t* digests, const uint64_t* n_dev, uint64_t max_n,
                            uint32_t n_owners, uint8_t* out, uint64_t* perm, uint64_t* msg, uint64_t* blk) {
    const uint32_t bits = 31 - __builtin_clz(n_owners | 1);
    const uint32_t shift = 8 - bits;
    const uint64_t nblk = (max_n + BP_CHUNK - 1) / BP_CHUNK;
    if (nblk)
        hipLaunchKernelGGL(k_bucket_pass<false>, dim3((unsigned)nblk), dim3(BP_THREADS), 0, st, digests, n_dev,
                           n_owners, shift, FLAT, blk, out, perm);
    hipLaunchKernelGGL(k_owner_top, dim3(1), dim3(256), 0, st, blk, nblk, n_owners, n_dev, msg);
    if (nblk)
        hipLaunchKernelGGL(k_bucket_pass<true>, dim3((unsigned)nblk), dim3(BP_THREADS), 0, st, digests, n_dev,
                           n_owners, shift, FLAT, blk, out, perm);
}

__global__ void k_copy_u64(const uint64_t* __restrict__ src, uint64_t* __restrict__ dst, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = src[i];
}

void launch_copy_u64(hipStream_t st, const uint64_t* src, uint64_t* dst, uint32_t n) {
    if (n) hipLaunchKernelGGL(k_copy_u64, dim3((n + 255) / 256), dim3(256), 0, st, src, dst, n);
}

// Verdicts of my owner sections (partition order) back to blob order, into is_dup and the records.
__global__ void k_owner_scatter(const uint8_t* __restrict__ verdict, const uint64_t* __restrict__ perm, uint64_t n,
                                uint8_t* __restrict__ is_dup, uint8_t* __restrict__ packed) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t j = perm[i];
    const uint8_t v = verdict[i];
    is_dup[j] = v;
    if (packed) packed[j * sizeof(bw_blob) + offsetof(bw_blob, is_dup)] = v;
}

void launch_owner_scatter(hipStream_t st, const uint8_t* verdict, const uint64_t* perm, uint64_t n, uint8_t* is_dup,
                          uint8_t* packed) {
    if (!n) return;
    hipLaunchKernelGGL(k_owner_scatter, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, verdict, perm, n, is_dup,
                       packed);
}

// Owner side: the received buckets (source-major = canonical) packed contiguously, n on device.
__global__ void k_bucket_gather(const uint8_t* __restrict__ buckets, const uint64_t* __restrict__ counts,
                                uint32_t n_src, uint64_t cap, uint8_t* __restrict__ out, uint64_t* __restrict__ n_out,
                                int expand, const uint8_t* __restrict__ v_in, uint8_t* __restrict__ v_out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t s = i / cap, k = i % cap;
    if (s >= n_src) return;
    uint64_t base = 0;
    for (uint32_t j = 0; j < s; j++) base += counts[j];
    if (!expand && i == 0) {
        uint64_t t = 0;
        for (uint32_t j = 0; j < n_src; j++) t += counts[j];
        *n_out = t;
    }
    if (k >= counts[s]) return;
    if (!expand) {
        const uint4* a = (const uint4*)(buckets + i * 32);
        uint4* d = (uint4*)(out + (base + k) * 32);
        d[0] = a[0];
        d[1] = a[1];
    } else {
        v_out[i] = v_in[base + k];  // verdicts back into the bucket layout
    }
}

void launch_bucket_gather(hipStream_t st, const uint8_t* buckets, const uint64_t* counts, uint32_t n_src, uint64_t cap,
                          uint8_t* out, uint64_t* n_out) {
    const uint64_t n = (uint64_t)n_src * cap;
    if (!n) return;
    hipLaunchKernelGGL(k_bucket_gather, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, buckets, counts, n_src, cap,
                       out, n_out, 0, nullptr, nullptr);
}

void launch_bucket_expand(hipStream_t st, const uint64_t* counts, uint32_t n_src, uint64_t cap, const uint8_t* v_in,
                          uint8_t* v_out) {
    const uint64_t n = (uint64_t)n_src * cap;
    if (!n) return;
    hipLaunchKernelGGL(k_bucket_gather, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, nullptr, counts, n_src,
                       cap, nullptr, nullptr, 1, v_in, v_out);
}

// Source side: verdicts of my buckets back to blob order.
__global__ void k_bucket_scatter(const uint8_t* __restrict__ verdict, const uint64_t* __restrict__ perm,
                                 const uint64_t* __restrict__ counts, uint32_t n_owners, uint64_t cap,
                                 uint8_t* __restrict__ is_dup, uint8_t* __restrict__ packed) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t o = i / cap, k = i % cap;
    if (o >= n_owners || k >= counts[o]) return;
    const uint64_t j = perm[i];
    const uint8_t v = verdict[i];
    is_dup[j] = v;
    if (packed) packed[j * sizeof(bw_blob) + offsetof(bw_blob, is_dup)] = v;
}

void launch_bucket_scatter(hipStream_t st, const uint8_t* verdict, const uint64_t* perm, const uint64_t* counts,
                           uint32_t n_owners, uint64_t cap, uint8_t* is_dup, uint8_t* packed) {
    const uint64_t n = (uint64_t)n_owners * cap;
    if (!n) return;
    hipLaunchKernelGGL(k_bucket_scatter, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, verdict, perm, counts,
                       n_owners, cap, is_dup, packed);
}

// ------------------------------------------------------------------ result records

__device__ __forceinline__ void index_snapshot(const uint64_t* dstate, uint64_t* ctr) {
    ctr[C_LOST] = dstate[D_LOST];
    ctr[C_NUNIQUE] = dstate[D_NUNIQUE];
    ctr[C_IX_OVF] = dstate[D_BUCKET_OVF];
    ctr[C_IX_LOGLEN] = dstate[D_LOGLEN];
    ctr[C_IX_VALID] = 1;
}

__global__ void k_index_snapshot(const uint64_t* dstate, uint64_t* ctr) { index_snapshot(dstate, ctr); }

void launch_index_snapshot(hipStream_t st, const uint64_t* dstate, uint64_t* ctr) {
    hipLaunchKernelGGL(k_index_snapshot, dim3(1), dim3(1), 0, st, dstate, ctr);
}

// host (may be null): pinned host memory that receives the counters (C_COUNT u64, the index
// snapshot included) and the first host_n records as well -- the batch's results reach the host
// without a copy operation on the stream (each one costs ~5 us of idle GPU plus its own time).
__global__ void k_pack(uint64_t* ctr, BlobArrays b, const uint64_t* __restrict__ file_start,
                       const uint8_t* __restrict__ digests, const uint8_t* __restrict__ is_dup, uint8_t* __restrict__ out,
                       const uint64_t* dstate, uint8_t* __restrict__ host, uint64_t host_n) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k == 0) {
        if (dstate) index_snapshot(dstate, ctr);  // the gate ran before this kernel on the stream
        if (host)
            for (int i = 0; i < C_COUNT; i++) ((uint64_t*)host)[i] = ctr[i];
    }
    if (k >= ctr[C_NBLOBS]) return;
    uint64_t* o = (uint64_t*)(out + k * 72);
    const uint32_t f = b.file[k];
    o[0] = f;
    o[1] = b.start[k] - file_start[f];
    o[2] = b.len[k];
    o[3] = b.ghash[k];
    const uint64_t* d = (const uint64_t*)(digests + k * 32);
    o[4] = d[0];
    o[5] = d[1];
    o[6] = d[2];
    o[7] = d[3];
    o[8] = is_dup ? (uint64_t)is_dup[k] : 0;
    if (host && k < host_n) {
        uint64_t* h = (uint64_t*)(host + C_COUNT * 8 + k * 72);
#pragma unroll
        for (int i = 0; i < 9; i++) h[i] = o[i];
    }
}

void launch_pack(hipStream_t st, uint64_t* ctr, BlobArrays b, const uint64_t* file_start, const uint8_t* digests,
                 const uint8_t* is_dup, uint8_t* out, uint64_t max_blobs, const uint64_t* dstate, uint8_t* host,
                 uint64_t host_n) {
    hipLaunchKernelGGL(k_pack, dim3((unsigned)((max_blobs + 255) / 256 + (max_blobs == 0))), dim3(256), 0, st, ctr, b,
                       file_start, digests, is_dup, out, dstate, host, host_n);
}

}  // namespace bw
