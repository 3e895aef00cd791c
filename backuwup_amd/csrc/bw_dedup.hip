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
// and an open-addressing table of {key = first 8 digest bytes, seq = min position}.
//   k_append  copy the batch digests to the log tail
//   k_claim   CAS the key into a slot, atomicMin the sequence number (first occurrence wins)
//   k_verdict dup iff the slot's winner is an earlier position holding the same 32 bytes; a
//             different digest behind the same 64-bit key is reported (BW_ECOLLISION), never
//             silently merged.
#include "bw_device.h"
#include "bw_internal.h"

namespace bw {

__device__ __forceinline__ uint64_t fmix64(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}

__device__ __forceinline__ uint64_t digest_key(const uint8_t* d) {
    const uint64_t k = *(const uint64_t*)d;
    return k ? k : 1;  // 0 marks an empty slot
}

__global__ void k_table_clear(uint64_t* __restrict__ table, uint64_t cap) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < cap) { table[2 * i] = 0; table[2 * i + 1] = ~0ull; }
}

void launch_table_clear(hipStream_t st, uint64_t* table, uint64_t cap) {
    hipLaunchKernelGGL(k_table_clear, dim3((unsigned)((cap + 255) / 256)), dim3(256), 0, st, table, cap);
}

__device__ __forceinline__ uint64_t batch_n(const uint64_t* n_dev, uint64_t n_host) {
    return n_dev ? *n_dev : n_host;
}

__global__ void k_append(uint8_t* __restrict__ log, const uint64_t* dstate, const uint8_t* __restrict__ digests,
                         const uint64_t* n_dev, uint64_t n_host) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= batch_n(n_dev, n_host)) return;
    const uint64_t base = dstate[D_LOGLEN];
    const uint4* s = (const uint4*)(digests + i * 32);
    uint4* d = (uint4*)(log + (base + i) * 32);
    d[0] = s[0];
    d[1] = s[1];
}

// Claim log[lo + i] for i < n into the table.
__device__ __forceinline__ void claim(uint64_t* table, uint64_t cap, const uint8_t* log, uint64_t seq) {
    const uint64_t key = digest_key(log + seq * 32), mask = cap - 1;
    uint64_t s = fmix64(key) & mask;
    for (;;) {
        unsigned long long* kp = (unsigned long long*)&table[2 * s];
        uint64_t k = *kp;
        if (k == 0) {
            const uint64_t prev = atomicCAS(kp, 0ull, (unsigned long long)key);
            k = prev == 0 ? key : prev;
        }
        if (k == key) {
            atomicMin((unsigned long long*)&table[2 * s + 1], (unsigned long long)seq);
            return;
        }
        s = (s + 1) & mask;
    }
}

__global__ void k_claim(uint64_t* __restrict__ table, uint64_t cap, const uint8_t* __restrict__ log,
                        const uint64_t* dstate, const uint64_t* n_dev, uint64_t n_host) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= batch_n(n_dev, n_host)) return;
    claim(table, cap, log, dstate[D_LOGLEN] + i);
}

__global__ void k_verdict(const uint64_t* __restrict__ table, uint64_t cap, const uint8_t* __restrict__ log,
                          uint64_t* dstate, const uint64_t* n_dev, uint64_t n_host, uint8_t* __restrict__ is_dup) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= batch_n(n_dev, n_host)) return;
    const uint64_t seq = dstate[D_LOGLEN] + i;
    const uint8_t* d = log + seq * 32;
    const uint64_t key = digest_key(d), mask = cap - 1;
    uint64_t s = fmix64(key) & mask;
    while (table[2 * s] != key) s = (s + 1) & mask;
    const uint64_t w = table[2 * s + 1];
    uint8_t v;
    if (w == seq) {
        v = 0;
        atomicAdd((unsigned long long*)&dstate[D_NUNIQUE], 1ull);
    } else {
        const uint4* a = (const uint4*)(log + w * 32);
        const uint4* b = (const uint4*)d;
        const uint4 a0 = a[0], a1 = a[1], b0 = b[0], b1 = b[1];
        const bool same = a0.x == b0.x && a0.y == b0.y && a0.z == b0.z && a0.w == b0.w && a1.x == b1.x &&
                          a1.y == b1.y && a1.z == b1.z && a1.w == b1.w;
        v = same ? 1 : 2;
        if (!same) atomicOr((unsigned long long*)&dstate[D_COLLIDE], 1ull);
    }
    if (is_dup) is_dup[i] = v;
}

__global__ void k_advance(uint64_t* dstate, const uint64_t* n_dev, uint64_t n_host) {
    if (threadIdx.x == 0 && blockIdx.x == 0) dstate[D_LOGLEN] += batch_n(n_dev, n_host);
}

void launch_dedup(hipStream_t st, uint64_t* table, uint64_t cap, uint8_t* log, uint64_t* dstate,
                  const uint8_t* digests, const uint64_t* n_dev, uint64_t n_host, uint64_t max_n, uint8_t* is_dup) {
    if (!max_n) return;
    const dim3 g((unsigned)((max_n + 255) / 256)), b(256);
    hipLaunchKernelGGL(k_append, g, b, 0, st, log, dstate, digests, n_dev, n_host);
    hipLaunchKernelGGL(k_claim, g, b, 0, st, table, cap, log, dstate, n_dev, n_host);
    hipLaunchKernelGGL(k_verdict, g, b, 0, st, table, cap, log, dstate, n_dev, n_host, is_dup);
    hipLaunchKernelGGL(k_advance, dim3(1), dim3(64), 0, st, dstate, n_dev, n_host);
}

__global__ void k_rehash(uint64_t* __restrict__ table, uint64_t cap, const uint8_t* __restrict__ log,
                         const uint64_t* dstate) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= dstate[D_LOGLEN]) return;
    claim(table, cap, log, i);
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

// ------------------------------------------------------------------ result records

__global__ void k_pack(const uint64_t* ctr, BlobArrays b, const uint64_t* __restrict__ file_start,
                       const uint8_t* __restrict__ digests, const uint8_t* __restrict__ is_dup, uint8_t* __restrict__ out) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
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
}

void launch_pack(hipStream_t st, const uint64_t* ctr, BlobArrays b, const uint64_t* file_start, const uint8_t* digests,
                 const uint8_t* is_dup, uint8_t* out, uint64_t max_blobs) {
    if (!max_blobs) return;
    hipLaunchKernelGGL(k_pack, dim3((unsigned)((max_blobs + 255) / 256)), dim3(256), 0, st, ctr, b, file_start,
                       digests, is_dup, out);
}

}  // namespace bw
