// bw_pack.hip -- packfile and index-file assembly on gfx950.
//
// Replaces the byte work of Manager::write_packfiles / serialize_packfile (client/src/backup/
// filesystem/packfile/pack.rs:115-227) and of BlobIndex::flush / load (blob_index.rs:167-226);
// the AES-256-GCM of every blob, header and index file runs in bw_seal.hip.
//
//   k_zstd_store  frames each blob as the magicless zstd frame that level 3 emits for
//                 incompressible input (pack.rs:58-64 settings): FHD 0x00, window descriptor,
//                 raw blocks of <= 128 KiB with 3-byte headers.  One wave per 64 KiB of frame;
//                 each lane writes 16 aligned bytes per step, read from the blob with one
//                 16-byte load unless the step straddles a block header (1 step in 8192).
//   k_pack_meta   one lane per queued blob: its PackfileHeaderBlob entry in bincode varint
//                 form (hash, kind, compression = Zstd, length, offset; filesystem/mod.rs:36-43)
//                 into the header staging area, and its 12-byte nonce in front of its sealed
//                 bytes in the packfile.
//   k_pack_files  one lane per packfile: the Vec length varint of the header and the u64 LE
//                 encrypted-header length that opens the packfile (pack.rs:222-224).
//   k_index_parse one lane per decrypted index file: the bincode varint Vec length, checked
//                 against the plaintext size (44-byte (BlobHash, PackfileId) records, trailing
//                 bytes rejected as bincode's DefaultOptions do).
//   k_index_gather one lane per record: digest (and optionally the whole record) to a
//                 contiguous array, which then seeds the dedup index (bw_dedup.hip).
#include "bw_device.h"
#include "bw_internal.h"

namespace bw {

// ------------------------------------------------------------------ zstd store frames
__device__ __forceinline__ uint8_t frame_byte(const uint8_t* __restrict__ src, uint32_t len, uint32_t nb, uint32_t wd,
                                              uint32_t f) {
    if (f == 0) return 0;  // Frame_Header_Descriptor: no FCS, no single segment, no checksum, no dict
    if (f == 1) return (uint8_t)wd;
    const uint32_t k = (f - 2) / ZSTD_STRIDE, r = (f - 2) - k * ZSTD_STRIDE;
    if (r < 3) {
        const uint32_t bl = k == nb - 1 ? len - k * ZSTD_BLOCK : ZSTD_BLOCK;
        const uint32_t h = (bl << 3) | (k == nb - 1 ? 1u : 0u);  // Raw_Block, Last_Block bit
        return (uint8_t)(h >> (8 * r));
    }
    return src[(uint64_t)k * ZSTD_BLOCK + r - 3];
}

__global__ __launch_bounds__(256) void k_zstd_store(const uint8_t* __restrict__ src, uint8_t* __restrict__ stage,
                                                    const StoreItem* __restrict__ items, uint64_t n_items,
                                                    uint64_t n_units) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t unit = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (unit >= n_units) return;
    uint64_t lo = 0, hi = n_items;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (items[mid].unit0 <= unit) lo = mid + 1;
        else hi = mid;
    }
    const StoreItem it = items[lo - 1];
    const uint32_t len = (uint32_t)it.len, nb = len ? (len + ZSTD_BLOCK - 1) / ZSTD_BLOCK : 1;
    const uint32_t framed = 2 + 3 * nb + len, wd = it.wd;
    const uint8_t* s = src + it.src_off;
    uint8_t* d = stage + it.stage_off;
    const uint32_t u0 = (uint32_t)(unit - it.unit0) * STORE_UNIT;
    const uint32_t u1 = u0 + STORE_UNIT < framed ? u0 + STORE_UNIT : framed;
    for (uint32_t f = u0 + 16 * lane; f < u1; f += 16 * 64) {
        const uint32_t k0 = f >= 2 ? (f - 2) / ZSTD_STRIDE : 0, r0 = f >= 2 ? (f - 2) - k0 * ZSTD_STRIDE : 0;
        if (f >= 2 && r0 >= 3 && r0 + 16 <= ZSTD_STRIDE && f + 16 <= framed) {
            // 16 data bytes of one block: one (unaligned) 16-byte load, one aligned store
            *(uint4*)(d + f) = *(const uint4*)(s + (uint64_t)k0 * ZSTD_BLOCK + r0 - 3);
        } else {
            uint32_t w[4] = {0, 0, 0, 0};
            for (uint32_t b = 0; b < 16 && f + b < framed; b++) w[b >> 2] |= (uint32_t)frame_byte(s, len, nb, wd, f + b) << (8 * (b & 3));
            if (f + 16 <= framed) {
                *(uint4*)(d + f) = make_uint4(w[0], w[1], w[2], w[3]);
            } else {
                for (uint32_t b = 0; f + b < framed; b++) d[f + b] = (uint8_t)(w[b >> 2] >> (8 * (b & 3)));
            }
        }
    }
}

void launch_zstd_store(hipStream_t st, const uint8_t* src, uint8_t* stage, const StoreItem* items, uint64_t n_items,
                       uint64_t n_units) {
    if (!n_units) return;
    hipLaunchKernelGGL(k_zstd_store, dim3((unsigned)((n_units + 3) / 4)), dim3(256), 0, st, src, stage, items, n_items,
                       n_units);
}

// ------------------------------------------------------------------ packfile header entries
__device__ __forceinline__ uint32_t put_varint(uint8_t* p, uint64_t v) {
    if (v < 251) {
        p[0] = (uint8_t)v;
        return 1;
    }
    const uint32_t n = v < (1ull << 16) ? 2 : (v < (1ull << 32) ? 4 : 8);
    p[0] = n == 2 ? 251 : (n == 4 ? 252 : 253);
    for (uint32_t i = 0; i < n; i++) p[1 + i] = (uint8_t)(v >> (8 * i));
    return 1 + n;
}

__global__ void k_pack_meta(const PackBlob* __restrict__ blobs, uint64_t n, uint8_t* __restrict__ hdr,
                            uint8_t* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const PackBlob& b = blobs[i];
    uint8_t* p = hdr + b.hdr_off;
    for (int k = 0; k < 32; k++) p[k] = b.hash[k];
    p += 32;
    p += put_varint(p, b.kind);
    p += put_varint(p, 1);  // CompressionKind::Zstd (pack.rs:136)
    p += put_varint(p, b.sealed_len);
    put_varint(p, b.section_off);
    uint8_t* q = out + b.nonce_off;
    for (int k = 0; k < 12; k++) q[k] = b.nonce[k];
}

__global__ void k_pack_files(const PackFileDesc* __restrict__ files, uint64_t n, uint8_t* __restrict__ hdr,
                             uint8_t* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const PackFileDesc& f = files[i];
    put_varint(hdr + f.hdr_off, f.count);
    uint8_t* q = out + f.out_off;
    for (int k = 0; k < 8; k++) q[k] = (uint8_t)(f.header_len >> (8 * k));
}

void launch_pack_meta(hipStream_t st, const PackBlob* blobs, uint64_t n, const PackFileDesc* files, uint64_t n_files,
                      uint8_t* hdr, uint8_t* out) {
    if (n) hipLaunchKernelGGL(k_pack_meta, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, blobs, n, hdr, out);
    if (n_files)
        hipLaunchKernelGGL(k_pack_files, dim3((unsigned)((n_files + 255) / 256)), dim3(256), 0, st, files, n_files, hdr,
                           out);
}

// ------------------------------------------------------------------ index files
// parsed[2 * f] = record count, parsed[2 * f + 1] = offset of the first record, or ~0 when the
// plaintext is not exactly one bincode varint Vec<([u8; 32], [u8; 12])>
__global__ void k_index_parse(const uint8_t* __restrict__ pt, const uint64_t* __restrict__ pt_off,
                              const uint64_t* __restrict__ pt_len, uint64_t n_files, uint64_t* __restrict__ parsed) {
    const uint64_t f = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= n_files) return;
    const uint8_t* p = pt + pt_off[f];
    const uint64_t len = pt_len[f];
    uint64_t cnt = ~0ull, at = ~0ull;
    if (len >= 1) {
        const uint32_t t = p[0];
        const uint32_t size = t < 251 ? 0 : (t == 251 ? 2 : (t == 252 ? 4 : (t == 253 ? 8 : 99)));
        if (size != 99 && len >= 1 + size) {
            uint64_t v = t;
            if (size) {
                v = 0;
                for (uint32_t i = 0; i < size; i++) v |= (uint64_t)p[1 + i] << (8 * i);
            }
            const uint64_t body = len - 1 - size;
            if (v <= body / 44 && v * 44 == body) {
                cnt = v;
                at = 1 + size;
            }
        }
    }
    parsed[2 * f] = cnt;
    parsed[2 * f + 1] = at;
}

void launch_index_parse(hipStream_t st, const uint8_t* pt, const uint64_t* pt_off, const uint64_t* pt_len,
                        uint64_t n_files, uint64_t* parsed) {
    if (!n_files) return;
    hipLaunchKernelGGL(k_index_parse, dim3((unsigned)((n_files + 255) / 256)), dim3(256), 0, st, pt, pt_off, pt_len,
                       n_files, parsed);
}

// rec_src[r]: byte offset of record r in the plaintext buffer (host-built from the parse)
__global__ void k_index_gather(const uint8_t* __restrict__ pt, const uint64_t* __restrict__ file_rec0,
                               const uint64_t* __restrict__ file_src, uint64_t n_files, uint64_t n_rec,
                               uint8_t* __restrict__ digests, uint8_t* __restrict__ records) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rec) return;
    uint64_t lo = 0, hi = n_files;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (file_rec0[mid] <= r) lo = mid + 1;
        else hi = mid;
    }
    const uint64_t f = lo - 1;
    const uint8_t* s = pt + file_src[f] + (r - file_rec0[f]) * 44;
    uint32_t w[11];
    for (int k = 0; k < 11; k++) w[k] = (uint32_t)s[4 * k] | (uint32_t)s[4 * k + 1] << 8 | (uint32_t)s[4 * k + 2] << 16 |
                                        (uint32_t)s[4 * k + 3] << 24;
    uint32_t* d = (uint32_t*)(digests + r * 32);
    for (int k = 0; k < 8; k++) d[k] = w[k];
    if (records) {
        uint32_t* e = (uint32_t*)(records + r * 44);
        for (int k = 0; k < 11; k++) e[k] = w[k];
    }
}

void launch_index_gather(hipStream_t st, const uint8_t* pt, const uint64_t* file_rec0, const uint64_t* file_src,
                         uint64_t n_files, uint64_t n_rec, uint8_t* digests, uint8_t* records) {
    if (!n_rec) return;
    hipLaunchKernelGGL(k_index_gather, dim3((unsigned)((n_rec + 255) / 256)), dim3(256), 0, st, pt, file_rec0,
                       file_src, n_files, n_rec, digests, records);
}

}  // namespace bw
