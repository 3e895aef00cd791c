// bw_pack.hip -- packfile and index-file assembly on gfx950.
//
// Replaces the byte work of Manager::write_packfiles / serialize_packfile (client/src/backup/
// filesystem/packfile/pack.rs:115-227) and of BlobIndex::flush / load (blob_index.rs:167-226);
// the AES-256-GCM of every blob, header and index file runs in bw_seal.hip.
//
//   (zstd store frames -- the magicless frame level 3 emits for incompressible input,
//    pack.rs:58-64 settings -- are built on the fly by k_seal_ctr<false, true> in bw_seal.hip,
//    so a blob is read once and its sealed frame written once.)
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
