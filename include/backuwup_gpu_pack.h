/* backuwup_gpu_pack.h -- the C ABI of the write side after the hot path:
 * blob sealing, per-blob zstd level 3, packfiles and index files, implemented by libbackuwup_amd.so
 * (backuwup_amd/csrc/bw_capi_pack.hip).  Included by backuwup_gpu.h, whose types it uses; kept in a
 * file of its own so the hot path's header (and the source digest the committed profiles carry,
 * backuwup_amd/build.py) does not change when this side does. */
#ifndef BACKUWUP_GPU_PACK_H
#define BACKUWUP_GPU_PACK_H
#include "backuwup_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- blob sealing ----
 * The encryption half of Manager::compress_encrypt_blob (pack.rs:70-80) for already compressed
 * payloads, and the packfile header / index keys (pack.rs:212-217, blob_index.rs:185-191,205-213):
 *   key_i = KeyManager::derive_backup_key(info_i)  (key_manager.rs:80-86:
 *           Hkdf::<Sha256>::from_prk(prk).expand(info_i, 32 bytes); prk = backup_secret_key)
 *   out_i = Aes256Gcm::new(key_i).encrypt_in_place(nonce_i, b"", src_i)  = ciphertext || 16-byte tag
 * Item i: src_i = src[src_off[i] .. + src_len[i]), info_i = info[i*info_len .. + info_len)
 * (info_len <= BW_SEAL_MAX_INFO: 32 for a blob hash, 6 for "header", 5 for "index"),
 * nonce_i = nonces[12*i .. + 12]; the output goes to dst + dst_off[i] (src_len[i] + 16 bytes).
 * Output ranges must not overlap each other or the inputs.  Tables are host arrays. */
#define BW_SEAL_MAX_INFO 54u
#define BW_SEAL_TAG_BYTES 16u
/* Device buffers; asynchronous on the context stream. */
int bw_seal_device(bw_ctx* ctx, const uint8_t prk[32], const uint8_t* d_src, const uint64_t* src_off,
                   const uint64_t* src_len, uint64_t n, const uint8_t* info, uint32_t info_len,
                   const uint8_t* nonces, uint8_t* d_dst, const uint64_t* dst_off);
/* decrypt_in_place: src_len[i] includes the tag (>= 16, else BW_EINVAL); plaintext (src_len[i] - 16
 * bytes) to dst + dst_off[i]; ok[i] (host) = 1 if the tag verified, 0 where the reference returns
 * Err(aes_gcm::Error) -- the plaintext of such an item must be discarded.  Synchronous. */
int bw_open_device(bw_ctx* ctx, const uint8_t prk[32], const uint8_t* d_src, const uint64_t* src_off,
                   const uint64_t* src_len, uint64_t n, const uint8_t* info, uint32_t info_len,
                   const uint8_t* nonces, uint8_t* d_dst, const uint64_t* dst_off, uint8_t* ok);
/* Same over host buffers (synchronous; only the output ranges are written). */
int bw_seal(bw_ctx* ctx, const uint8_t prk[32], const uint8_t* src, const uint64_t* src_off,
            const uint64_t* src_len, uint64_t n, const uint8_t* info, uint32_t info_len,
            const uint8_t* nonces, uint8_t* dst, const uint64_t* dst_off);
int bw_open(bw_ctx* ctx, const uint8_t prk[32], const uint8_t* src, const uint64_t* src_off,
            const uint64_t* src_len, uint64_t n, const uint8_t* info, uint32_t info_len,
            const uint8_t* nonces, uint8_t* dst, const uint64_t* dst_off, uint8_t* ok);

/* ---- packfiles and index files ----
 * Manager::write_packfiles + serialize_packfile (pack.rs:115-227): the queue of unique blobs
 * (already gated by the index, so write_packfiles' re-check at :131 finds nothing) becomes
 * packfiles laid out back to back in one buffer:
 *   u64 LE header_len || AES-GCM(key "header", nonce = packfile id)(bincode varint
 *   Vec<PackfileHeaderBlob{hash, kind, compression = Zstd, length, offset}>) || (nonce || sealed)*
 * where sealed = AES-GCM(derive_backup_key(hash), nonce)(zstd payload) (pack.rs:58-80).  A
 * packfile closes when its blob section reaches BW_PACKFILE_TARGET_SIZE or it holds
 * BW_PACKFILE_MAX_BLOBS blobs (pack.rs:147).  Packfile ids and blob nonces come from the
 * caller (the reference draws them from getrandom, pack.rs:74-76, :207-208). */
#define BW_PACKFILE_TARGET_SIZE 3145728u /* packfile/mod.rs:25 */
#define BW_PACKFILE_MAX_SIZE 16777216u   /* packfile/mod.rs:27 */
#define BW_PACKFILE_MAX_BLOBS 100000u    /* packfile/mod.rs:29 */
#define BW_BLOB_NONCE_SIZE 12u
#define BW_INDEX_MAX_FILE_ENTRIES 50000u /* blob_index.rs:16 */
#define BW_INDEX_ENTRY_BYTES 44u         /* (BlobHash, PackfileId) */
enum { BW_BLOB_FILE_CHUNK = 0, BW_BLOB_TREE = 1 }; /* BlobKind, filesystem/mod.rs:13-17 */

/* payload_len[i] is the raw blob length: each blob is framed on the GPU as the magicless zstd
 * frame of raw blocks that zstd level 3 emits for incompressible input (2-byte frame header,
 * 3-byte header per 128 KiB block).  Without this flag payloads are caller-made zstd frames. */
#define BW_PACK_ZSTD_STORE 1u

typedef struct bw_packfile {
    uint64_t first_blob; /* queue position of its first blob                         */
    uint64_t n_blobs;
    uint64_t offset;     /* start of the packfile in the output buffer               */
    uint64_t size;       /* 8 + header_len + blob section                            */
    uint64_t header_len; /* encrypted header bytes (the u64 LE prefix)                */
} bw_packfile;

/* ---- per-blob zstd level 3 ----
 * Manager::compress_encrypt_blob's compression (pack.rs:58-64): for every blob, the frame
 * zstd::bulk::Compressor::new(3) writes with include_checksum(false), include_contentsize(false),
 * include_magicbytes(false) -- byte for byte the level-3 output of libzstd's dfast compressor
 * (pinned against the system libzstd 1.4.8; the reference links 1.5.5).
 * Blob i: src + src_off[i] (src_len[i] <= 3 MiB, else BW_EINVAL like add_blob's BlobTooLarge,
 * pack.rs:32-34); its frame goes to dst + dst_off[i], which must hold bw_zstd_store_size(src_len[i])
 * bytes (level 3 never writes more); frame_len[i] (host) = the frame's size.  Synchronous. */
int bw_zstd_compress_device(bw_ctx* ctx, const uint8_t* d_src, const uint64_t* src_off, const uint64_t* src_len,
                            uint64_t n, uint8_t* d_dst, const uint64_t* dst_off, uint64_t* frame_len);
/* Same over host buffers (staged through the device). */
int bw_zstd_compress(bw_ctx* ctx, const uint8_t* src, const uint64_t* src_off, const uint64_t* src_len, uint64_t n,
                     uint8_t* dst, const uint64_t* dst_off, uint64_t* frame_len);
/* Asynchronous form: one call lasts as long as its largest blob's serial parse, so a packer keeps
 * several batches in flight.  bw_zstd_submit_device copies the offset tables, starts the batch on
 * one of the context's BW_ZSTD_LANES lanes (each its own hash tables and a stream of its own,
 * ordered after the work already on the context's stream: lanes 0-3 high-priority streams, which
 * the runtime serves from a hardware-queue pool of their own, lanes 4-5 normal ones; 1 GiB text
 * batches from one host thread, HIP's default 4 queues per pool: 4 lanes 3.5 GB/s, 6 lanes 4.4-4.6)
 * and returns at once with *ticket; BW_ESTATE when every lane holds
 * a batch (wait for one first).  Hash tables: per lane, 768 KiB per blob for sub-batches of more
 * than 2,048 blobs and 2.5 MiB per blob for smaller ones (two pools, each grown to the largest
 * sub-batch of its layout seen: at most BW_OPT_ZSTD_SLOTS x 768 KiB + 2,048 x 2.5 MiB).  d_src and d_dst stay untouched by the caller until
 * bw_zstd_wait(ticket), which blocks for the batch and writes its n frame sizes to frame_len. */
#define BW_ZSTD_LANES 6
int bw_zstd_submit_device(bw_ctx* ctx, const uint8_t* d_src, const uint64_t* src_off, const uint64_t* src_len,
                          uint64_t n, uint8_t* d_dst, const uint64_t* dst_off, uint64_t* ticket);
int bw_zstd_wait(bw_ctx* ctx, uint64_t ticket, uint64_t* frame_len);

/* compress_encrypt_blob + write_packfiles end to end (pack.rs:58-80, 115-227) for a queue of
 * unique blobs in device memory, in two calls around the caller's plan:
 *   1. bw_pack_compress_device: zstd level 3 of blob i (d_src + src_off[i], src_len[i] <= 3 MiB,
 *      else BW_EINVAL) into a staging area the context owns; frame_len[i] (host) = its frame's
 *      size (synchronous);
 *   2. the caller plans over those sizes -- bw_pack_plan(frame_len, n, 0, ...) or
 *      bw_pack_plan_session(..., frame_len, ..., 0, ...) -- and draws one id per packfile;
 *   3. bw_pack_build_compressed: the staged frames sealed (derive_backup_key(hashes[i]), nonces[i])
 *      and laid out as bw_pack_build_device does with flags 0 (asynchronous on the context stream).
 * The staged frames stay valid until the next bw_pack_compress_device on the same context. */
int bw_pack_compress_device(bw_ctx* ctx, const uint8_t* d_src, const uint64_t* src_off, const uint64_t* src_len,
                            uint64_t n, uint64_t* frame_len);
int bw_pack_build_compressed(bw_ctx* ctx, const uint8_t prk[32], const uint8_t* hashes, const uint8_t* kinds,
                             const uint8_t* nonces, const bw_packfile* plan, uint64_t npf, const uint8_t* ids,
                             uint8_t* d_out);
/* Host-buffer forms (synchronous): the blobs are staged through the device; the packfiles land
 * in out (plan[npf-1].offset + plan[npf-1].size bytes). */
int bw_pack_compress(bw_ctx* ctx, const uint8_t* src, const uint64_t* src_off, const uint64_t* src_len, uint64_t n,
                     uint64_t* frame_len);
int bw_pack_build_compressed_host(bw_ctx* ctx, const uint8_t prk[32], const uint8_t* hashes, const uint8_t* kinds,
                                  const uint8_t* nonces, const bw_packfile* plan, uint64_t npf, const uint8_t* ids,
                                  uint8_t* out);
/* Size of the zstd store frame of a len-byte blob. */
uint64_t bw_zstd_store_size(uint64_t len);
/* Grouping and sizes (host only).  out may be NULL with cap 0 to query *n_out; BW_ENOSPC when
 * cap is too small; *total_bytes = the output buffer size. */
int bw_pack_plan(const uint64_t* payload_len, uint64_t n, uint32_t flags, bw_packfile* out, uint64_t cap,
                 uint64_t* n_out, uint64_t* total_bytes);
/* The reference's write cadence over one session (Manager::add_blob -> trigger_write_if_desired ->
 * write_packfiles, then Manager::flush; pack.rs:31-55, 82-162): n blobs in canonical (add) order
 * with their gate verdicts (bw_blob.is_dup) and payload lengths.  The packfiles hold the blobs with
 * is_dup == 0 in that order (*n_unique of them; first_blob counts among them), cut where the
 * reference cuts: a drain starts when the pending queue -- including copies of still-pending blobs,
 * which add_blob does not catch -- reaches BW_PACKFILE_TARGET_SIZE sealed bytes or
 * BW_PACKFILE_MAX_BLOBS blobs, and drains everything queued (its last packfile is a remainder);
 * the final flush drains the rest.  Host only. */
int bw_pack_plan_session(const uint8_t* digests, const uint8_t* is_dup, const uint64_t* payload_len, uint64_t n,
                         uint32_t flags, bw_packfile* out, uint64_t cap, uint64_t* n_out, uint64_t* total_bytes,
                         uint64_t* n_unique);
/* Build the planned packfiles.  Blob i: payload d_src + src_off[i] (src_len[i] bytes), hashes
 * 32 B, kinds 1 B (BW_BLOB_*), nonces 12 B; packfile_ids 12 B per packfile (host arrays).
 * d_out (device, plan's total_bytes) receives the packfiles.  Asynchronous on the context
 * stream; plan = bw_pack_plan's or bw_pack_plan_session's; BW_EINVAL when the plan does not match the blobs or a packfile exceeds
 * BW_PACKFILE_MAX_SIZE (the reference's assert, pack.rs:152-156). */
int bw_pack_build_device(bw_ctx* ctx, const uint8_t prk[32], const uint8_t* d_src, const uint64_t* src_off,
                         const uint64_t* src_len, uint64_t n, const uint8_t* hashes, const uint8_t* kinds,
                         const uint8_t* nonces, uint32_t flags, const bw_packfile* plan, uint64_t n_packfiles,
                         const uint8_t* packfile_ids, uint8_t* d_out);
/* Same over host buffers (synchronous). */
int bw_pack_build(bw_ctx* ctx, const uint8_t prk[32], const uint8_t* src, const uint64_t* src_off,
                  const uint64_t* src_len, uint64_t n, const uint8_t* hashes, const uint8_t* kinds,
                  const uint8_t* nonces, uint32_t flags, const bw_packfile* plan, uint64_t n_packfiles,
                  const uint8_t* packfile_ids, uint8_t* out);

/* Index files: BlobIndex::push/flush (blob_index.rs:151-164, 202-226).  file =
 * AES-GCM(key "index", nonce = u32 LE file number || 0^8)(bincode varint Vec<(BlobHash,
 * PackfileId)>). */
typedef struct bw_index_file {
    uint32_t file_num; /* the file name, "{file_num:0>10}"               */
    uint32_t pad;
    uint64_t offset;   /* start of the file in the buffer                  */
    uint64_t size;     /* bytes (plaintext + 16)                           */
    uint64_t n_entries;
} bw_index_file;
/* entries (host, n x 44 B) pushed in order from last_file_num: one file per
 * BW_INDEX_MAX_FILE_ENTRIES entries plus the final unconditional flush (Manager::flush,
 * pack.rs:84-90), so n = 0 still writes one empty file.  out (host) receives the files back to
 * back; files[] their table.  out = NULL or a small cap: BW_ENOSPC with *n_files and
 * *total_bytes set.  Sealed on the GPU; synchronous. */
int bw_index_files_build(bw_ctx* ctx, const uint8_t prk[32], const uint8_t* entries, uint64_t n,
                         uint32_t last_file_num, uint8_t* out, uint64_t cap, bw_index_file* files, uint64_t files_cap,
                         uint64_t* n_files, uint64_t* total_bytes);
/* BlobIndex::load (blob_index.rs:167-200) fused with the device seed: n_files index files (host
 * buffer `data`, table files[] with file_num/offset/size) are decrypted and parsed on the GPU
 * and every digest is seeded into the context's index (as bw_index_seed).  entries (optional,
 * host, cap x 44 B) receives the records in file order (the reference sorts its `items` by hash
 * afterwards).  A file whose tag fails -> BW_ECRYPTO, one that is not exactly one varint Vec ->
 * BW_EFORMAT; *bad_file = its position and nothing is seeded.  Synchronous. */
int bw_index_load_files(bw_ctx* ctx, const uint8_t prk[32], const uint8_t* data, const bw_index_file* files,
                        uint64_t n_files, uint8_t* entries, uint64_t cap, uint64_t* n_entries, uint64_t* bad_file);

#ifdef __cplusplus
}
#endif
#endif /* BACKUWUP_GPU_PACK_H */
