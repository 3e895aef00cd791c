/*
 * bw_oracle.h -- CPU restatement of backuwup's dedup front end.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this.  The
 * product path (backuwup_amd/, libbackuwup_amd.so) never links, imports or calls it.
 *
 * PARITY STATUS: the reference's arithmetic lives in two third-party Rust crates that are
 * absent from /root/reference and unbuildable here (no cargo/rustc, no network):
 *   - fastcdc 3.0.3 (Cargo.lock:557-560), module v2020, Normalization::Level1
 *   - blake3  1.3.3 (Cargo.lock:149-159), blake3::hash()
 * The reference's own tests pin none of this path, so parity is UNPINNED BY THE
 * REFERENCE.  This restatement is pinned instead by: the published BLAKE3 known answers
 * (SURVEY.md A.4), the GEAR derivation rule + sha256 (A.2), the MASKS popcount identity (A.3),
 * an independent pure-Python BLAKE3/FastCDC restatement (tests/golden/make_golden.py), and the
 * cross-check vector of A.5.
 */
#ifndef BW_ORACLE_H
#define BW_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Same layout as bw_blob in include/backuwup_gpu.h (checked by tests). */
typedef struct orc_blob {
    uint64_t file;      /* index of the file in the batch (canonical order)             */
    uint64_t offset;    /* byte offset of the blob inside its file                       */
    uint64_t length;    /* blob length in bytes                                          */
    uint64_t gear_hash; /* fastcdc Chunk.hash for CDC chunks, 0 for whole-file blobs     */
    uint8_t digest[32]; /* blake3::hash(blob)                                            */
    uint8_t is_dup;     /* 1 if Manager::add_blob would return Ok(None) (dedup hit)       */
    uint8_t pad[7];
} orc_blob;

typedef struct orc_index orc_index;

void orc_gear_table(uint64_t out[256]);
/* FastCDC::with_level(.., Level1) parameter validation + mask selection.  0 ok, -1 = the crate
 * would panic on an assert. */
int orc_fastcdc_masks(uint32_t min, uint32_t avg, uint32_t max, uint64_t* mask_s, uint64_t* mask_l);
/* fastcdc::v2020::cut() on src[0..len): returns the cut length, writes the gear hash; or
 * ORC_CUT_PANIC where the crate indexes past the source (only with avg > max). */
#define ORC_CUT_PANIC ((size_t)-1)
size_t orc_fastcdc_cut(const uint8_t* src, size_t len, uint32_t min, uint32_t avg, uint32_t max,
                       uint64_t mask_s, uint64_t mask_l, uint64_t* hash);
/* FastCDC::new(src, min, avg, max).collect(): chunks as (hash, offset, length) triples.  -1: the
 * crate's asserts fail; -2: cap too small; -3: the crate panics while iterating (avg > max). */
int orc_fastcdc_chunks(const uint8_t* src, size_t len, uint32_t min, uint32_t avg, uint32_t max,
                       uint64_t* out_hash, uint64_t* out_off, uint64_t* out_len, size_t cap,
                       size_t* n_out);
void orc_blake3(const uint8_t* data, size_t len, uint8_t out[32]);
/* tree pieces of orc_blake3 (for bw_oracle_simd.c) */
void orc_blake3_chunk_cv(const uint8_t* in, size_t len, uint64_t t, uint32_t out[8]);
void orc_blake3_parent_cv(const uint32_t l[8], const uint32_t r[8], uint32_t flags, uint32_t out[8]);
/* The crate's SIMD strategy (16 chunks / parents per AVX-512 compression), bit-identical to
 * orc_blake3; falls back to it without AVX-512 (bw_oracle_simd.c). */
void orc_blake3_fast(const uint8_t* data, size_t len, uint8_t out[32]);
int orc_blake3_simd_available(void);
/* orc_process_files hashes with orc_blake3_fast (1) or orc_blake3 (0, default); returns the
 * mode in effect. */
int orc_set_blake3_simd(int on);

orc_index* orc_index_new(const uint8_t* sorted_digests, size_t n);
void orc_index_free(orc_index* ix);
int orc_index_is_duplicate(orc_index* ix, const uint8_t digest[32]);
int orc_index_insert(orc_index* ix, const uint8_t digest[32]);

/* The whole front end over a batch of files laid out back to back in `data`:
 * process_file policy (dir_packer.rs:231-282) -> blake3 -> dedup gate in canonical order.
 * Chunk + hash run on `threads` pthreads, parallel across files and serial within a file
 * (the reference's task-per-file model, dir_packer.rs:148-166); dedup runs serially in
 * canonical order on `ix` (may be NULL = empty index). */
int orc_process_files(const uint8_t* data, const uint64_t* file_off, const uint64_t* file_len,
                      size_t n_files, uint32_t min, uint32_t avg, uint32_t max,
                      uint64_t small_file_threshold, orc_index* ix, int threads,
                      orc_blob* out, size_t cap, size_t* n_out);

/* ---- sealing (bw_oracle_seal.c): pack.rs:58-80, key_manager.rs:80-86 ---- */
void orc_sha256(const uint8_t* data, size_t len, uint8_t out[32]);
void orc_hmac_sha256(const uint8_t* key, size_t klen, const uint8_t* msg, size_t mlen, uint8_t out[32]);
void orc_hkdf_expand32(const uint8_t prk[32], const uint8_t* info, size_t info_len, uint8_t out[32]);
void orc_aes256_encrypt_block(const uint8_t key[32], const uint8_t in[16], uint8_t out[16]);
void orc_aes256_gcm_seal(const uint8_t key[32], const uint8_t nonce[12], const uint8_t* pt, size_t len,
                         uint8_t* out /* len + 16 */);
int orc_aes256_gcm_open(const uint8_t key[32], const uint8_t nonce[12], const uint8_t* ct,
                        size_t len_with_tag, uint8_t* out);
void orc_seal_blob(const uint8_t prk[32], const uint8_t* info, size_t info_len, const uint8_t nonce[12],
                   const uint8_t* payload, size_t len, uint8_t* out);
int orc_open_blob(const uint8_t prk[32], const uint8_t* info, size_t info_len, const uint8_t nonce[12],
                  const uint8_t* sealed, size_t len_with_tag, uint8_t* out);

/* ---- zstd level 3 (bw_oracle_zstd.c): pack.rs:58-64 ---- */
void bwo_zstd3_params(size_t n, unsigned out[4]);  /* wlog, small-hash log, long-hash log, mls */
size_t bwo_zstd3_bound(size_t n);
size_t bwo_zstd3_compress(const uint8_t* src, size_t n, uint8_t* dst);

#ifdef __cplusplus
}
#endif
#endif
