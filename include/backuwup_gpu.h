/*
 * backuwup_gpu.h -- C ABI of the MI355X (gfx950) dedup front end for backuwup.
 *
 * The reference has no FFI layer on this path; it reaches three Rust call sites directly
 * (SURVEY.md §8b).  Each entry point below replaces one of them and keeps its argument
 * meaning and error behaviour; INTEGRATION.md shows the Rust `extern "C"` binding:
 *
 *   fastcdc::v2020::FastCDC::new(&[u8], min, avg, max) + Iterator<Item = Chunk>
 *       client/src/backup/filesystem/dir_packer.rs:254-266          -> bw_fastcdc_chunks
 *   blake3::hash(&[u8]) -> Hash  (then .into(): [u8; 32])
 *       client/src/backup/filesystem/dir_packer.rs:286, :320, :353  -> bw_blake3_hash(_many)
 *   BlobIndex::load() (sorted `items`)            blob_index.rs:167-200  -> bw_index_seed
 *   Manager::add_blob dedup gate -> BlobIndex::is_blob_duplicate, then blobs_queued.insert
 *       pack.rs:37-39, blob_index.rs:109,130-148                     -> bw_index_check_insert
 *   dir_packer::process_file + add_file_blob for a batch of files (dir_packer.rs:231-311)
 *                                                                   -> bw_process_files(_device)
 *
 * Conventions: every function returns an int status (BW_OK = 0, negative = error) and never
 * unwinds across the boundary.  Where the fastcdc crate panics on an assert (parameter ranges)
 * this returns BW_EINVAL.  Output arrays are caller-owned; when one is too small BW_ENOSPC is
 * returned and *n_out holds the required count.  Device buffers, streams and the dedup table
 * are owned by the opaque bw_ctx.  A context is not thread-safe: callers hashing from several
 * threads use one context per thread, all attached to one shared bw_index (the reference
 * serializes index access under the packer mutex, packfile/mod.rs:77; so does bw_index).
 *
 * Scalars: "device pointer" arguments are HIP device addresses (e.g. from hipMalloc or a
 * torch tensor's data_ptr()), 16-byte aligned; everything else is host memory.
 */
#ifndef BACKUWUP_GPU_H
#define BACKUWUP_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BW_API_VERSION 1

enum {
    BW_OK = 0,
    BW_EINVAL = -1,     /* parameter outside the fastcdc crate's asserted ranges, bad pointer  */
    BW_ENOSPC = -2,     /* caller's output array too small; *n_out = required count            */
    BW_EHIP = -3,       /* HIP runtime error (message in bw_last_error)                        */
    BW_ENOMEM = -4,     /* device or host allocation failed                                    */
    BW_ECOLLISION = -5, /* not returned since round 4: the index compares whole digests        */
    BW_ESTATE = -6,     /* call order violated (e.g. bw_results before a batch was submitted)   */
    BW_ECRYPTO = -7,    /* an AES-GCM tag did not verify (PackfileError::CryptoError)           */
    BW_EFORMAT = -8,    /* bincode deserialization failed (PackfileError::SerializationError)   */
    BW_ECOMM = -9,      /* the exchange transport failed (RCCL, or the caller's host all-to-all) */
    BW_EAGAIN = -10     /* bw_blake3_hash_dropin_device only: the device's hash service could not
                           take this call (message over BW_COALESCE_MAX_MSG, service unavailable,
                           or no digest within its bound); nothing was changed, retry the message
                           through a context (bw_blake3_hash_many)                                 */
};

/* fastcdc::v2020 size bounds (asserted by FastCDC::with_level).  avg > max passes those asserts, but
 * the crate's cut() then reads past max (a chunk longer than max, or an index panic): the ABI refuses
 * it with BW_EINVAL too.  min > max is legal: a remainder <= min is one chunk, longer than max. */
#define BW_MINIMUM_MIN 64u
#define BW_MINIMUM_MAX 1048576u
#define BW_AVERAGE_MIN 256u
#define BW_AVERAGE_MAX 4194304u
#define BW_MAXIMUM_MIN 1024u
#define BW_MAXIMUM_MAX 16777216u

/* backuwup's chunker constants, client/src/defaults.rs:61-68 */
#define BW_BLOB_MINIMUM_TARGET_SIZE 262144u  /* 256 KiB */
#define BW_BLOB_DESIRED_TARGET_SIZE 1048576u /* 1 MiB   */
#define BW_BLOB_MAX_UNCOMPRESSED_SIZE 3145728u /* 3 MiB */

typedef struct bw_ctx bw_ctx;

/* fastcdc::v2020::Chunk { hash: u64, offset: usize, length: usize } */
typedef struct bw_chunk {
    uint64_t hash;
    uint64_t offset;
    uint64_t length;
} bw_chunk;

/* One blob produced by process_file/add_file_blob (dir_packer.rs:231-311), in canonical order
 * (files in the order given, chunks in offset order). */
typedef struct bw_blob {
    uint64_t file;      /* index of the source file in the batch                            */
    uint64_t offset;    /* offset of the blob inside its file                                */
    uint64_t length;    /* blob length                                                       */
    uint64_t gear_hash; /* Chunk.hash for CDC chunks; 0 for whole-file blobs                 */
    uint8_t digest[32]; /* blake3::hash(blob) = BlobHash                                     */
    uint8_t is_dup;     /* 1 = Manager::add_blob returns Ok(None) (already seen)             */
    uint8_t pad[7];
} bw_blob;

/* Batch parameters.  Defaults (bw_params_default): backuwup's 256 KiB / 1 MiB / 3 MiB and the
 * small-file rule `len > BLOB_DESIRED_TARGET_SIZE` -> CDC (dir_packer.rs:246). */
typedef struct bw_params {
    uint32_t min_size;
    uint32_t avg_size;
    uint32_t max_size;
    uint32_t flags;                /* BW_F_* below                                      */
    uint64_t small_file_threshold; /* files with len > threshold are chunked by CDC     */
} bw_params;

#define BW_F_NO_HASH 1u        /* chunk only (digests left zero)                           */
#define BW_F_NO_DEDUP 2u       /* skip the index (is_dup left 0); digests still logged     */
#define BW_F_SERIAL_RESOLVE 4u /* force the serial boundary walker (test/diagnostic path)  */

void bw_params_default(bw_params* p);
const char* bw_strerror(int rc);

int bw_create(int device, bw_ctx** out);
void bw_destroy(bw_ctx* ctx);
const char* bw_last_error(const bw_ctx* ctx);
/* Run on a caller stream (hipStream_t as void*); NULL selects the context's own stream. */
int bw_set_stream(bw_ctx* ctx, void* hip_stream);
void* bw_get_stream(bw_ctx* ctx);

/* FastCDC::new(src, min, avg, max).collect::<Vec<Chunk>>() over a host buffer. */
int bw_fastcdc_chunks(bw_ctx* ctx, const uint8_t* src, uint64_t len, uint32_t min_size,
                      uint32_t avg_size, uint32_t max_size, bw_chunk* out, uint64_t cap,
                      uint64_t* n_out);

/* The reference's per-file call pattern (dir_packer.rs:254-266 then :286 per chunk) without a second
 * trip per chunk: FastCDC::new(src, min, avg, max).collect() as bw_fastcdc_chunks, with every
 * chunk's BLAKE3 digest computed in the same submit and kept under *handle until
 * bw_fastcdc_release(handle).  Until then bw_blake3_hash_dropin of exactly one of these chunks
 * (pointer src + offset, that length; any context, any thread) returns the kept digest without
 * touching the GPU.  The caller keeps src unchanged until the release: the Rust drop-in's FastCDC
 * borrows the mmap immutably for its lifetime and releases in Drop (rust/backuwup-gpu,
 * INTEGRATION.md).  The registry of live handles is an ordered interval map under a reader lock
 * with a per-thread cache, so lookups from many threads neither serialize nor scan every handle. */
int bw_fastcdc_chunks_hashed(bw_ctx* ctx, const uint8_t* src, uint64_t len, uint32_t min_size,
                             uint32_t avg_size, uint32_t max_size, bw_chunk* out, uint64_t cap,
                             uint64_t* n_out, uint64_t* handle);
void bw_fastcdc_release(uint64_t handle);
/* digests answered from kept chunk digests since the process started (diagnostic) */
uint64_t bw_blake3_kept_hits(void);

/* blake3::hash(data) -> 32 bytes, host buffer; always hashes the bytes given.  Messages up to
 * BW_COALESCE_MAX_MSG (a small file, a tree blob) go to the device's hash service: each caller
 * copies its message into a staging buffer of its own and posts a request into a ring of slots that
 * a persistent kernel's workers poll (with a large BAR both sit in HBM, written by the CPU through
 * the BAR; otherwise in pinned host memory, or so with BW_SVC_HOST_RING=1); the digest lands in a
 * response slot in pinned memory, where the caller spins briefly and then sleeps until a library
 * thread wakes it.  No kernel launch per call: ~7 us for a tree blob, ~20 us for 16 KiB on one
 * thread, and concurrent callers (any contexts, any threads) are served in parallel.  The service's
 * instance ends by itself after 5 ms without messages (or 500 ms of life; the next call starts
 * another).  It runs on a non-blocking stream of the least priority, so neither the process's
 * streams nor the legacy null stream wait for it; a device-wide synchronization does, up to the
 * life (BW_SVC_LIFE_US=1000..500000 shortens it).  BW_DROPIN_SERVICE=0 in the
 * environment selects the earlier batching path (launches coalesced over four lanes).  For such
 * messages the context is only read for its device, so any number of threads may pass the same
 * context; larger messages run on the context itself (one thread at a time). */
#define BW_COALESCE_MAX_MSG 65536u
int bw_blake3_hash(bw_ctx* ctx, const uint8_t* data, uint64_t len, uint8_t out[32]);
/* The Rust blake3::hash drop-in's entry (dir_packer.rs:286, :320, :353): as bw_blake3_hash, except
 * that a chunk slice of a live bw_fastcdc_chunks_hashed source is answered from its kept digest.
 * Only for callers that guarantee those bytes are unchanged while the handle lives. */
int bw_blake3_hash_dropin(bw_ctx* ctx, const uint8_t* data, uint64_t len, uint8_t out[32]);
/* The same without a context, for callers that hold none (the Rust blake3::hash drop-in: each thread
 * names the device it hashes on, INTEGRATION.md "every GPU of the node"): the kept digests first,
 * then messages up to BW_COALESCE_MAX_MSG through `device`'s hash service.  Returns BW_EAGAIN, with
 * nothing changed, where bw_blake3_hash_dropin would have used its context: a larger message, a
 * service that is unavailable, or a call that got no slot or digest within 10 s (its ticket is then
 * cancelled and its ring slot handed on, so later calls are unaffected).  The caller then hashes the
 * message through a context it holds (bw_blake3_hash_many). */
int bw_blake3_hash_dropin_device(int device, const uint8_t* data, uint64_t len, uint8_t out[32]);
/* launches (hash-service instances, or coalesced batches) and the messages they carried on
 * `device` since the process started */
int bw_blake3_coalesce_stats(int device, uint64_t* batches, uint64_t* messages);
/* hash-service calls on `device` that gave up (BW_EAGAIN) and whose tickets were abandoned; of
 * those, tickets already handed back; and instances found finished without having published their
 * end (the host then marks them ended itself) */
int bw_blake3_service_faults(int device, uint64_t* abandoned, uint64_t* reclaimed, uint64_t* recovered);
/* visible HIP devices (the Rust drop-ins' pool spreads over them) */
int bw_device_count(int* n);
/* n independent messages data[offsets[i] .. offsets[i]+lengths[i]) -> out[32*i..] */
int bw_blake3_hash_many(bw_ctx* ctx, const uint8_t* data, uint64_t data_len,
                        const uint64_t* offsets, const uint64_t* lengths, uint64_t n,
                        uint8_t* out);

/* BlobIndex: empty the in-HBM index (capacity_hint = expected entries, 0 = default). */
int bw_index_reset(bw_ctx* ctx, uint64_t capacity_hint);
/* BlobIndex::load: seed with prior backups' sorted digests (n x 32 bytes). */
int bw_index_seed(bw_ctx* ctx, const uint8_t* sorted_digests, uint64_t n);
/* n digests in canonical order: is_dup[i] = is_blob_duplicate(d_i) at its turn, and every
 * non-duplicate is then inserted (pack.rs:37 + blob_index.rs:109).  Host buffers. */
int bw_index_check_insert(bw_ctx* ctx, const uint8_t* digests, uint64_t n, uint8_t* is_dup);
/* number of distinct digests currently in the index */
int bw_index_size(bw_ctx* ctx, uint64_t* n);

/* Any index error is sticky until the next reset: BW_ENOSPC if an exchange bucket overflowed
 * (synchronizes; the device-side gate below does not check).  Distinct digests that share any
 * prefix are distinct entries: slots are compared by all 32 bytes, as the reference's HashSet and
 * binary search do (blob_index.rs:109,130-148). */
int bw_index_check(bw_ctx* ctx);

/* ---- one index shared by several contexts (one backup session, several batches in flight) ----
 * The reference keeps one BlobIndex behind the packer mutex (packfile/mod.rs:77, blob_index.rs:
 * 44-57) and every task of a backup gates against it.  A context owns a private index; attached
 * to a shared one, every index operation of every attached context (reset, seed, gate of a batch,
 * check_insert) is ordered on the GPU after the previous one, in the order the host issued them
 * (an event chain across the contexts' streams), so the batches of a session are gated in
 * submission order whichever stream runs them.  Index calls through different contexts may come
 * from different threads; each context itself stays single-threaded. */
typedef struct bw_index bw_index;
int bw_index_create(int device, bw_index** out);
/* Drops the caller's reference; the index lives on while contexts are attached to it. */
void bw_index_destroy(bw_index* index);
/* Gate this context's batches through `index` (NULL: back to the context's private index).
 * Waits for the context's pending work first. */
int bw_attach_index(bw_ctx* ctx, bw_index* index);

/* ---- context options ---- */
enum {
    /* Options 5, 6, 7, 10, 11 (value 2) and 14 (value 1) select variants measured slower than the
     * shipped kernels.  They are compiled only into the diagnostic build (BW_DIAG,
     * libbackuwup_amd_debug.so); the product library accepts them at the shipped value only and
     * returns BW_EINVAL otherwise. */
    BW_OPT_DEPTH = 1,            /* batches a context keeps addressable (result slots), 1..8; default 2 */
    BW_OPT_SCAN_SMALL_BYTES = 2, /* batches below this many bytes scan half-size tiles (default 4 GiB) */
    BW_OPT_CAND_CAP = 3,         /* test hook: fixed candidate array capacity (0 = sized per batch)  */
    BW_OPT_STAGE_CHUNK = 4,      /* pinned staging chunk for pageable bw_submit_host input (64 MiB)  */
    BW_OPT_B3_LOADS = 5,         /* BLAKE3 leaf pass loads: 0 = one block ahead, 1 = 132-byte block pairs,
                                    2 = aligned 128-byte lines through registers (k_b3_lines, default) */
    BW_OPT_SCAN_WAVES = 6,       /* gear-scan workgroup: 16 waves (default) or 8 (leaves LDS for BLAKE3) */
    BW_OPT_LATENCY_STREAM = 7,   /* 1: the small kernels between the passes on a high-priority stream */
    BW_OPT_ZSTD_SLOTS = 8,       /* bw_zstd_*: blobs compressed at once (16384); hash tables 768 KiB per blob,
                                    2.5 MiB per blob in sub-batches of at most 2,048 blobs */
    BW_OPT_ZSTD_BATCH_BYTES = 9, /* bw_zstd_*: input bytes per internal batch (~4.2x in scratch; 8 GiB) */
    BW_OPT_ORDER_HASH = 10,      /* 1: the scans and the BLAKE3 leaf passes of the contexts sharing an
                                    index run one at a time each, in submission order (a batch's scan
                                    then overlaps the previous batch's hashing); 0 (default): as soon
                                    as their inputs are ready */
    BW_OPT_SPLIT = 11,           /* 2: a batch of >= 2 files between 64 MiB and 4 GiB that gates
                                    through the index runs as two parts on two streams (head files
                                    here, tail files on a helper context), scans and BLAKE3 passes in
                                    order, meant to keep the scan beside the hashing with one batch
                                    in flight; 1 (default): off -- measured slower (the tail's scan
                                    waits for CUs held by the head's hashing).  bw_batch_views /
                                    bw_batch_device_views of a split batch return BW_ESTATE */
    BW_OPT_PROFILE_MASK = 12,    /* bw_profile_*: bit i = mark the start of stage i (BW_STAGE_*), bit
                                    BW_N_STAGES = the batch end; a stage's time runs to the next mark,
                                    the last mark closes the batch (at least two bits).  Default: all.
                                    Each mark costs the stream ~5 us of idle time */
    BW_OPT_SCAN_FIRST = 13,      /* when a batch's gear scan is enqueued: 1 = before the host builds
                                    and uploads the batch tables (the scan needs none of them), 0 =
                                    after the upload, 2 (default) = first for batches under
                                    BW_OPT_SCAN_SMALL_BYTES, where the host's share of a batch shows */
    BW_OPT_B3_UPPER = 14,        /* BLAKE3 levels above the 4-leaf groups: 0 (default) = a launch of
                                    their own after the leaf pass (k_b3_upper), 1 = inside the leaf pass
                                    (k_b3_lines; the wave that finishes a blob's last group builds them)
                                    -- measured 15-21 % slower on C1/C2/C4.  Only the aligned-line leaf
                                    pass (BW_OPT_B3_LOADS 2) fuses them */
    BW_OPT_B3_GROUP = 15         /* BLAKE3 leaves per lane of the aligned-line leaf pass: 4, 2 or 1, or
                                    0 (default) = 2 for batches under BW_OPT_SCAN_SMALL_BYTES or of
                                    small blobs, else 4.  Smaller groups cut the pass's last partial
                                    round of waves and ragged lanes (the levels above them move to the
                                    upper pass) */
};
int bw_set_option(bw_ctx* ctx, int option, uint64_t value);

/* Whole front end for a batch of files stored back to back in a host buffer: chunk -> hash
 * -> dedup; synchronous; results in canonical order.  Like every synchronous helper here
 * (bw_fastcdc_chunks, bw_blake3_hash(_many), bw_tree_blobs) it runs in a slot of its own outside
 * the ticket ring: it neither drops a batch the caller holds a ticket for nor changes which batch
 * bw_results / bw_batch_views(0) name.  A too-small cap gives BW_ENOSPC (call again). */
int bw_process_files(bw_ctx* ctx, const uint8_t* data, uint64_t data_len,
                     const uint64_t* file_off, const uint64_t* file_len, uint64_t n_files,
                     const bw_params* params, bw_blob* out, uint64_t cap, uint64_t* n_out);

/* ---- pipelined batches ----
 * A context holds the results of its last BW_OPT_DEPTH batches, each addressed by the ticket its
 * submit returned; submitting into a full ring drops the oldest batch (its ticket then gives
 * BW_ESTATE).  Batches of one context run one after another on its stream; batch k+1 can be
 * queued before batch k's results are read.  File tables are host arrays, copied at submit. */
/* Bytes already resident in HBM (d_data = device pointer, 16-byte aligned).  Asynchronous. */
int bw_submit_device(bw_ctx* ctx, const uint8_t* d_data, uint64_t data_len, const uint64_t* file_off,
                     const uint64_t* file_len, uint64_t n_files, const bw_params* params, uint64_t* ticket);
/* Bytes in host memory (the mmap'd files of dir_packer.rs:247-266, gathered back to back).  The
 * batch is copied to HBM on the context's copy stream while earlier batches compute: pinned or
 * bw_host_register'ed memory by DMA straight from `data`; pageable memory through a ring of
 * pinned staging chunks (the call returns once every byte is staged).  `data` must stay
 * unchanged until the call returns (pageable) or until bw_wait(ticket) returns (pinned). */
int bw_submit_host(bw_ctx* ctx, const uint8_t* data, uint64_t data_len, const uint64_t* file_off,
                   const uint64_t* file_len, uint64_t n_files, const bw_params* params, uint64_t* ticket);
/* Wait for batch `ticket` and copy its blobs out (repeatable while the ticket is held). */
int bw_wait(bw_ctx* ctx, uint64_t ticket, bw_blob* out, uint64_t cap, uint64_t* n_out);
/* Page-lock a host range (e.g. an mmap'd file) so bw_submit_host DMAs it without staging. */
int bw_host_register(void* ptr, uint64_t len);
int bw_host_unregister(void* ptr);

/* bw_submit_device without a ticket (results via bw_results). */
int bw_process_files_device(bw_ctx* ctx, const uint8_t* d_data, uint64_t data_len,
                            const uint64_t* file_off, const uint64_t* file_len, uint64_t n_files,
                            const bw_params* params);
/* Wait for the most recently submitted batch and copy its blobs out. */
int bw_results(bw_ctx* ctx, bw_blob* out, uint64_t cap, uint64_t* n_out);
/* Device views of the most recent batch (valid until the ring reuses its slot): n blobs
 * (synchronizes), digests (n x 32 B, canonical order) and is_dup bytes. */
int bw_batch_device_views(bw_ctx* ctx, uint64_t* n_blobs, const uint8_t** d_digests,
                          uint8_t** d_is_dup);

/* ---- multi-GPU digest exchange (index partitioned by digest prefix, RCCL all-to-all) ----
 * owner(d) = d[0] >> (8 - log2(n_owners)), n_owners a power of two <= 256.
 * Stable partition of n device digests by owner: d_out (n x 32 B, grouped by owner, canonical
 * order kept inside each group), d_perm[n] = source index of each output digest,
 * h_counts[n_owners] (host) = digests per owner.  Synchronizes (the counts size the exchange). */
int bw_partition_by_owner(bw_ctx* ctx, const uint8_t* d_digests, uint64_t n, uint32_t n_owners,
                          uint8_t* d_out, uint64_t* d_perm, uint64_t* h_counts);
/* Owner side: n device digests in canonical order (an all-to-all output is source-rank-major,
 * which is canonical when files are sharded rank-major) -> d_is_dup[n] (device). */
int bw_index_check_insert_device(bw_ctx* ctx, const uint8_t* d_digests, uint64_t n,
                                 uint8_t* d_is_dup);
/* Scatter owner verdicts back to source order: d_is_dup[d_perm[i]] = d_verdict[i]. */
int bw_scatter_verdicts(bw_ctx* ctx, const uint8_t* d_verdict, const uint64_t* d_perm,
                        uint64_t n, uint8_t* d_is_dup);

/* Building blocks of a fixed-capacity exchange (round 3; bw_exchange_dedup below no longer uses
 * them): every rank sends every owner a bucket of `cap` digest slots, so the all-to-alls have equal
 * splits and the counts stay on the device; a batch with more digests for one owner than cap sets
 * a sticky error that bw_index_check reports as BW_ENOSPC.
 * Device views of batch `ticket` (0 = the most recent), no synchronization: d_n_blobs points at
 * the batch's blob count in HBM; *max_blobs = its host-side upper bound.  The verdicts of an
 * exchanged batch are final once bw_wait(ticket) returned. */
int bw_batch_views(bw_ctx* ctx, uint64_t ticket, const uint64_t** d_n_blobs, const uint8_t** d_digests,
                   uint8_t** d_is_dup, uint64_t* max_blobs);
/* d_buckets[n_owners][cap][32] = digests by owner, canonical order inside each bucket;
 * d_perm[n_owners][cap] = source index; d_counts[n_owners] (device u64).  n = *d_n (device),
 * max_n its host bound. */
int bw_partition_buckets(bw_ctx* ctx, const uint8_t* d_digests, const uint64_t* d_n, uint64_t max_n, uint64_t cap,
                         uint32_t n_owners, uint8_t* d_buckets, uint64_t* d_perm, uint64_t* d_counts);
/* Owner: gate the received buckets (n_src x cap, counts d_counts[n_src] on the device) in
 * source-major order; d_verdicts in the same bucket layout. */
int bw_index_check_insert_buckets(bw_ctx* ctx, const uint8_t* d_buckets, const uint64_t* d_counts, uint32_t n_src,
                                  uint64_t cap, uint8_t* d_verdicts);
/* Source: d_is_dup[d_perm[o][i]] = d_verdicts[o][i] for i < d_counts[o]. */
int bw_scatter_buckets(bw_ctx* ctx, const uint8_t* d_verdicts, const uint64_t* d_perm, const uint64_t* d_counts,
                       uint32_t n_owners, uint64_t cap, uint8_t* d_is_dup);

/* ---- multi-GPU dedup behind one call per batch (RCCL over xGMI) ----
 * The index partitioned by digest prefix across the ranks of a node replaces the one BlobIndex
 * behind the packer mutex (packfile/mod.rs:77, blob_index.rs:130-148, pack.rs:37).  Every rank
 * keeps its shard in its own context's index (or a bw_index its contexts share), submits its
 * batches with BW_F_NO_DEDUP, and then calls bw_exchange_dedup once per batch, in the same batch
 * order on every rank.  Files are sharded rank-major (rank r's batch k holds canonical files
 * before rank r+1's batch k), so the owner gates the received digests in canonical order.
 * A communicator moves bytes between the ranks, either
 *   - over RCCL: rank 0 draws an id with bw_comm_unique_id, the caller hands those 128 bytes to
 *     every rank (any channel), and each rank calls bw_comm_init (blocks until all joined); or
 *   - through the caller's own host transport (bw_comm_init_host): fn(user, send, recv, bytes)
 *     must deliver send[r * bytes ..] to rank r's recv[my_rank * bytes ..] for every rank r
 *     (equal splits: the library pads every rank's sections to the largest one); buffers are
 *     pinned host memory, world * bytes long; nonzero return = failure. */
#define BW_COMM_ID_BYTES 128u
typedef struct bw_comm bw_comm;
typedef int (*bw_host_all_to_all)(void* user, const void* send, void* recv, uint64_t bytes_per_rank);
int bw_comm_unique_id(uint8_t id[BW_COMM_ID_BYTES]);
/* world: a power of two <= 256; device must be the device of the contexts it serves.
 * Every wait on the peers has a deadline (the reference's transport sends with timeouts,
 * net_p2p/transport.rs:127-128): initialisation, each collective's enqueue, the arrival of an
 * exchange's counts (counted from its bw_exchange_dedup) and bw_wait of an exchanged batch.  On an RCCL error or a missed deadline the
 * communicator is aborted (ncclCommAbort), the call returns BW_ECOMM, and so does every later
 * call on it; bw_comm_destroy then only releases it.  bw_comm_init uses the default deadline. */
#define BW_COMM_DEFAULT_TIMEOUT_MS 120000u
int bw_comm_init(int device, int rank, int world, const uint8_t id[BW_COMM_ID_BYTES], bw_comm** out);
int bw_comm_init_timeout(int device, int rank, int world, const uint8_t id[BW_COMM_ID_BYTES], uint32_t timeout_ms,
                         bw_comm** out);
int bw_comm_set_timeout(bw_comm* comm, uint32_t timeout_ms);
/* BW_OK, or BW_ECOMM once the communicator was aborted (a peer failed or stalled). */
int bw_comm_status(const bw_comm* comm);
int bw_comm_init_host(int device, int rank, int world, bw_host_all_to_all fn, void* user, bw_comm** out);
/* The N ranks of ONE process (the reference packs a backup in one process, backup/mod.rs:64):
 * out[0..n) get ranks 0..n-1 on devices[r] (a device may repeat).  The ranks are driven from n
 * threads, one per rank, each calling bw_exchange_dedup with its own context and out[r] in the
 * same batch order (INTEGRATION.md "One process, every GPU").
 *   bw_comm_init_all:   RCCL over xGMI (draws the id and initialises the n ranks concurrently;
 *                       RCCL refuses two ranks on one device);
 *   bw_comm_init_local: an in-process host transport (threads exchange through host memory; any
 *                       devices, the same device for several ranks included).
 * On failure every communicator created is destroyed and out[] is NULL. */
int bw_comm_init_all(const int* devices, int n, uint32_t timeout_ms, bw_comm** out);
int bw_comm_init_local(const int* devices, int n, bw_comm** out);
void bw_comm_destroy(bw_comm* comm);
const char* bw_comm_last_error(const bw_comm* comm);
/* Obsolete since round 5 (accepted and ignored): every transfer of bw_exchange_dedup is sized
 * exactly from the counts the exchange carries, so there is no bucket capacity to fix or agree. */
int bw_comm_set_capacity(bw_comm* comm, uint64_t cap);
/* Batch `ticket` of ctx (0 = the most recent; submitted with BW_F_NO_DEDUP, hashed and not split,
 * else BW_ESTATE) through the exchange: its digests are grouped by owner = digest[0] >> (8 - log2
 * world), and the per-owner counts go to every rank (16 bytes per rank, on a control communicator
 * split off at bw_comm_init and a stream of its own).  The call returns without waiting for any
 * peer.  Once the counts have arrived -- noticed by any later call on the communicator (the next
 * bw_exchange_dedup, bw_comm_progress, bw_wait of an exchanged batch, a submit that reuses its
 * slot) -- the digests travel to their owners (each transfer exactly its digests), the owner gates
 * them against ctx's index in source-rank order (canonical when files are sharded rank-major), and
 * the verdicts come back into the batch's is_dup and records (bw_wait).  Exchanges finish in the
 * order they were issued; every rank calls this for its k-th batch in the same order, and the
 * contexts sharing a communicator are driven from one thread.  The host transport runs the whole
 * exchange inside the call (its all-to-all is synchronous). */
int bw_exchange_dedup(bw_ctx* ctx, bw_comm* comm, uint64_t ticket);
/* Finish the queued exchanges whose counts have arrived (never waits).  BW_ECOMM once aborted. */
int bw_comm_progress(bw_comm* comm);

/* ---- one long file split across the ranks (SURVEY.md §8e "single long stream") ----
 * The reference chunks a file serially from its start (a new FastCDC per file, dir_packer.rs:254-266);
 * here the W ranks of a communicator chunk one file together.  Rank r owns the file bytes [S_r,
 * S_{r+1}), S_k = file_len * k / W, and holds its window [lo, hi) (bw_stream_window: the owned range
 * widened by max_size on both sides, clipped to the file) in HBM.  bw_chunk_stream_shard chunks and
 * hashes the window from a speculative start and settles with the other ranks (rounds of a 16-byte
 * allgather on the communicator's control communicator; random data settles in one round, data with
 * no content-defined cut in at most W + 1) where each rank's true chain enters: the chunks every rank
 * emits are, in rank order, exactly FastCDC::new(file, min, avg, max)'s chunks (boundaries, Chunk.hash
 * and digests), the chunk straddling a split hashed once, by the rank after it.
 * out->ticket names the batch (in ctx's ring, submitted with BW_F_NO_DEDUP) that holds this rank's
 * final chain: bw_wait(ticket) returns the chain's blobs with offsets relative to out->chain_start,
 * of which [first_blob, first_blob + n_blobs) are the ones this rank emits; bw_exchange_dedup(ctx,
 * comm, ticket) sends only those to their owners.  d_window = file byte lo in device memory, any
 * alignment (the library may read up to 15 bytes before it, inside its 16-byte granule).  Every rank
 * calls it for the same file at the same point in its sequence of calls on the communicator; it
 * returns once the ranks settled (host-synchronous, deadline-bounded like every wait on peers).
 * min_size > max_size (legal in the crate, whose cut() then returns a remainder <= min whole, longer
 * than max) is refused with BW_EINVAL: the windows rest on every chunk being <= max. */
typedef struct bw_stream_shard {
    uint64_t ticket;      /* batch holding this rank's final chain                             */
    uint64_t first_blob;  /* the chunks this rank emits: blobs [first_blob, first_blob + n_blobs) */
    uint64_t n_blobs;
    uint64_t chain_start; /* file offset where the chain starts (its blobs' offsets count from it) */
    uint32_t rounds;      /* settlement rounds                                                  */
    uint32_t pad;
} bw_stream_shard;
int bw_stream_window(uint64_t file_len, int rank, int world, uint32_t max_size, uint64_t* lo, uint64_t* hi);
int bw_chunk_stream_shard(bw_ctx* ctx, bw_comm* comm, const uint8_t* d_window, uint64_t file_len,
                          const bw_params* params, bw_stream_shard* out);

/* ---- tree blobs: split_serialize_tree + add_tree_to_blobs, dir_packer.rs:314-390 ----
 * Tree { kind: TreeKind, name: String, metadata: TreeMetadata { size, mtime, ctime: Option<u64> },
 *        children: Vec<BlobHash>, next_sibling: Option<BlobHash> }   (filesystem/mod.rs:63-77)
 * serialized with bincode 1.3.3 `bincode::serialize` (fixint, little endian). */
#define BW_TREE_FILE 0u /* TreeKind::File */
#define BW_TREE_DIR 1u  /* TreeKind::Dir  */
#define BW_TREE_HAS_SIZE 1u
#define BW_TREE_HAS_MTIME 2u
#define BW_TREE_HAS_CTIME 4u
#define BW_TREE_BLOB_MAX_CHILDREN 10000u /* dir_packer.rs:35 */

typedef struct bw_tree {
    uint32_t kind;            /* BW_TREE_FILE or BW_TREE_DIR                               */
    uint32_t flags;           /* BW_TREE_HAS_*: which metadata options are Some            */
    uint64_t size, mtime, ctime;
    const uint8_t* name;      /* UTF-8 bytes (the reference's to_string_lossy), no NUL     */
    uint64_t name_len;
    const uint8_t* children;  /* n_children x 32-byte BlobHash, in the parent's order      */
    uint64_t n_children;
} bw_tree;

/* One tree blob (a piece of a split tree), canonical order: trees as given, pieces in order. */
typedef struct bw_tree_blob {
    uint64_t tree;      /* index of the tree                                 */
    uint64_t piece;     /* 0 = the blob whose hash represents the tree        */
    uint64_t length;    /* serialized bytes                                  */
    uint8_t hash[32];   /* blake3 of the serialized piece                     */
    uint8_t is_dup;     /* Manager::add_blob returns Ok(None)                 */
    uint8_t pad[7];
} bw_tree_blob;

/* bincode of one Tree (no splitting); next_sibling NULL = None.  Host only.  BW_ENOSPC with the
 * required size in *n_out when cap is too small. */
int bw_tree_serialize(const bw_tree* tree, const uint8_t* next_sibling, uint8_t* out, uint64_t cap,
                      uint64_t* n_out);
/* n trees: split (> 10,000 children), serialize, BLAKE3 every piece on the GPU (the last pieces
 * first, each earlier piece with its successor's hash as next_sibling), then the dedup gate over
 * all pieces in canonical order (skipped with BW_F_NO_DEDUP in flags).  tree_hashes[32*i] = the
 * tree's hash (its first piece).  out (may be NULL) receives every piece; *n_out = pieces.
 * Synchronous; runs in the context's own helper slot, so batches held by ticket stay readable. */
int bw_tree_blobs(bw_ctx* ctx, const bw_tree* trees, uint64_t n, uint32_t flags, uint8_t* tree_hashes,
                  bw_tree_blob* out, uint64_t cap, uint64_t* n_out);

/* ---- stage timing (HIP events on the context stream, accumulated over profiled batches) ---- */
enum {
    BW_STAGE_SCAN = 0,     /* gear candidate scan (k_scan)                                 */
    BW_STAGE_COMPACT = 1,  /* candidate compaction                                          */
    BW_STAGE_RESOLVE = 2,  /* speculative chains + merge resolution + serial walker         */
    BW_STAGE_ASSEMBLE = 3, /* blob table + Chunk.hash                                       */
    BW_STAGE_B3LEAF = 4,   /* BLAKE3 4-leaf groups (k_b3_groups)                            */
    BW_STAGE_B3TREE = 5,   /* BLAKE3 upper tree levels (k_b3_tree)                          */
    BW_STAGE_DEDUP = 6,    /* index append/claim/verdict                                    */
    BW_STAGE_PACK = 7,     /* result records                                                */
    BW_N_STAGES = 8
};
int bw_profile_enable(bw_ctx* ctx, int on); /* also clears the accumulators */
/* stage_ms[BW_N_STAGES] = summed milliseconds; *n_batches = batches accumulated.  Syncs. */
int bw_profile_read(bw_ctx* ctx, double* stage_ms, uint64_t* n_batches);
/* The profiled batches' intervals of one stage, out[2k] = start, out[2k+1] = end, in ms on the
 * device's timeline (every context of a device shares its origin, so a caller can take the union
 * of a stage over contexts).  *n = intervals; BW_ENOSPC if cap < *n.  Syncs. */
int bw_profile_intervals(bw_ctx* ctx, int stage, double* out, uint64_t cap, uint64_t* n);

/* ---- roofline calibration (diagnostic; replaces no reference call, touches no batch state) ----
 * The BLAKE3 leaf pass's compression run from registers (no memory traffic) on every CU at the
 * leaf pass's occupancy, for about `ms` milliseconds on the context stream: the integer-issue
 * ceiling of that pass measured on the running chip.  out[0] = GB/s of message compressed,
 * out[1] = mean shader clock over the run in GHz, out[2] = bytes per shader clock per CU,
 * out[3] = the measured launch's milliseconds.  Synchronous. */
int bw_calibrate_b3(bw_ctx* ctx, double ms, double out[4]);

#ifdef __cplusplus
}
#endif
/* the write side after the hot path: sealing, zstd, packfiles, index files */
#include "backuwup_gpu_pack.h"

#endif /* BACKUWUP_GPU_H */
