// bw_internal.h -- host-side declarations shared by the backuwup_amd translation units.
#pragma once
#include <algorithm>
#include <string>
#include <thread>
#include <vector>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/backuwup_gpu.h"

// BW_DIAG: compile the variants measured slower than the shipped path (the 8-wave scan, the
// prefetch / block-pair leaf loaders, the upper levels fused into the leaf pass, the split batch,
// serialized passes, the latency stream).  Only the diagnostic build defines it
// (libbackuwup_amd_debug.so, with BW_DEBUG); the product library holds one scan kernel per tile
// size, one leaf kernel and one upper-level kernel.
#ifndef BW_DIAG
#define BW_DIAG 0
#endif

namespace bw {

// ------------------------------------------------------------------ tunables
constexpr int SCAN_BLOCK = 1024;                                   // 16 waves, 1 block per CU (LDS)
#ifndef BW_SCAN_STRIP
#define BW_SCAN_STRIP 2048
#endif
#ifndef BW_SCAN_CAP
#define BW_SCAN_CAP 16
#endif
constexpr int SCAN_STRIP = BW_SCAN_STRIP;                          // bytes per lane
constexpr uint64_t SCAN_TILE = 64ull * SCAN_STRIP;                 // one wave's sub-tile (128 KiB)
constexpr int SCAN_STRIP_SMALL = SCAN_STRIP / 2;                   // batches below SCAN_SMALL_BYTES
constexpr uint64_t SCAN_SMALL_BYTES = 4ull << 30;                  // (one tile per wave otherwise: slow)
constexpr uint32_t SCAN_TILE_SHIFT = __builtin_ctzll(SCAN_TILE);
constexpr int SCAN_CAP = BW_SCAN_CAP;                              // candidate slots per tile
constexpr int SCAN_STEP = 64;                                      // bytes per lane per staged step
constexpr int STAGE_ROW = SCAN_STEP + 16;                          // padded LDS staging row
constexpr int GEAR_REP = 32;                                      // LDS gear replicas
constexpr int CHAIN_CAP = 128;                                    // cuts stored per segment

// device counter slots (uint64 each)
enum Ctr : int {
    C_NCAND = 0,     // gear candidates stored (clamped to the candidate array capacity)
    C_NOVF = 1,      // tiles whose candidates overflowed SCAN_CAP
    C_NBLOBS = 2,    // blobs produced by the batch
    C_NGROUPS = 3,   // BLAKE3 4-leaf groups
    C_SEQBASE = 4,   // dedup log position of the batch's first blob
    C_LOST = 5,      // a gated digest found no table slot (internal error; the table is kept half empty)
    C_NINVALID = 6,  // files that needed the serial boundary walker
    C_NUNIQUE = 7,   // distinct digests in the index
    C_CANDTOTAL = 8, // gear candidates found (> C_NCAND: the array was too small, see C_TRUNC)
    C_DEDUPN = 9,    // blobs handed to the index
    C_TRUNC = 10,    // first byte position whose candidates did not fit the array (BW_NONE: all fit);
                     // the walkers scan the bytes themselves from there on
    // the index's state right after the batch's gate (snapshot by k_pack / k_index_snapshot), read
    // back with the staged results: C_LOST, C_NUNIQUE and these
    C_IX_OVF = 11,    // an exchange bucket overflowed (D_BUCKET_OVF)
    C_IX_LOGLEN = 12, // log length (D_LOGLEN)
    C_IX_VALID = 13,  // 1 = the snapshot was taken
    C_DONE_TILES = 14, // blocks of the tile-count scan that finished (its last block scans the totals)
    C_DONE_UNITS = 15, // blocks of the unit-count scan that finished (likewise)
    C_COUNT = 16
};
static_assert(SCAN_STRIP_SMALL % (4 * SCAN_STEP) == 0, "k_scan consumes four 64-byte steps per iteration");
static_assert(SCAN_STRIP % (4 * SCAN_STEP) == 0, "k_scan consumes four 64-byte steps per iteration");

struct Masks {
    uint32_t min, avg, max, s0;  // s0 = 2 * (min / 2): first position the crate hashes
    uint64_t mask_s, mask_l, mask_pre;  // mask_pre = mask_s & mask_l (scan prefilter)
    uint32_t pre_shift;  // the scan carries h << pre_shift; 63 - top bit of (mask_s | mask_l)
    uint32_t pre_hi;     // bits of mask_pre inside the high dword of h << pre_shift
    uint32_t tile_shift; // log2 of the scan tile in bytes (SCAN_TILE, or half of it for small batches)
};

// One boundary-resolution segment: a window [start, end) of one CDC file.
struct SegDesc {
    uint64_t start, end, file_end;
    uint32_t cfile;  // index among the batch's CDC files
    uint32_t last;   // 1 = last segment of its file
};

struct CFileDesc {
    uint64_t start, end;  // global byte range of the file
    uint64_t fb_off;      // offset into the serial-walker output buffer
    uint32_t first_seg, nseg;
};

// Canonical-order unit: either a whole small file (kind 0) or one CDC segment (kind 1).
struct UnitDesc {
    uint64_t start, len;  // small file: its range; segment: unused
    uint32_t file;        // batch file index
    uint32_t kind;        // 0 = small-file blob, 1 = CDC segment
    uint32_t seg;         // segment index (kind 1)
    uint32_t cfile;       // CDC file index (kind 1)
};

// Blob table (struct of arrays), canonical order.
struct BlobArrays {
    uint64_t* start;  // global byte position
    uint64_t* len;
    uint64_t* goff;   // first BLAKE3 group
    uint32_t* file;
    uint32_t* kind;   // 0 = whole-file blob, 1 = CDC chunk
    uint64_t* fend;   // end of the owning file (for Chunk.hash of CDC chunks)
    uint64_t* ghash;  // Chunk.hash
    uint64_t cap;       // entries the arrays hold (BW_DEBUG checks)
    uint64_t data_len;  // bytes of the batch buffer (BW_DEBUG checks)
    uint32_t* gdone = nullptr;  // per blob: BLAKE3 groups finished (zero between passes); null = the
                                // upper levels run as a launch of their own (k_b3_upper)
    uint32_t gshift = 2;        // log2 of the leaves per BLAKE3 group (k_b3_lines: 0..2; others: 2)
};

// ------------------------------------------------------------------ launchers (bw_cdc.hip)
// returns false (nothing launched) when mk.tile_shift names no compiled tile size
bool launch_scan(hipStream_t st, const uint8_t* data, uint64_t n_bytes, uint64_t n_tiles,
                 const Masks& mk, uint32_t* tile_count, uint64_t* tile_slots, uint32_t* ovf_list,
                 uint64_t* ctr, int waves /* 16 or 8 per block */);
void launch_compact(hipStream_t st, const uint8_t* data, uint64_t n_bytes, uint64_t n_tiles,
                    const Masks& mk, uint32_t* tile_count, uint64_t* tile_slots,
                    uint64_t* tile_off, uint64_t* cand, uint64_t cand_cap, uint32_t* ovf_list,
                    uint64_t* ctr, uint64_t* scratch /* >= n_tiles / 1024 + 1 entries */);
void launch_chains(hipStream_t st, const uint8_t* data, uint64_t data_len, const Masks& mk, const uint64_t* cand,
                   const uint64_t* tile_off, uint64_t* ctr, const SegDesc* segs, uint64_t nseg,
                   uint64_t* chains, uint32_t* chain_n, uint64_t* chain_cptr, uint64_t* merge,
                   int force_serial);
void launch_resolve(hipStream_t st, const uint8_t* data, uint64_t data_len, const Masks& mk, const uint64_t* cand,
                    const uint64_t* tile_off, uint64_t* ctr, const SegDesc* segs, uint64_t nseg,
                    const CFileDesc* cfiles, uint64_t ncf, const uint64_t* chains,
                    const uint32_t* chain_n, const uint64_t* merge, uint64_t* seg_M,
                    uint32_t* seg_cnt, uint32_t* cf_invalid, uint64_t* fb_starts,
                    uint64_t* fb_count, int force_serial);
void launch_assemble(hipStream_t st, uint64_t* ctr, const UnitDesc* units, uint64_t nunits,
                     const SegDesc* segs, const CFileDesc* cfiles, const uint64_t* chains,
                     const uint32_t* chain_n, const uint64_t* seg_M, const uint32_t* cf_invalid,
                     const uint64_t* fb_starts, const uint64_t* fb_count, BlobArrays b,
                     uint64_t* ucnt /* 2 * nunits */, uint64_t* ubtot /* 2 * (nunits / 256 + 2) */);
// bytes (rounded up to 16) from device-accessible pinned host memory into HBM, by a kernel on st
void launch_upload(hipStream_t st, const void* host_src, void* dst, uint64_t bytes);
void launch_zero(hipStream_t st, uint64_t* p, uint32_t n);  // n u64 (<= a few hundred) to 0
void launch_cut_hash(hipStream_t st, const uint8_t* data, const Masks& mk, const uint64_t* ctr,
                     BlobArrays b, uint64_t max_blobs);


// ------------------------------------------------------------------ launchers (bw_blake3.hip)
// how the leaf pass feeds its compressions: one 64-byte block ahead (prefetch), block pairs, or
// whole aligned 128-byte lines through a register ring (k_b3_lines)
enum { B3_LOADS_PREFETCH = 0, B3_LOADS_PAIRS = 1, B3_LOADS_LINES = 2 };
void launch_blake3(hipStream_t st, const uint8_t* data, const uint64_t* ctr, BlobArrays b,
                   uint64_t max_blobs, uint64_t max_groups, uint32_t* cv_buf,
                   uint32_t* cv_tmp /* like cv_buf */, uint8_t* digests, int max_leaves,
                   hipEvent_t between /* may be null */, int loads,
                   hipStream_t upper /* stream of the upper tree levels; `between` must order it */,
                   hipEvent_t leaf_done = nullptr /* recorded on st right after the leaf pass */,
                   hipEvent_t mark = nullptr /* a timing mark, likewise */);
// The leaf pass's compression from registers (roofline calibration): n_blocks blocks of 256,
// stamps[2 * block] = shader cycles, stamps[2 * block + 1] = 100 MHz ticks of wave 0.
void launch_b3_calib(hipStream_t st, uint32_t n_blocks, uint32_t blocks_per_lane, uint32_t* sink, uint64_t* stamps);
uint32_t b3_calib_blocks_per_cu();  // the leaf pass's occupancy (blocks of 256 per CU)
// ------------------------------------------------------------------ launchers (bw_dedup.hip)
// Dedup state (device, persistent across batches): st[0] = log length (next seq),
// st[1] = distinct digests, st[2] = a digest found no slot (internal error; never set while the
// table is kept at most half full).
// st[3] = an exchange bucket overflowed (a batch had more blobs than the agreed capacity).
// st[4] = blocks of the running gate's verdict pass that finished (its last block advances st[0]).
enum DState : int { D_LOGLEN = 0, D_NUNIQUE = 1, D_LOST = 2, D_BUCKET_OVF = 3, D_DONE = 4, D_COUNT = 5 };
void launch_table_clear(hipStream_t st, uint64_t* table, uint64_t cap);
// Append n digests (n from *n_dev if non-null, else n_host) to the log and decide them in
// order: is_dup[i] (may be null) = digest seen at an earlier log position.
void launch_dedup(hipStream_t st, uint64_t* table, uint64_t cap, uint8_t* log, uint64_t* dstate,
                  const uint8_t* digests, const uint64_t* n_dev, uint64_t n_host, uint64_t max_n,
                  uint8_t* is_dup);
// Re-claim log[0 .. *len) into a fresh table (growth).  The table holds one u64 per slot.
void launch_rehash(hipStream_t st, uint64_t* table, uint64_t cap, const uint8_t* log,
                   const uint64_t* dstate, uint64_t max_n);
void launch_partition(hipStream_t st, const uint8_t* digests, uint64_t n, uint32_t n_owners,
                      uint8_t* out, uint64_t* perm, uint64_t* counts_dev);
void launch_scatter(hipStream_t st, const uint8_t* verdict, const uint64_t* perm, uint64_t n,
                    uint8_t* is_dup);
// fixed-capacity owner buckets (multi-GPU exchange without host round trips); blk holds
// ceil(max_n / 4096) * n_owners u64, err is set when a bucket would exceed cap
void launch_bucket_partition(hipStream_t st, const uint8_t* digests, const uint64_t* n_dev, uint64_t max_n,
                             uint32_t n_owners, uint64_t cap, uint8_t* out, uint64_t* perm, uint64_t* counts,
                             uint64_t* blk, uint64_t* err);
void launch_bucket_gather(hipStream_t st, const uint8_t* buckets, const uint64_t* counts, uint32_t n_src, uint64_t cap,
                          uint8_t* out, uint64_t* n_out);
void launch_bucket_expand(hipStream_t st, const uint64_t* counts, uint32_t n_src, uint64_t cap, const uint8_t* v_in,
                          uint8_t* v_out);
// packed (may be null): the batch's bw_blob records, whose is_dup byte is written as well
void launch_bucket_scatter(hipStream_t st, const uint8_t* verdict, const uint64_t* perm, const uint64_t* counts,
                           uint32_t n_owners, uint64_t cap, uint8_t* is_dup, uint8_t* packed = nullptr);
// dstate (may be null): the index state snapshot into ctr[C_LOST, C_NUNIQUE, C_IX_*]
// host (may be null): pinned memory that also receives ctr and the first host_n records
void launch_pack(hipStream_t st, uint64_t* ctr, BlobArrays b, const uint64_t* file_start,
                 const uint8_t* digests, const uint8_t* is_dup, uint8_t* out, uint64_t max_blobs,
                 const uint64_t* dstate, uint8_t* host = nullptr, uint64_t host_n = 0);
void launch_index_snapshot(hipStream_t st, const uint64_t* dstate, uint64_t* ctr);
// bw_exchange_dedup: the batch's digests grouped by owner back to back (out, perm: n_max entries),
// msg[2o] = digests for owner o, msg[2o + 1] = the largest section; blk as for the buckets
void launch_owner_partition(hipStream_t st, const uint8_t* digests, const uint64_t* n_dev, uint64_t max_n,
                            uint32_t n_owners, uint8_t* out, uint64_t* perm, uint64_t* msg, uint64_t* blk);
// n u64 from device memory into device-accessible pinned host memory, by a kernel on st
void launch_copy_u64(hipStream_t st, const uint64_t* src, uint64_t* dst, uint32_t n);
// is_dup[perm[i]] = verdict[i] (and the records' is_dup byte, packed may be null), i < n
void launch_owner_scatter(hipStream_t st, const uint8_t* verdict, const uint64_t* perm, uint64_t n, uint8_t* is_dup,
                          uint8_t* packed);

// ------------------------------------------------------------------ sealing (bw_seal.hip)
// BW_SEAL_MAX_INFO (include/backuwup_gpu.h): HKDF info bytes that fit one HMAC block with 0x01 + padding
constexpr uint32_t PIECE_BLOCKS = 8192;  // 16-byte blocks per k_seal_ctr wave task (128 KiB)
constexpr int SEAL_THREADS = 1024;       // 16 waves: one LDS set per CU

struct SealItem {
    uint64_t src_off, len, dst_off, piece0;  // len = plaintext bytes; piece0 = first piece
    uint32_t nonce[3];                       // big-endian words of the 12-byte nonce
    uint32_t info_len;
    uint8_t info[56];
    uint32_t raw_len, wd;  // store-framed items: the plaintext is the zstd store frame of raw_len
                           // source bytes with window descriptor wd (launch_seal(framed = true))
};

struct SealKey {
    uint32_t rk[60];   // AES-256 round keys, big-endian words
    uint32_t H[4], E0[4], HP[4], H64[4];  // E(0), E(J0), H^PIECE_BLOCKS, H^64
    uint32_t P[6][4];  // H^(2^k), k = 0..5
    uint32_t R1[4];    // AES round 1 minus its counter-word terms (the nonce words are constant)
};

struct SealPads {
    uint32_t istate[8], ostate[8];  // SHA-256 states after the HMAC key ^ ipad / ^ opad blocks
};
void seal_pads(const uint8_t prk[32], SealPads* pads);
uint64_t seal_pieces(uint64_t len);  // k_seal_ctr wave tasks of an item of len bytes
void seal_fill_item(SealItem* it, uint64_t src_off, uint64_t len, uint64_t dst_off, uint64_t piece0,
                    const uint8_t nonce[12], const uint8_t* info, uint32_t info_len);
// dec = false: dst = ciphertext || tag; dec = true: dst = plaintext, ok[i] = tag verified
// framed (sealing only): item plaintexts are zstd store frames built on the fly from the source
void launch_seal(hipStream_t st, bool dec, bool framed, const uint8_t* src, uint8_t* dst, const SealItem* items,
                 uint64_t n, const SealPads& pads, SealKey* keys, uint64_t n_pieces, uint32_t* parts, uint8_t* ok);
uint32_t zstd_window_descriptor(uint64_t raw_len);

// ------------------------------------------------------------------ host helpers
// fn(lo, hi) over [0, n) on up to 16 threads: the host-side table work of million-item batches
// (16 = this GPU's share of the box's cores).  `work` (default n) sizes the thread count; small
// work runs inline.
template <typename F>
void parallel_ranges(uint64_t n, F fn, uint64_t work = 0) {
    if (!work) work = n;
    const uint64_t hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    const uint64_t t = work < 65536 ? 1 : std::min<uint64_t>(std::min<uint64_t>(hw, work / 32768), n);
    if (t <= 1) {
        fn(0, n);
        return;
    }
    std::vector<std::thread> th;
    for (uint64_t k = 0; k < t; k++) th.emplace_back(fn, n * k / t, n * (k + 1) / t);
    for (auto& x : th) x.join();
}

// ------------------------------------------------------------------ many small messages (bw_capi.hip)
int ctx_device(const bw_ctx* c);
// the blobs of batch `ticket` that bw_exchange_dedup sends to their owners: [first, first + n)
// (default: all of them); bw_chunk_stream_shard's rank keeps only the chunks it owns
int batch_set_exchange_range(bw_ctx* c, uint64_t ticket, uint64_t first, uint64_t n);
// Pinned host staging owned by the context (valid until the next call that uses it).
uint8_t* message_stage(bw_ctx* c, size_t bytes);
// BLAKE3 of n whole messages lying in `staged` (from message_stage) at offs/lens, in one batch;
// with dedup the digests go through the index in order (add_blob's gate) and dup[i] is the
// verdict.  Synchronous; hashes (n x 32) and dup are host arrays.
int hash_messages(bw_ctx* c, const uint8_t* staged, uint64_t total, const uint64_t* offs, const uint64_t* lens,
                  uint64_t n, bool dedup, uint8_t* hashes, uint8_t* dup);

// ------------------------------------------------------------------ exchange transport (bw_comm.hip)
int comm_rank(const bw_comm* c);
int comm_world(const bw_comm* c);
int comm_device(const bw_comm* c);
bool comm_failed(const bw_comm* c);
void*& comm_exq(bw_comm* c);  // the exchanges waiting for their counts (owned by bw_capi.hip)
uint64_t comm_now_ns();
// wait for ev (after work that includes the communicator's collectives) to the communicator's
// deadline, polling RCCL's async errors; aborts the communicator on error or timeout (BW_ECOMM)
int comm_wait_event(bw_comm* c, hipEvent_t ev, std::string& err);
// one non-blocking look at ev (enqueued at since_ns): *ready, or BW_ECOMM past the deadline
int comm_poll(bw_comm* c, hipEvent_t ev, uint64_t since_ns, bool* ready, std::string& err);
// the exchange's counts, 16 B per rank: d_recv[2k, 2k + 1] = rank k's d_send[2r, 2r + 1].  RCCL:
// enqueued on st (the caller stages d_send/d_recv to the host and records its event); host
// transport: synchronous, h[0, 2W) = d_send, h[2W, 4W) = received, *now = true
int comm_counts(bw_comm* c, const uint64_t* d_send, uint64_t* d_recv, uint64_t* h, hipStream_t st, bool* now,
                std::string& err);
// variable all-to-all of elem-byte elements: scnt[k] to rank k, rcnt[k] from rank k (sections back
// to back in rank order); the host transport pads every section to `pad` elements.  On st.
int comm_all_to_allv(bw_comm* c, const void* d_send, const uint64_t* scnt, void* d_recv, const uint64_t* rcnt,
                     uint64_t elem, uint64_t pad, hipStream_t st, std::string& err);
// all[2k, 2k + 1] = rank k's mine[0, 1] (host-synchronous, deadline-bounded; control communicator)
int comm_allgather2(bw_comm* c, const uint64_t mine[2], uint64_t* all, std::string& err);
// bw_capi.hip: finish the queued exchanges whose counts arrived, in issue order (until = null: those
// ready now; else every one up to and including the exchange of slot `until`, waiting for them)
int exchange_progress(bw_comm* c, const void* until);
void exchange_drain(bw_comm* c);  // every queued exchange, waiting (bw_comm_destroy)

// ------------------------------------------------------------------ packfiles / index files (bw_pack.hip)
constexpr uint32_t ZSTD_BLOCK = 131072;           // zstd ZSTD_BLOCKSIZE_MAX
constexpr uint32_t ZSTD_STRIDE = ZSTD_BLOCK + 3;  // a raw block with its 3-byte header

struct PackBlob {
    uint8_t hash[32];
    uint8_t nonce[12];
    uint32_t kind;          // BlobKind tag
    uint64_t sealed_len;    // PackfileHeaderBlob.length (compressed + 16-byte tag)
    uint64_t section_off;   // PackfileHeaderBlob.offset (from the blob section start, at the nonce)
    uint64_t hdr_off;       // entry position in the header staging buffer
    uint64_t nonce_off;     // nonce position in the output
};

struct PackFileDesc {
    uint64_t hdr_off, count, out_off, header_len;
};

void launch_pack_meta(hipStream_t st, const PackBlob* blobs, uint64_t n, const PackFileDesc* files, uint64_t n_files,
                      uint8_t* hdr, uint8_t* out);
void launch_index_parse(hipStream_t st, const uint8_t* pt, const uint64_t* pt_off, const uint64_t* pt_len,
                        uint64_t n_files, uint64_t* parsed);
void launch_index_gather(hipStream_t st, const uint8_t* pt, const uint64_t* file_rec0, const uint64_t* file_src,
                         uint64_t n_files, uint64_t n_rec, uint8_t* digests, uint8_t* records);

// ------------------------------------------------------------------ zstd level 3 (bw_zstd.hip)
struct ZstdWork;
void zstd_work_free(ZstdWork* w);
void zstd_work_limits(ZstdWork*& w, uint64_t max_slots, uint64_t max_bytes);
void zstd_work_copy_limits(ZstdWork*& dst, const ZstdWork* src);  // dst created if null
// frames of n blobs (device buffers, host offset tables); synchronous on st; frame_len is host
int zstd_compress(hipStream_t st, ZstdWork*& w, const uint8_t* d_src, const uint64_t* src_off, const uint64_t* src_len,
                  uint64_t n, uint8_t* d_dst, const uint64_t* dst_off, uint64_t* frame_len, std::string& err);

}  // namespace bw
