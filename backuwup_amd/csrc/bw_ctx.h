// bw_ctx.h -- the context, its batch slots and the shared index: the private state behind the C ABI
// (include/backuwup_gpu.h), shared by the translation units that implement it: bw_capi.hip (contexts,
// the batch pipeline, the index, the multi-GPU exchange, stage timing), bw_dropin.hip / bw_stream.hip
// (the drop-in entry points) and bw_capi_pack.hip (sealing, zstd, packfiles and index files).
#pragma once
#include <atomic>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/backuwup_gpu.h"
#include "bw_internal.h"

using namespace bw;

namespace bwx {

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
};

struct PinBuf {
    void* p = nullptr;
    size_t cap = 0;
};

constexpr int MAX_DEPTH = 8;
constexpr int STAGE_RING = 4;

// One batch's outputs (kept until the ring wraps) and its host-streamed input.
struct Slot {
    // `res_dev`: the batch's device counters (C_COUNT u64) followed by its packed bw_blob records,
    // one buffer so that the results come back to the host in one copy
    DevBuf res_dev, digests, is_dup, input;
    PinBuf meta;                      // pinned metadata staging of this slot's batch
    hipEvent_t meta_done = nullptr;   // `meta` reusable once this fired (or `done`: meta_on_done)
    hipEvent_t input_free = nullptr;  // the batch's last read of its input (BLAKE3) finished
    hipEvent_t copied = nullptr;      // host-streamed input arrived in `input`
    bool meta_pending = false, input_used = false;
    bool meta_on_done = false;  // the staging's last upload is covered by `done` (no event of its own)
    uint64_t ticket = 0;  // 0: empty
    uint64_t max_blobs = 0;
    bool dedup = false;
    bool hashed = false;          // digests computed (not BW_F_NO_HASH): the exchange may gate them
    bw_comm* comm = nullptr;      // the batch went through this communicator's exchange: waits on it
                                  // are deadline-bounded (bw::comm_wait_event)
    // Results staged for the host as the batch's last stream operations: the counters (with the
    // index's state after the batch's gate) and the first res_n packed records, in pinned memory,
    // so a wait is one event synchronization and a memcpy instead of three device round trips.
    PinBuf res;
    uint64_t res_n = 0;
    hipEvent_t done = nullptr;   // the staged copies landed
    uint64_t mark = 0;           // the index's enq_total right after this batch's gate
    // a batch split by BW_OPT_SPLIT: its tail part is ticket tail_ticket of the context's helper,
    // holding files [tail_file0, n_files)
    uint64_t tail_ticket = 0, tail_file0 = 0;
    // bw_exchange_dedup of this batch: its digests grouped by owner (ex_dig, source positions
    // ex_perm), the counts message (ex_msg, device) and the counts of every rank (ex_h, pinned:
    // [0, 2W) mine, [2W, 4W) received); ex_part fires after the partition, ex_ready once ex_h holds
    // the counts.  ex_state: 0 = none, 1 = queued (waiting for the counts), 2 = enqueued, 3 = failed.
    DevBuf ex_dig, ex_perm, ex_msg;
    PinBuf ex_h;
    hipEvent_t ex_part = nullptr, ex_ready = nullptr;
    int ex_state = 0, ex_rc = 0;
    bool ex_now = false;     // the counts arrived synchronously (host transport)
    uint64_t ex_since = 0;   // when the counts were enqueued (steady clock, ns)
    uint64_t ex_first = 0, ex_n = ~0ull;  // the blobs the exchange sends (batch_set_exchange_range)
};

}  // namespace bwx

using namespace bwx;

// The seen-chunk index (BlobIndex, blob_index.rs:44-57): a digest log + an open-addressing table
// in HBM.  Shared by every context attached to it; operations are serialized by `mu` on the host
// and by the `tail` event on the GPU (each one waits for the previous one, on whatever stream).
struct bw_index {
    int device = 0;
    std::mutex mu;
    std::atomic<int> refs{1};
    DevBuf table, log, dstate;
    uint64_t table_cap = 0, log_cap = 0;
    uint64_t log_hi = 0;     // host upper bound of the log length, in-flight appends included
    uint64_t enq_total = 0;  // sum of the upper bounds of every append ever enqueued
    hipEvent_t tail = nullptr;
    bool tail_set = false;
    hipStream_t tail_stream = nullptr;  // the stream `tail` was last recorded on
    // With BW_OPT_ORDER_HASH, the scans and the BLAKE3 leaf passes of the contexts attached here
    // run one at a time each, in submission order, so a batch's scan shares the GPU with the
    // previous batch's hashing rather than two hashing passes sharing it while the scans wait.
    // Measured: scan/hash concurrency 10 % -> 28 % of the C2 timeline, throughput
    // unchanged, so it is off by default.
    hipEvent_t hash_tail = nullptr, scan_tail = nullptr;
    bool hash_tail_set = false, scan_tail_set = false;
};

struct bw_ctx {
    int device = 0;
    hipStream_t own = nullptr, stream = nullptr, copy = nullptr;
    std::string err;

    // per-batch device workspace (shared by the slots: batches run one after another on `stream`)
    DevBuf tile_count, tile_slots, tile_off, tile_btot, cand, ovf;
    DevBuf meta, chains, chain_n, chain_cptr, merge, seg_M, seg_cnt, cf_invalid, fb_starts, fb_count;
    DevBuf b_start, b_len, b_goff, b_file, b_kind, b_fend, b_ghash;
    DevBuf b_gdone;  // per blob: BLAKE3 groups finished (fused upper levels); zero between passes
    DevBuf cv, cv2, data, scratch, ucnt, ubtot;
    DevBuf bk_blk, bk_pack, bk_v;  // multi-GPU exchange buckets (bw_partition_buckets, ...)
    // bw_exchange_dedup: the digests received (source-major), the owner's verdicts on them, and
    // the verdicts on this rank's digests that come back; the exchange's transfers, gate and
    // scatter run on ex_st once its counts arrived (the per-batch parts live in the slot)
    DevBuf ex_rbk, ex_v, ex_rv;
    hipStream_t ex_st = nullptr;

    // batches in flight: ring of result slots addressed by ticket
    Slot slots[MAX_DEPTH];
    int depth = 2;
    uint64_t next_ticket = 1, last_ticket = 0;
    uint64_t last_n = 0;  // blobs of the last batch read back (sizes the next batches' staged results)
    // Intra-batch pipelining (BW_OPT_SPLIT): a multi-file batch below split_max bytes is cut by
    // bytes into a head (this context) and a tail (a helper context on its own stream, attached to
    // the same index), with the two scans and the two BLAKE3 passes each run in order, so the
    // tail's scan runs beside the head's hashing: one batch in flight still keeps the scan (HBM)
    // and BLAKE3 (VALU) side by side.  The gates stay in file order (head, then tail).
    int split = 1;  // off by default: measured slower on C1
    uint64_t split_min = 64ull << 20, split_max = 4ull << 30;
    bw_ctx* helper = nullptr;
    bool is_helper = false;
    hipEvent_t e_split = nullptr, e_tail = nullptr;
    // the synchronous helpers (bw_process_files, bw_fastcdc_chunks, bw_blake3_hash(_many), tree
    // blobs) run in a slot of their own outside the ring: they never drop a batch the caller still
    // holds a ticket for, and leave last_ticket (bw_results, bw_batch_views) unchanged
    Slot sync_slot;

    // pageable host input: ring of pinned staging chunks on the copy stream
    PinBuf ring[STAGE_RING];
    hipEvent_t ring_ev[STAGE_RING] = {};
    bool ring_set[STAGE_RING] = {};
    uint64_t stage_chunk = 64ull << 20;

    // options (bw_set_option)
    uint64_t scan_small_bytes = SCAN_SMALL_BYTES;
    bool order_hash = false;  // BW_OPT_ORDER_HASH
    uint64_t cand_cap_forced = 0;
    int b3_group = 0;   // BW_OPT_B3_GROUP: leaves per BLAKE3 group of the aligned-line leaf pass (0 = auto)
    bool b3_fused = false;  // BW_OPT_B3_UPPER: the upper levels inside the leaf pass (measured slower)
    int b3_loads = B3_LOADS_LINES;  // k_b3_lines: 1.07x fetch (pairs 1.42x), -6 % time isolated
    int scan_waves = 16;
    // latency stream: the small kernels between the two big passes (compaction, boundary
    // resolution, assembly, upper tree levels, gate, records) on a high-priority stream, so they
    // get CUs ahead of another batch's big kernels (BW_OPT_LATENCY_STREAM)
    bool lat_split = false;
    hipStream_t hi = nullptr;
    hipEvent_t e_scan = nullptr, e_lat = nullptr, e_b3 = nullptr, e_end = nullptr;
    uint64_t cand_override = 0;  // raised when a batch found more candidates than its array held

    // blob sealing (bw_seal.hip): item table staging + per-item key material + piece partials
    DevBuf seal_items, seal_keys, seal_parts, seal_ok, seal_io;
    PinBuf seal_stage;
    hipEvent_t seal_done = nullptr;  // seal_stage reusable once this fired
    bool seal_pending = false;

    // packfiles / index files (bw_pack.hip): tables, zstd staging, header plaintexts, host I/O
    DevBuf pk_blobs, pk_files, pk_hdr, pk_src, pk_out, ix_io, ix_tab, ix_dig;
    std::vector<PackBlob> h_pk_blobs;
    std::vector<PackFileDesc> h_pk_files;
    hipEvent_t pk_done = nullptr;  // the host tables above reusable once this fired
    bool pk_pending = false;

    // many small messages (tree blobs): pinned staging of the serialized bytes
    PinBuf msg_stage;

    // per-blob zstd level 3 (bw_zstd.hip): hash-table slots and scratch; zs_io = host-call staging
    ZstdWork* zw = nullptr;
    // asynchronous zstd (bw_zstd_submit_device / bw_zstd_wait): each lane runs one batch on its own
    // stream and hash tables, driven by a library thread through the batch's host round trips
    struct ZsLane {
        hipStream_t st = nullptr;      // the stream the lane's batch runs on (own_st or the context's)
        hipStream_t own_st = nullptr;  // created on first use by a lane that runs on a stream of its own
        hipEvent_t ready = nullptr;  // the context stream's work before the submit
        ZstdWork* w = nullptr;
        std::thread th;
        uint64_t ticket = 0;  // 0: free
        std::vector<uint64_t> so, sl, dof, fl;
        int rc = 0;
        std::string err;
    };
    ZsLane zs_lanes[BW_ZSTD_LANES];
    uint64_t zs_next = 1;
    DevBuf zs_io;
    // bw_pack_compress_device: level-3 frames staged for bw_pack_build_compressed
    DevBuf pk_stage;
    std::vector<uint64_t> pk_stage_off, pk_stage_len;

    // dedup index: `idx` is `own` unless the context is attached to a shared one
    bw_index* own_idx = nullptr;
    bw_index* idx = nullptr;
    uint64_t idx_mark = 0;  // idx->enq_total right after this context's last append

    // host-side time of submit's phases (diagnostic: BW_HOST_TIMING=1 at bw_create prints them at
    // bw_destroy): metadata, device buffers, metadata upload, chunk/hash launches, gate, tail
    bool host_timing = false;
    double host_ms[6] = {};
    uint64_t host_batches = 0;

    // stage timing: two event sets, alternated per batch so recording never waits on the GPU
    bool prof = false;
    uint32_t prof_mask = (2u << BW_N_STAGES) - 1;  // marks recorded (BW_OPT_PROFILE_MASK)
    int scan_first = 2;                             // BW_OPT_SCAN_FIRST
    hipEvent_t ev[2][BW_N_STAGES + 1] = {};
    bool ev_pending[2] = {false, false};
    int ev_set = 0;
    double stage_ms[BW_N_STAGES] = {};
    std::vector<double> intervals[BW_N_STAGES];  // [start, end) ms since the device's reference event
    uint64_t prof_batches = 0;
};

#define HIPCHK(ctx, expr)                                                                   \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess) {                                                             \
            (ctx)->err = std::string(#expr) + ": " + hipGetErrorString(e_);                 \
            return BW_EHIP;                                                                 \
        }                                                                                   \
    } while (0)

int ensure(bw_ctx* c, DevBuf& b, size_t bytes);       // device buffer of at least `bytes`
int ensure_host(bw_ctx* c, PinBuf& b, size_t bytes);  // pinned host buffer of at least `bytes`
void free_dev(DevBuf& b);
void free_host(PinBuf& b);

template <typename T>
inline T* P(DevBuf& b) { return (T*)b.p; }

constexpr size_t CTR_BYTES = C_COUNT * 8;

// Event kinds.  An event recorded between two kernels costs the stream ~5.5 us of idle time with
// the default system-scope fence (a cache writeback and invalidate); the events that only order GPU
// work (or tell the host that the GPU finished reading something) release at device scope, and the
// stage marks, which only time, take no system fence at all.  `done`, after which the host reads
// results the GPU wrote into pinned memory, keeps the system scope.
constexpr unsigned EV_ORDER = hipEventDisableTiming | hipEventReleaseToDevice;
constexpr unsigned EV_TIMING = hipEventDisableSystemFence;
inline uint64_t* slot_ctr(Slot& s) { return (uint64_t*)s.res_dev.p; }
inline uint8_t* slot_records(Slot& s) { return (uint8_t*)s.res_dev.p + CTR_BYTES; }

// shared by the translation units of the C ABI (bw_capi.hip defines them)
Slot* slot_of(bw_ctx* c, uint64_t ticket);
int stage_results(bw_ctx* c, Slot& s, bool written = false, uint64_t want = 0, hipStream_t st = nullptr);
int dedup_device(bw_ctx* c, const uint8_t* d_digests, const uint64_t* n_dev, uint64_t n_host, uint64_t max_n,
                 uint8_t* d_is_dup, hipStream_t st = nullptr, const std::function<void(hipStream_t)>& then = nullptr);
int check_collision(bw_ctx* c, bool all = false);

