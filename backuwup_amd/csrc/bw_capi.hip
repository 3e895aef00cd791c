// bw_capi.hip -- the C ABI (include/backuwup_gpu.h) and the host-side batch orchestration.
//
// The host side only turns file sizes into small metadata tables (segments, canonical units);
// every byte of file data is read on the GPU.  A batch is enqueued on one HIP stream with no
// host synchronisation until results are requested, so a caller can keep batches in flight:
//   * a context keeps the outputs of its last `depth` batches in a ring of slots, addressed by
//     the ticket bw_submit_* returns (bw_wait), so batch k+1 can be queued before batch k is read;
//   * bw_submit_host copies a batch from host memory on the context's copy stream, into the slot's
//     own HBM buffer, while the previous batch computes (pinned memory is DMA'd directly, pageable
//     memory goes through a ring of pinned staging chunks);
//   * one dedup index (bw_index) can be shared by several contexts on several streams: every
//     index operation waits for the index's previous operation (an event chain), so the batches of
//     one backup session are gated in submission order whichever stream runs them.
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/backuwup_gpu.h"
#include "bw_device.h"
#include "bw_internal.h"
#include "bw_tables.inc"

using namespace bw;

static const uint64_t H_MASKS[26] = BW_MASKS_INIT;

#include "bw_ctx.h"

// ------------------------------------------------------------------ helpers

int ensure(bw_ctx* c, DevBuf& b, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (b.cap >= bytes) return BW_OK;
    if (b.p) {
        hipStreamSynchronize(c->stream);
        if (c->copy) hipStreamSynchronize(c->copy);
        if (c->ex_st) hipStreamSynchronize(c->ex_st);
        hipFree(b.p);
        b.p = nullptr;
        b.cap = 0;
    }
    size_t want = bytes + bytes / 4 + 256;
    if (hipMalloc(&b.p, want) != hipSuccess) {
        c->err = "hipMalloc(" + std::to_string(want) + ") failed";
        b.p = nullptr;
        return BW_ENOMEM;
    }
    b.cap = want;
    return BW_OK;
}

int ensure_host(bw_ctx* c, PinBuf& b, size_t bytes) {
    if (b.cap >= bytes) return BW_OK;
    if (b.p) hipHostFree(b.p);
    b.p = nullptr;
    b.cap = 0;
    size_t want = bytes + bytes / 4 + 4096;
    if (hipHostMalloc(&b.p, want, hipHostMallocDefault) != hipSuccess) {
        c->err = "hipHostMalloc(" + std::to_string(want) + ") failed";
        return BW_ENOMEM;
    }
    b.cap = want;
    return BW_OK;
}

void free_dev(DevBuf& b) {
    if (b.p) hipFree(b.p);
    b.p = nullptr;
    b.cap = 0;
}

void free_host(PinBuf& b) {
    if (b.p) hipHostFree(b.p);
    b.p = nullptr;
    b.cap = 0;
}

static int make_masks(uint32_t mn, uint32_t av, uint32_t mx, Masks* mk) {
    // FastCDC::with_level asserts (fastcdc 3.0.3 v2020) -> BW_EINVAL instead of a panic.
    if (mn < BW_MINIMUM_MIN || mn > BW_MINIMUM_MAX) return BW_EINVAL;
    if (av < BW_AVERAGE_MIN || av > BW_AVERAGE_MAX) return BW_EINVAL;
    if (mx < BW_MAXIMUM_MIN || mx > BW_MAXIMUM_MAX) return BW_EINVAL;
    // avg > max passes the crate's asserts, but then cut() keeps center = avg past remaining = max:
    // its first loop reads beyond max (a cut there makes a chunk longer than max) and, where the
    // source ends first, indexes out of bounds -- a panic, on most inputs (oracle/bw_oracle.c
    // ORC_CUT_PANIC restates it).  backuwup never passes such sizes (dir_packer.rs:254-259); the
    // ABI refuses them instead of returning chunks the crate would not.
    if (av > mx) return BW_EINVAL;
    const uint32_t bits = (uint32_t)lround(log2((double)av));  // logarithm2(): round(log2(avg))
    mk->min = mn;
    mk->avg = av;
    mk->max = mx;
    mk->s0 = 2 * (mn / 2);
    mk->mask_s = H_MASKS[bits + 1];  // Normalization::Level1
    mk->mask_l = H_MASKS[bits - 1];
    mk->mask_pre = mk->mask_s & mk->mask_l;
    mk->pre_shift = (uint32_t)__builtin_clzll(mk->mask_s | mk->mask_l);  // 63 - top bit
    mk->pre_hi = (uint32_t)((mk->mask_pre << mk->pre_shift) >> 32);
    mk->tile_shift = SCAN_TILE_SHIFT;
    return BW_OK;
}

static uint64_t seg_len_for(const Masks& mk, bool small_batch) {
    // Segments are a multiple of max_size so that chains through data without candidates
    // (e.g. zeros: every chunk is exactly max) stay phase-aligned and merge immediately; the
    // multiple keeps a segment's own cuts within CHAIN_CAP / 2.  Small batches take at most 2 x max:
    // their chain walk is latency on the critical path (one wave walks a segment's cuts one after
    // another, ~1.7 us each), and more, shorter segments walk in parallel.
    uint64_t k = (uint64_t)(CHAIN_CAP / 2) * std::min<uint64_t>(mk.s0, mk.max) / mk.max;
    if (k < 1) k = 1;
    if (k > (small_batch ? 2 : 8)) k = small_batch ? 2 : 8;
    return k * mk.max;
}

// ------------------------------------------------------------------ stage timing

// prof_mask bit i (i <= BW_N_STAGES, the batch end) = record mark i; stage i's time runs from its
// mark to the next recorded one, and the last recorded mark closes the batch.  Every event
// recorded between two kernels costs the stream ~5.5 us of idle time (profiles/r03: k_scan ->
// k_tile_partial with a mark between them 5.7 us, kernels without one 0), so the bench's timed
// region marks only the leaf pass.
// One timing event per device, recorded when a context of the device first enables profiling: the
// stage intervals of every context of the device are placed on its timeline, so a caller can take
// the union of one stage's launches across contexts (bw_profile_intervals).
static std::mutex g_ref_mu;
static hipEvent_t g_ref[64] = {};

static hipEvent_t prof_reference(int device, hipStream_t st) {
    std::lock_guard<std::mutex> lk(g_ref_mu);
    if (device < 0 || device >= 64) return nullptr;
    if (!g_ref[device] && hipEventCreateWithFlags(&g_ref[device], EV_TIMING) == hipSuccess) {
        hipEventRecord(g_ref[device], st);
        hipEventSynchronize(g_ref[device]);
    }
    return g_ref[device];
}

static void prof_collect(bw_ctx* c, int set) {
    if (!c->ev_pending[set]) return;
    const uint32_t mask = c->prof_mask;
    const int last = 31 - __builtin_clz(mask);
    hipEventSynchronize(c->ev[set][last]);
    hipEvent_t ref = prof_reference(c->device, c->stream);
    for (int i = 0; i < last; i++) {
        if (!((mask >> i) & 1)) continue;
        int j = i + 1;
        while (!((mask >> j) & 1)) j++;
        float ms = 0;
        if (hipEventElapsedTime(&ms, c->ev[set][i], c->ev[set][j]) == hipSuccess) c->stage_ms[i] += ms;
        float t0 = 0;
        if (ref && hipEventElapsedTime(&t0, ref, c->ev[set][i]) == hipSuccess) {
            c->intervals[i].push_back(t0);
            c->intervals[i].push_back((double)t0 + ms);
        }
    }
    c->prof_batches++;
    c->ev_pending[set] = false;
}

static void prof_mark(bw_ctx* c, int stage, hipStream_t st = nullptr) {
    if (c->prof && ((c->prof_mask >> stage) & 1)) hipEventRecord(c->ev[c->ev_set][stage], st ? st : c->stream);
}

// ------------------------------------------------------------------ the index object

static int index_init(bw_index* x, int device) {
    x->device = device;
    if (hipSetDevice(device) != hipSuccess) return BW_EHIP;
    if (hipEventCreateWithFlags(&x->tail, EV_ORDER) != hipSuccess) return BW_EHIP;
    if (hipEventCreateWithFlags(&x->hash_tail, EV_ORDER) != hipSuccess) return BW_EHIP;
    if (hipEventCreateWithFlags(&x->scan_tail, EV_ORDER) != hipSuccess) return BW_EHIP;
    if (hipMalloc(&x->dstate.p, D_COUNT * 8) != hipSuccess) return BW_ENOMEM;
    x->dstate.cap = D_COUNT * 8;
    if (hipMemset(x->dstate.p, 0, D_COUNT * 8) != hipSuccess) return BW_EHIP;
    return BW_OK;
}

static void index_release(bw_index* x) {
    if (!x || --x->refs > 0) return;
    hipSetDevice(x->device);
    if (x->tail_set) hipEventSynchronize(x->tail);
    free_dev(x->table);
    free_dev(x->log);
    free_dev(x->dstate);
    if (x->hash_tail_set) hipEventSynchronize(x->hash_tail);
    if (x->tail) hipEventDestroy(x->tail);
    if (x->hash_tail) hipEventDestroy(x->hash_tail);
    if (x->scan_tail_set) hipEventSynchronize(x->scan_tail);
    if (x->scan_tail) hipEventDestroy(x->scan_tail);
    delete x;
}

// Scope of one index operation issued on context c's stream: holds the index lock, makes the
// stream wait for the previous operation (from any context) and records this one as the new tail.
struct IndexOp {
    bw_ctx* c;
    bw_index* x;
    hipStream_t st;
    std::lock_guard<std::mutex> lk;
    explicit IndexOp(bw_ctx* cc, hipStream_t s = nullptr)
        : c(cc), x(cc->idx), st(s ? s : cc->stream), lk(cc->idx->mu) {
        // the previous operation on this same stream is ordered already (and a wait costs the
        // stream an idle gap like any event operation)
        if (x->tail_set && x->tail_stream != st) hipStreamWaitEvent(st, x->tail, 0);
    }
    ~IndexOp() {
        hipEventRecord(x->tail, st);
        x->tail_set = true;
        x->tail_stream = st;
    }
};

// Room for `incoming` more log entries (lock held).  Growth waits for every earlier operation of
// the index (its tail) before the old buffers are replaced; sessions pre-size with bw_index_reset.
static int index_capacity(bw_ctx* c, uint64_t incoming, hipStream_t st) {
    bw_index* x = c->idx;
    if (x->table_cap && ((x->log_hi + incoming) > x->log_cap || (x->log_hi + incoming) * 2 > x->table_cap)) {
        // Before growing, replace the host's bound by the real log length.  The bound adds every
        // gate's max_n (a batch's len/min + 2 blobs, an exchange gate's n_src x cap slots) and only
        // a result read tightens it, so without this a session whose batches are never read back
        // (the multi-GPU exchange) would grow the table by its bounds, not its digests.  `st`
        // already waits for the index tail and the lock is held, so once it drains the length is
        // exact; growing synchronizes anyway.
        uint64_t len = 0;
        HIPCHK(c, hipMemcpyAsync(&len, P<uint64_t>(x->dstate) + D_LOGLEN, 8, hipMemcpyDeviceToHost, st));
        HIPCHK(c, hipStreamSynchronize(st));
        x->log_hi = std::min(x->log_hi, len);
    }
    const uint64_t need_log = x->log_hi + incoming;
    if (need_log >> 40) {  // table words hold a 40-bit log position
        c->err = "index log beyond 2^40 entries";
        return BW_ENOMEM;
    }
    if (need_log > x->log_cap) {
        uint64_t cap = x->log_cap ? x->log_cap : 1 << 16;
        while (cap < need_log) cap *= 2;
        DevBuf nb;
        if (hipMalloc(&nb.p, cap * 32) != hipSuccess) {
            c->err = "hipMalloc of the index log failed";
            return BW_ENOMEM;
        }
        nb.cap = cap * 32;
        if (x->log.p) {
            HIPCHK(c, hipMemcpyAsync(nb.p, x->log.p, x->log_cap * 32, hipMemcpyDeviceToDevice, st));
            HIPCHK(c, hipStreamSynchronize(st));
            hipFree(x->log.p);
        }
        x->log = nb;
        x->log_cap = cap;
    }
    // keep the table at most half full (upper bound: every logged digest distinct)
    if (need_log * 2 > x->table_cap) {
        uint64_t cap = x->table_cap ? x->table_cap : 1 << 16;
        while (cap < need_log * 2) cap *= 2;
        if (x->table.p) {
            HIPCHK(c, hipStreamSynchronize(st));
            hipFree(x->table.p);
            x->table.p = nullptr;
        }
        if (hipMalloc(&x->table.p, cap * 8) != hipSuccess) {
            c->err = "hipMalloc of the index table failed";
            return BW_ENOMEM;
        }
        x->table.cap = cap * 8;
        const uint64_t old = x->table_cap;
        x->table_cap = cap;
        launch_table_clear(st, P<uint64_t>(x->table), cap);
        if (old) launch_rehash(st, P<uint64_t>(x->table), cap, P<uint8_t>(x->log), P<uint64_t>(x->dstate),
                               x->log_hi);
    }
    return BW_OK;
}

static int index_reset_locked(bw_ctx* c, uint64_t hint, hipStream_t st) {
    bw_index* x = c->idx;
    x->log_hi = 0;
    HIPCHK(c, hipMemsetAsync(x->dstate.p, 0, D_COUNT * 8, st));
    if (int rc = index_capacity(c, hint ? hint : 1024, st)) return rc;
    launch_table_clear(st, P<uint64_t>(x->table), x->table_cap);
    HIPCHK(c, hipGetLastError());
    return BW_OK;
}

// Append + gate n digests (n read on the device from n_dev when given; max_n bounds it).
// `then` (may be empty) is enqueued after the gate and before the index's tail event, i.e. inside
// the index operation: a batch's k_pack snapshots the index state there, and its launch does not
// sit behind an event record (each costs the stream ~5.5 us of idle time).
int dedup_device(bw_ctx* c, const uint8_t* d_digests, const uint64_t* n_dev, uint64_t n_host, uint64_t max_n,
                 uint8_t* d_is_dup, hipStream_t st, const std::function<void(hipStream_t)>& then) {
    IndexOp op(c, st);
    st = op.st;
    bw_index* x = c->idx;
    if (!x->table_cap)
        if (int rc = index_reset_locked(c, 0, st)) return rc;
    if (int rc = index_capacity(c, max_n, st)) return rc;
    launch_dedup(st, P<uint64_t>(x->table), x->table_cap, P<uint8_t>(x->log), P<uint64_t>(x->dstate),
                 d_digests, n_dev, n_host, max_n, d_is_dup);
    x->log_hi += max_n;
    x->enq_total += max_n;
    c->idx_mark = x->enq_total;
    if (then) then(st);
    HIPCHK(c, hipGetLastError());
    return BW_OK;
}

// Read the index state (synchronizes the context stream): after every operation issued so far
// from any context (all = true), or after this context's own last one (all = false: reading a
// batch's results must not wait for batches queued behind it on other streams).
static int read_index_state(bw_ctx* c, uint64_t st[D_COUNT], bool all) {
    bw_index* x = c->idx;
    uint64_t mark = c->idx_mark;  // appends at or before the read position
    if (all) {
        std::lock_guard<std::mutex> lk(x->mu);
        if (x->tail_set) hipStreamWaitEvent(c->stream, x->tail, 0);
        mark = x->enq_total;
    }
    HIPCHK(c, hipMemcpyAsync(st, x->dstate.p, D_COUNT * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    // tighten the host bound: appends enqueued after the read position add at most their bounds
    std::lock_guard<std::mutex> lk(x->mu);
    x->log_hi = std::min(x->log_hi, st[D_LOGLEN] + (x->enq_total - std::min(x->enq_total, mark)));
    return BW_OK;
}

int check_collision(bw_ctx* c, bool all) {
    uint64_t st[D_COUNT];
    if (int rc = read_index_state(c, st, all)) return rc;
    if (st[D_LOST]) {
        c->err = "index lookup found no slot (internal error)";
        return BW_EHIP;
    }
    if (st[D_BUCKET_OVF]) {
        c->err = "a batch had more blobs than its exchange bucket capacity (verdicts incomplete)";
        return BW_ENOSPC;
    }
    return BW_OK;
}

// ------------------------------------------------------------------ C ABI: basics

extern "C" void bw_params_default(bw_params* p) {
    if (!p) return;
    p->min_size = BW_BLOB_MINIMUM_TARGET_SIZE;
    p->avg_size = BW_BLOB_DESIRED_TARGET_SIZE;
    p->max_size = BW_BLOB_MAX_UNCOMPRESSED_SIZE;
    p->flags = 0;
    p->small_file_threshold = BW_BLOB_DESIRED_TARGET_SIZE;  // dir_packer.rs:246
}

extern "C" const char* bw_strerror(int rc) {
    switch (rc) {
        case BW_OK: return "ok";
        case BW_EINVAL: return "invalid argument (fastcdc parameter range or pointer)";
        case BW_ENOSPC: return "output capacity too small";
        case BW_EHIP: return "HIP runtime error";
        case BW_ENOMEM: return "out of memory";
        case BW_ECOLLISION: return "64-bit digest key collision in the index (no longer returned)";
        case BW_ESTATE: return "invalid call order";
        case BW_ECRYPTO: return "AES-GCM authentication failed";
        case BW_EFORMAT: return "malformed bincode data";
        case BW_ECOMM: return "the exchange transport failed (communicator aborted)";
        case BW_EAGAIN: return "the hash service could not take the call; retry through a context";
        default: return "unknown error";
    }
}

extern "C" int bw_create(int device, bw_ctx** out) {
    if (!out) return BW_EINVAL;
    *out = nullptr;
    bw_ctx* c = new bw_ctx();
    c->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return BW_EHIP;
    }
    c->stream = c->own;
    c->host_timing = getenv("BW_HOST_TIMING") != nullptr;
    c->own_idx = new bw_index();
    c->idx = c->own_idx;
    if (int rc = index_init(c->own_idx, device)) {
        bw_destroy(c);
        return rc;
    }
    for (int s = 0; s <= MAX_DEPTH; s++) {
        Slot& sl = s < MAX_DEPTH ? c->slots[s] : c->sync_slot;
        if (hipEventCreateWithFlags(&sl.meta_done, EV_ORDER) != hipSuccess ||
            hipEventCreateWithFlags(&sl.input_free, EV_ORDER) != hipSuccess ||
            hipEventCreateWithFlags(&sl.copied, EV_ORDER) != hipSuccess ||
            hipEventCreateWithFlags(&sl.ex_part, EV_ORDER) != hipSuccess ||
            hipEventCreateWithFlags(&sl.ex_ready, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&sl.done, hipEventDisableTiming) != hipSuccess) {
            bw_destroy(c);
            return BW_EHIP;
        }
    }
    *out = c;
    return BW_OK;
}

extern "C" void bw_destroy(bw_ctx* c) {
    if (!c) return;
    if (c->helper) bw_destroy(c->helper);  // its batches end before this context's buffers go
    for (hipEvent_t e : {c->e_split, c->e_tail})
        if (e) hipEventDestroy(e);
    if (c->host_timing && c->host_batches)
        fprintf(stderr, "bw host ms/batch over %llu batches: meta %.3f bufs %.3f upload %.3f launch %.3f gate %.3f tail %.3f\n",
                (unsigned long long)c->host_batches, c->host_ms[0] / c->host_batches, c->host_ms[1] / c->host_batches,
                c->host_ms[2] / c->host_batches, c->host_ms[3] / c->host_batches, c->host_ms[4] / c->host_batches,
                c->host_ms[5] / c->host_batches);
    hipSetDevice(c->device);
    for (int k = 0; k <= MAX_DEPTH; k++) {  // exchanges of this context still waiting for their counts
        Slot& s = k < MAX_DEPTH ? c->slots[k] : c->sync_slot;
        if (s.ex_state == 1 && s.comm) exchange_progress(s.comm, &s);
    }
    if (c->stream) hipStreamSynchronize(c->stream);
    if (c->copy) hipStreamSynchronize(c->copy);
    if (c->ex_st) hipStreamSynchronize(c->ex_st);
    DevBuf* all[] = {&c->tile_count, &c->tile_slots, &c->tile_off, &c->tile_btot, &c->cand, &c->ovf, &c->meta,
                     &c->chains, &c->chain_n, &c->chain_cptr, &c->merge, &c->seg_M,
                     &c->seg_cnt, &c->cf_invalid, &c->fb_starts, &c->fb_count, &c->b_start, &c->b_len,
                     &c->b_goff, &c->b_file, &c->b_kind, &c->b_fend, &c->b_ghash, &c->b_gdone, &c->cv, &c->cv2,
                     &c->data, &c->scratch, &c->ucnt, &c->ubtot, &c->seal_items, &c->seal_keys, &c->seal_parts,
                     &c->seal_ok, &c->seal_io, &c->pk_blobs, &c->pk_files, &c->pk_hdr, &c->pk_src, &c->pk_out,
                     &c->ix_io, &c->ix_tab, &c->ix_dig, &c->bk_blk, &c->bk_pack, &c->bk_v, &c->zs_io, &c->pk_stage,
                     &c->ex_rbk, &c->ex_v, &c->ex_rv};
    for (auto& L : c->zs_lanes) {  // batches still in flight finish first
        if (L.th.joinable()) L.th.join();
        if (L.own_st) hipStreamDestroy(L.own_st);  // (lane 0's own stream leaked)
        if (L.ready) hipEventDestroy(L.ready);
        zstd_work_free(L.w);
        L.w = nullptr;
    }
    for (DevBuf* b : all) free_dev(*b);
    zstd_work_free(c->zw);
    c->zw = nullptr;
    for (int k = 0; k <= MAX_DEPTH; k++) {
        Slot& s = k < MAX_DEPTH ? c->slots[k] : c->sync_slot;
        free_dev(s.res_dev);
        free_dev(s.digests);
        free_dev(s.is_dup);
        free_dev(s.input);
        free_dev(s.ex_dig);
        free_dev(s.ex_perm);
        free_dev(s.ex_msg);
        free_host(s.meta);
        free_host(s.res);
        free_host(s.ex_h);
        if (s.ex_part) hipEventDestroy(s.ex_part);
        if (s.ex_ready) hipEventDestroy(s.ex_ready);
        if (s.done) hipEventDestroy(s.done);
        if (s.meta_done) hipEventDestroy(s.meta_done);
        if (s.input_free) hipEventDestroy(s.input_free);
        if (s.copied) hipEventDestroy(s.copied);
    }
    for (int r = 0; r < STAGE_RING; r++) {
        free_host(c->ring[r]);
        if (c->ring_ev[r]) hipEventDestroy(c->ring_ev[r]);
    }
    free_host(c->seal_stage);
    free_host(c->msg_stage);
    if (c->seal_done) hipEventDestroy(c->seal_done);
    if (c->pk_done) hipEventDestroy(c->pk_done);
    for (int k = 0; k < 2; k++)
        for (int i = 0; i <= BW_N_STAGES; i++)
            if (c->ev[k][i]) hipEventDestroy(c->ev[k][i]);
    if (c->idx != c->own_idx) index_release(c->idx);
    index_release(c->own_idx);
    if (c->hi) hipStreamSynchronize(c->hi);
    for (hipEvent_t e : {c->e_scan, c->e_lat, c->e_b3, c->e_end})
        if (e) hipEventDestroy(e);
    if (c->hi) hipStreamDestroy(c->hi);
    if (c->copy) hipStreamDestroy(c->copy);
    if (c->ex_st) hipStreamDestroy(c->ex_st);
    if (c->own) hipStreamDestroy(c->own);
    delete c;
}

extern "C" const char* bw_last_error(const bw_ctx* c) { return c ? c->err.c_str() : "null context"; }

extern "C" int bw_set_stream(bw_ctx* c, void* s) {
    if (!c) return BW_EINVAL;
    hipStream_t want = s ? (hipStream_t)s : c->own;
    if (want == c->stream) return BW_OK;
    hipSetDevice(c->device);
    hipStreamSynchronize(c->stream);  // work queued on the old stream is done before the switch
    c->stream = want;
    return BW_OK;
}

extern "C" void* bw_get_stream(bw_ctx* c) { return c ? (void*)c->stream : nullptr; }

// Variants measured slower than the shipped path are compiled only into the
// diagnostic build (BW_DIAG: libbackuwup_amd_debug.so); the product library accepts their
// options at the shipped value only.
static int diag_only(bw_ctx* c, int opt, uint64_t v, uint64_t shipped) {
    if (BW_DIAG || v == shipped) return 1;  // go on to the option's own case
    c->err = "option " + std::to_string(opt) + " = " + std::to_string(v) +
             " selects a diagnostic variant: load the BW_DIAG build (libbackuwup_amd_debug.so)";
    return BW_EINVAL;
}

extern "C" int bw_set_option(bw_ctx* c, int opt, uint64_t v) {
    if (!c) return BW_EINVAL;
    int d = 1;
    switch (opt) {
        case BW_OPT_SPLIT: d = v == 2 ? diag_only(c, opt, v, 1) : 1; break;
        case BW_OPT_ORDER_HASH: d = diag_only(c, opt, v, 0); break;
        case BW_OPT_SCAN_WAVES: d = diag_only(c, opt, v, 16); break;
        case BW_OPT_LATENCY_STREAM: d = diag_only(c, opt, v, 0); break;
        case BW_OPT_B3_LOADS: d = diag_only(c, opt, v, B3_LOADS_LINES); break;
        case BW_OPT_B3_UPPER: d = diag_only(c, opt, v, 0); break;
        default: break;
    }
    if (d != 1) return d;
    switch (opt) {
        case BW_OPT_DEPTH:
            if (v < 1 || v > MAX_DEPTH) return BW_EINVAL;
            hipSetDevice(c->device);
            hipStreamSynchronize(c->stream);
            if (c->copy) hipStreamSynchronize(c->copy);
            c->depth = (int)v;
            for (Slot& s : c->slots) s.ticket = 0;  // earlier tickets are no longer addressable
            c->last_ticket = 0;
            if (c->helper) return bw_set_option(c->helper, opt, v);
            return BW_OK;
        case BW_OPT_SPLIT:
            if (v < 1 || v > 2) return BW_EINVAL;
            c->split = (int)v;
            return BW_OK;
        case BW_OPT_SCAN_SMALL_BYTES:
            c->scan_small_bytes = v;
            return c->helper ? bw_set_option(c->helper, opt, v) : BW_OK;
        case BW_OPT_ORDER_HASH:
            if (v > 1) return BW_EINVAL;
            c->order_hash = v != 0;
            return BW_OK;
        case BW_OPT_CAND_CAP:
            c->cand_cap_forced = v;
            return c->helper ? bw_set_option(c->helper, opt, v) : BW_OK;
        case BW_OPT_SCAN_WAVES:
            if (v != 8 && v != 16) return BW_EINVAL;
            c->scan_waves = (int)v;
            return c->helper ? bw_set_option(c->helper, opt, v) : BW_OK;
        case BW_OPT_LATENCY_STREAM:
            if (v && !c->hi) {
                hipSetDevice(c->device);
                int least = 0, greatest = 0;
                HIPCHK(c, hipDeviceGetStreamPriorityRange(&least, &greatest));
                HIPCHK(c, hipStreamCreateWithPriority(&c->hi, hipStreamNonBlocking, greatest));
                for (hipEvent_t* e : {&c->e_scan, &c->e_lat, &c->e_b3, &c->e_end})
                    HIPCHK(c, hipEventCreateWithFlags(e, EV_ORDER));
            }
            c->lat_split = v != 0;
            return BW_OK;
        case BW_OPT_ZSTD_SLOTS:
            if (v < 1 || v > (1u << 20)) return BW_EINVAL;
            hipSetDevice(c->device);
            hipStreamSynchronize(c->stream);
            zstd_work_limits(c->zw, v, 0);
            return BW_OK;
        case BW_OPT_ZSTD_BATCH_BYTES:
            if (v < (1u << 20)) return BW_EINVAL;
            zstd_work_limits(c->zw, 0, v);
            return BW_OK;
        case BW_OPT_B3_LOADS:
            if (v > B3_LOADS_LINES) return BW_EINVAL;
            c->b3_loads = (int)v;
            return c->helper ? bw_set_option(c->helper, opt, v) : BW_OK;
        case BW_OPT_PROFILE_MASK:
            if (__builtin_popcountll(v) < 2 || v >= (2u << BW_N_STAGES)) return BW_EINVAL;
            c->prof_mask = (uint32_t)v;
            return c->helper ? bw_set_option(c->helper, opt, v) : BW_OK;
        case BW_OPT_B3_GROUP:
            if (v != 0 && v != 1 && v != 2 && v != 4) return BW_EINVAL;
            c->b3_group = (int)v;
            return c->helper ? bw_set_option(c->helper, opt, v) : BW_OK;
        case BW_OPT_B3_UPPER:
            if (v > 1) return BW_EINVAL;
            c->b3_fused = v == 1;
            return c->helper ? bw_set_option(c->helper, opt, v) : BW_OK;
        case BW_OPT_SCAN_FIRST:
            if (v > 2) return BW_EINVAL;
            c->scan_first = (int)v;
            return c->helper ? bw_set_option(c->helper, opt, v) : BW_OK;
        case BW_OPT_STAGE_CHUNK:
            if (v < 4096) return BW_EINVAL;
            hipSetDevice(c->device);
            if (c->copy) hipStreamSynchronize(c->copy);
            for (int r = 0; r < STAGE_RING; r++) free_host(c->ring[r]);
            c->stage_chunk = v;
            return BW_OK;
        default: return BW_EINVAL;
    }
}

// ------------------------------------------------------------------ dedup index (C ABI)

extern "C" int bw_index_create(int device, bw_index** out) {
    if (!out) return BW_EINVAL;
    *out = nullptr;
    bw_index* x = new bw_index();
    if (int rc = index_init(x, device)) {
        index_release(x);
        return rc;
    }
    *out = x;
    return BW_OK;
}

extern "C" void bw_index_destroy(bw_index* x) { index_release(x); }

extern "C" int bw_attach_index(bw_ctx* c, bw_index* x) {
    if (!c) return BW_EINVAL;
    if (!x) x = c->own_idx;
    if (x->device != c->device) {
        c->err = "index and context live on different devices";
        return BW_EINVAL;
    }
    if (x == c->idx) return BW_OK;
    hipSetDevice(c->device);
    HIPCHK(c, hipStreamSynchronize(c->stream));  // this context's work on the old index is done
    bw_index* old = c->idx;
    if (x != c->own_idx) x->refs++;
    c->idx = x;
    c->idx_mark = 0;
    if (old != c->own_idx) index_release(old);
    if (c->helper) return bw_attach_index(c->helper, x);
    return BW_OK;
}

extern "C" int bw_index_reset(bw_ctx* c, uint64_t hint) {
    if (!c) return BW_EINVAL;
    hipSetDevice(c->device);
    IndexOp op(c);
    return index_reset_locked(c, hint, c->stream);
}

extern "C" int bw_index_seed(bw_ctx* c, const uint8_t* sorted, uint64_t n) {
    if (!c || (n && !sorted)) return BW_EINVAL;
    if (!n) return BW_OK;
    hipSetDevice(c->device);
    if (int rc = ensure(c, c->scratch, n * 32)) return rc;
    HIPCHK(c, hipMemcpyAsync(c->scratch.p, sorted, n * 32, hipMemcpyHostToDevice, c->stream));
    if (int rc = dedup_device(c, P<uint8_t>(c->scratch), nullptr, n, n, nullptr)) return rc;
    return check_collision(c);
}

extern "C" int bw_index_check_insert(bw_ctx* c, const uint8_t* digests, uint64_t n, uint8_t* is_dup) {
    if (!c || (n && (!digests || !is_dup))) return BW_EINVAL;
    if (!n) return BW_OK;
    hipSetDevice(c->device);
    if (int rc = ensure(c, c->scratch, n * 33)) return rc;
    uint8_t* dd = P<uint8_t>(c->scratch);
    HIPCHK(c, hipMemcpyAsync(dd, digests, n * 32, hipMemcpyHostToDevice, c->stream));
    if (int rc = dedup_device(c, dd, nullptr, n, n, dd + n * 32)) return rc;
    HIPCHK(c, hipMemcpyAsync(is_dup, dd + n * 32, n, hipMemcpyDeviceToHost, c->stream));
    return check_collision(c);
}

extern "C" int bw_index_check_insert_device(bw_ctx* c, const uint8_t* d_digests, uint64_t n, uint8_t* d_is_dup) {
    if (!c || (n && (!d_digests || !d_is_dup))) return BW_EINVAL;
    if (!n) return BW_OK;
    hipSetDevice(c->device);
    return dedup_device(c, d_digests, nullptr, n, n, d_is_dup);
}

extern "C" int bw_index_check(bw_ctx* c) {
    if (!c) return BW_EINVAL;
    hipSetDevice(c->device);
    return check_collision(c, true);
}

extern "C" int bw_index_size(bw_ctx* c, uint64_t* n) {
    if (!c || !n) return BW_EINVAL;
    hipSetDevice(c->device);
    uint64_t st[D_COUNT];
    if (int rc = read_index_state(c, st, true)) return rc;
    *n = st[D_NUNIQUE];
    return BW_OK;
}

// ------------------------------------------------------------------ the batch pipeline

Slot* slot_of(bw_ctx* c, uint64_t ticket) {
    if (!ticket || ticket >= c->next_ticket) return nullptr;
    Slot* s = &c->slots[(ticket - 1) % (uint64_t)c->depth];
    return s->ticket == ticket ? s : nullptr;
}

static int validate_batch(bw_ctx* c, uint64_t data_len, const uint64_t* foff, const uint64_t* flen, uint64_t nf,
                          const bw_params* prm, Masks* mk) {
    if (int rc = make_masks(prm->min_size, prm->avg_size, prm->max_size, mk)) {
        c->err = "fastcdc parameters out of range";
        return rc;
    }
    if (nf && (!foff || !flen)) return BW_EINVAL;
    for (uint64_t f = 0; f < nf; f++)
        if (foff[f] > data_len || flen[f] > data_len - foff[f]) {
            c->err = "file " + std::to_string(f) + " lies outside the data buffer";
            return BW_EINVAL;
        }
    return BW_OK;
}

// Queue the host copies of a batch's results behind its kernels on the context stream: the
// counters and the first res_n packed records (about twice the previous batch's blob count: a
// guess, the rest is copied at the wait if the batch has more) into the slot's pinned buffer.
// The results a bw_wait returns without touching the device: the counters and the first `want`
// records in the slot's pinned buffer.  stage_prepare sizes the buffer (before the batch's last
// kernel, which may write it directly: `*zero_copy`); stage_results copies what that kernel did not
// write and records `done`.
constexpr uint64_t ZERO_COPY_MAX = 4ull << 20;  // larger result sets go by DMA copy
static int stage_prepare(bw_ctx* c, Slot& s, uint64_t max_blobs, uint64_t* want_out, bool* zero_copy) {
    const uint64_t want = std::min<uint64_t>(max_blobs, std::max<uint64_t>(1024, 2 * c->last_n + 1024));
    if (s.res.cap < C_COUNT * 8 + want * sizeof(bw_blob)) {
        HIPCHK(c, hipEventSynchronize(s.done));  // the buffer may still be the target of the slot's last copy
        if (int rc = ensure_host(c, s.res, C_COUNT * 8 + want * sizeof(bw_blob))) return rc;
    }
    *want_out = want;
    if (zero_copy) *zero_copy = CTR_BYTES + want * sizeof(bw_blob) <= ZERO_COPY_MAX;
    return BW_OK;
}

int stage_results(bw_ctx* c, Slot& s, bool written, uint64_t want, hipStream_t st) {
    if (!st) st = c->stream;
    if (!written) {
        if (int rc = stage_prepare(c, s, s.max_blobs, &want, nullptr)) return rc;
        // one copy: the counters and the first `want` records lie back to back on the device (two
        // copies cost the stream a ~12 us gap between them with one batch in flight, profiles/r03)
        HIPCHK(c, hipMemcpyAsync(s.res.p, s.res_dev.p, CTR_BYTES + want * sizeof(bw_blob), hipMemcpyDeviceToHost,
                                 st));
    }
    HIPCHK(c, hipEventRecord(s.done, st));
    s.res_n = want;
    return BW_OK;
}

// Enqueue one batch (bytes at d_data, in HBM) into slot `s` on the context stream.
static int submit(bw_ctx* c, Slot& s, const uint8_t* d_data, uint64_t data_len, const uint64_t* foff,
                  const uint64_t* flen, uint64_t nf, const bw_params* prm, bool stage = true, bool order_force = false) {
    Masks mk;
    if (int rc = validate_batch(c, data_len, foff, flen, nf, prm, &mk)) return rc;
    if (data_len && !d_data) return BW_EINVAL;
    if (((uintptr_t)d_data & 15) != 0) {
        c->err = "device data pointer must be 16-byte aligned";
        return BW_EINVAL;
    }
    hipSetDevice(c->device);
    auto clk = [] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    double t_mark = c->host_timing ? clk() : 0;
    auto phase = [&](int k) {
        if (!c->host_timing) return;
        const double t = clk();
        c->host_ms[k] += t - t_mark;
        t_mark = t;
    };
    const bool force_serial = (prm->flags & BW_F_SERIAL_RESOLVE) != 0;
    const bool do_hash = !(prm->flags & BW_F_NO_HASH);
    const bool do_dedup = do_hash && !(prm->flags & BW_F_NO_DEDUP);

    // ---- the scan's tiles and buffers
    // CDC files and the blob bound (the same bound as the tables below give): the result buffer
    // holds the counters the scan writes, so it is sized before the scan is enqueued
    uint64_t ncf_pre = 0, mb_pre = 0;
    {
        const uint64_t mc = std::min<uint64_t>(mk.s0, mk.max);
        for (uint64_t f = 0; f < nf; f++) {
            const bool cdc = flen[f] > prm->small_file_threshold && flen[f] > 0;
            ncf_pre += cdc;
            mb_pre += cdc ? flen[f] / mc + 2 : 1;
        }
    }
    // small batches scan half-size tiles: with one 128 KiB tile per wave the per-tile start
    // costs dominate (C1: 0.50 -> 0.33 ms per GiB); large ones keep the longer strips
    // (BW_OPT_SCAN_SMALL_BYTES moves the threshold, so the tests can run either tile size on any input)
    mk.tile_shift = data_len < c->scan_small_bytes ? SCAN_TILE_SHIFT - 1 : SCAN_TILE_SHIFT;
    const uint64_t tile_bytes = 1ull << mk.tile_shift;
    const uint64_t n_tiles = ncf_pre ? (data_len + tile_bytes - 1) / tile_bytes : 0;
    {
        int rc0 = 0;
        rc0 |= ensure(c, c->tile_count, n_tiles * 4);
        rc0 |= ensure(c, c->tile_slots, n_tiles * SCAN_CAP * 8);
        rc0 |= ensure(c, c->ovf, n_tiles * 4);
        rc0 |= ensure(c, s.res_dev, CTR_BYTES + mb_pre * sizeof(bw_blob));
        if (rc0) return BW_ENOMEM;
    }
    // ---- the gear scan: counters zeroed, then the scan; it reads only the batch bytes and the
    // tile buffers above
    auto enqueue_scan = [&]() -> int {
        // (a kernel of ours: after hipMemsetAsync's fill the scan started ~5.4 us later)
        launch_zero(c->stream, slot_ctr(s), C_COUNT);
        if (c->prof) {
            c->ev_set ^= 1;
            prof_collect(c, c->ev_set);  // the set about to be reused belongs to batch k-2
        }
        prof_mark(c, BW_STAGE_SCAN);
        if (!ncf_pre) return BW_OK;
        bw_index* x = c->idx;
        std::unique_lock<std::mutex> lk(x->mu, std::defer_lock);
        if (c->order_hash || order_force) {
            lk.lock();
            if (x->scan_tail_set) HIPCHK(c, hipStreamWaitEvent(c->stream, x->scan_tail, 0));
        }
        if (!launch_scan(c->stream, d_data, data_len, n_tiles, mk, P<uint32_t>(c->tile_count),
                         P<uint64_t>(c->tile_slots), P<uint32_t>(c->ovf), slot_ctr(s), c->scan_waves)) {
            c->err = "no scan kernel for tile size 2^" + std::to_string(mk.tile_shift);
            return BW_EINVAL;
        }
        if (c->order_hash || order_force) {
            HIPCHK(c, hipEventRecord(x->scan_tail, c->stream));
            x->scan_tail_set = true;
        }
        return BW_OK;
    };
    // Small batches enqueue it before the host tables, so the GPU starts while the host builds
    // them (one batch in flight: the host's share of a 1 GiB batch sits on the critical path).
    // Large ones keep it behind the upload: enqueued first, it made C3's two contexts fall into a
    // slower phase in one run of two (1,647 vs 1,871 GB/s; profiles/r02/s31_reorder).
    const bool scan_first = c->scan_first == 2 ? data_len < c->scan_small_bytes : c->scan_first == 1;
    if (scan_first)
        if (int r6 = enqueue_scan()) return r6;

    // ---- host metadata: CDC files, segments, canonical units
    const uint64_t L = seg_len_for(mk, data_len < c->scan_small_bytes);
    // every chunk but a file's last is >= min(2*(min/2), max) bytes (max < min is legal in the crate)
    const uint64_t min_chunk = std::min<uint64_t>(mk.s0, mk.max);
    // Two passes over file ranges (in parallel for large batches: C4's million files took ~4 ms on
    // one thread): count each range's segments, CDC files, units and bounds, then fill the tables
    // at the ranges' prefix offsets.  The tables are the same as one serial walk in file order.
    struct Part {
        uint64_t nseg = 0, ncf = 0, nunits = 0, fb = 0, max_blobs = 0, total_len = 0, max_blob_len = 0;
    };
    const uint64_t T = nf >= 65536 ? 64 : 1;
    std::vector<Part> part(T), base(T);
    auto is_cdc = [&](uint64_t f) { return flen[f] > prm->small_file_threshold && flen[f] > 0; };
    parallel_ranges(T, [&](uint64_t k0, uint64_t k1) {
        for (uint64_t k = k0; k < k1; k++) {
            Part& q = part[k];
            for (uint64_t f = nf * k / T; f < nf * (k + 1) / T; f++) {
                q.total_len += flen[f];
                if (is_cdc(f)) {
                    const uint64_t ns = (flen[f] + L - 1) / L, nb = flen[f] / min_chunk + 2;
                    q.nseg += ns;
                    q.nunits += ns;
                    q.ncf++;
                    q.fb += nb;
                    q.max_blobs += nb;
                } else {
                    q.nunits++;
                    q.max_blobs++;
                    q.max_blob_len = std::max<uint64_t>(q.max_blob_len, flen[f]);
                }
            }
        }
    }, nf);
    Part tot;
    // a CDC chunk is <= max, or <= min where cut() returns a remainder <= min whole before clipping
    // to max (min > max is legal in the crate; round-6 fuzz: a 70,325 B chunk under max = 1,520)
    tot.max_blob_len = std::max<uint64_t>(mk.max, mk.min);
    for (uint64_t k = 0; k < T; k++) {
        base[k] = tot;
        tot.nseg += part[k].nseg;
        tot.ncf += part[k].ncf;
        tot.nunits += part[k].nunits;
        tot.fb += part[k].fb;
        tot.max_blobs += part[k].max_blobs;
        tot.total_len += part[k].total_len;
        tot.max_blob_len = std::max(tot.max_blob_len, part[k].max_blob_len);
    }
    // the tables are written straight into the slot's pinned staging, from which they are uploaded
    // (a million files' 40 MB of tables were a vector build plus one serial memcpy before)
    const uint64_t nseg = tot.nseg, ncf = tot.ncf, nunits = tot.nunits;
    const size_t meta_bytes = nseg * sizeof(SegDesc) + ncf * sizeof(CFileDesc) + nunits * sizeof(UnitDesc) + nf * 8;
    if (s.meta_pending) {
        hipEventSynchronize(s.meta_on_done ? s.done : s.meta_done);
        s.meta_pending = false;
    }
    if (int r3 = ensure_host(c, s.meta, meta_bytes + 64)) return r3;
    SegDesc* segs = (SegDesc*)s.meta.p;
    CFileDesc* cfs = (CFileDesc*)(segs + nseg);
    UnitDesc* units = (UnitDesc*)(cfs + ncf);
    uint64_t* fstart_h = (uint64_t*)(units + nunits);
    static_assert(sizeof(SegDesc) % 8 == 0 && sizeof(CFileDesc) % 8 == 0 && sizeof(UnitDesc) % 8 == 0, "staging alignment");
    parallel_ranges(T, [&](uint64_t k0, uint64_t k1) {
        for (uint64_t k = k0; k < k1; k++) {
            uint64_t si = base[k].nseg, ci = base[k].ncf, ui = base[k].nunits, fb = base[k].fb;
            const uint64_t f0 = nf * k / T, f1 = nf * (k + 1) / T;
            if (f1 > f0) memcpy(fstart_h + f0, foff + f0, (f1 - f0) * 8);
            for (uint64_t f = f0; f < f1; f++) {
                if (is_cdc(f)) {
                    CFileDesc cf;
                    cf.start = foff[f];
                    cf.end = foff[f] + flen[f];
                    cf.fb_off = fb;
                    cf.first_seg = (uint32_t)si;
                    const uint64_t ns = (flen[f] + L - 1) / L;
                    cf.nseg = (uint32_t)ns;
                    for (uint64_t j = 0; j < ns; j++) {
                        SegDesc sd;
                        sd.start = cf.start + j * L;
                        sd.end = std::min(cf.start + (j + 1) * L, cf.end);
                        sd.file_end = cf.end;
                        sd.cfile = (uint32_t)ci;
                        sd.last = j + 1 == ns;
                        UnitDesc u;
                        u.start = 0;
                        u.len = 0;
                        u.file = (uint32_t)f;
                        u.kind = 1;
                        u.seg = (uint32_t)si;
                        u.cfile = sd.cfile;
                        units[ui++] = u;
                        segs[si++] = sd;
                    }
                    fb += flen[f] / min_chunk + 2;
                    cfs[ci++] = cf;
                } else {
                    UnitDesc u;
                    u.start = foff[f];
                    u.len = flen[f];
                    u.file = (uint32_t)f;
                    u.kind = 0;
                    u.seg = 0;
                    u.cfile = 0;
                    units[ui++] = u;
                }
            }
        }
    }, nf);
    const uint64_t max_blobs = tot.max_blobs, fb_total = tot.fb, max_blob_len = tot.max_blob_len,
                   total_len = tot.total_len;
    // Leaves per BLAKE3 group (one lane each) of the aligned-line leaf pass.  Auto: 2 for small
    // batches (under BW_OPT_SCAN_SMALL_BYTES: the pass's last partial round of waves is a large share
    // of it) and for batches of small blobs (mean blob bound under 128 KiB: fewer lanes idle in a
    // blob's ragged last group); 4 otherwise (the upper levels' extra work is not paid back).
    // Measured (profiles/r03/s05_group): C1 one batch in flight +3 %, C1 three +1.7 %, C4 +9.5 %,
    // C2 -1.3 % with 2.
    const bool small_groups = data_len < c->scan_small_bytes || total_len < max_blobs * (128ull << 10);
    const int grp = c->b3_group ? c->b3_group : (small_groups ? 2 : 4);
    const uint32_t gshift = c->b3_loads != B3_LOADS_LINES ? 2 : (grp == 1 ? 0 : grp == 2 ? 1 : 2);
    const uint64_t max_groups = total_len / (1024ull << gshift) + max_blobs + 1;  // 1 KiB BLAKE3 leaves
    const int max_leaves = (int)std::min<uint64_t>((max_blob_len + 1023) / 1024, 1u << 30);
    if (ncf != ncf_pre || max_blobs != mb_pre) return BW_ESTATE;  // the same sums as the pre-count; cannot differ

    // ---- device buffers
    phase(0);
    int rc = 0;
    rc |= ensure(c, c->tile_off, (n_tiles + 1) * 8);
    rc |= ensure(c, c->tile_btot, (n_tiles / 1024 + 2) * 8);
    rc |= ensure(c, c->meta, meta_bytes);  // segs | cfiles | units | fstart, as staged
    rc |= ensure(c, c->chains, nseg * CHAIN_CAP * 8);
    rc |= ensure(c, c->chain_n, nseg * 4);
    rc |= ensure(c, c->chain_cptr, nseg * 8);
    rc |= ensure(c, c->merge, nseg * 8);
    rc |= ensure(c, c->seg_M, nseg * 8);
    rc |= ensure(c, c->seg_cnt, nseg * 4);
    rc |= ensure(c, c->cf_invalid, ncf * 4);
    rc |= ensure(c, c->fb_starts, fb_total * 8);
    rc |= ensure(c, c->fb_count, ncf * 8);
    rc |= ensure(c, c->b_start, max_blobs * 8);
    rc |= ensure(c, c->b_len, max_blobs * 8);
    rc |= ensure(c, c->b_goff, max_blobs * 8);
    rc |= ensure(c, c->b_file, max_blobs * 4);
    rc |= ensure(c, c->b_kind, max_blobs * 4);
    rc |= ensure(c, c->b_fend, max_blobs * 8);
    rc |= ensure(c, c->b_ghash, max_blobs * 8);
    if (c->b_gdone.cap < max_blobs * 4) {  // the passes leave it zeroed; a new buffer starts so
        rc |= ensure(c, c->b_gdone, max_blobs * 4);
        if (!rc) HIPCHK(c, hipMemsetAsync(c->b_gdone.p, 0, c->b_gdone.cap, c->stream));
    }
    rc |= ensure(c, c->cv, max_groups * 32);
    rc |= ensure(c, c->cv2, max_leaves > 64 ? max_groups * 32 : 16);
    rc |= ensure(c, s.digests, max_blobs * 32);
    rc |= ensure(c, s.is_dup, max_blobs);
    rc |= ensure(c, c->ucnt, 2 * nunits * 8);
    rc |= ensure(c, c->ubtot, 2 * (nunits / 256 + 2) * 8);
    if (rc) return BW_ENOMEM;
    // candidate array: 4x the expected count (2^-popcount(mask) per byte) plus slack.  A batch that
    // finds more stays exact (the walkers test the bytes past the array's end, C_TRUNC) and the
    // next batch gets the room it would have needed.
    uint64_t cand_cap = 16;
    if (ncf) {
        const int bits = __builtin_popcountll(mk.mask_pre);
        cand_cap = 4 * (data_len >> bits) + 2 * n_tiles + 4096;
        cand_cap = std::max(cand_cap, c->cand_override);
        if (c->cand_cap_forced) cand_cap = c->cand_cap_forced;
    }
    if (int r2 = ensure(c, c->cand, cand_cap * 8)) return r2;

    // ---- metadata upload through the slot's pinned staging
    phase(1);
    auto up = [&](DevBuf& dst, const void* src, size_t bytes) -> hipError_t {
        return bytes ? hipMemcpyAsync(dst.p, src, bytes, hipMemcpyHostToDevice, c->stream) : hipSuccess;
    };
    // one copy: the tables lie back to back in the staging and keep that layout on the device.
    // Up to 1 MiB a kernel reads them over PCIe (no copy-engine round trip on the stream); more
    // (C4's million units, ~40 MB) go by DMA.
    if (meta_bytes <= (1u << 20)) launch_upload(c->stream, segs, c->meta.p, meta_bytes);
    else HIPCHK(c, up(c->meta, segs, meta_bytes));
    SegDesc* d_segs = P<SegDesc>(c->meta);
    CFileDesc* d_cfs = (CFileDesc*)(d_segs + nseg);
    UnitDesc* d_units = (UnitDesc*)(d_cfs + ncf);
    uint64_t* d_fstart = (uint64_t*)(d_units + nunits);
    // The staging is refilled when the slot comes round again, `depth` batches later: for a staged
    // batch of a context that keeps two or more, the batch's own end (`done`) covers the upload, so
    // no event goes between the upload and the next kernel (each costs the stream ~5.5 us)
    s.meta_on_done = stage && c->depth >= 2;
    if (!s.meta_on_done) HIPCHK(c, hipEventRecord(s.meta_done, c->stream));
    s.meta_pending = true;
    phase(2);

    if (!scan_first)
        if (int r6 = enqueue_scan()) return r6;
    uint64_t* ctr = slot_ctr(s);
    hipStream_t st = c->stream;

    BlobArrays b{P<uint64_t>(c->b_start), P<uint64_t>(c->b_len), P<uint64_t>(c->b_goff), P<uint32_t>(c->b_file),
                 P<uint32_t>(c->b_kind), P<uint64_t>(c->b_fend), P<uint64_t>(c->b_ghash), max_blobs, data_len,
                 c->b3_fused ? P<uint32_t>(c->b_gdone) : nullptr, gshift};

    // ---- chunking (the scan on the context stream, the latency-bound kernels after it on `lat`)
    const bool split = c->lat_split;
    hipStream_t lat = split ? c->hi : st;
    if (split) {
        HIPCHK(c, hipEventRecord(c->e_scan, st));
        HIPCHK(c, hipStreamWaitEvent(lat, c->e_scan, 0));
    }
    prof_mark(c, BW_STAGE_COMPACT, lat);
    if (ncf)
        launch_compact(lat, d_data, data_len, n_tiles, mk, P<uint32_t>(c->tile_count), P<uint64_t>(c->tile_slots),
                       P<uint64_t>(c->tile_off), P<uint64_t>(c->cand), cand_cap, P<uint32_t>(c->ovf), ctr,
                       P<uint64_t>(c->tile_btot));
    prof_mark(c, BW_STAGE_RESOLVE, lat);
    if (ncf) {
        launch_chains(lat, d_data, data_len, mk, P<uint64_t>(c->cand), P<uint64_t>(c->tile_off), ctr, d_segs,
                      nseg, P<uint64_t>(c->chains), P<uint32_t>(c->chain_n), P<uint64_t>(c->chain_cptr),
                      P<uint64_t>(c->merge), force_serial);
        launch_resolve(lat, d_data, data_len, mk, P<uint64_t>(c->cand), P<uint64_t>(c->tile_off), ctr,
                       d_segs, nseg, d_cfs, ncf, P<uint64_t>(c->chains),
                       P<uint32_t>(c->chain_n), P<uint64_t>(c->merge), P<uint64_t>(c->seg_M), P<uint32_t>(c->seg_cnt),
                       P<uint32_t>(c->cf_invalid), P<uint64_t>(c->fb_starts), P<uint64_t>(c->fb_count), force_serial);
    }
    prof_mark(c, BW_STAGE_ASSEMBLE, lat);
    launch_assemble(lat, ctr, d_units, nunits, d_segs, d_cfs,
                    P<uint64_t>(c->chains), P<uint32_t>(c->chain_n), P<uint64_t>(c->seg_M), P<uint32_t>(c->cf_invalid),
                    P<uint64_t>(c->fb_starts), P<uint64_t>(c->fb_count), b, P<uint64_t>(c->ucnt),
                    P<uint64_t>(c->ubtot));
    // Chunk.hash: one wave per chunk (a thread-serial version inside k_unit_emit made C1's
    // assembly 0.03 -> 0.31 ms: 64 dependent byte loads per chunk)
    if (ncf) launch_cut_hash(lat, d_data, mk, ctr, b, max_blobs);
    else HIPCHK(c, hipMemsetAsync(c->b_ghash.p, 0, max_blobs * 8, lat));
    if (split) {
        HIPCHK(c, hipEventRecord(c->e_lat, lat));
        HIPCHK(c, hipStreamWaitEvent(st, c->e_lat, 0));
    }

    // ---- hashing (the leaf pass on the context stream, the upper levels on lat) + dedup on lat
    prof_mark(c, BW_STAGE_B3LEAF, st);
    if (do_hash) {
        // the B3TREE stage mark (timing only) and the event that orders the upper levels' stream
        // after the leaf pass (split latency stream) are separate events
        hipEvent_t mark = c->prof && ((c->prof_mask >> BW_STAGE_B3TREE) & 1) ? c->ev[c->ev_set][BW_STAGE_B3TREE] : nullptr;
        hipEvent_t between = split ? c->e_b3 : nullptr;
        bw_index* x = c->idx;
        std::unique_lock<std::mutex> lk(x->mu, std::defer_lock);
        const bool order = c->order_hash || order_force;
        if (order) {
            lk.lock();
            if (x->hash_tail_set) HIPCHK(c, hipStreamWaitEvent(st, x->hash_tail, 0));
        }
        launch_blake3(st, d_data, ctr, b, max_blobs, max_groups, P<uint32_t>(c->cv), P<uint32_t>(c->cv2),
                      P<uint8_t>(s.digests), max_leaves, between, c->b3_loads, lat, order ? x->hash_tail : nullptr, mark);
        if (order) x->hash_tail_set = true;
    } else {
        prof_mark(c, BW_STAGE_B3TREE, st);
        if (split) {
            HIPCHK(c, hipEventRecord(c->e_b3, st));
            HIPCHK(c, hipStreamWaitEvent(lat, c->e_b3, 0));
        }
        HIPCHK(c, hipMemsetAsync(s.digests.p, 0, max_blobs * 32, lat));
    }
    // no kernel of this batch reads d_data after here; only the slot's own input buffer (host
    // batches, stream_in) is ever refilled behind this event
    if (d_data == P<uint8_t>(s.input)) HIPCHK(c, hipEventRecord(s.input_free, st));
    phase(3);
    prof_mark(c, BW_STAGE_DEDUP, lat);
    // small result sets are written to the slot's pinned buffer by k_pack itself (no copy on the
    // stream: pack -> copy cost a 12 us gap with one batch in flight, profiles/r03/s07_upper_block)
    uint64_t want = 0;
    bool zero_copy = false;
    if (stage)
        if (int r5 = stage_prepare(c, s, max_blobs, &want, &zero_copy)) return r5;
    auto pack = [&](hipStream_t ps) {
        prof_mark(c, BW_STAGE_PACK, ps);
        launch_pack(ps, ctr, b, d_fstart, P<uint8_t>(s.digests), do_dedup ? P<uint8_t>(s.is_dup) : nullptr,
                    slot_records(s), max_blobs, do_dedup ? P<uint64_t>(c->idx->dstate) : nullptr,
                    zero_copy ? (uint8_t*)s.res.p : nullptr, want);
    };
    if (do_dedup) {  // the pack runs inside the index operation (before its tail event)
        if (int r4 = dedup_device(c, P<uint8_t>(s.digests), ctr + C_DEDUPN, 0, max_blobs, P<uint8_t>(s.is_dup), lat,
                                  pack))
            return r4;
        s.mark = c->idx_mark;
    } else {
        pack(lat);
    }
    phase(4);
    if (split) {  // the batch ends on the context stream (the caller's order)
        prof_mark(c, BW_N_STAGES, lat);
        HIPCHK(c, hipEventRecord(c->e_end, lat));
        HIPCHK(c, hipStreamWaitEvent(st, c->e_end, 0));
    }
    if (!split) prof_mark(c, BW_N_STAGES);
    if (c->prof) c->ev_pending[c->ev_set] = true;
    HIPCHK(c, hipGetLastError());
    s.max_blobs = max_blobs;
    s.dedup = do_dedup;
    s.hashed = do_hash;
    s.comm = nullptr;
    s.ex_state = 0;
    s.ex_rc = 0;
    s.ex_first = 0;
    s.ex_n = ~0ull;
    if (stage)
        if (int r5 = stage_results(c, s, zero_copy, want)) return r5;
    phase(5);
    c->host_batches += c->host_timing;
    return BW_OK;
}

// Claim the next slot of the ring (the batch it held, if any, is dropped) and give it a ticket.
// A dropped batch whose exchange is still queued is finished first, and the new batch's kernels
// wait for the exchange's transfers, gate and scatter on ex_st (they use the slot's buffers).
static Slot& claim_slot(bw_ctx* c, uint64_t* ticket) {
    const uint64_t t = c->next_ticket++;
    Slot& s = c->slots[(t - 1) % (uint64_t)c->depth];
    if (s.ex_state == 1 && s.comm) exchange_progress(s.comm, &s);
    if (s.ex_state == 2) hipStreamWaitEvent(c->stream, s.done, 0);
    s.ticket = t;
    c->last_ticket = t;
    if (ticket) *ticket = t;
    return s;
}

static const bw_params* params_or_default(const bw_params* prm, bw_params* def) {
    if (prm) return prm;
    bw_params_default(def);
    return def;
}

// The helper context of BW_OPT_SPLIT: same device, index and kernel options, its own stream.
static int ensure_helper(bw_ctx* c) {
    if (c->helper) return BW_OK;
    bw_ctx* h = nullptr;
    if (int rc = bw_create(c->device, &h)) return rc;
    h->is_helper = true;
    h->depth = c->depth;
    h->scan_small_bytes = c->scan_small_bytes;
    h->cand_cap_forced = c->cand_cap_forced;
    // every per-context kernel and profiling option (the tail parts ran with defaults)
    h->b3_loads = c->b3_loads;
    h->scan_waves = c->scan_waves;
    h->b3_group = c->b3_group;
    h->b3_fused = c->b3_fused;
    h->prof_mask = c->prof_mask;
    h->scan_first = c->scan_first;
    if (c->lat_split && bw_set_option(h, BW_OPT_LATENCY_STREAM, 1) != BW_OK) {
        bw_destroy(h);
        return BW_EHIP;
    }
    if (int rc = bw_attach_index(h, c->idx)) {
        bw_destroy(h);
        return rc;
    }
    if (c->prof) bw_profile_enable(h, 1);
    if (!c->e_split) HIPCHK(c, hipEventCreateWithFlags(&c->e_split, EV_ORDER));
    if (!c->e_tail) HIPCHK(c, hipEventCreateWithFlags(&c->e_tail, EV_ORDER));
    c->helper = h;
    return BW_OK;
}

// First file of the tail part, or 0 = do not split.  Splits only batches that gate through the
// index (a NO_DEDUP batch's device views feed the multi-GPU exchange whole), hold at least two
// files, and are large enough to amortise the second submission but small enough that one batch
// in flight leaves the scan and BLAKE3 passes apart (large batches fill the chip either way).
static uint64_t split_point(bw_ctx* c, uint64_t data_len, const uint64_t* flen, uint64_t nf, const bw_params* prm) {
    if (c->split < 2 || c->is_helper || nf < 2 || (prm->flags & (BW_F_NO_DEDUP | BW_F_NO_HASH))) return 0;
    if (data_len > c->split_max) return 0;
    uint64_t total = 0;
    for (uint64_t f = 0; f < nf; f++) total += flen[f];
    if (total < c->split_min) return 0;
    uint64_t acc = 0;
    for (uint64_t f = 0; f + 1 < nf; f++) {  // the head ends at the first file that reaches half the bytes
        acc += flen[f];
        if (2 * acc >= total) return f + 1;
    }
    return nf - 1;
}

// Submit into slot s of c, split into a head (here) and a tail (c's helper) when split_point says
// so.  d_data is already ordered on c's stream (caller data, or the slot's input after stream_in).
static int submit_split(bw_ctx* c, Slot& s, const uint8_t* d_data, uint64_t data_len, const uint64_t* foff,
                        const uint64_t* flen, uint64_t nf, const bw_params* prm) {
    s.tail_ticket = 0;
    Masks mk;
    if (int rc = validate_batch(c, data_len, foff, flen, nf, prm, &mk)) return rc;
    const uint64_t f0 = split_point(c, data_len, flen, nf, prm);
    if (!f0) return submit(c, s, d_data, data_len, foff, flen, nf, prm);
    if (int rc = ensure_helper(c)) return rc;
    bw_ctx* h = c->helper;
    HIPCHK(c, hipEventRecord(c->e_split, c->stream));  // the tail sees what the caller ordered before
    if (int rc = submit(c, s, d_data, data_len, foff, flen, f0, prm, true, true)) return rc;
    HIPCHK(c, hipStreamWaitEvent(h->stream, c->e_split, 0));
    uint64_t t2 = 0;
    Slot& s2 = claim_slot(h, &t2);
    if (int rc = submit(h, s2, d_data, data_len, foff + f0, flen + f0, nf - f0, prm, true, true)) {
        s2.ticket = 0;
        c->err = "tail part: " + h->err;
        return rc;
    }
    // the batch ends on c's stream once both parts have (the caller's order, and the slot's input
    // is free only after the tail's BLAKE3 read it too)
    HIPCHK(c, hipEventRecord(c->e_tail, h->stream));
    HIPCHK(c, hipStreamWaitEvent(c->stream, c->e_tail, 0));
    if (d_data == P<uint8_t>(s.input)) HIPCHK(c, hipEventRecord(s.input_free, c->stream));
    s.tail_ticket = t2;
    s.tail_file0 = f0;
    return BW_OK;
}

extern "C" int bw_submit_device(bw_ctx* c, const uint8_t* d_data, uint64_t data_len, const uint64_t* foff,
                                const uint64_t* flen, uint64_t nf, const bw_params* prm, uint64_t* ticket) {
    if (!c) return BW_EINVAL;
    if (ticket) *ticket = 0;
    bw_params def;
    prm = params_or_default(prm, &def);
    hipSetDevice(c->device);
    Slot& s = claim_slot(c, ticket);
    if (int rc = submit_split(c, s, d_data, data_len, foff, flen, nf, prm)) {
        s.ticket = 0;
        if (ticket) *ticket = 0;
        return rc;
    }
    return BW_OK;
}

extern "C" int bw_process_files_device(bw_ctx* c, const uint8_t* d_data, uint64_t data_len, const uint64_t* foff,
                                       const uint64_t* flen, uint64_t nf, const bw_params* prm) {
    return bw_submit_device(c, d_data, data_len, foff, flen, nf, prm, nullptr);
}

static bool is_pinned(const void* p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();  // pageable memory: clear the sticky error
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

// H2D of a host batch into s.input on the copy stream (ordered after the slot's previous batch
// stopped reading that buffer); the compute stream then waits for it.  Pinned or registered
// memory is DMA'd directly; pageable memory is copied chunk by chunk into a ring of pinned
// staging buffers (16 host threads per chunk) while the previous chunks are in flight.
static int stream_in(bw_ctx* c, Slot& s, const uint8_t* data, uint64_t len) {
    if (!c->copy) HIPCHK(c, hipStreamCreateWithFlags(&c->copy, hipStreamNonBlocking));
    if (int rc = ensure(c, s.input, len + 64)) return rc;
    if (s.input_used) HIPCHK(c, hipStreamWaitEvent(c->copy, s.input_free, 0));
    uint8_t* dst = P<uint8_t>(s.input);
    if (len && is_pinned(data)) {
        HIPCHK(c, hipMemcpyAsync(dst, data, len, hipMemcpyHostToDevice, c->copy));
    } else {
        for (uint64_t off = 0, k = 0; off < len; off += c->stage_chunk, k++) {
            const int r = (int)(k % STAGE_RING);
            const uint64_t n = std::min<uint64_t>(c->stage_chunk, len - off);
            if (!c->ring_ev[r]) HIPCHK(c, hipEventCreateWithFlags(&c->ring_ev[r], hipEventDisableTiming));
            if (c->ring_set[r]) HIPCHK(c, hipEventSynchronize(c->ring_ev[r]));
            if (int rc = ensure_host(c, c->ring[r], c->stage_chunk)) return rc;
            uint8_t* pin = (uint8_t*)c->ring[r].p;
            parallel_ranges(
                n, [&](uint64_t lo, uint64_t hi) { memcpy(pin + lo, data + off + lo, hi - lo); }, n / 16);
            HIPCHK(c, hipMemcpyAsync(dst + off, pin, n, hipMemcpyHostToDevice, c->copy));
            HIPCHK(c, hipEventRecord(c->ring_ev[r], c->copy));
            c->ring_set[r] = true;
        }
    }
    HIPCHK(c, hipEventRecord(s.copied, c->copy));
    HIPCHK(c, hipStreamWaitEvent(c->stream, s.copied, 0));
    s.input_used = true;
    return BW_OK;
}

extern "C" int bw_submit_host(bw_ctx* c, const uint8_t* data, uint64_t data_len, const uint64_t* foff,
                              const uint64_t* flen, uint64_t nf, const bw_params* prm, uint64_t* ticket) {
    if (!c || (data_len && !data)) return BW_EINVAL;
    if (ticket) *ticket = 0;
    bw_params def;
    prm = params_or_default(prm, &def);
    Masks mk;
    if (int rc = validate_batch(c, data_len, foff, flen, nf, prm, &mk)) return rc;
    hipSetDevice(c->device);
    Slot& s = claim_slot(c, ticket);
    int rc = stream_in(c, s, data, data_len);
    if (!rc) rc = submit_split(c, s, P<uint8_t>(s.input), data_len, foff, flen, nf, prm);
    if (rc) {
        s.ticket = 0;
        if (ticket) *ticket = 0;
    }
    return rc;
}

extern "C" int bw_host_register(void* p, uint64_t len) {
    if (!p || !len) return BW_EINVAL;
    return hipHostRegister(p, len, hipHostRegisterDefault) == hipSuccess ? BW_OK : BW_EHIP;
}

extern "C" int bw_host_unregister(void* p) {
    if (!p) return BW_EINVAL;
    return hipHostUnregister(p) == hipSuccess ? BW_OK : BW_EHIP;
}

// Results of the batch in slot s (waits for it).  Repeatable until the ring reuses the slot.
static int slot_results(bw_ctx* c, Slot& s, bw_blob* out, uint64_t cap, uint64_t* n_out) {
    hipSetDevice(c->device);
    if (s.ex_state == 1)  // queued exchange: its counts first, then its transfers are enqueued
        if (int rc = exchange_progress(s.comm, &s)) return rc;
    if (s.ex_state == 3) return s.ex_rc ? s.ex_rc : BW_ECOMM;
    if (s.comm) {  // an exchange in flight: a failed or stalled peer must not hang the wait
        if (int rc = comm_wait_event(s.comm, s.done, c->err)) return rc;
    } else {
        HIPCHK(c, hipEventSynchronize(s.done));  // the staged counters and records have landed
    }
    const uint64_t* ctr = (const uint64_t*)s.res.p;
    if (ctr[C_CANDTOTAL] > ctr[C_NCAND])  // exact anyway; give later batches the room they need
        c->cand_override = std::max(c->cand_override, ctr[C_CANDTOTAL] + 1024);
    const uint64_t n = ctr[C_NBLOBS];
    *n_out = n;
    c->last_n = n;
    if (s.dedup) {
        if (ctr[C_IX_VALID]) {  // the index state right after this batch's gate
            bw_index* x = c->idx;
            {
                std::lock_guard<std::mutex> lk(x->mu);
                x->log_hi = std::min(x->log_hi, ctr[C_IX_LOGLEN] + (x->enq_total - std::min(x->enq_total, s.mark)));
            }
            if (ctr[C_LOST]) {
                c->err = "index lookup found no slot (internal error)";
                return BW_EHIP;
            }
            if (ctr[C_IX_OVF]) {
                c->err = "a batch had more blobs than its exchange bucket capacity (verdicts incomplete)";
                return BW_ENOSPC;
            }
        } else if (int rc = check_collision(c)) {
            return rc;
        }
    }
    if (n > cap) return BW_ENOSPC;
    if (n && out) {
        const uint64_t k = std::min(n, s.res_n);
        memcpy(out, (const uint8_t*)s.res.p + C_COUNT * 8, k * sizeof(bw_blob));
        if (n > k)  // more blobs than staged: the rest straight from the device
            HIPCHK(c, hipMemcpy(out + k, slot_records(s) + k * sizeof(bw_blob), (n - k) * sizeof(bw_blob),
                                hipMemcpyDeviceToHost));
    }
    return BW_OK;
}

// Results of a batch that may have been split: the head's blobs, then the tail's with their file
// indices shifted back to the batch's numbering.
static int batch_results(bw_ctx* c, Slot& s, bw_blob* out, uint64_t cap, uint64_t* n_out) {
    if (!s.tail_ticket) return slot_results(c, s, out, cap, n_out);
    Slot* t = c->helper ? slot_of(c->helper, s.tail_ticket) : nullptr;
    if (!t) {
        c->err = "the batch's tail part is no longer held by the helper context";
        return BW_ESTATE;
    }
    uint64_t na = 0, nb = 0;  // the parts' counts first (no copy, no capacity limit)
    if (int rc = slot_results(c, s, nullptr, ~0ull, &na)) return rc;
    if (int rc = slot_results(c->helper, *t, nullptr, ~0ull, &nb)) {
        c->err = "tail part: " + c->helper->err;
        return rc;
    }
    *n_out = na + nb;
    c->last_n = na + nb;
    if (na + nb > cap) return BW_ENOSPC;
    if (!out) return BW_OK;
    if (int rc = slot_results(c, s, out, na, &na)) return rc;
    if (int rc = slot_results(c->helper, *t, out + na, nb, &nb)) return rc;
    for (uint64_t i = 0; i < nb; i++) out[na + i].file += s.tail_file0;
    return BW_OK;
}

extern "C" int bw_wait(bw_ctx* c, uint64_t ticket, bw_blob* out, uint64_t cap, uint64_t* n_out) {
    if (!c || !n_out) return BW_EINVAL;
    Slot* s = slot_of(c, ticket);
    if (!s) {
        c->err = "ticket " + std::to_string(ticket) + " is not (or no longer) held by the context";
        return BW_ESTATE;
    }
    return batch_results(c, *s, out, cap, n_out);
}

extern "C" int bw_results(bw_ctx* c, bw_blob* out, uint64_t cap, uint64_t* n_out) {
    if (!c || !n_out) return BW_EINVAL;
    Slot* s = slot_of(c, c->last_ticket);
    if (!s) return BW_ESTATE;
    return batch_results(c, *s, out, cap, n_out);
}

extern "C" int bw_batch_device_views(bw_ctx* c, uint64_t* n_blobs, const uint8_t** d_digests, uint8_t** d_is_dup) {
    if (!c) return BW_EINVAL;
    Slot* s = slot_of(c, c->last_ticket);
    if (!s) return BW_ESTATE;
    if (s->tail_ticket) {
        c->err = "the batch was split in two parts (BW_OPT_SPLIT): no single device view";
        return BW_ESTATE;
    }
    hipSetDevice(c->device);
    uint64_t n = 0;
    HIPCHK(c, hipMemcpyAsync(&n, slot_ctr(*s) + C_NBLOBS, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (n_blobs) *n_blobs = n;
    if (d_digests) *d_digests = P<uint8_t>(s->digests);
    if (d_is_dup) *d_is_dup = P<uint8_t>(s->is_dup);
    return BW_OK;
}

static int upload_data(bw_ctx* c, const uint8_t* data, uint64_t len) {
    if (int rc = ensure(c, c->data, len + 64)) return rc;
    if (len) HIPCHK(c, hipMemcpyAsync(c->data.p, data, len, hipMemcpyHostToDevice, c->stream));
    return BW_OK;
}

// A synchronous helper's batch: bytes already in c->data, enqueued into the context's own slot
// (outside the ticket ring).
static int submit_sync(bw_ctx* c, uint64_t data_len, const uint64_t* foff, const uint64_t* flen, uint64_t nf,
                       const bw_params* prm, bool stage = true) {
    Slot& s = c->sync_slot;
    s.ticket = 0;
    return submit(c, s, P<uint8_t>(c->data), data_len, foff, flen, nf, prm, stage);
}

extern "C" int bw_process_files(bw_ctx* c, const uint8_t* data, uint64_t data_len, const uint64_t* foff,
                                const uint64_t* flen, uint64_t nf, const bw_params* prm, bw_blob* out, uint64_t cap,
                                uint64_t* n_out) {
    if (!c || !n_out || (data_len && !data)) return BW_EINVAL;
    hipSetDevice(c->device);
    bw_params def;
    prm = params_or_default(prm, &def);
    if (int rc = upload_data(c, data, data_len)) return rc;
    if (int rc = submit_sync(c, data_len, foff, flen, nf, prm)) return rc;
    return slot_results(c, c->sync_slot, out, cap, n_out);
}

extern "C" int bw_fastcdc_chunks(bw_ctx* c, const uint8_t* src, uint64_t len, uint32_t mn, uint32_t av, uint32_t mx,
                                 bw_chunk* out, uint64_t cap, uint64_t* n_out) {
    if (!c || !n_out || (len && !src)) return BW_EINVAL;
    Masks mk;
    if (int rc = make_masks(mn, av, mx, &mk)) return rc;
    *n_out = 0;
    if (len == 0) return BW_OK;  // the iterator yields nothing for an empty source
    bw_params p;
    p.min_size = mn;
    p.avg_size = av;
    p.max_size = mx;
    p.flags = BW_F_NO_HASH;
    p.small_file_threshold = 0;
    const uint64_t off = 0;
    std::vector<bw_blob> tmp(len / std::min<uint64_t>(mk.s0, mk.max) + 2);
    uint64_t n = 0;
    if (int rc = bw_process_files(c, src, len, &off, &len, 1, &p, tmp.data(), tmp.size(), &n)) return rc;
    *n_out = n;
    if (n > cap) return BW_ENOSPC;
    for (uint64_t i = 0; i < n; i++) {
        out[i].hash = tmp[i].gear_hash;
        out[i].offset = tmp[i].offset;
        out[i].length = tmp[i].length;
    }
    return BW_OK;
}

extern "C" int bw_blake3_hash_many(bw_ctx* c, const uint8_t* data, uint64_t data_len, const uint64_t* offsets,
                                   const uint64_t* lengths, uint64_t n, uint8_t* out) {
    if (!c || (n && (!offsets || !lengths || !out))) return BW_EINVAL;
    if (!n) return BW_OK;
    bw_params p;
    bw_params_default(&p);
    p.flags = BW_F_NO_DEDUP;
    p.small_file_threshold = ~0ull;  // every message is one whole blob
    std::vector<bw_blob> tmp(n);
    uint64_t got = 0;
    if (int rc = bw_process_files(c, data, data_len, offsets, lengths, n, &p, tmp.data(), n, &got)) return rc;
    if (got != n) return BW_EHIP;
    for (uint64_t i = 0; i < n; i++) memcpy(out + 32 * i, tmp[i].digest, 32);
    return BW_OK;
}

int bw::ctx_device(const bw_ctx* c) { return c->device; }

int bw::batch_set_exchange_range(bw_ctx* c, uint64_t ticket, uint64_t first, uint64_t n) {
    Slot* s = slot_of(c, ticket);
    if (!s || s->ex_state) return BW_ESTATE;
    s->ex_first = first;
    s->ex_n = n;
    return BW_OK;
}

uint8_t* bw::message_stage(bw_ctx* c, size_t bytes) {
    hipSetDevice(c->device);
    if (c->msg_stage.cap < bytes) {
        hipStreamSynchronize(c->stream);
        if (ensure_host(c, c->msg_stage, bytes)) return nullptr;
    }
    return (uint8_t*)c->msg_stage.p;
}

int bw::hash_messages(bw_ctx* c, const uint8_t* staged, uint64_t total, const uint64_t* offs, const uint64_t* lens,
                      uint64_t n, bool dedup, uint8_t* hashes, uint8_t* dup) {
    if (!n) return BW_OK;
    hipSetDevice(c->device);
    if (int rc = upload_data(c, staged, total)) return rc;
    bw_params p;
    bw_params_default(&p);
    p.flags = dedup ? 0 : BW_F_NO_DEDUP;
    p.small_file_threshold = ~0ull;  // every message is one whole blob, in the order given
    if (int rc = submit_sync(c, total, offs, lens, n, &p, false)) return rc;
    Slot& s = c->sync_slot;
    HIPCHK(c, hipMemcpyAsync(hashes, s.digests.p, n * 32, hipMemcpyDeviceToHost, c->stream));
    if (dedup) HIPCHK(c, hipMemcpyAsync(dup, s.is_dup.p, n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return dedup ? check_collision(c) : BW_OK;
}

// ------------------------------------------------------------------ multi-GPU helpers

extern "C" int bw_partition_by_owner(bw_ctx* c, const uint8_t* d_digests, uint64_t n, uint32_t n_owners,
                                     uint8_t* d_out, uint64_t* d_perm, uint64_t* h_counts) {
    if (!c || !h_counts || n_owners == 0 || n_owners > 256 || (n_owners & (n_owners - 1))) return BW_EINVAL;
    hipSetDevice(c->device);
    if (int rc = ensure(c, c->scratch, 256 * 8)) return rc;
    launch_partition(c->stream, d_digests, n, n_owners, d_out, d_perm, P<uint64_t>(c->scratch));
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(h_counts, c->scratch.p, n_owners * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return BW_OK;
}

extern "C" int bw_batch_views(bw_ctx* c, uint64_t ticket, const uint64_t** d_n_blobs, const uint8_t** d_digests,
                              uint8_t** d_is_dup, uint64_t* max_blobs) {
    if (!c) return BW_EINVAL;
    Slot* s = slot_of(c, ticket ? ticket : c->last_ticket);
    if (!s) return BW_ESTATE;
    if (s->tail_ticket) {
        c->err = "the batch was split in two parts (BW_OPT_SPLIT): no single device view";
        return BW_ESTATE;
    }
    if (d_n_blobs) *d_n_blobs = slot_ctr(*s) + C_NBLOBS;
    if (d_digests) *d_digests = P<uint8_t>(s->digests);
    if (d_is_dup) *d_is_dup = P<uint8_t>(s->is_dup);
    if (max_blobs) *max_blobs = s->max_blobs;
    return BW_OK;
}

static bool owners_ok(uint32_t n) { return n >= 1 && n <= 256 && (n & (n - 1)) == 0; }

extern "C" int bw_partition_buckets(bw_ctx* c, const uint8_t* d_digests, const uint64_t* d_n, uint64_t max_n,
                                    uint64_t cap, uint32_t n_owners, uint8_t* d_buckets, uint64_t* d_perm,
                                    uint64_t* d_counts) {
    if (!c || !d_n || !d_counts || !owners_ok(n_owners) || (cap && (!d_buckets || !d_perm))) return BW_EINVAL;
    if (max_n && !d_digests) return BW_EINVAL;
    hipSetDevice(c->device);
    const uint64_t nblk = (max_n + 4095) / 4096;
    if (int rc = ensure(c, c->bk_blk, (nblk + 1) * n_owners * 8)) return rc;
    launch_bucket_partition(c->stream, d_digests, d_n, max_n, n_owners, cap, d_buckets, d_perm, d_counts,
                            P<uint64_t>(c->bk_blk), P<uint64_t>(c->idx->dstate) + D_BUCKET_OVF);
    HIPCHK(c, hipGetLastError());
    return BW_OK;
}

extern "C" int bw_index_check_insert_buckets(bw_ctx* c, const uint8_t* d_buckets, const uint64_t* d_counts,
                                             uint32_t n_src, uint64_t cap, uint8_t* d_verdicts) {
    if (!c || !d_counts || !n_src || (cap && (!d_buckets || !d_verdicts))) return BW_EINVAL;
    const uint64_t total = (uint64_t)n_src * cap;
    if (!total) return BW_OK;
    hipSetDevice(c->device);
    if (int rc = ensure(c, c->bk_pack, total * 32 + 16)) return rc;
    if (int rc = ensure(c, c->bk_v, total)) return rc;
    uint8_t* pack = P<uint8_t>(c->bk_pack);
    uint64_t* n_dev = (uint64_t*)(pack + total * 32);
    launch_bucket_gather(c->stream, d_buckets, d_counts, n_src, cap, pack, n_dev);
    if (int rc = dedup_device(c, pack, n_dev, 0, total, P<uint8_t>(c->bk_v))) return rc;
    launch_bucket_expand(c->stream, d_counts, n_src, cap, P<uint8_t>(c->bk_v), d_verdicts);
    HIPCHK(c, hipGetLastError());
    return BW_OK;
}

extern "C" int bw_scatter_buckets(bw_ctx* c, const uint8_t* d_verdicts, const uint64_t* d_perm,
                                  const uint64_t* d_counts, uint32_t n_owners, uint64_t cap, uint8_t* d_is_dup) {
    if (!c || !d_counts || !owners_ok(n_owners) || (cap && (!d_verdicts || !d_perm || !d_is_dup))) return BW_EINVAL;
    hipSetDevice(c->device);
    launch_bucket_scatter(c->stream, d_verdicts, d_perm, d_counts, n_owners, cap, d_is_dup);
    HIPCHK(c, hipGetLastError());
    return BW_OK;
}

extern "C" int bw_scatter_verdicts(bw_ctx* c, const uint8_t* d_verdict, const uint64_t* d_perm, uint64_t n,
                                   uint8_t* d_is_dup) {
    if (!c) return BW_EINVAL;
    hipSetDevice(c->device);
    launch_scatter(c->stream, d_verdict, d_perm, n, d_is_dup);
    HIPCHK(c, hipGetLastError());
    return BW_OK;
}

// ---- one batch through the digest-prefix exchange (include/backuwup_gpu.h, bw_exchange_dedup)
// At the call, on the context stream: the batch's digests grouped by owner (owner sections back to
// back) with the per-owner counts, then the counts all-to-all on the communicator's control stream.
// Nothing waits for the peers.  Once the counts are in (exchange_progress, called by every later
// exchange, by bw_wait of an exchanged batch, by claim_slot and by bw_comm_progress), on the
// context's exchange stream: the digests to their owners (every transfer exactly its digests), the
// owner's gate over what it received (source-major = canonical order), the verdicts back, scattered
// into the batch's is_dup and records.  Exchanges finish in issue order, the same on every rank.
namespace {
struct ExPending {
    bw_ctx* c;
    Slot* s;
};
struct ExQueue {
    std::mutex mu;
    std::vector<ExPending> q;  // FIFO (front = index 0)
};

// Created once per communicator under a lock: two contexts exchanging on one
// communicator from two threads must share one FIFO, or the issue order stops being the same on
// every rank.
std::mutex g_exq_create_mu;
ExQueue* exq_of(bw_comm* comm, bool create) {
    std::lock_guard<std::mutex> lk(g_exq_create_mu);
    void*& p = comm_exq(comm);
    if (!p && create) p = new ExQueue();
    return (ExQueue*)p;
}

// The transfers, gate and scatter of one exchange whose counts arrived (ex_h holds them).
int exchange_finish(bw_comm* comm, bw_ctx* c, Slot& s) {
    hipSetDevice(c->device);
    const uint32_t W = (uint32_t)comm_world(comm);
    const uint64_t* h = (const uint64_t*)s.ex_h.p;
    std::vector<uint64_t> scnt(W), rcnt(W);
    uint64_t n = 0, rtot = 0, pad = 0;
    for (uint32_t k = 0; k < W; k++) {
        scnt[k] = h[2 * k];
        rcnt[k] = h[2 * W + 2 * k];
        pad = std::max(pad, h[2 * W + 2 * k + 1]);  // every rank's largest section: the same on all ranks
        n += scnt[k];
        rtot += rcnt[k];
    }
    if (n > (s.ex_n == ~0ull ? s.max_blobs : s.ex_n)) {
        c->err = "exchange counts exceed the batch's blob bound (internal error)";
        return BW_EHIP;
    }
    if (!c->ex_st) HIPCHK(c, hipStreamCreateWithFlags(&c->ex_st, hipStreamNonBlocking));
    hipStream_t st = c->ex_st;
    int rc = 0;
    rc |= ensure(c, c->ex_rbk, rtot * 32);
    rc |= ensure(c, c->ex_v, rtot);
    rc |= ensure(c, c->ex_rv, n);
    if (rc) return BW_ENOMEM;
    HIPCHK(c, hipStreamWaitEvent(st, s.ex_now ? s.ex_part : s.ex_ready, 0));
    if (int r = comm_all_to_allv(comm, s.ex_dig.p, scnt.data(), c->ex_rbk.p, rcnt.data(), 32, pad, st, c->err))
        return r;
    if (rtot)
        if (int r = dedup_device(c, P<uint8_t>(c->ex_rbk), nullptr, rtot, rtot, P<uint8_t>(c->ex_v), st)) return r;
    if (int r = comm_all_to_allv(comm, c->ex_v.p, rcnt.data(), c->ex_rv.p, scnt.data(), 1, pad, st, c->err)) return r;
    const uint64_t first = s.ex_n == ~0ull ? 0 : s.ex_first;  // perm counts from the range's first blob
    launch_owner_scatter(st, P<uint8_t>(c->ex_rv), P<uint64_t>(s.ex_perm), n, P<uint8_t>(s.is_dup) + first,
                         slot_records(s) + first * sizeof(bw_blob));
    launch_index_snapshot(st, P<uint64_t>(c->idx->dstate), slot_ctr(s));
    HIPCHK(c, hipGetLastError());
    s.dedup = true;  // bw_wait now reports the index's sticky errors for this batch
    s.mark = c->idx_mark;
    // the records staged at submit predate the verdicts: stage them again behind the scatter
    if (int r = stage_results(c, s, false, 0, st)) return r;
    s.ex_state = 2;
    return BW_OK;
}
}  // namespace

int bw::exchange_progress(bw_comm* comm, const void* until) {
    ExQueue* q = exq_of(comm, false);
    if (!q) return BW_OK;
    const Slot* u = (const Slot*)until;
    if (u && u->ex_state != 1) u = nullptr;  // not queued (finished, failed or never exchanged)
    if (until && !u) return ((const Slot*)until)->ex_state == 3 ? ((const Slot*)until)->ex_rc : BW_OK;
    std::lock_guard<std::mutex> lk(q->mu);
    while (!q->q.empty()) {
        ExPending e = q->q.front();
        hipSetDevice(e.c->device);
        bool ready = e.s->ex_now;
        int rc = ready ? BW_OK : comm_poll(comm, e.s->ex_ready, e.s->ex_since, &ready, e.c->err);
        if (!rc && !ready) {
            if (!u) return BW_OK;  // nothing more has its counts yet
            rc = comm_wait_event(comm, e.s->ex_ready, e.c->err);
        }
        if (!rc) rc = exchange_finish(comm, e.c, *e.s);
        if (rc) {  // the ranks no longer agree on what follows: fail every queued exchange
            const std::string why = e.c->err;
            for (ExPending& f : q->q) {
                f.s->ex_state = 3;
                f.s->ex_rc = comm_failed(comm) ? BW_ECOMM : rc;
                if (f.c != e.c) f.c->err = "an earlier exchange on the communicator failed: " + why;
            }
            q->q.clear();
            return comm_failed(comm) ? BW_ECOMM : rc;
        }
        q->q.erase(q->q.begin());
        if (u && e.s == u) return BW_OK;
    }
    return BW_OK;
}

void bw::exchange_drain(bw_comm* comm) {
    ExQueue* q = exq_of(comm, false);
    if (!q) return;
    const Slot* last = nullptr;
    {
        std::lock_guard<std::mutex> lk(q->mu);
        if (!q->q.empty()) last = q->q.back().s;
    }
    if (last) exchange_progress(comm, last);
    delete q;
    comm_exq(comm) = nullptr;
}

extern "C" int bw_exchange_dedup(bw_ctx* c, bw_comm* comm, uint64_t ticket) {
    if (!c || !comm) return BW_EINVAL;
    if (comm_device(comm) != c->device) {
        c->err = "communicator and context live on different devices";
        return BW_EINVAL;
    }
    Slot* s = slot_of(c, ticket ? ticket : c->last_ticket);
    if (!s) {
        c->err = "ticket " + std::to_string(ticket) + " is not (or no longer) held by the context";
        return BW_ESTATE;
    }
    if (comm_failed(comm)) {
        c->err = "the communicator was aborted by an earlier failure";
        return BW_ECOMM;
    }
    if (s->dedup || s->ex_state) {
        c->err = "the batch was gated already (submit it with BW_F_NO_DEDUP and exchange it once)";
        return BW_ESTATE;
    }
    if (!s->hashed) {  // BW_F_NO_HASH: its digest array holds no digests
        c->err = "the batch was submitted with BW_F_NO_HASH: no digests to exchange";
        return BW_ESTATE;
    }
    if (s->tail_ticket) {
        c->err = "the batch was split in two parts (BW_OPT_SPLIT): no single digest array";
        return BW_ESTATE;
    }
    if (comm_failed(comm)) {
        c->err = "the communicator was aborted by an earlier failure";
        return BW_ECOMM;
    }
    hipSetDevice(c->device);
    const uint32_t W = (uint32_t)comm_world(comm);
    const bool ranged = s->ex_n != ~0ull;  // a range of the batch's blobs (bw_chunk_stream_shard)
    const uint64_t max_n = ranged ? s->ex_n : s->max_blobs;
    const uint64_t nblk = (max_n + 4095) / 4096;
    int rc = 0;
    rc |= ensure(c, s->ex_dig, max_n * 32);
    rc |= ensure(c, s->ex_perm, max_n * 8);
    rc |= ensure(c, s->ex_msg, 4 * W * 8 + 8);  // [0, 2W) sent, [2W, 4W) received, [4W] a range's length
    rc |= ensure(c, c->bk_blk, (nblk + 1) * W * 8);
    if (rc) return BW_ENOMEM;
    if (int r = ensure_host(c, s->ex_h, 4 * W * 8 + 8)) return r;
    uint64_t* msg = P<uint64_t>(s->ex_msg);
    uint64_t* h = (uint64_t*)s->ex_h.p;
    const uint64_t* d_n = slot_ctr(*s) + C_NBLOBS;
    if (ranged) {  // the range's length as a device count (pinned source: the copy is asynchronous)
        h[4 * W] = max_n;
        HIPCHK(c, hipMemcpyAsync(msg + 4 * W, h + 4 * W, 8, hipMemcpyHostToDevice, c->stream));
        d_n = msg + 4 * W;
    }
    launch_owner_partition(c->stream, P<uint8_t>(s->digests) + (ranged ? 32 * s->ex_first : 0), d_n, max_n, W,
                           P<uint8_t>(s->ex_dig), P<uint64_t>(s->ex_perm), msg, P<uint64_t>(c->bk_blk));
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipEventRecord(s->ex_part, c->stream));
    s->comm = comm;
    s->ex_since = comm_now_ns();
    s->ex_rc = 0;
    bool now = false;
    if (int r = comm_counts(comm, msg, msg + 2 * W, h, c->stream, &now, c->err)) {
        s->ex_state = 3;
        s->ex_rc = r;
        return r;
    }
    if (!now) {  // RCCL: the counts to the slot's pinned buffer by a kernel behind the all-to-all
        launch_copy_u64(c->stream, msg, h, 4 * W);
        HIPCHK(c, hipGetLastError());
        HIPCHK(c, hipEventRecord(s->ex_ready, c->stream));
    }
    s->ex_now = now;
    s->ex_state = 1;
    {
        ExQueue* q = exq_of(comm, true);
        std::lock_guard<std::mutex> lk(q->mu);
        q->q.push_back(ExPending{c, s});
    }
    // the host transport delivered the counts already: finish now; RCCL: whatever is ready
    return exchange_progress(comm, now ? s : nullptr);
}

// ------------------------------------------------------------------ clock stamps (diagnostic build)
#if BW_CLOCK_STAMPS
namespace bw {
void clock_log_register_cdc(void* log);
void clock_log_register_b3(void* log);
}
static ClockLog* g_clock_log = nullptr;  // device: the header; its records follow it
// (re)arm the log of `device` with room for cap records and switch stamping on or off; the kernels
// of every context of the process stamp into it.  Not in the C ABI header: libbackuwup_amd_clock.so
// only (tools/clock_windows.py).
extern "C" int bw_clock_log(int device, uint64_t cap, int on) {
    hipSetDevice(device);
    if (!g_clock_log) {
        if (hipMalloc(&g_clock_log, sizeof(ClockLog) + cap * sizeof(ClockRec)) != hipSuccess) return BW_ENOMEM;
        ClockLog h{(ClockRec*)(g_clock_log + 1), cap, 0, 0};
        if (hipMemcpy(g_clock_log, &h, sizeof h, hipMemcpyHostToDevice) != hipSuccess) return BW_EHIP;
        clock_log_register_cdc(g_clock_log);
        clock_log_register_b3(g_clock_log);
    }
    hipDeviceSynchronize();
    ClockLog h;
    if (hipMemcpy(&h, g_clock_log, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return BW_EHIP;
    if (on && !h.on) h.n = 0;  // a new window
    h.on = on ? 1 : 0;
    return hipMemcpy(g_clock_log, &h, sizeof h, hipMemcpyHostToDevice) == hipSuccess ? BW_OK : BW_EHIP;
}
// the records (40 B each: kind, pad, t0, t1 at 100 MHz, c0, c1 shader cycles); *n = logged (may
// exceed cap: the rest were dropped)
extern "C" int bw_clock_log_read(void* out, uint64_t cap, uint64_t* n) {
    if (!g_clock_log || !n) return BW_ESTATE;
    hipDeviceSynchronize();
    ClockLog h;
    if (hipMemcpy(&h, g_clock_log, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return BW_EHIP;
    *n = h.n;
    const uint64_t k = std::min<uint64_t>(std::min<uint64_t>(h.n, h.cap), cap);
    if (k && out && hipMemcpy(out, g_clock_log + 1, k * sizeof(ClockRec), hipMemcpyDeviceToHost) != hipSuccess)
        return BW_EHIP;
    return BW_OK;
}
#endif

// ------------------------------------------------------------------ stage timing API

extern "C" int bw_profile_enable(bw_ctx* c, int on) {
    if (!c) return BW_EINVAL;
    if (c->helper)
        if (int rc = bw_profile_enable(c->helper, on)) return rc;
    hipSetDevice(c->device);
    hipStreamSynchronize(c->stream);
    for (int k = 0; k < 2; k++) {
        c->ev_pending[k] = false;
        for (int i = 0; i <= BW_N_STAGES; i++)
            if (!c->ev[k][i]) HIPCHK(c, hipEventCreateWithFlags(&c->ev[k][i], EV_TIMING));
    }
    c->prof = on != 0;
    if (c->prof) prof_reference(c->device, c->stream);
    for (int i = 0; i < BW_N_STAGES; i++) {
        c->stage_ms[i] = 0;
        c->intervals[i].clear();
    }
    c->prof_batches = 0;
    return BW_OK;
}

extern "C" int bw_profile_read(bw_ctx* c, double* stage_ms, uint64_t* n_batches) {
    if (!c) return BW_EINVAL;
    prof_collect(c, 0);
    prof_collect(c, 1);
    if (c->helper) {  // split batches: the tail parts' stage times add to the batch's
        prof_collect(c->helper, 0);
        prof_collect(c->helper, 1);
    }
    if (stage_ms)
        for (int i = 0; i < BW_N_STAGES; i++) stage_ms[i] = c->stage_ms[i] + (c->helper ? c->helper->stage_ms[i] : 0);
    if (n_batches) *n_batches = c->prof_batches;
    return BW_OK;
}

extern "C" int bw_profile_intervals(bw_ctx* c, int stage, double* out, uint64_t cap, uint64_t* n) {
    if (!c || !n || stage < 0 || stage >= BW_N_STAGES || (cap && !out)) return BW_EINVAL;
    prof_collect(c, 0);
    prof_collect(c, 1);
    const std::vector<double>& v = c->intervals[stage];
    *n = v.size() / 2;
    if (*n > cap) return BW_ENOSPC;
    if (*n) memcpy(out, v.data(), v.size() * sizeof(double));
    return BW_OK;
}

extern "C" int bw_calibrate_b3(bw_ctx* c, double ms, double out[4]) {
    if (!c || !out || !(ms > 0) || ms > 10000) return BW_EINVAL;
    hipSetDevice(c->device);
    int n_cu = 0;
    HIPCHK(c, hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, c->device));
    if (n_cu <= 0) return BW_ESTATE;
    const uint32_t nblk = (uint32_t)n_cu * b3_calib_blocks_per_cu();
    DevBuf stamps, sink;
    auto release = [&] {
        free_dev(stamps);
        free_dev(sink);
    };
    if (ensure(c, stamps, (size_t)nblk * 16) || ensure(c, sink, 64)) {
        release();
        return BW_ENOMEM;
    }
    hipEvent_t e0 = nullptr, e1 = nullptr;
    auto fail = [&](hipError_t e) {
        c->err = std::string("calibration: ") + hipGetErrorString(e);
        if (e0) hipEventDestroy(e0);
        if (e1) hipEventDestroy(e1);
        release();
        return BW_EHIP;
    };
    hipError_t e;
    if ((e = hipEventCreate(&e0)) || (e = hipEventCreate(&e1))) return fail(e);
    // a short probe sizes the run: blocks per lane so that one launch lasts about `ms`
    uint32_t bpl = 256;
    float t = 0;
    for (int pass = 0; pass < 2; pass++) {
        hipEventRecord(e0, c->stream);
        launch_b3_calib(c->stream, nblk, bpl, P<uint32_t>(sink), P<uint64_t>(stamps));
        hipEventRecord(e1, c->stream);
        if ((e = hipEventSynchronize(e1)) || (e = hipEventElapsedTime(&t, e0, e1))) return fail(e);
        if (pass == 0) {
            const double scale = ms / std::max(1e-3, (double)t);
            bpl = (uint32_t)std::min(1e8, std::max(256.0, bpl * scale));
        }
    }
    std::vector<uint64_t> h((size_t)nblk * 2);
    if ((e = hipMemcpy(h.data(), stamps.p, h.size() * 8, hipMemcpyDeviceToHost))) return fail(e);
    double cyc = 0, ticks = 0;
    for (uint32_t i = 0; i < nblk; i++) {
        cyc += (double)h[2 * i];
        ticks += (double)h[2 * i + 1];
    }
    const double bytes = (double)nblk * 256 * bpl * 64;
    const double ghz = ticks > 0 ? cyc / ticks * 0.1 : 0;  // s_memrealtime counts at 100 MHz
    out[0] = t > 0 ? bytes / (t * 1e-3) / 1e9 : 0;
    out[1] = ghz;
    out[2] = ghz > 0 && t > 0 ? out[0] / ghz / n_cu : 0;  // bytes per shader clock per CU
    out[3] = t;
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    release();
    return BW_OK;
}
