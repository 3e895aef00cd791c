// bw_capi.hip -- the C ABI (include/backuwup_gpu.h) and the host-side batch orchestration.
//
// The host side only turns file sizes into small metadata tables (segments, canonical units);
// every byte of file data is read on the GPU.  A batch is enqueued on one HIP stream with no
// host synchronisation until results are requested, so a caller can keep batches in flight.
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../include/backuwup_gpu.h"
#include "bw_internal.h"
#include "bw_tables.inc"

using namespace bw;

static const uint64_t H_MASKS[26] = BW_MASKS_INIT;

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
};

struct PinBuf {
    void* p = nullptr;
    size_t cap = 0;
};

}  // namespace

struct bw_ctx {
    int device = 0;
    hipStream_t own = nullptr, stream = nullptr;
    std::string err;
    hipEvent_t meta_done = nullptr;  // staging buffer reusable once this fired
    bool meta_pending = false;

    // per-batch device buffers
    DevBuf tile_count, tile_slots, tile_off, tile_btot, cand, ovf, ctr;
    DevBuf segs, cfiles, units, chains, chain_n, chain_cptr, merge, seg_M, seg_cnt, cf_invalid, fb_starts, fb_count;
    DevBuf b_start, b_len, b_goff, b_file, b_kind, b_fend, b_ghash;
    DevBuf cv, cv2, digests, is_dup, packed, fstart, data, scratch, ucnt, ubtot;
    PinBuf stage;

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

    // persistent dedup index
    DevBuf table, log, dstate;
    uint64_t table_cap = 0, log_cap = 0, log_hi = 0;  // log_hi: host upper bound of log length

    // stage timing: two event sets, alternated per batch so recording never waits on the GPU
    bool prof = false;
    hipEvent_t ev[2][BW_N_STAGES + 1] = {};
    bool ev_pending[2] = {false, false};
    int ev_set = 0;
    double stage_ms[BW_N_STAGES] = {};
    uint64_t prof_batches = 0;

    // last batch (kept so a batch whose candidate array overflowed can be re-run exactly)
    uint64_t cand_override = 0;
    const uint8_t* last_data = nullptr;
    uint64_t last_len = 0;
    std::vector<uint64_t> last_off, last_flen;
    bw_params last_prm{};
    bool pending = false;
    uint64_t last_max_blobs = 0;
    uint64_t last_nfiles = 0;
    bool last_dedup = false;
};

// ------------------------------------------------------------------ helpers

#define HIPCHK(ctx, expr)                                                                   \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess) {                                                             \
            (ctx)->err = std::string(#expr) + ": " + hipGetErrorString(e_);                 \
            return BW_EHIP;                                                                 \
        }                                                                                   \
    } while (0)

static int ensure(bw_ctx* c, DevBuf& b, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (b.cap >= bytes) return BW_OK;
    if (b.p) {
        hipStreamSynchronize(c->stream);
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

static int ensure_pinned(bw_ctx* c, PinBuf& b, size_t bytes) {
    if (c->meta_pending) {
        hipEventSynchronize(c->meta_done);
        c->meta_pending = false;
    }
    if (b.cap >= bytes) return BW_OK;
    if (b.p) hipHostFree(b.p);
    size_t want = bytes + bytes / 4 + 4096;
    if (hipHostMalloc(&b.p, want, hipHostMallocDefault) != hipSuccess) {
        c->err = "hipHostMalloc failed";
        b.p = nullptr;
        b.cap = 0;
        return BW_ENOMEM;
    }
    b.cap = want;
    return BW_OK;
}

template <typename T>
static T* P(DevBuf& b) { return (T*)b.p; }

static int make_masks(uint32_t mn, uint32_t av, uint32_t mx, Masks* mk) {
    // FastCDC::with_level asserts (fastcdc 3.0.3 v2020) -> BW_EINVAL instead of a panic.
    if (mn < BW_MINIMUM_MIN || mn > BW_MINIMUM_MAX) return BW_EINVAL;
    if (av < BW_AVERAGE_MIN || av > BW_AVERAGE_MAX) return BW_EINVAL;
    if (mx < BW_MAXIMUM_MIN || mx > BW_MAXIMUM_MAX) return BW_EINVAL;
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

static uint64_t seg_len_for(const Masks& mk) {
    // Segments are a multiple of max_size so that chains through data without candidates
    // (e.g. zeros: every chunk is exactly max) stay phase-aligned and merge immediately; the
    // multiple keeps a segment's own cuts within CHAIN_CAP / 2.
    uint64_t k = (uint64_t)(CHAIN_CAP / 2) * std::min<uint64_t>(mk.s0, mk.max) / mk.max;
    if (k < 1) k = 1;
    if (k > 8) k = 8;
    return k * mk.max;
}

// ------------------------------------------------------------------ stage timing

static void prof_collect(bw_ctx* c, int set) {
    if (!c->ev_pending[set]) return;
    hipEventSynchronize(c->ev[set][BW_N_STAGES]);
    for (int i = 0; i < BW_N_STAGES; i++) {
        float ms = 0;
        if (hipEventElapsedTime(&ms, c->ev[set][i], c->ev[set][i + 1]) == hipSuccess) c->stage_ms[i] += ms;
    }
    c->prof_batches++;
    c->ev_pending[set] = false;
}

static void prof_mark(bw_ctx* c, int stage) {
    if (c->prof) hipEventRecord(c->ev[c->ev_set][stage], c->stream);
}

// ------------------------------------------------------------------ C ABI: basics

extern "C" void bw_params_default(bw_params* p) {
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
        case BW_ECOLLISION: return "64-bit digest key collision in the index";
        case BW_ESTATE: return "invalid call order";
        case BW_ECRYPTO: return "AES-GCM authentication failed";
        case BW_EFORMAT: return "malformed bincode data";
        default: return "unknown error";
    }
}

extern "C" int bw_create(int device, bw_ctx** out) {
    if (!out) return BW_EINVAL;
    *out = nullptr;
    bw_ctx* c = new bw_ctx();
    c->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&c->meta_done, hipEventDisableTiming) != hipSuccess) {
        delete c;
        return BW_EHIP;
    }
    c->stream = c->own;
    if (ensure(c, c->dstate, D_COUNT * 8) || ensure(c, c->ctr, C_COUNT * 8)) {
        delete c;
        return BW_ENOMEM;
    }
    hipMemsetAsync(c->dstate.p, 0, D_COUNT * 8, c->stream);
    hipMemsetAsync(c->ctr.p, 0, C_COUNT * 8, c->stream);
    *out = c;
    return BW_OK;
}

extern "C" void bw_destroy(bw_ctx* c) {
    if (!c) return;
    hipSetDevice(c->device);
    if (c->stream) hipStreamSynchronize(c->stream);
    DevBuf* all[] = {&c->tile_count, &c->tile_slots, &c->tile_off, &c->tile_btot, &c->cand, &c->ovf, &c->ctr, &c->segs,
                     &c->cfiles, &c->units, &c->chains, &c->chain_n, &c->chain_cptr, &c->merge, &c->seg_M,
                     &c->seg_cnt, &c->cf_invalid, &c->fb_starts, &c->fb_count, &c->b_start, &c->b_len,
                     &c->b_goff, &c->b_file, &c->b_kind, &c->b_fend, &c->b_ghash, &c->cv, &c->cv2, &c->digests,
                     &c->is_dup, &c->packed, &c->fstart, &c->data, &c->scratch, &c->ucnt, &c->ubtot, &c->table,
                     &c->log, &c->dstate, &c->seal_items, &c->seal_keys, &c->seal_parts, &c->seal_ok,
                     &c->seal_io, &c->pk_blobs, &c->pk_files, &c->pk_hdr,
                     &c->pk_src, &c->pk_out, &c->ix_io, &c->ix_tab, &c->ix_dig};
    for (DevBuf* b : all)
        if (b->p) hipFree(b->p);
    if (c->stage.p) hipHostFree(c->stage.p);
    if (c->seal_stage.p) hipHostFree(c->seal_stage.p);
    if (c->msg_stage.p) hipHostFree(c->msg_stage.p);
    if (c->seal_done) hipEventDestroy(c->seal_done);
    if (c->pk_done) hipEventDestroy(c->pk_done);
    if (c->meta_done) hipEventDestroy(c->meta_done);
    for (int k = 0; k < 2; k++)
        for (int i = 0; i <= BW_N_STAGES; i++)
            if (c->ev[k][i]) hipEventDestroy(c->ev[k][i]);
    if (c->own) hipStreamDestroy(c->own);
    delete c;
}

extern "C" const char* bw_last_error(const bw_ctx* c) { return c ? c->err.c_str() : "null context"; }

extern "C" int bw_set_stream(bw_ctx* c, void* s) {
    if (!c) return BW_EINVAL;
    hipStreamSynchronize(c->stream);
    c->stream = s ? (hipStream_t)s : c->own;
    return BW_OK;
}

extern "C" void* bw_get_stream(bw_ctx* c) { return c ? (void*)c->stream : nullptr; }

// ------------------------------------------------------------------ dedup index

static int index_capacity(bw_ctx* c, uint64_t incoming) {
    const uint64_t need_log = c->log_hi + incoming;
    if (need_log > c->log_cap) {
        uint64_t cap = c->log_cap ? c->log_cap : 1 << 16;
        while (cap < need_log) cap *= 2;
        DevBuf nb;
        if (hipMalloc(&nb.p, cap * 32) != hipSuccess) return BW_ENOMEM;
        nb.cap = cap * 32;
        if (c->log.p) {
            hipMemcpyAsync(nb.p, c->log.p, c->log_cap * 32, hipMemcpyDeviceToDevice, c->stream);
            hipStreamSynchronize(c->stream);
            hipFree(c->log.p);
        }
        c->log = nb;
        c->log_cap = cap;
    }
    // keep the table at most half full (upper bound: every logged digest distinct)
    if (need_log * 2 > c->table_cap) {
        uint64_t cap = c->table_cap ? c->table_cap : 1 << 16;
        while (cap < need_log * 2) cap *= 2;
        if (c->table.p) {
            hipStreamSynchronize(c->stream);
            hipFree(c->table.p);
            c->table.p = nullptr;
        }
        if (hipMalloc(&c->table.p, cap * 16) != hipSuccess) return BW_ENOMEM;
        c->table.cap = cap * 16;
        const uint64_t old = c->table_cap;
        c->table_cap = cap;
        launch_table_clear(c->stream, P<uint64_t>(c->table), cap);
        if (old) launch_rehash(c->stream, P<uint64_t>(c->table), cap, P<uint8_t>(c->log), P<uint64_t>(c->dstate),
                               c->log_hi);
    }
    return BW_OK;
}

extern "C" int bw_index_reset(bw_ctx* c, uint64_t hint) {
    if (!c) return BW_EINVAL;
    hipSetDevice(c->device);
    c->log_hi = 0;
    hipMemsetAsync(c->dstate.p, 0, D_COUNT * 8, c->stream);
    if (int rc = index_capacity(c, hint ? hint : 1024)) return rc;
    launch_table_clear(c->stream, P<uint64_t>(c->table), c->table_cap);
    HIPCHK(c, hipGetLastError());
    return BW_OK;
}

static int dedup_device(bw_ctx* c, const uint8_t* d_digests, const uint64_t* n_dev, uint64_t n_host, uint64_t max_n,
                        uint8_t* d_is_dup) {
    if (!c->table_cap)
        if (int rc = bw_index_reset(c, 0)) return rc;
    if (int rc = index_capacity(c, max_n)) return rc;
    launch_dedup(c->stream, P<uint64_t>(c->table), c->table_cap, P<uint8_t>(c->log), P<uint64_t>(c->dstate),
                 d_digests, n_dev, n_host, max_n, d_is_dup);
    c->log_hi += max_n;
    HIPCHK(c, hipGetLastError());
    return BW_OK;
}

static int check_collision(bw_ctx* c) {
    uint64_t st[D_COUNT];
    HIPCHK(c, hipMemcpyAsync(st, c->dstate.p, sizeof st, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->log_hi = st[D_LOGLEN];  // tighten the host bound
    if (st[D_COLLIDE]) {
        c->err = "64-bit key collision between distinct digests";
        return BW_ECOLLISION;
    }
    return BW_OK;
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

extern "C" int bw_index_size(bw_ctx* c, uint64_t* n) {
    if (!c || !n) return BW_EINVAL;
    uint64_t st[D_COUNT];
    HIPCHK(c, hipMemcpyAsync(st, c->dstate.p, sizeof st, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    *n = st[D_NUNIQUE];
    return BW_OK;
}

// ------------------------------------------------------------------ the batch pipeline

static int submit(bw_ctx* c, const uint8_t* d_data, uint64_t data_len, const uint64_t* foff, const uint64_t* flen,
                  uint64_t nf, const bw_params* prm) {
    Masks mk;
    if (int rc = make_masks(prm->min_size, prm->avg_size, prm->max_size, &mk)) {
        c->err = "fastcdc parameters out of range";
        return rc;
    }
    if (nf && (!foff || !flen)) return BW_EINVAL;
    if (data_len && !d_data) return BW_EINVAL;
    if (((uintptr_t)d_data & 15) != 0) {
        c->err = "device data pointer must be 16-byte aligned";
        return BW_EINVAL;
    }
    for (uint64_t f = 0; f < nf; f++)
        if (foff[f] > data_len || flen[f] > data_len - foff[f]) {
            c->err = "file " + std::to_string(f) + " lies outside the data buffer";
            return BW_EINVAL;
        }
    hipSetDevice(c->device);
    const bool force_serial = (prm->flags & BW_F_SERIAL_RESOLVE) != 0;
    const bool do_hash = !(prm->flags & BW_F_NO_HASH);
    const bool do_dedup = do_hash && !(prm->flags & BW_F_NO_DEDUP);

    // ---- host metadata: CDC files, segments, canonical units
    const uint64_t L = seg_len_for(mk);
    // every chunk but a file's last is >= min(2*(min/2), max) bytes (max < min is legal in the crate)
    const uint64_t min_chunk = std::min<uint64_t>(mk.s0, mk.max);
    std::vector<SegDesc> segs;
    std::vector<CFileDesc> cfs;
    std::vector<UnitDesc> units;
    units.reserve(nf);
    uint64_t max_blobs = 0, fb_total = 0, max_blob_len = mk.max, total_len = 0;
    for (uint64_t f = 0; f < nf; f++) {
        total_len += flen[f];
        if (flen[f] > prm->small_file_threshold && flen[f] > 0) {
            CFileDesc cf;
            cf.start = foff[f];
            cf.end = foff[f] + flen[f];
            cf.fb_off = fb_total;
            cf.first_seg = (uint32_t)segs.size();
            const uint64_t ns = (flen[f] + L - 1) / L;
            cf.nseg = (uint32_t)ns;
            for (uint64_t j = 0; j < ns; j++) {
                SegDesc sd;
                sd.start = cf.start + j * L;
                sd.end = std::min(cf.start + (j + 1) * L, cf.end);
                sd.file_end = cf.end;
                sd.cfile = (uint32_t)cfs.size();
                sd.last = j + 1 == ns;
                UnitDesc u;
                u.start = 0;
                u.len = 0;
                u.file = (uint32_t)f;
                u.kind = 1;
                u.seg = (uint32_t)segs.size();
                u.cfile = sd.cfile;
                units.push_back(u);
                segs.push_back(sd);
            }
            const uint64_t nb = flen[f] / min_chunk + 2;
            fb_total += nb;
            max_blobs += nb;
            cfs.push_back(cf);
        } else {
            UnitDesc u;
            u.start = foff[f];
            u.len = flen[f];
            u.file = (uint32_t)f;
            u.kind = 0;
            u.seg = 0;
            u.cfile = 0;
            units.push_back(u);
            max_blobs += 1;
            max_blob_len = std::max<uint64_t>(max_blob_len, flen[f]);
        }
    }
    const uint64_t nseg = segs.size(), ncf = cfs.size(), nunits = units.size();
    const uint64_t max_groups = total_len / 4096 + max_blobs + 1;
    const int max_leaves = (int)std::min<uint64_t>((max_blob_len + 1023) / 1024, 1u << 30);
    // small batches scan half-size tiles: with one 128 KiB tile per wave the per-tile start
    // costs dominate (C1: 0.50 -> 0.33 ms per GiB); large ones keep the longer strips
    // (BW_SCAN_SMALL_BYTES overrides the threshold, so the tests can run either tile size on any input)
    const char* sb = getenv("BW_SCAN_SMALL_BYTES");
    const uint64_t small_bytes = sb ? strtoull(sb, nullptr, 10) : SCAN_SMALL_BYTES;
    mk.tile_shift = data_len < small_bytes ? SCAN_TILE_SHIFT - 1 : SCAN_TILE_SHIFT;
    const uint64_t tile_bytes = 1ull << mk.tile_shift;
    const uint64_t n_tiles = ncf ? (data_len + tile_bytes - 1) / tile_bytes : 0;

    // ---- device buffers
    int rc = 0;
    rc |= ensure(c, c->tile_count, n_tiles * 4);
    rc |= ensure(c, c->tile_slots, n_tiles * SCAN_CAP * 8);
    rc |= ensure(c, c->tile_off, (n_tiles + 1) * 8);
    rc |= ensure(c, c->tile_btot, (n_tiles / 1024 + 2) * 8);
    rc |= ensure(c, c->ovf, n_tiles * 4);
    rc |= ensure(c, c->segs, nseg * sizeof(SegDesc));
    rc |= ensure(c, c->cfiles, ncf * sizeof(CFileDesc));
    rc |= ensure(c, c->units, nunits * sizeof(UnitDesc));
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
    rc |= ensure(c, c->cv, max_groups * 32);
    rc |= ensure(c, c->cv2, max_leaves > 64 ? max_groups * 32 : 16);
    rc |= ensure(c, c->digests, max_blobs * 32);
    rc |= ensure(c, c->is_dup, max_blobs);
    rc |= ensure(c, c->packed, max_blobs * sizeof(bw_blob));
    rc |= ensure(c, c->fstart, nf * 8);
    rc |= ensure(c, c->ucnt, 2 * nunits * 8);
    rc |= ensure(c, c->ubtot, 2 * (nunits / 1024 + 2) * 8);
    if (rc) return BW_ENOMEM;
    // candidate array: 4x the expected count (2^-popcount(mask) per byte) plus slack; a batch
    // that finds more is re-run by bw_results with the exact count (pathological inputs only)
    uint64_t cand_cap = 16;
    if (ncf) {
        const int bits = __builtin_popcountll(mk.mask_pre);
        cand_cap = 4 * (data_len >> bits) + 2 * n_tiles + 4096;
        cand_cap = std::max(cand_cap, c->cand_override);
    }
    if (int r2 = ensure(c, c->cand, cand_cap * 8)) return r2;

    // ---- metadata upload through pinned staging
    const size_t meta_bytes = nseg * sizeof(SegDesc) + ncf * sizeof(CFileDesc) + nunits * sizeof(UnitDesc) + nf * 8;
    if (int r3 = ensure_pinned(c, c->stage, meta_bytes + 64)) return r3;
    uint8_t* sp = (uint8_t*)c->stage.p;
    size_t o = 0;
    auto up = [&](DevBuf& dst, const void* src, size_t bytes) -> hipError_t {
        if (!bytes) return hipSuccess;
        memcpy(sp + o, src, bytes);
        hipError_t e = hipMemcpyAsync(dst.p, sp + o, bytes, hipMemcpyHostToDevice, c->stream);
        o += bytes;
        return e;
    };
    HIPCHK(c, up(c->segs, segs.data(), nseg * sizeof(SegDesc)));
    HIPCHK(c, up(c->cfiles, cfs.data(), ncf * sizeof(CFileDesc)));
    HIPCHK(c, up(c->units, units.data(), nunits * sizeof(UnitDesc)));
    HIPCHK(c, up(c->fstart, foff, nf * 8));
    hipEventRecord(c->meta_done, c->stream);
    c->meta_pending = true;
    HIPCHK(c, hipMemsetAsync(c->ctr.p, 0, C_COUNT * 8, c->stream));

    if (c->prof) {
        c->ev_set ^= 1;
        prof_collect(c, c->ev_set);  // the set about to be reused belongs to batch k-2
    }
    prof_mark(c, BW_STAGE_SCAN);
    BlobArrays b{P<uint64_t>(c->b_start), P<uint64_t>(c->b_len), P<uint64_t>(c->b_goff), P<uint32_t>(c->b_file),
                 P<uint32_t>(c->b_kind), P<uint64_t>(c->b_fend), P<uint64_t>(c->b_ghash)};
    uint64_t* ctr = P<uint64_t>(c->ctr);
    hipStream_t st = c->stream;

    // ---- chunking
    if (ncf) {
        launch_scan(st, d_data, data_len, n_tiles, mk, P<uint32_t>(c->tile_count), P<uint64_t>(c->tile_slots),
                    P<uint32_t>(c->ovf), ctr);
        prof_mark(c, BW_STAGE_COMPACT);
        launch_compact(st, d_data, data_len, n_tiles, mk, P<uint32_t>(c->tile_count), P<uint64_t>(c->tile_slots),
                       P<uint64_t>(c->tile_off), P<uint64_t>(c->cand), cand_cap, P<uint32_t>(c->ovf), ctr,
                       P<uint64_t>(c->tile_btot));
        prof_mark(c, BW_STAGE_RESOLVE);
        launch_chains(st, d_data, mk, P<uint64_t>(c->cand), P<uint64_t>(c->tile_off), ctr, P<SegDesc>(c->segs), nseg,
                      P<uint64_t>(c->chains), P<uint32_t>(c->chain_n), P<uint64_t>(c->chain_cptr),
                      P<uint64_t>(c->merge), force_serial);
        launch_resolve(st, d_data, mk, P<uint64_t>(c->cand), P<uint64_t>(c->tile_off), ctr, P<SegDesc>(c->segs), nseg,
                       P<CFileDesc>(c->cfiles), ncf, P<uint64_t>(c->chains), P<uint32_t>(c->chain_n),
                       P<uint64_t>(c->merge), P<uint64_t>(c->seg_M), P<uint32_t>(c->seg_cnt),
                       P<uint32_t>(c->cf_invalid), P<uint64_t>(c->fb_starts), P<uint64_t>(c->fb_count), force_serial);
    } else {
        prof_mark(c, BW_STAGE_COMPACT);
        prof_mark(c, BW_STAGE_RESOLVE);
    }
    prof_mark(c, BW_STAGE_ASSEMBLE);
    launch_assemble(st, ctr, P<UnitDesc>(c->units), nunits, P<SegDesc>(c->segs), P<CFileDesc>(c->cfiles),
                    P<uint64_t>(c->chains), P<uint32_t>(c->chain_n), P<uint64_t>(c->seg_M), P<uint32_t>(c->cf_invalid),
                    P<uint64_t>(c->fb_starts), P<uint64_t>(c->fb_count), b, P<uint64_t>(c->ucnt),
                    P<uint64_t>(c->ubtot));
    if (ncf) launch_cut_hash(st, d_data, mk, ctr, b, max_blobs);
    else HIPCHK(c, hipMemsetAsync(c->b_ghash.p, 0, max_blobs * 8, st));

    // ---- hashing + dedup
    prof_mark(c, BW_STAGE_B3LEAF);
    if (do_hash) {
        launch_blake3(st, d_data, ctr, b, max_blobs, max_groups, P<uint32_t>(c->cv), P<uint32_t>(c->cv2),
                      P<uint8_t>(c->digests), max_leaves, c->prof ? c->ev[c->ev_set][BW_STAGE_B3TREE] : nullptr);
    } else {
        prof_mark(c, BW_STAGE_B3TREE);
        HIPCHK(c, hipMemsetAsync(c->digests.p, 0, max_blobs * 32, st));
    }
    prof_mark(c, BW_STAGE_DEDUP);
    if (do_dedup) {
        if (int r4 = dedup_device(c, P<uint8_t>(c->digests), ctr + C_DEDUPN, 0, max_blobs, P<uint8_t>(c->is_dup)))
            return r4;
    }
    prof_mark(c, BW_STAGE_PACK);
    launch_pack(st, ctr, b, P<uint64_t>(c->fstart), P<uint8_t>(c->digests), do_dedup ? P<uint8_t>(c->is_dup) : nullptr,
                P<uint8_t>(c->packed), max_blobs);
    prof_mark(c, BW_N_STAGES);
    if (c->prof) c->ev_pending[c->ev_set] = true;
    HIPCHK(c, hipGetLastError());
    c->pending = true;
    c->last_data = d_data;
    c->last_len = data_len;
    c->last_off.assign(foff, foff + nf);
    c->last_flen.assign(flen, flen + nf);
    c->last_prm = *prm;
    c->last_max_blobs = max_blobs;
    c->last_nfiles = nf;
    c->last_dedup = do_dedup;
    return BW_OK;
}

extern "C" int bw_process_files_device(bw_ctx* c, const uint8_t* d_data, uint64_t data_len, const uint64_t* foff,
                                       const uint64_t* flen, uint64_t nf, const bw_params* prm) {
    if (!c) return BW_EINVAL;
    bw_params def;
    if (!prm) {
        bw_params_default(&def);
        prm = &def;
    }
    return submit(c, d_data, data_len, foff, flen, nf, prm);
}

extern "C" int bw_results(bw_ctx* c, bw_blob* out, uint64_t cap, uint64_t* n_out) {
    if (!c || !n_out) return BW_EINVAL;
    if (!c->pending) return BW_ESTATE;
    hipSetDevice(c->device);
    uint64_t ctr[C_COUNT];
    HIPCHK(c, hipMemcpyAsync(ctr, c->ctr.p, sizeof ctr, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (ctr[C_CANDTOTAL] > ctr[C_NCAND]) {
        // candidate array overflowed: the chunk lists are incomplete -> re-run with exact room.
        // (k_assemble handed 0 blobs to the index, so the re-run sees the same index.)
        c->cand_override = ctr[C_CANDTOTAL] + 1024;
        std::vector<uint64_t> fo = c->last_off, fl = c->last_flen;
        if (int rc = submit(c, c->last_data, c->last_len, fo.data(), fl.data(), fo.size(), &c->last_prm)) return rc;
        return bw_results(c, out, cap, n_out);
    }
    *n_out = ctr[C_NBLOBS];
    if (c->last_dedup)
        if (int rc = check_collision(c)) return rc;
    if (ctr[C_NBLOBS] > cap) return BW_ENOSPC;
    if (ctr[C_NBLOBS] && out)
        HIPCHK(c, hipMemcpy(out, c->packed.p, ctr[C_NBLOBS] * sizeof(bw_blob), hipMemcpyDeviceToHost));
    return BW_OK;
}

extern "C" int bw_batch_device_views(bw_ctx* c, uint64_t* n_blobs, const uint8_t** d_digests, uint8_t** d_is_dup) {
    if (!c) return BW_EINVAL;
    if (!c->pending) return BW_ESTATE;
    uint64_t n = 0;
    HIPCHK(c, hipMemcpyAsync(&n, (uint64_t*)c->ctr.p + C_NBLOBS, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (n_blobs) *n_blobs = n;
    if (d_digests) *d_digests = P<uint8_t>(c->digests);
    if (d_is_dup) *d_is_dup = P<uint8_t>(c->is_dup);
    return BW_OK;
}

static int upload_data(bw_ctx* c, const uint8_t* data, uint64_t len) {
    if (int rc = ensure(c, c->data, len + 64)) return rc;
    if (len) HIPCHK(c, hipMemcpyAsync(c->data.p, data, len, hipMemcpyHostToDevice, c->stream));
    return BW_OK;
}

extern "C" int bw_process_files(bw_ctx* c, const uint8_t* data, uint64_t data_len, const uint64_t* foff,
                                const uint64_t* flen, uint64_t nf, const bw_params* prm, bw_blob* out, uint64_t cap,
                                uint64_t* n_out) {
    if (!c || !n_out || (data_len && !data)) return BW_EINVAL;
    hipSetDevice(c->device);
    if (int rc = upload_data(c, data, data_len)) return rc;
    if (int rc = bw_process_files_device(c, P<uint8_t>(c->data), data_len, foff, flen, nf, prm)) return rc;
    return bw_results(c, out, cap, n_out);
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

uint8_t* bw::message_stage(bw_ctx* c, size_t bytes) {
    hipSetDevice(c->device);
    if (c->msg_stage.cap < bytes) {
        hipStreamSynchronize(c->stream);
        if (c->msg_stage.p) hipHostFree(c->msg_stage.p);
        c->msg_stage.p = nullptr;
        c->msg_stage.cap = 0;
        const size_t want = bytes + bytes / 4 + 4096;
        if (hipHostMalloc(&c->msg_stage.p, want, hipHostMallocDefault) != hipSuccess) {
            c->err = "hipHostMalloc failed";
            return nullptr;
        }
        c->msg_stage.cap = want;
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
    if (int rc = submit(c, P<uint8_t>(c->data), total, offs, lens, n, &p)) return rc;
    HIPCHK(c, hipMemcpyAsync(hashes, c->digests.p, n * 32, hipMemcpyDeviceToHost, c->stream));
    if (dedup) HIPCHK(c, hipMemcpyAsync(dup, c->is_dup.p, n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->pending = false;
    return dedup ? check_collision(c) : BW_OK;
}

extern "C" int bw_blake3_hash(bw_ctx* c, const uint8_t* data, uint64_t len, uint8_t out[32]) {
    const uint64_t off = 0;
    static const uint8_t empty[16] = {0};
    return bw_blake3_hash_many(c, len ? data : empty, len, &off, &len, 1, out);
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

extern "C" int bw_scatter_verdicts(bw_ctx* c, const uint8_t* d_verdict, const uint64_t* d_perm, uint64_t n,
                                   uint8_t* d_is_dup) {
    if (!c) return BW_EINVAL;
    hipSetDevice(c->device);
    launch_scatter(c->stream, d_verdict, d_perm, n, d_is_dup);
    HIPCHK(c, hipGetLastError());
    return BW_OK;
}

// ------------------------------------------------------------------ stage timing API

extern "C" int bw_profile_enable(bw_ctx* c, int on) {
    if (!c) return BW_EINVAL;
    hipSetDevice(c->device);
    hipStreamSynchronize(c->stream);
    for (int k = 0; k < 2; k++) {
        c->ev_pending[k] = false;
        for (int i = 0; i <= BW_N_STAGES; i++)
            if (!c->ev[k][i]) HIPCHK(c, hipEventCreate(&c->ev[k][i]));
    }
    c->prof = on != 0;
    for (int i = 0; i < BW_N_STAGES; i++) c->stage_ms[i] = 0;
    c->prof_batches = 0;
    return BW_OK;
}

extern "C" int bw_profile_read(bw_ctx* c, double* stage_ms, uint64_t* n_batches) {
    if (!c) return BW_EINVAL;
    prof_collect(c, 0);
    prof_collect(c, 1);
    if (stage_ms)
        for (int i = 0; i < BW_N_STAGES; i++) stage_ms[i] = c->stage_ms[i];
    if (n_batches) *n_batches = c->prof_batches;
    return BW_OK;
}

// ------------------------------------------------------------------ blob sealing (§8f row 3)
// compress_encrypt_blob's HKDF key + AES-256-GCM (pack.rs:70-80) and the inverse
// (unpack.rs:58-63, blob_index.rs:185-191); kernels in bw_seal.hip.

// raw_len (sealing only, may be null): item i's plaintext is the zstd store frame of raw_len[i]
// source bytes at d_src + src_off[i], built inside k_seal_ctr; src_len[i] is the frame length.
static int seal_submit(bw_ctx* c, bool dec, const uint8_t* prk, const uint8_t* d_src, const uint64_t* src_off,
                       const uint64_t* src_len, uint64_t n, const uint8_t* info, uint32_t info_len,
                       const uint8_t* nonces, uint8_t* d_dst, const uint64_t* dst_off, uint8_t* ok,
                       const uint64_t* raw_len = nullptr) {
    if (!c || !prk || info_len > BW_SEAL_MAX_INFO) return BW_EINVAL;
    if (n && (!d_src || !src_off || !src_len || !nonces || !d_dst || !dst_off || (info_len && !info))) return BW_EINVAL;
    if (dec && n && !ok) return BW_EINVAL;
    hipSetDevice(c->device);
    if (!n) return BW_OK;
    if (dec)
        for (uint64_t i = 0; i < n; i++)
            if (src_len[i] < 16) return BW_EINVAL;  // shorter than the tag: decrypt_in_place fails
    if (!c->seal_done) HIPCHK(c, hipEventCreateWithFlags(&c->seal_done, hipEventDisableTiming));
    if (c->seal_pending) {
        hipEventSynchronize(c->seal_done);
        c->seal_pending = false;
    }
    const size_t bytes = n * sizeof(SealItem);
    if (c->seal_stage.cap < bytes) {
        if (c->seal_stage.p) hipHostFree(c->seal_stage.p);
    if (c->msg_stage.p) hipHostFree(c->msg_stage.p);
        c->seal_stage.p = nullptr;
        c->seal_stage.cap = 0;
        const size_t want = bytes + bytes / 4 + 4096;
        if (hipHostMalloc(&c->seal_stage.p, want, hipHostMallocDefault) != hipSuccess) {
            c->err = "hipHostMalloc failed";
            return BW_ENOMEM;
        }
        c->seal_stage.cap = want;
    }
    SealItem* it = (SealItem*)c->seal_stage.p;
    std::vector<uint64_t> piece0(n);
    uint64_t pieces = 0;
    for (uint64_t i = 0; i < n; i++) {
        piece0[i] = pieces;
        pieces += seal_pieces(dec ? src_len[i] - 16 : src_len[i]);
    }
    parallel_ranges(n, [&](uint64_t lo, uint64_t hi) {
        for (uint64_t i = lo; i < hi; i++) {
            const uint64_t len = dec ? src_len[i] - 16 : src_len[i];
            seal_fill_item(&it[i], src_off[i], len, dst_off[i], piece0[i], nonces + 12 * i,
                           info + (uint64_t)info_len * i, info_len);
            if (raw_len) {
                it[i].raw_len = (uint32_t)raw_len[i];
                it[i].wd = zstd_window_descriptor(raw_len[i]);
            }
        }
    });
    if (int rc = ensure(c, c->seal_items, bytes)) return rc;
    if (int rc = ensure(c, c->seal_keys, n * sizeof(SealKey))) return rc;
    if (int rc = ensure(c, c->seal_parts, (pieces + 1) * 16)) return rc;
    if (dec)
        if (int rc = ensure(c, c->seal_ok, n)) return rc;
    HIPCHK(c, hipMemcpyAsync(c->seal_items.p, it, bytes, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipEventRecord(c->seal_done, c->stream));
    c->seal_pending = true;
    SealPads pads;
    seal_pads(prk, &pads);
    launch_seal(c->stream, dec, raw_len != nullptr, d_src, d_dst, P<SealItem>(c->seal_items), n, pads,
                P<SealKey>(c->seal_keys), pieces,
                P<uint32_t>(c->seal_parts), dec ? P<uint8_t>(c->seal_ok) : nullptr);
    HIPCHK(c, hipGetLastError());
    if (dec) {
        HIPCHK(c, hipMemcpyAsync(ok, c->seal_ok.p, n, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    return BW_OK;
}

extern "C" int bw_seal_device(bw_ctx* c, const uint8_t prk[32], const uint8_t* d_src, const uint64_t* src_off,
                              const uint64_t* src_len, uint64_t n, const uint8_t* info, uint32_t info_len,
                              const uint8_t* nonces, uint8_t* d_dst, const uint64_t* dst_off) {
    return seal_submit(c, false, prk, d_src, src_off, src_len, n, info, info_len, nonces, d_dst, dst_off, nullptr);
}

extern "C" int bw_open_device(bw_ctx* c, const uint8_t prk[32], const uint8_t* d_src, const uint64_t* src_off,
                              const uint64_t* src_len, uint64_t n, const uint8_t* info, uint32_t info_len,
                              const uint8_t* nonces, uint8_t* d_dst, const uint64_t* dst_off, uint8_t* ok) {
    return seal_submit(c, true, prk, d_src, src_off, src_len, n, info, info_len, nonces, d_dst, dst_off, ok);
}

// Host-buffer forms: both buffers go through one device staging area ([src | dst]).
static int seal_host(bw_ctx* c, bool dec, const uint8_t* prk, const uint8_t* src, const uint64_t* src_off,
                     const uint64_t* src_len, uint64_t n, const uint8_t* info, uint32_t info_len,
                     const uint8_t* nonces, uint8_t* dst, const uint64_t* dst_off, uint8_t* ok) {
    if (!c || (n && (!src || !src_off || !src_len || !dst || !dst_off))) return BW_EINVAL;
    hipSetDevice(c->device);
    uint64_t s_end = 0, d_end = 0;
    for (uint64_t i = 0; i < n; i++) {
        if (dec && src_len[i] < 16) return BW_EINVAL;
        s_end = std::max(s_end, src_off[i] + src_len[i]);
        d_end = std::max(d_end, dst_off[i] + (dec ? src_len[i] - 16 : src_len[i] + 16));
    }
    const uint64_t d_base = (s_end + 255) & ~255ull;
    if (int rc = ensure(c, c->seal_io, d_base + d_end + 16)) return rc;
    uint8_t* io = P<uint8_t>(c->seal_io);
    if (s_end) HIPCHK(c, hipMemcpyAsync(io, src, s_end, hipMemcpyHostToDevice, c->stream));
    int rc = seal_submit(c, dec, prk, io, src_off, src_len, n, info, info_len, nonces, io + d_base, dst_off, ok);
    if (rc) return rc;
    // copy back only the written ranges (the caller's gaps stay untouched)
    for (uint64_t i = 0; i < n; i++) {
        const uint64_t len = dec ? src_len[i] - 16 : src_len[i] + 16;
        if (len) HIPCHK(c, hipMemcpyAsync(dst + dst_off[i], io + d_base + dst_off[i], len, hipMemcpyDeviceToHost, c->stream));
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return BW_OK;
}

extern "C" int bw_seal(bw_ctx* c, const uint8_t prk[32], const uint8_t* src, const uint64_t* src_off,
                       const uint64_t* src_len, uint64_t n, const uint8_t* info, uint32_t info_len,
                       const uint8_t* nonces, uint8_t* dst, const uint64_t* dst_off) {
    return seal_host(c, false, prk, src, src_off, src_len, n, info, info_len, nonces, dst, dst_off, nullptr);
}

extern "C" int bw_open(bw_ctx* c, const uint8_t prk[32], const uint8_t* src, const uint64_t* src_off,
                       const uint64_t* src_len, uint64_t n, const uint8_t* info, uint32_t info_len,
                       const uint8_t* nonces, uint8_t* dst, const uint64_t* dst_off, uint8_t* ok) {
    return seal_host(c, true, prk, src, src_off, src_len, n, info, info_len, nonces, dst, dst_off, ok);
}

// ------------------------------------------------------------------ packfiles (§8f row 4)
// Manager::write_packfiles / serialize_packfile (pack.rs:115-227); kernels in bw_pack.hip.

static uint32_t varint_len(uint64_t v) { return v < 251 ? 1 : (v < (1ull << 16) ? 3 : (v < (1ull << 32) ? 5 : 9)); }

extern "C" uint64_t bw_zstd_store_size(uint64_t len) {
    const uint64_t nb = len ? (len + ZSTD_BLOCK - 1) / ZSTD_BLOCK : 1;
    return 2 + 3 * nb + len;
}

static uint64_t sealed_len_of(uint64_t payload, uint32_t flags) {
    return (flags & BW_PACK_ZSTD_STORE ? bw_zstd_store_size(payload) : payload) + BW_SEAL_TAG_BYTES;
}

// header plaintext bytes of a PackfileHeaderBlob entry
static uint64_t entry_len(uint64_t sealed, uint64_t section_off) {
    return 32 + 1 + 1 + varint_len(sealed) + varint_len(section_off);
}

static void plan_packfiles(const uint64_t* payload_len, uint64_t n, uint32_t flags, std::vector<bw_packfile>& out) {
    uint64_t i = 0, off = 0;
    while (i < n) {
        bw_packfile p{};
        p.first_blob = i;
        uint64_t written = 0, hdr = 0;
        while (i < n) {
            const uint64_t sealed = sealed_len_of(payload_len[i], flags);
            hdr += entry_len(sealed, written);
            written += sealed + BW_BLOB_NONCE_SIZE;
            p.n_blobs++;
            i++;
            if (written >= BW_PACKFILE_TARGET_SIZE || p.n_blobs >= BW_PACKFILE_MAX_BLOBS) break;
        }
        hdr += varint_len(p.n_blobs);
        p.header_len = hdr + BW_SEAL_TAG_BYTES;
        p.offset = off;
        p.size = 8 + p.header_len + written;
        off += p.size;
        out.push_back(p);
    }
}

extern "C" int bw_pack_plan(const uint64_t* payload_len, uint64_t n, uint32_t flags, bw_packfile* out, uint64_t cap,
                            uint64_t* n_out, uint64_t* total_bytes) {
    if (!n_out || !total_bytes || (n && !payload_len) || (cap && !out)) return BW_EINVAL;
    std::vector<bw_packfile> pl;
    plan_packfiles(payload_len, n, flags, pl);
    *n_out = pl.size();
    *total_bytes = pl.empty() ? 0 : pl.back().offset + pl.back().size;
    if (pl.size() > cap) return BW_ENOSPC;
    std::copy(pl.begin(), pl.end(), out);
    return BW_OK;
}

static int pack_submit(bw_ctx* c, const uint8_t* prk, const uint8_t* d_src, const uint64_t* src_off,
                       const uint64_t* src_len, uint64_t n, const uint8_t* hashes, const uint8_t* kinds,
                       const uint8_t* nonces, uint32_t flags, const bw_packfile* plan, uint64_t npf,
                       const uint8_t* ids, uint8_t* d_out) {
    if (!c || !prk || (flags & ~BW_PACK_ZSTD_STORE)) return BW_EINVAL;
    if (n && (!d_src || !src_off || !src_len || !hashes || !kinds || !nonces)) return BW_EINVAL;
    if (npf && (!plan || !ids || !d_out)) return BW_EINVAL;
    hipSetDevice(c->device);
    // the plan must be the reference's grouping of exactly these blobs
    std::vector<bw_packfile> want;
    plan_packfiles(src_len, n, flags, want);
    if (want.size() != npf) return BW_EINVAL;
    for (uint64_t p = 0; p < npf; p++) {
        const bw_packfile &a = want[p], &b = plan[p];
        if (a.first_blob != b.first_blob || a.n_blobs != b.n_blobs || a.offset != b.offset || a.size != b.size ||
            a.header_len != b.header_len) {
            c->err = "packfile plan does not match the blobs (use bw_pack_plan)";
            return BW_EINVAL;
        }
        if (a.size > BW_PACKFILE_MAX_SIZE) {
            c->err = "bug: violated packfile size limit";  // pack.rs:152-156 asserts
            return BW_EINVAL;
        }
    }
    for (uint64_t i = 0; i < n; i++)
        if (kinds[i] > BW_BLOB_TREE || ((flags & BW_PACK_ZSTD_STORE) && src_len[i] > (1ull << 31))) return BW_EINVAL;
    if (!n) return BW_OK;
    if (!c->pk_done) HIPCHK(c, hipEventCreateWithFlags(&c->pk_done, hipEventDisableTiming));
    if (c->pk_pending) {
        hipEventSynchronize(c->pk_done);
        c->pk_pending = false;
    }
    const bool store = flags & BW_PACK_ZSTD_STORE;
    c->h_pk_blobs.resize(n);
    c->h_pk_files.resize(npf);
    std::vector<uint64_t> s_off(n), s_len(n), d_off(n), h_off(npf), h_len(npf), h_dst(npf);
    uint64_t hdr_total = 0;
    for (uint64_t p = 0; p < npf; p++) {
        const bw_packfile& f = plan[p];
        h_off[p] = hdr_total;
        h_len[p] = f.header_len - BW_SEAL_TAG_BYTES;
        h_dst[p] = f.offset + 8;
        c->h_pk_files[p] = PackFileDesc{hdr_total, f.n_blobs, f.offset, f.header_len};
        hdr_total += h_len[p];
    }
    // packfiles are independent once their header offsets are known: fill their blobs in parallel
    parallel_ranges(
        npf,
        [&](uint64_t p_lo, uint64_t p_hi) {
            for (uint64_t p = p_lo; p < p_hi; p++) {
                const bw_packfile& f = plan[p];
                uint64_t entry = h_off[p] + varint_len(f.n_blobs), section = 0;
                const uint64_t data0 = f.offset + 8 + f.header_len;
                for (uint64_t i = f.first_blob; i < f.first_blob + f.n_blobs; i++) {
                    const uint64_t frame = store ? bw_zstd_store_size(src_len[i]) : src_len[i];
                    const uint64_t sealed = frame + BW_SEAL_TAG_BYTES;
                    PackBlob& b = c->h_pk_blobs[i];
                    memcpy(b.hash, hashes + 32 * i, 32);
                    memcpy(b.nonce, nonces + 12 * i, 12);
                    b.kind = kinds[i];
                    b.sealed_len = sealed;
                    b.section_off = section;
                    b.hdr_off = entry;
                    b.nonce_off = data0 + section;
                    entry += entry_len(sealed, section);
                    section += sealed + BW_BLOB_NONCE_SIZE;
                    s_len[i] = frame;
                    s_off[i] = src_off[i];
                    d_off[i] = b.nonce_off + BW_BLOB_NONCE_SIZE;
                }
            }
        },
        n);
    if (int rc = ensure(c, c->pk_blobs, n * sizeof(PackBlob))) return rc;
    if (int rc = ensure(c, c->pk_files, npf * sizeof(PackFileDesc))) return rc;
    if (int rc = ensure(c, c->pk_hdr, hdr_total)) return rc;
    HIPCHK(c, hipMemcpyAsync(c->pk_blobs.p, c->h_pk_blobs.data(), n * sizeof(PackBlob), hipMemcpyHostToDevice,
                             c->stream));
    HIPCHK(c, hipMemcpyAsync(c->pk_files.p, c->h_pk_files.data(), npf * sizeof(PackFileDesc), hipMemcpyHostToDevice,
                             c->stream));
    HIPCHK(c, hipEventRecord(c->pk_done, c->stream));
    c->pk_pending = true;
    launch_pack_meta(c->stream, P<PackBlob>(c->pk_blobs), n, P<PackFileDesc>(c->pk_files), npf, P<uint8_t>(c->pk_hdr),
                     d_out);
    HIPCHK(c, hipGetLastError());
    // every blob: derive_backup_key(hash) + AES-GCM(nonce) of its payload (its store frame, built
    // while it is encrypted) into its place behind its nonce
    if (int rc = seal_submit(c, false, prk, d_src, s_off.data(), s_len.data(), n, hashes, 32, nonces, d_out,
                             d_off.data(), nullptr, store ? src_len : nullptr))
        return rc;
    // every header: derive_backup_key(b"header") + AES-GCM(packfile id) behind the length prefix
    std::vector<uint8_t> info(npf * 6);
    for (uint64_t p = 0; p < npf; p++) memcpy(&info[6 * p], "header", 6);
    return seal_submit(c, false, prk, P<uint8_t>(c->pk_hdr), h_off.data(), h_len.data(), npf, info.data(), 6, ids,
                       d_out, h_dst.data(), nullptr);
}

extern "C" int bw_pack_build_device(bw_ctx* c, const uint8_t prk[32], const uint8_t* d_src, const uint64_t* src_off,
                                    const uint64_t* src_len, uint64_t n, const uint8_t* hashes, const uint8_t* kinds,
                                    const uint8_t* nonces, uint32_t flags, const bw_packfile* plan, uint64_t npf,
                                    const uint8_t* ids, uint8_t* d_out) {
    return pack_submit(c, prk, d_src, src_off, src_len, n, hashes, kinds, nonces, flags, plan, npf, ids, d_out);
}

extern "C" int bw_pack_build(bw_ctx* c, const uint8_t prk[32], const uint8_t* src, const uint64_t* src_off,
                             const uint64_t* src_len, uint64_t n, const uint8_t* hashes, const uint8_t* kinds,
                             const uint8_t* nonces, uint32_t flags, const bw_packfile* plan, uint64_t npf,
                             const uint8_t* ids, uint8_t* out) {
    if (!c || (n && (!src || !src_off || !src_len)) || (npf && (!plan || !out))) return BW_EINVAL;
    hipSetDevice(c->device);
    uint64_t s_end = 0;
    for (uint64_t i = 0; i < n; i++) s_end = std::max(s_end, src_off[i] + src_len[i]);
    const uint64_t total = npf ? plan[npf - 1].offset + plan[npf - 1].size : 0;
    if (int rc = ensure(c, c->pk_src, s_end)) return rc;
    if (int rc = ensure(c, c->pk_out, total)) return rc;
    if (s_end) HIPCHK(c, hipMemcpyAsync(c->pk_src.p, src, s_end, hipMemcpyHostToDevice, c->stream));
    if (int rc = pack_submit(c, prk, P<uint8_t>(c->pk_src), src_off, src_len, n, hashes, kinds, nonces, flags, plan,
                             npf, ids, P<uint8_t>(c->pk_out)))
        return rc;
    if (total) HIPCHK(c, hipMemcpyAsync(out, c->pk_out.p, total, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return BW_OK;
}

// ------------------------------------------------------------------ index files (§8f row 4)
// BlobIndex::push/flush/load (blob_index.rs:151-240).

static void counter_to_nonce(uint32_t num, uint8_t nonce[12]) {
    memset(nonce, 0, 12);
    for (int k = 0; k < 4; k++) nonce[k] = (uint8_t)(num >> (8 * k));
}

extern "C" int bw_index_files_build(bw_ctx* c, const uint8_t prk[32], const uint8_t* entries, uint64_t n,
                                    uint32_t last_file_num, uint8_t* out, uint64_t cap, bw_index_file* files,
                                    uint64_t files_cap, uint64_t* n_files, uint64_t* total_bytes) {
    if (!c || !prk || !n_files || !total_bytes || (n && !entries)) return BW_EINVAL;
    const uint64_t nf = n / BW_INDEX_MAX_FILE_ENTRIES + 1;  // full files, then the final flush
    if ((uint64_t)last_file_num + nf > 0xffffffffull) {
        c->err = "bug: index file counter overflow";  // blob_index.rs:207-210 expects
        return BW_EINVAL;
    }
    std::vector<bw_index_file> tab(nf);
    std::vector<uint64_t> pt_off(nf), pt_len(nf), dst_off(nf);
    uint64_t off = 0, pt = 0;
    for (uint64_t f = 0; f < nf; f++) {
        const uint64_t cnt = f + 1 < nf ? BW_INDEX_MAX_FILE_ENTRIES : n - f * BW_INDEX_MAX_FILE_ENTRIES;
        pt_off[f] = pt;
        pt_len[f] = varint_len(cnt) + BW_INDEX_ENTRY_BYTES * cnt;
        tab[f] = bw_index_file{(uint32_t)(last_file_num + 1 + f), 0, off, pt_len[f] + BW_SEAL_TAG_BYTES, cnt};
        dst_off[f] = off;
        pt += pt_len[f];
        off += tab[f].size;
    }
    *n_files = nf;
    *total_bytes = off;
    if (!out || cap < off || !files || files_cap < nf) return BW_ENOSPC;
    // plaintexts: bincode varint Vec<([u8; 32], [u8; 12])>
    std::vector<uint8_t> plain(pt);
    std::vector<uint8_t> nonces(12 * nf), info(5 * nf);
    for (uint64_t f = 0; f < nf; f++) {
        uint8_t* p = plain.data() + pt_off[f];
        const uint64_t cnt = tab[f].n_entries;
        if (cnt < 251) {
            *p++ = (uint8_t)cnt;
        } else {
            *p++ = 251;  // cnt <= 50 000 < 2^16
            *p++ = (uint8_t)cnt;
            *p++ = (uint8_t)(cnt >> 8);
        }
        memcpy(p, entries + f * BW_INDEX_MAX_FILE_ENTRIES * BW_INDEX_ENTRY_BYTES, cnt * BW_INDEX_ENTRY_BYTES);
        counter_to_nonce(tab[f].file_num, &nonces[12 * f]);
        memcpy(&info[5 * f], "index", 5);
    }
    if (int rc = bw_seal(c, prk, plain.data(), pt_off.data(), pt_len.data(), nf, info.data(), 5, nonces.data(), out,
                         dst_off.data()))
        return rc;
    std::copy(tab.begin(), tab.end(), files);
    return BW_OK;
}

extern "C" int bw_index_load_files(bw_ctx* c, const uint8_t prk[32], const uint8_t* data, const bw_index_file* files,
                                   uint64_t nf, uint8_t* entries, uint64_t cap, uint64_t* n_entries,
                                   uint64_t* bad_file) {
    if (!c || !prk || !n_entries || (nf && (!data || !files))) return BW_EINVAL;
    *n_entries = 0;
    if (bad_file) *bad_file = ~0ull;
    if (!nf) return BW_OK;
    hipSetDevice(c->device);
    uint64_t end = 0, pt_total = 0;
    std::vector<uint64_t> src_off(nf), src_len(nf), pt_off(nf), pt_len(nf);
    std::vector<uint8_t> nonces(12 * nf), info(5 * nf);
    for (uint64_t f = 0; f < nf; f++) {
        if (files[f].size < BW_SEAL_TAG_BYTES) {  // decrypt_in_place fails on a buffer shorter than the tag
            if (bad_file) *bad_file = f;
            c->err = "index file shorter than the GCM tag";
            return BW_ECRYPTO;
        }
        src_off[f] = files[f].offset;
        src_len[f] = files[f].size;
        end = std::max(end, files[f].offset + files[f].size);
        pt_off[f] = pt_total;
        pt_len[f] = files[f].size - BW_SEAL_TAG_BYTES;
        pt_total += (pt_len[f] + 15) & ~15ull;
        counter_to_nonce(files[f].file_num, &nonces[12 * f]);
        memcpy(&info[5 * f], "index", 5);
    }
    const uint64_t pt_base = (end + 255) & ~255ull;
    if (int rc = ensure(c, c->ix_io, pt_base + pt_total + 16)) return rc;
    uint8_t* io = P<uint8_t>(c->ix_io);
    HIPCHK(c, hipMemcpyAsync(io, data, end, hipMemcpyHostToDevice, c->stream));
    std::vector<uint8_t> ok(nf);
    if (int rc = seal_submit(c, true, prk, io, src_off.data(), src_len.data(), nf, info.data(), 5, nonces.data(),
                             io + pt_base, pt_off.data(), ok.data()))
        return rc;
    for (uint64_t f = 0; f < nf; f++)
        if (!ok[f]) {
            if (bad_file) *bad_file = f;
            c->err = "index file " + std::to_string(files[f].file_num) + " failed authentication";
            return BW_ECRYPTO;
        }
    // parse the Vec length of every file
    if (int rc = ensure(c, c->ix_tab, nf * 8 * 4)) return rc;
    uint64_t* tab = P<uint64_t>(c->ix_tab);
    std::vector<uint64_t> up(2 * nf);
    std::copy(pt_off.begin(), pt_off.end(), up.begin());
    std::copy(pt_len.begin(), pt_len.end(), up.begin() + nf);
    HIPCHK(c, hipMemcpyAsync(tab, up.data(), 2 * nf * 8, hipMemcpyHostToDevice, c->stream));
    launch_index_parse(c->stream, io + pt_base, tab, tab + nf, nf, tab + 2 * nf);
    HIPCHK(c, hipGetLastError());
    std::vector<uint64_t> parsed(2 * nf);
    HIPCHK(c, hipMemcpyAsync(parsed.data(), tab + 2 * nf, 2 * nf * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    std::vector<uint64_t> rec0(nf), fsrc(nf);
    uint64_t R = 0;
    for (uint64_t f = 0; f < nf; f++) {
        if (parsed[2 * f] == ~0ull) {
            if (bad_file) *bad_file = f;
            c->err = "index file " + std::to_string(files[f].file_num) + " is not a bincode Vec<(BlobHash, PackfileId)>";
            return BW_EFORMAT;
        }
        rec0[f] = R;
        fsrc[f] = pt_off[f] + parsed[2 * f + 1];
        R += parsed[2 * f];
    }
    *n_entries = R;
    if (entries && cap < R) return BW_ENOSPC;
    if (!R) return BW_OK;
    std::copy(rec0.begin(), rec0.end(), up.begin());
    std::copy(fsrc.begin(), fsrc.end(), up.begin() + nf);
    HIPCHK(c, hipMemcpyAsync(tab, up.data(), 2 * nf * 8, hipMemcpyHostToDevice, c->stream));
    if (int rc = ensure(c, c->ix_dig, R * 32 + (entries ? R * BW_INDEX_ENTRY_BYTES : 0))) return rc;
    uint8_t* dig = P<uint8_t>(c->ix_dig);
    uint8_t* rec = entries ? dig + R * 32 : nullptr;
    launch_index_gather(c->stream, io + pt_base, tab, tab + nf, nf, R, dig, rec);
    HIPCHK(c, hipGetLastError());
    if (entries) HIPCHK(c, hipMemcpyAsync(entries, rec, R * BW_INDEX_ENTRY_BYTES, hipMemcpyDeviceToHost, c->stream));
    if (int rc = dedup_device(c, dig, nullptr, R, R, nullptr)) return rc;
    return check_collision(c);
}
