// bw_capi_pack.hip -- the C ABI of the write side after the hot path (include/backuwup_gpu.h):
// blob sealing, per-blob zstd, packfiles and index files.  Shares the
// context's private state (bw_ctx.h) with bw_capi.hip.
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
#include "bw_ctx.h"

using namespace bw;

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
    if (int rc = ensure_host(c, c->seal_stage, bytes)) return rc;
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

// ------------------------------------------------------------------ zstd level 3

extern "C" int bw_zstd_compress_device(bw_ctx* c, const uint8_t* d_src, const uint64_t* src_off, const uint64_t* src_len,
                                       uint64_t n, uint8_t* d_dst, const uint64_t* dst_off, uint64_t* frame_len) {
    if (!c || (n && (!d_src || !src_off || !src_len || !d_dst || !dst_off || !frame_len))) return BW_EINVAL;
    hipSetDevice(c->device);
    return zstd_compress(c->stream, c->zw, d_src, src_off, src_len, n, d_dst, dst_off, frame_len, c->err);
}

extern "C" int bw_zstd_submit_device(bw_ctx* c, const uint8_t* d_src, const uint64_t* src_off, const uint64_t* src_len,
                                     uint64_t n, uint8_t* d_dst, const uint64_t* dst_off, uint64_t* ticket) {
    if (!c || !ticket || (n && (!d_src || !src_off || !src_len || !d_dst || !dst_off))) return BW_EINVAL;
    *ticket = 0;
    for (uint64_t i = 0; i < n; i++)
        if (src_len[i] > 3ull * 1024 * 1024) {
            c->err = "zstd: blob larger than BLOB_MAX_UNCOMPRESSED_SIZE (3 MiB)";
            return BW_EINVAL;
        }
    bw_ctx::ZsLane* L = nullptr;
    for (auto& x : c->zs_lanes)
        if (!x.ticket) {
            L = &x;
            break;
        }
    // Every lane on a stream of its own, each on a hardware queue of its own where the runtime has
    // one: HIP maps a process's streams of one priority onto GPU_MAX_HW_QUEUES queues (4 by
    // default), and two lanes sharing a queue run one after the other.  The runtime keeps a queue
    // pool per priority, so lanes 0-3 take high-priority streams (a pool nothing else in the library
    // uses, except BW_OPT_LATENCY_STREAM) and lanes 4-5 normal ones.  1 GiB text batches from one
    // host thread with the default 4 queues (profiles/r05/s28_zstd_lanes .. s31): 3 lanes 2.86-2.90
    // GB/s (round 4's normal-priority lanes, lane 0 on the context's stream: 2.32), 4 lanes 3.52-3.56,
    // 5 lanes 4.04, 6 lanes 4.43-4.56; 8 lanes 3.46 (two share the context's queues; 5.01 with 8
    // queues).  BW_ZSTD_LANE_PRIO=normal restores round 4's placement (A/B): with fewer than
    // BW_ZSTD_LANES + 2 queues lane 0 then runs on the context's stream.
    static const int hw_queues = [] {
        const char* q = getenv("GPU_MAX_HW_QUEUES");
        return q && atoi(q) > 0 ? atoi(q) : 4;
    }();
    static const bool lane_high = [] {
        const char* e = getenv("BW_ZSTD_LANE_PRIO");
        return !(e && !strcmp(e, "normal"));
    }();
    const bool own = lane_high || L != &c->zs_lanes[0] || hw_queues >= BW_ZSTD_LANES + 2;  // + the context's, the caller's
    if (!L) {
        c->err = "every zstd lane holds a batch (BW_ZSTD_LANES = " + std::to_string(BW_ZSTD_LANES) +
                 "): bw_zstd_wait for one first";
        return BW_ESTATE;
    }
    hipSetDevice(c->device);
    if (own) {
        if (!L->own_st) {
            int least = 0, greatest = 0;
            HIPCHK(c, hipDeviceGetStreamPriorityRange(&least, &greatest));
            const bool hi = lane_high && L - c->zs_lanes < 4;  // (the high pool's default 4 queues)
            HIPCHK(c, hipStreamCreateWithPriority(&L->own_st, hipStreamNonBlocking, hi ? greatest : 0));
        }
        if (!L->ready) HIPCHK(c, hipEventCreateWithFlags(&L->ready, hipEventDisableTiming));
        HIPCHK(c, hipEventRecord(L->ready, c->stream));
        HIPCHK(c, hipStreamWaitEvent(L->own_st, L->ready, 0));
        L->st = L->own_st;
    } else {
        // lane 0 on the context's stream: its library thread synchronizes that stream, so work the
        // caller queues there after this submit is waited for too (include/backuwup_gpu.h)
        L->st = c->stream;
    }
    zstd_work_copy_limits(L->w, c->zw);  // the context's BW_OPT_ZSTD_* limits
    L->so.assign(src_off, src_off + n);
    L->sl.assign(src_len, src_len + n);
    L->dof.assign(dst_off, dst_off + n);
    L->fl.assign(n, 0);
    L->rc = BW_OK;
    L->err.clear();
    L->ticket = c->zs_next++;
    const int dev = c->device;
    L->th = std::thread([L, dev, d_src, d_dst, n] {
        hipSetDevice(dev);
        L->rc = zstd_compress(L->st, L->w, d_src, L->so.data(), L->sl.data(), n, d_dst, L->dof.data(), L->fl.data(),
                              L->err);
    });
    *ticket = L->ticket;
    return BW_OK;
}

extern "C" int bw_zstd_wait(bw_ctx* c, uint64_t ticket, uint64_t* frame_len) {
    if (!c || !ticket) return BW_EINVAL;
    for (auto& L : c->zs_lanes) {
        if (L.ticket != ticket) continue;
        if (L.th.joinable()) L.th.join();
        L.ticket = 0;
        if (L.rc) {
            c->err = L.err;
            return L.rc;
        }
        if (!L.fl.empty()) {
            if (!frame_len) return BW_EINVAL;
            memcpy(frame_len, L.fl.data(), L.fl.size() * 8);
        }
        return BW_OK;
    }
    c->err = "zstd ticket " + std::to_string(ticket) + " is not (or no longer) held by the context";
    return BW_ESTATE;
}

extern "C" int bw_zstd_compress(bw_ctx* c, const uint8_t* src, const uint64_t* src_off, const uint64_t* src_len, uint64_t n,
                                uint8_t* dst, const uint64_t* dst_off, uint64_t* frame_len) {
    if (!c || (n && (!src || !src_off || !src_len || !dst || !dst_off || !frame_len))) return BW_EINVAL;
    hipSetDevice(c->device);
    // inputs packed back to back on the device, frames at their store-frame capacity
    std::vector<uint64_t> so(n), fo(n);
    uint64_t in = 0, out = 0;
    for (uint64_t i = 0; i < n; i++) {
        if (src_len[i] > 3ull * 1024 * 1024) return BW_EINVAL;
        so[i] = in;
        in += (src_len[i] + 15) & ~15ull;
        fo[i] = out;
        out += bw_zstd_store_size(src_len[i]);
    }
    if (int rc = ensure(c, c->zs_io, in + out + 16)) return rc;
    uint8_t* io = P<uint8_t>(c->zs_io);
    for (uint64_t i = 0; i < n; i++)
        if (src_len[i]) HIPCHK(c, hipMemcpyAsync(io + so[i], src + src_off[i], src_len[i], hipMemcpyHostToDevice, c->stream));
    if (int rc = zstd_compress(c->stream, c->zw, io, so.data(), src_len, n, io + in, fo.data(), frame_len, c->err)) return rc;
    for (uint64_t i = 0; i < n; i++)
        HIPCHK(c, hipMemcpyAsync(dst + dst_off[i], io + in + fo[i], frame_len[i], hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return BW_OK;
}

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

// write_packfiles' drain (pack.rs:123-148) over queue positions [i, to): packfiles close when their
// blob section reaches PACKFILE_TARGET_SIZE or PACKFILE_MAX_BLOBS blobs; the last may be a remainder.
static void plan_range(const uint64_t* payload_len, uint64_t i, uint64_t to, uint32_t flags,
                       std::vector<bw_packfile>& out, uint64_t& off) {
    while (i < to) {
        bw_packfile p{};
        p.first_blob = i;
        uint64_t written = 0, hdr = 0;
        while (i < to) {
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

static void plan_packfiles(const uint64_t* payload_len, uint64_t n, uint32_t flags, std::vector<bw_packfile>& out) {
    uint64_t off = 0;
    plan_range(payload_len, 0, n, flags, out, off);
}

// A plan is acceptable if it is what write_packfiles could have produced for this queue: packfiles
// cover the queue in order, none closes later than the target size / blob count allows (earlier
// is a remainder: a drain ended there), and every size and offset is consistent.
static bool plan_valid(const uint64_t* payload_len, uint64_t n, uint32_t flags, const bw_packfile* plan, uint64_t npf,
                       std::string& why) {
    uint64_t next = 0, off = 0;
    for (uint64_t p = 0; p < npf; p++) {
        const bw_packfile& f = plan[p];
        if (f.first_blob != next || f.n_blobs == 0 || f.n_blobs > n - next || f.offset != off) {
            why = "packfile " + std::to_string(p) + " does not continue the queue";
            return false;
        }
        uint64_t written = 0, hdr = 0;
        for (uint64_t k = 0; k < f.n_blobs; k++) {
            if (k && (written >= BW_PACKFILE_TARGET_SIZE || k >= BW_PACKFILE_MAX_BLOBS)) {
                why = "packfile " + std::to_string(p) + " holds blobs past its close point";
                return false;
            }
            const uint64_t sealed = sealed_len_of(payload_len[f.first_blob + k], flags);
            hdr += entry_len(sealed, written);
            written += sealed + BW_BLOB_NONCE_SIZE;
        }
        const uint64_t header_len = hdr + varint_len(f.n_blobs) + BW_SEAL_TAG_BYTES;
        if (f.header_len != header_len || f.size != 8 + header_len + written) {
            why = "packfile " + std::to_string(p) + " sizes do not match its blobs";
            return false;
        }
        next += f.n_blobs;
        off += f.size;
    }
    if (next != n) {
        why = "the plan does not cover every blob";
        return false;
    }
    return true;
}

namespace {
struct DigestKey {
    const uint8_t* d;
    bool operator==(const DigestKey& o) const { return memcmp(d, o.d, 32) == 0; }
};
struct DigestHash {
    size_t operator()(const DigestKey& k) const {
        uint64_t v;
        memcpy(&v, k.d, 8);
        return (size_t)v;
    }
};
}  // namespace

extern "C" int bw_pack_plan_session(const uint8_t* digests, const uint8_t* is_dup, const uint64_t* payload_len,
                                    uint64_t n, uint32_t flags, bw_packfile* out, uint64_t cap, uint64_t* n_out,
                                    uint64_t* total_bytes, uint64_t* n_unique) {
    if (!n_out || !total_bytes || (n && (!digests || !is_dup || !payload_len)) || (cap && !out)) return BW_EINVAL;
    // the queue = the blobs the gate found new (is_dup == 0), in canonical order
    std::vector<uint64_t> ulen;
    std::unordered_map<DigestKey, uint64_t, DigestHash> first;  // digest -> its queue position
    ulen.reserve(n);
    for (uint64_t i = 0; i < n; i++)
        if (!is_dup[i]) {
            first.emplace(DigestKey{digests + 32 * i}, ulen.size());
            ulen.push_back(payload_len[i]);
        }
    // Manager::add_blob + trigger_write_if_desired (pack.rs:31-55, 92-113) in canonical order: a
    // copy of a blob that is still pending passes add_blob's gate and is queued too (it counts
    // toward the trigger and is dropped when its drain reaches it); a copy of a written or seeded
    // blob is dropped at once.  Between drains the index does not change, so the trigger's rescan
    // of the queue is a running sum.
    std::vector<bw_packfile> pl;
    uint64_t off = 0, placed = 0, queued_to = 0, pend_bytes = 0, pend_cnt = 0;
    for (uint64_t i = 0; i < n; i++) {
        uint64_t sealed;
        if (!is_dup[i]) {
            sealed = sealed_len_of(ulen[queued_to++], flags);
        } else {
            auto it = first.find(DigestKey{digests + 32 * i});
            if (it == first.end() || it->second < placed) continue;  // seeded or already written
            sealed = sealed_len_of(ulen[it->second], flags);
        }
        pend_bytes += sealed;
        pend_cnt++;
        if (pend_bytes >= BW_PACKFILE_TARGET_SIZE || pend_cnt >= BW_PACKFILE_MAX_BLOBS) {
            plan_range(ulen.data(), placed, queued_to, flags, pl, off);  // write_packfiles(true)
            placed = queued_to;
            pend_bytes = pend_cnt = 0;
        }
    }
    plan_range(ulen.data(), placed, queued_to, flags, pl, off);  // Manager::flush
    *n_out = pl.size();
    *total_bytes = off;
    if (n_unique) *n_unique = ulen.size();
    if (pl.size() > cap) return BW_ENOSPC;
    std::copy(pl.begin(), pl.end(), out);
    return BW_OK;
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
    // the plan must be a grouping write_packfiles could produce for exactly these blobs
    // (bw_pack_plan: one drain; bw_pack_plan_session: the reference's cadence)
    std::string why;
    if (!plan_valid(src_len, n, flags, plan, npf, why)) {
        c->err = "packfile plan does not match the blobs: " + why;
        return BW_EINVAL;
    }
    for (uint64_t p = 0; p < npf; p++)
        if (plan[p].size > BW_PACKFILE_MAX_SIZE) {
            c->err = "bug: violated packfile size limit";  // pack.rs:152-156 asserts
            return BW_EINVAL;
        }
    for (uint64_t i = 0; i < n; i++)
        if (kinds[i] > BW_BLOB_TREE) return BW_EINVAL;
        else if ((flags & BW_PACK_ZSTD_STORE) && src_len[i] > BW_BLOB_MAX_UNCOMPRESSED_SIZE) {
            // add_blob rejects it (PackfileError::BlobTooLarge, pack.rs:32-34) and the reader
            // decompresses into a 3 MiB buffer (unpack.rs:67)
            c->err = "blob " + std::to_string(i) + " exceeds BLOB_MAX_UNCOMPRESSED_SIZE";
            return BW_EINVAL;
        }
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

// compress_encrypt_blob + write_packfiles end to end on the device (pack.rs:58-80, 115-227):
// level-3 frames of the queue's blobs into the context's staging area, then -- after the host's
// plan over the frame lengths -- sealing and packfile layout straight from that staging.
extern "C" int bw_pack_compress_device(bw_ctx* c, const uint8_t* d_src, const uint64_t* src_off,
                                       const uint64_t* src_len, uint64_t n, uint64_t* frame_len) {
    if (!c || (n && (!d_src || !src_off || !src_len || !frame_len))) return BW_EINVAL;
    hipSetDevice(c->device);
    // whatever was staged before is gone; a call that fails leaves nothing staged, so a later
    // bw_pack_build_compressed cannot seal stale staging bytes under a plan of empty frames
    c->pk_stage_off.clear();
    c->pk_stage_len.clear();
    for (uint64_t i = 0; i < n; i++)
        if (src_len[i] > BW_BLOB_MAX_UNCOMPRESSED_SIZE) {  // BlobTooLarge, pack.rs:32-34
            c->err = "blob " + std::to_string(i) + " is larger than BLOB_MAX_UNCOMPRESSED_SIZE";
            return BW_EINVAL;
        }
    std::vector<uint64_t> off(n);
    uint64_t out = 0;
    for (uint64_t i = 0; i < n; i++) {
        off[i] = out;
        out += (bw_zstd_store_size(src_len[i]) + 15) & ~15ull;
    }
    if (int rc = ensure(c, c->pk_stage, out + 16)) return rc;
    if (int rc = zstd_compress(c->stream, c->zw, d_src, src_off, src_len, n, P<uint8_t>(c->pk_stage), off.data(),
                               frame_len, c->err))
        return rc;
    c->pk_stage_off = std::move(off);
    c->pk_stage_len.assign(frame_len, frame_len + n);
    return BW_OK;
}

extern "C" int bw_pack_build_compressed(bw_ctx* c, const uint8_t prk[32], const uint8_t* hashes, const uint8_t* kinds,
                                        const uint8_t* nonces, const bw_packfile* plan, uint64_t npf,
                                        const uint8_t* ids, uint8_t* d_out) {
    if (!c) return BW_EINVAL;
    hipSetDevice(c->device);
    const uint64_t n = c->pk_stage_len.size();
    if (npf && plan[npf - 1].first_blob + plan[npf - 1].n_blobs != n) {
        c->err = "the plan does not cover the staged blobs";
        return BW_EINVAL;
    }
    return pack_submit(c, prk, P<uint8_t>(c->pk_stage), c->pk_stage_off.data(), c->pk_stage_len.data(), n, hashes,
                       kinds, nonces, 0, plan, npf, ids, d_out);
}

// Host-buffer forms of the chain: the blobs are uploaded back to back into the context's
// staging source, the packfiles come back into the caller's buffer (synchronous).
extern "C" int bw_pack_compress(bw_ctx* c, const uint8_t* src, const uint64_t* src_off, const uint64_t* src_len,
                                uint64_t n, uint64_t* frame_len) {
    if (!c || (n && (!src_off || !src_len || !frame_len))) return BW_EINVAL;
    // src may be NULL when every blob is empty (a queue of empty files has no bytes to point at)
    for (uint64_t i = 0; i < n && !src; i++)
        if (src_len[i]) return BW_EINVAL;
    hipSetDevice(c->device);
    std::vector<uint64_t> so(n);
    uint64_t in = 0;
    for (uint64_t i = 0; i < n; i++) {
        if (src_len[i] > BW_BLOB_MAX_UNCOMPRESSED_SIZE) return BW_EINVAL;
        so[i] = in;
        in += (src_len[i] + 15) & ~15ull;
    }
    if (int rc = ensure(c, c->pk_src, in + 16)) return rc;
    for (uint64_t i = 0; i < n; i++)
        if (src_len[i])
            HIPCHK(c, hipMemcpyAsync(P<uint8_t>(c->pk_src) + so[i], src + src_off[i], src_len[i], hipMemcpyHostToDevice,
                                     c->stream));
    return bw_pack_compress_device(c, P<uint8_t>(c->pk_src), so.data(), src_len, n, frame_len);
}

extern "C" int bw_pack_build_compressed_host(bw_ctx* c, const uint8_t prk[32], const uint8_t* hashes,
                                             const uint8_t* kinds, const uint8_t* nonces, const bw_packfile* plan,
                                             uint64_t npf, const uint8_t* ids, uint8_t* out) {
    if (!c || (npf && (!plan || !out))) return BW_EINVAL;
    hipSetDevice(c->device);
    const uint64_t total = npf ? plan[npf - 1].offset + plan[npf - 1].size : 0;
    if (int rc = ensure(c, c->pk_out, total + 16)) return rc;
    if (int rc = bw_pack_build_compressed(c, prk, hashes, kinds, nonces, plan, npf, ids, P<uint8_t>(c->pk_out)))
        return rc;
    if (total) HIPCHK(c, hipMemcpyAsync(out, c->pk_out.p, total, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return BW_OK;
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
