// bw_dropin.hip -- the two-`use`-line integration: the entry points behind the Rust
// drop-ins for `fastcdc::v2020::FastCDC` and `blake3::hash`, called the way the reference calls the
// crates, one task per file from tokio's worker threads (dir_packer.rs:166):
//
//   * CDC files (dir_packer.rs:254-266, then :286 per chunk): bw_fastcdc_chunks_hashed chunks AND
//     hashes the file in one submit and keeps the chunk digests under a handle; the per-chunk
//     blake3::hash drop-in (bw_blake3_hash_dropin) finds its digest there by (pointer, length) while
//     the handle lives.  The registry is an ordered map of the live sources (an interval lookup under
//     a reader lock) with a per-thread cache of the last source hit, so callers on many threads do
//     not serialize on one mutex and a lookup does not scan every open file.
//   * whole-file blobs and tree blobs (dir_packer.rs:267-271 -> :286, :274 -> :320/:353): one small
//     message per call.  Concurrent calls from many threads are coalesced: each caller reserves room
//     in the open batch's pinned staging, copies its own message there (the copies run in parallel
//     on the callers' threads), and one of them -- the leader -- sends the whole batch through one
//     hash_messages launch while the next batch fills; every waiter takes its digest from the batch.
//     One batch is in flight per device at a time, so a batch holds what the other threads brought
//     while the previous one ran (group commit).
//
// Only bw_blake3_hash_dropin consults the kept digests: its caller guarantees that the bytes under a
// live handle do not change (the Rust FastCDC drop-in borrows the mmap immutably for the handle's
// lifetime).  bw_blake3_hash always hashes the bytes it is given (a rewritten buffer must
// never be answered from an earlier chunking).
#include <string.h>

#include <atomic>
#include <condition_variable>
#include <map>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <thread>
#include <vector>

#include "bw_internal.h"

using namespace bw;

namespace {

// ------------------------------------------------------------------ kept chunk digests
struct Kept {
    uint64_t handle;
    const uint8_t* base;
    uint64_t len;
    std::vector<uint64_t> off, clen;  // chunk offsets (ascending) and lengths
    std::vector<uint8_t> dig;         // 32 B per chunk
    std::atomic<bool> live{true};
};

std::shared_mutex g_kept_mu;
// live sources by base address (several handles may share a base: the vector); a lookup takes the
// greatest base <= the pointer and walks down while the ranges could still contain it
std::map<uintptr_t, std::vector<std::shared_ptr<Kept>>> g_kept_by_base;
std::map<uint64_t, std::shared_ptr<Kept>> g_kept_by_handle;
std::atomic<uint64_t> g_kept_next{1}, g_kept_hits{0};
uint64_t g_kept_maxlen = 0;  // the longest live source: bounds the walk down from the greatest base
thread_local std::weak_ptr<Kept> t_last;

bool answer(const Kept& k, const uint8_t* data, uint64_t len, uint8_t out[32]) {
    if (!k.live.load(std::memory_order_acquire) || data < k.base || data >= k.base + k.len) return false;
    const uint64_t o = (uint64_t)(data - k.base);
    auto it = std::lower_bound(k.off.begin(), k.off.end(), o);
    if (it == k.off.end() || *it != o) return false;
    const size_t i = it - k.off.begin();
    if (k.clen[i] != len) return false;
    memcpy(out, k.dig.data() + 32 * i, 32);
    return true;
}

bool kept_lookup(const uint8_t* data, uint64_t len, uint8_t out[32]) {
    if (auto k = t_last.lock())  // the task's own file, almost always
        if (answer(*k, data, len, out)) {
            g_kept_hits.fetch_add(1, std::memory_order_relaxed);
            return true;
        }
    std::shared_lock<std::shared_mutex> lk(g_kept_mu);
    if (g_kept_by_base.empty()) return false;
    auto it = g_kept_by_base.upper_bound((uintptr_t)data);
    while (it != g_kept_by_base.begin()) {
        --it;
        if ((uintptr_t)data - it->first >= g_kept_maxlen) break;  // no live source reaches this far
        for (const auto& k : it->second)
            if (answer(*k, data, len, out)) {
                t_last = k;
                g_kept_hits.fetch_add(1, std::memory_order_relaxed);
                return true;
            }
    }
    return false;
}

// ------------------------------------------------------------------ coalesced small messages
constexpr uint64_t CO_MAX_MSG = BW_COALESCE_MAX_MSG;  // larger messages go through the caller's context
constexpr uint64_t CO_STAGE = 64ull << 20;      // pinned staging per batch
constexpr uint32_t CO_MAX_N = 1u << 16;         // messages per batch
constexpr int CO_BUFS = 2;                      // staging buffers: one in flight, one filling

struct CoBatch {
    uint8_t* stage = nullptr;
    int buf = -1;
    uint64_t used = 0;
    uint32_t n = 0;
    std::vector<uint64_t> off, len;
    std::atomic<uint32_t> copied{0};
    std::vector<uint8_t> dig;
    int rc = 0;
    bool done = false;
};

struct Combiner {
    int device = 0;
    std::mutex mu;
    std::condition_variable cv;
    bw_ctx* ctx = nullptr;  // used by one leader at a time
    uint8_t* bufs[CO_BUFS] = {};
    bool buf_busy[CO_BUFS] = {};
    std::shared_ptr<CoBatch> open;
    bool in_flight = false;
    std::atomic<uint64_t> batches{0}, messages{0};
};

std::mutex g_co_mu;
Combiner* g_co[64] = {};

Combiner* combiner(int device) {
    if (device < 0 || device >= 64) return nullptr;
    std::lock_guard<std::mutex> lk(g_co_mu);
    if (!g_co[device]) {
        auto* c = new Combiner();  // lives as long as the process (the drop-ins have no teardown call)
        c->device = device;
        if (bw_create(device, &c->ctx) != BW_OK) {
            delete c;
            return nullptr;
        }
        hipSetDevice(device);
        for (auto& b : c->bufs)
            if (hipHostMalloc((void**)&b, CO_STAGE, hipHostMallocDefault) != hipSuccess) return nullptr;
        g_co[device] = c;
    }
    return g_co[device];
}

// Lock held.  A fresh open batch on a free staging buffer, or false when both are busy.
bool open_batch(Combiner* co) {
    for (int b = 0; b < CO_BUFS; b++)
        if (!co->buf_busy[b]) {
            auto nb = std::make_shared<CoBatch>();
            nb->buf = b;
            nb->stage = co->bufs[b];
            nb->off.reserve(256);
            nb->len.reserve(256);
            co->buf_busy[b] = true;
            co->open = std::move(nb);
            return true;
        }
    return false;
}

// Lock held on entry and exit: close `my` (the open batch), send it, publish the digests.
void lead(Combiner* co, std::unique_lock<std::mutex>& lk, const std::shared_ptr<CoBatch>& my) {
    co->open.reset();
    co->in_flight = true;
    lk.unlock();
    while (my->copied.load(std::memory_order_acquire) != my->n) std::this_thread::yield();  // reservers' copies
    my->dig.resize(32ull * my->n);
    hipSetDevice(co->device);
    my->rc = hash_messages(co->ctx, my->stage, my->used, my->off.data(), my->len.data(), my->n, false,
                           my->dig.data(), nullptr);
    co->batches.fetch_add(1, std::memory_order_relaxed);
    co->messages.fetch_add(my->n, std::memory_order_relaxed);
    lk.lock();
    my->done = true;
    co->buf_busy[my->buf] = false;
    co->in_flight = false;
    co->cv.notify_all();
}

int coalesced_hash(Combiner* co, const uint8_t* data, uint64_t len, uint8_t out[32]) {
    const uint64_t room = (len + 15) & ~15ull;
    std::unique_lock<std::mutex> lk(co->mu);
    for (;;) {
        if (!co->open && !open_batch(co)) {
            co->cv.wait(lk);
            continue;
        }
        CoBatch& b = *co->open;
        if (b.used + room <= CO_STAGE && b.n < CO_MAX_N) break;
        if (!co->in_flight) {  // full and nothing in flight: send it, then take the next one
            std::shared_ptr<CoBatch> full = co->open;
            lead(co, lk, full);
        } else {
            co->cv.wait(lk);
        }
    }
    std::shared_ptr<CoBatch> my = co->open;
    const uint32_t i = my->n++;
    const uint64_t at = my->used;
    my->used += room;
    my->off.push_back(at);
    my->len.push_back(len);
    lk.unlock();
    if (len) memcpy(my->stage + at, data, len);
    my->copied.fetch_add(1, std::memory_order_release);
    lk.lock();
    while (!my->done) {
        if (!co->in_flight && co->open == my) {
            lead(co, lk, my);
            break;
        }
        co->cv.wait(lk);
    }
    const int rc = my->rc;
    lk.unlock();
    if (!rc) memcpy(out, my->dig.data() + 32ull * i, 32);
    return rc;
}

int hash_one(bw_ctx* c, const uint8_t* data, uint64_t len, uint8_t out[32]) {
    if (len <= CO_MAX_MSG)
        if (Combiner* co = combiner(ctx_device(c))) return coalesced_hash(co, data, len, out);
    const uint64_t off = 0;
    static const uint8_t empty[16] = {0};
    return bw_blake3_hash_many(c, len ? data : empty, len, &off, &len, 1, out);
}

}  // namespace

extern "C" int bw_fastcdc_chunks_hashed(bw_ctx* c, const uint8_t* src, uint64_t len, uint32_t mn, uint32_t av,
                                        uint32_t mx, bw_chunk* out, uint64_t cap, uint64_t* n_out, uint64_t* handle) {
    if (!c || !n_out || !handle || (len && !src)) return BW_EINVAL;
    *handle = 0;
    *n_out = 0;
    // FastCDC::with_level's asserts hold for an empty source too
    if (mn < BW_MINIMUM_MIN || mn > BW_MINIMUM_MAX || av < BW_AVERAGE_MIN || av > BW_AVERAGE_MAX ||
        mx < BW_MAXIMUM_MIN || mx > BW_MAXIMUM_MAX)
        return BW_EINVAL;
    if (len == 0) return BW_OK;
    bw_params p;
    p.min_size = mn;
    p.avg_size = av;
    p.max_size = mx;
    p.flags = BW_F_NO_DEDUP;  // chunk + hash; the gate stays the caller's (add_blob)
    p.small_file_threshold = 0;
    const uint64_t off = 0;
    std::vector<bw_blob> tmp(len / std::min<uint64_t>(2 * (mn / 2), mx) + 2);
    uint64_t n = 0;
    // the file goes up as one pageable hipMemcpy, not through the context's pinned staging ring: the
    // reference's tasks call this from many threads at once (one mmap'd file each), and 16 callers
    // each fanning their memcpy out over 16 ring threads ran at 35 GB/s on C1 against 47-56 for
    // the runtime's own pageable copies (profiles/r04/s05_keptab)
    if (int rc = bw_process_files(c, src, len, &off, &len, 1, &p, tmp.data(), tmp.size(), &n)) return rc;
    *n_out = n;
    if (n > cap) return BW_ENOSPC;
    auto k = std::make_shared<Kept>();
    k->base = src;
    k->len = len;
    k->off.resize(n);
    k->clen.resize(n);
    k->dig.resize(32 * n);
    for (uint64_t i = 0; i < n; i++) {
        out[i].hash = tmp[i].gear_hash;
        out[i].offset = tmp[i].offset;
        out[i].length = tmp[i].length;
        k->off[i] = tmp[i].offset;
        k->clen[i] = tmp[i].length;
        memcpy(k->dig.data() + 32 * i, tmp[i].digest, 32);
    }
    k->handle = g_kept_next++;
    {
        std::unique_lock<std::shared_mutex> lk(g_kept_mu);
        g_kept_by_base[(uintptr_t)src].push_back(k);
        g_kept_by_handle[k->handle] = k;
        g_kept_maxlen = std::max(g_kept_maxlen, len);
    }
    t_last = k;  // this thread's next lookups are its chunks (dir_packer.rs:261-266)
    *handle = k->handle;
    return BW_OK;
}

extern "C" void bw_fastcdc_release(uint64_t handle) {
    if (!handle) return;
    std::unique_lock<std::shared_mutex> lk(g_kept_mu);
    auto h = g_kept_by_handle.find(handle);
    if (h == g_kept_by_handle.end()) return;
    std::shared_ptr<Kept> k = h->second;
    k->live.store(false, std::memory_order_release);
    g_kept_by_handle.erase(h);
    auto b = g_kept_by_base.find((uintptr_t)k->base);
    if (b != g_kept_by_base.end()) {
        auto& v = b->second;
        v.erase(std::remove(v.begin(), v.end(), k), v.end());
        if (v.empty()) g_kept_by_base.erase(b);
    }
    if (g_kept_by_handle.empty()) g_kept_maxlen = 0;  // (otherwise it stays an upper bound)
}

extern "C" uint64_t bw_blake3_kept_hits(void) { return g_kept_hits.load(); }

extern "C" int bw_blake3_coalesce_stats(int device, uint64_t* batches, uint64_t* messages) {
    if (device < 0 || device >= 64) return BW_EINVAL;
    std::lock_guard<std::mutex> lk(g_co_mu);
    const Combiner* co = g_co[device];
    if (batches) *batches = co ? co->batches.load() : 0;
    if (messages) *messages = co ? co->messages.load() : 0;
    return BW_OK;
}

extern "C" int bw_blake3_hash(bw_ctx* c, const uint8_t* data, uint64_t len, uint8_t out[32]) {
    if (!c || !out || (len && !data)) return BW_EINVAL;
    return hash_one(c, data, len, out);
}

extern "C" int bw_blake3_hash_dropin(bw_ctx* c, const uint8_t* data, uint64_t len, uint8_t out[32]) {
    if (!c || !out || (len && !data)) return BW_EINVAL;
    if (len && kept_lookup(data, len, out)) return BW_OK;
    return hash_one(c, data, len, out);
}
