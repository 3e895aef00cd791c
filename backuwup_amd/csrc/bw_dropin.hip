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
//     message per call.  Concurrent calls of at most 64 KiB from many threads are coalesced: each
//     caller copies its message into pinned memory of its own (the copies run in parallel on the
//     callers' threads) and adds it to the open batch; a library thread launches the open batch as
//     soon as one of four lanes (streams) is free, and a second one waits for the launched batches
//     and wakes their callers, so under load a batch holds what the other threads brought while the
//     lanes were busy (group commit).  A batch is one kernel that reads the messages from the
//     callers' pinned copies over PCIe and writes the digests into the batch's pinned table
//     (k_b3_msgs).  Larger messages run through the caller's own context (the batch pipeline, in
//     parallel across the callers' contexts): gathered into the one launcher thread they measured
//     30 GB/s on C1 against 55 through the callers' own contexts.
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
static_assert(CO_MAX_MSG == B3_MSG_MAX, "a coalesced batch is one k_b3_msgs launch");
constexpr uint32_t CO_MAX_N = 1u << 16;         // messages per batch
// a batch's table in pinned memory: message addresses, lengths and digests (the small-message
// kernel reads and writes them there, over PCIe)
constexpr uint64_t CO_META = (uint64_t)CO_MAX_N * (8 + 8 + 32);
constexpr int CO_LANES = 4;                     // batches on the GPU at once, a stream each
constexpr int CO_BUFS = CO_LANES + 2;           // tables: in flight, filling, being read

// Each calling thread copies its message into pinned memory of its own before it joins a batch, so
// a batch is complete the moment it is closed: the launcher never waits for a caller that was
// descheduled between reserving room and finishing its copy (with 256 threads on 16 cores it
// waited milliseconds).  The buffer is reused by the thread's next call, after this one returned.
struct TlStage {
    uint8_t* p = nullptr;
    uint64_t cap = 0;
    ~TlStage() {
        if (p) hipHostFree(p);
    }
};
thread_local TlStage t_stage;

struct CoBatch {
    int buf = -1, lane = -1;
    uint8_t* meta = nullptr;
    uint64_t maxlen = 0;
    uint32_t n = 0;
    std::atomic<uint32_t> readers{0};
    std::vector<uint64_t> ptr, len;  // message addresses (each caller's pinned copy) and lengths
    const uint8_t* digp = nullptr;   // the digests (the table's digest area)
    bool sync = false;               // the launch failed: nothing to wait for
    int rc = 0;
    std::mutex mu;                   // its waiters
    std::condition_variable cv;
    bool done = false;
};

// One per device.  Callers add their message to the open batch; a launcher thread closes the open
// batch as soon as a lane is free and launches it; a completer thread waits for the launched batches
// in order and wakes their waiters.  Under load the open batch fills while every lane is busy (group
// commit); idle, a lone call is launched at once.  (Measured against letting the callers launch and
// complete their own batches: the library threads win once the callers outnumber the cores, where a
// caller that owns a finished batch waits for a core before it can hand its lane on.)
struct Combiner {
    int device = 0;
    std::mutex mu;
    std::condition_variable cv_work, cv_done, cv_room;
    bw_ctx* ctx[CO_LANES] = {};  // a lane's context: its stream
    hipEvent_t ev[CO_LANES] = {};
    bool lane_busy[CO_LANES] = {};
    uint8_t* bufs[CO_BUFS] = {};
    bool buf_busy[CO_BUFS] = {};
    std::shared_ptr<CoBatch> open;
    std::vector<std::shared_ptr<CoBatch>> launched;  // FIFO
    std::atomic<uint64_t> batches{0}, messages{0};
};

std::mutex g_co_mu;
Combiner* g_co[64] = {};

void launcher(Combiner* co) {
    hipSetDevice(co->device);
    std::unique_lock<std::mutex> lk(co->mu);
    for (;;) {
        int lane = -1;
        for (;;) {
            lane = -1;
            for (int k = 0; k < CO_LANES; k++)
                if (!co->lane_busy[k]) lane = k;
            if (lane >= 0 && co->open && co->open->n) break;
            co->cv_work.wait(lk);
        }
        std::shared_ptr<CoBatch> b = std::move(co->open);
        co->open.reset();
        co->lane_busy[lane] = true;
        b->lane = lane;
        co->cv_room.notify_all();  // callers waiting for room open the next batch
        lk.unlock();
        {
            // every message fits one wave: one launch reads them from the callers' pinned copies and
            // writes the digests into the batch's pinned table (no copy operations, no batch tables)
            uint64_t* ptrs = (uint64_t*)b->meta;
            uint64_t* lens = ptrs + CO_MAX_N;
            uint8_t* dig = (uint8_t*)(lens + CO_MAX_N);
            memcpy(ptrs, b->ptr.data(), 8ull * b->n);
            memcpy(lens, b->len.data(), 8ull * b->n);
            hipStream_t st = (hipStream_t)bw_get_stream(co->ctx[lane]);
            launch_b3_msgs(st, nullptr, ptrs, lens, b->n, (uint32_t)b->maxlen, dig);
            const hipError_t e = hipGetLastError();
            if (e == hipSuccess) hipEventRecord(co->ev[lane], st);
            b->rc = e == hipSuccess ? BW_OK : BW_EHIP;
            b->sync = e != hipSuccess;
            b->digp = dig;
        }
        co->batches.fetch_add(1, std::memory_order_relaxed);
        co->messages.fetch_add(b->n, std::memory_order_relaxed);
        lk.lock();
        co->launched.push_back(std::move(b));
        co->cv_done.notify_one();
    }
}

void completer(Combiner* co) {
    hipSetDevice(co->device);
    std::unique_lock<std::mutex> lk(co->mu);
    for (;;) {
        while (co->launched.empty()) co->cv_done.wait(lk);
        std::shared_ptr<CoBatch> b = co->launched.front();
        lk.unlock();
        if (!b->sync && hipEventSynchronize(co->ev[b->lane]) != hipSuccess) b->rc = BW_EHIP;
        {
            std::lock_guard<std::mutex> bl(b->mu);
            b->done = true;
        }
        b->cv.notify_all();
        lk.lock();
        co->launched.erase(co->launched.begin());
        co->lane_busy[b->lane] = false;
        co->cv_work.notify_one();
    }
}

Combiner* combiner(int device) {
    if (device < 0 || device >= 64) return nullptr;
    std::lock_guard<std::mutex> lk(g_co_mu);
    if (!g_co[device]) {
        // lives as long as the process (the drop-ins have no teardown call), and so do its threads
        auto* c = new Combiner();
        c->device = device;
        hipSetDevice(device);
        for (int k = 0; k < CO_LANES; k++)
            if (bw_create(device, &c->ctx[k]) != BW_OK ||
                hipEventCreateWithFlags(&c->ev[k], hipEventDisableTiming) != hipSuccess)
                return nullptr;
        for (auto& b : c->bufs)
            if (hipHostMalloc((void**)&b, CO_META, hipHostMallocDefault) != hipSuccess) return nullptr;
        std::thread(launcher, c).detach();
        std::thread(completer, c).detach();
        g_co[device] = c;
    }
    return g_co[device];
}

int coalesced_hash(Combiner* co, const uint8_t* data, uint64_t len, uint8_t out[32]) {
    TlStage& ts = t_stage;
    if (ts.cap < len + 16) {  // this thread's pinned copy of its message
        if (ts.p) hipHostFree(ts.p);
        ts.p = nullptr;
        ts.cap = 0;
        const uint64_t want = std::max<uint64_t>(65536 + 64, len + 16);
        if (hipHostMalloc((void**)&ts.p, want, hipHostMallocDefault) != hipSuccess) return BW_ENOMEM;
        ts.cap = want;
    }
    if (len) memcpy(ts.p, data, len);
    std::shared_ptr<CoBatch> my;
    uint32_t i = 0;
    {
        std::unique_lock<std::mutex> lk(co->mu);
        for (;;) {
            if (!co->open) {
                int b = -1;
                for (int k = 0; k < CO_BUFS && b < 0; k++)
                    if (!co->buf_busy[k]) b = k;
                if (b >= 0) {
                    auto nb = std::make_shared<CoBatch>();
                    nb->buf = b;
                    nb->meta = co->bufs[b];
                    nb->ptr.reserve(256);
                    nb->len.reserve(256);
                    co->buf_busy[b] = true;
                    co->open = std::move(nb);
                }
            }
            if (co->open && co->open->n < CO_MAX_N) break;
            co->cv_room.wait(lk);  // no table free, or the open batch is full: the launcher frees one
        }
        my = co->open;
        i = my->n++;
        my->ptr.push_back((uint64_t)(uintptr_t)ts.p);
        my->len.push_back(len);
        my->maxlen = std::max(my->maxlen, len);
        my->readers.fetch_add(1, std::memory_order_relaxed);
        if (i == 0) co->cv_work.notify_one();  // a new batch: the launcher may take it now
    }
    {
        std::unique_lock<std::mutex> bl(my->mu);
        while (!my->done) my->cv.wait(bl);
    }
    const int rc = my->rc;
    if (!rc) memcpy(out, my->digp + 32ull * i, 32);
    if (my->readers.fetch_sub(1, std::memory_order_acq_rel) == 1) {  // the last reader gives the table back
        std::lock_guard<std::mutex> lk(co->mu);
        co->buf_busy[my->buf] = false;
        co->cv_room.notify_all();
    }
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
