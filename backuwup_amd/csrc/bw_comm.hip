// bw_comm.hip -- the transport of the multi-GPU digest exchange (include/backuwup_gpu.h, bw_comm_*).
//
// The reference keeps one BlobIndex behind the packer mutex (packfile/mod.rs:77, blob_index.rs:
// 130-148).  Across the GPUs of a node the index is partitioned by digest prefix and every batch's
// digests travel to their owner and its verdicts back (bw_exchange_dedup in bw_capi.hip).  The one
// collective that needs is an all-to-all with equal splits, which this file provides over either
//   * RCCL (ncclSend/ncclRecv pairs in one group, on the batch's stream, over xGMI), or
//   * a caller's host function (staged through pinned memory; synchronous) -- for a transport the
//     caller already has, e.g. several processes on one GPU in tests, where RCCL refuses a
//     communicator with two ranks on the same device.
//
// Failure path (round 4).  The reference never lets one peer stall the packer: its transport sends
// with timeouts (net_p2p/transport.rs:127-128).  Here every wait on a peer has a deadline:
//   * the RCCL communicators are non-blocking (ncclConfig_t.blocking = 0), so initialisation and
//     every enqueue return at once and are polled with ncclCommGetAsyncError against the deadline;
//   * a wait for a batch whose exchange is in flight polls its event and the async error state;
//   * on an error or a missed deadline both communicators are aborted (ncclCommAbort stops the
//     kernels that wait on a dead peer), the communicator is marked failed, and every later call
//     returns BW_ECOMM at once.
#include <string.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <rccl/rccl.h>

#include "bw_internal.h"

static_assert(BW_COMM_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "the C ABI's id size is RCCL's");

struct bw_comm {
    int device = 0, rank = 0, world = 1;
    ncclComm_t nccl = nullptr;            // RCCL transport: the data path (digests out, verdicts back)
    ncclComm_t ctl = nullptr;             // split of `nccl` at initialisation: the per-exchange counts,
                                          // on a stream of its own
    hipStream_t ctl_st = nullptr;
    uint64_t* ctl_buf = nullptr;          // device, 6 x world u64: [0, 2W) the counts received,
                                          // [2W, 4W) / [4W, 6W) an allgather's send / receive
    bw_host_all_to_all host_fn = nullptr;  // or the caller's host transport
    void* user = nullptr;
    void (*user_free)(void*) = nullptr;    // releases `user` with the communicator (bw_comm_init_local)
    void* exq = nullptr;                   // exchanges waiting for their counts (bw_capi.hip)
    uint32_t timeout_ms = BW_COMM_DEFAULT_TIMEOUT_MS;
    bool failed = false;                   // aborted: every call returns BW_ECOMM
    void* pin_send = nullptr;              // host transport: pinned staging, 2 x pin_cap
    size_t pin_cap = 0;
    // The communicator's collectives run in the order the host issued them, whatever streams they
    // were issued on: every one waits for the previous one's `tail`.  Contexts with batches in
    // flight issue their exchanges on their own streams, and two RCCL operations of one
    // communicator running at once on one GPU can wait on each other forever.
    hipEvent_t tail = nullptr;
    hipStream_t tail_stream = nullptr;
    hipEvent_t ctl_tail = nullptr;  // likewise for the control communicator (counts, allgathers)
    hipStream_t ctl_tail_stream = nullptr;
    std::string err;
};

namespace {

using Clock = std::chrono::steady_clock;

int comm_err(bw_comm* c, std::string& err, const std::string& what) {
    err = what;
    if (c) c->err = what;
    return BW_ECOMM;
}

void abort_all(bw_comm* c) {
    if (c->failed) return;
    c->failed = true;
    if (c->ctl) ncclCommAbort(c->ctl);
    if (c->nccl) ncclCommAbort(c->nccl);
    c->ctl = nullptr;
    c->nccl = nullptr;
}

int fail(bw_comm* c, std::string& err, const std::string& what) {
    abort_all(c);
    return comm_err(c, err, what + " (communicator aborted)");
}

Clock::time_point deadline_of(const bw_comm* c) { return Clock::now() + std::chrono::milliseconds(c->timeout_ms); }

// Between two polls of a wait on the GPU or the peers: yield for the first 2 ms (an exchange's
// counts or an RCCL enqueue normally settle within tens of microseconds, and the batch pipeline
// waits for them), then sleep 50 us.
void pace(Clock::time_point since) {
    if (Clock::now() - since < std::chrono::milliseconds(2))
        std::this_thread::yield();
    else
        std::this_thread::sleep_for(std::chrono::microseconds(50));
}

// An error reported by either communicator (ncclInProgress = still enqueuing, not an error).
ncclResult_t async_state(bw_comm* c) {
    for (ncclComm_t k : {c->nccl, c->ctl}) {
        if (!k) continue;
        ncclResult_t r = ncclSuccess;
        if (ncclCommGetAsyncError(k, &r) != ncclSuccess) return ncclInternalError;
        if (r != ncclSuccess) return r;
    }
    return ncclSuccess;
}

// A non-blocking call returned r: wait (to the deadline) until communicator k has finished it.
int settle(bw_comm* c, ncclComm_t k, ncclResult_t r, const char* what, std::string& err) {
    if (r != ncclSuccess && r != ncclInProgress) return fail(c, err, std::string(what) + ": " + ncclGetErrorString(r));
    const auto t0 = Clock::now(), dl = deadline_of(c);
    for (;;) {
        ncclResult_t s = ncclSuccess;
        if (ncclCommGetAsyncError(k, &s) != ncclSuccess) return fail(c, err, std::string(what) + ": async state");
        if (s == ncclSuccess) return BW_OK;
        if (s != ncclInProgress) return fail(c, err, std::string(what) + ": " + ncclGetErrorString(s));
        if (Clock::now() > dl)
            return fail(c, err, std::string(what) + ": no progress within " + std::to_string(c->timeout_ms) + " ms");
        pace(t0);
    }
}

}  // namespace

int bw::comm_rank(const bw_comm* c) { return c->rank; }
int bw::comm_world(const bw_comm* c) { return c->world; }
int bw::comm_device(const bw_comm* c) { return c->device; }
void*& bw::comm_exq(bw_comm* c) { return c->exq; }
bool bw::comm_failed(const bw_comm* c) { return c->failed; }

// Wait for `ev` (recorded after work that includes this communicator's collectives): polls the
// event and the communicators' async error state until the deadline; aborts on either.
int bw::comm_wait_event(bw_comm* c, hipEvent_t ev, std::string& err) {
    if (c->failed) return comm_err(c, err, "the communicator was aborted by an earlier failure");
    const auto t0 = Clock::now(), dl = deadline_of(c);
    for (;;) {
        const hipError_t q = hipEventQuery(ev);
        if (q == hipSuccess) return BW_OK;
        if (q != hipErrorNotReady) return fail(c, err, std::string("hipEventQuery: ") + hipGetErrorString(q));
        if (c->nccl) {
            const ncclResult_t a = async_state(c);
            if (a != ncclSuccess && a != ncclInProgress)
                return fail(c, err, std::string("RCCL async error: ") + ncclGetErrorString(a));
        }
        if (Clock::now() > dl)
            return fail(c, err, "a collective did not complete within " + std::to_string(c->timeout_ms) +
                                    " ms (a peer failed or stalled)");
        pace(t0);
    }
}

// The per-exchange counts (16 bytes per rank, include/backuwup_gpu.h bw_exchange_dedup): d_send[2r, 2r+1]
// goes to rank r, d_recv[2k, 2k+1] = what rank k sent here.  RCCL: on the control communicator,
// enqueued on st right behind the partition that wrote d_send (no host synchronization); the
// control communicator's operations wait for each other across streams like the data ones.  It is
// a split of the data communicator, so a later exchange's counts never queue behind an earlier
// exchange's transfers, which are enqueued once the host has read those counts
// (bw_capi.hip, exchange_progress).  Host transport: synchronous through pinned h (4 x world u64:
// [0, 2W) sent, [2W, 4W) received), *now = true.
int bw::comm_counts(bw_comm* c, const uint64_t* d_send, uint64_t* d_recv, uint64_t* h, hipStream_t st, bool* now,
                    std::string& err) {
    if (c->failed) return comm_err(c, err, "the communicator was aborted by an earlier failure");
    const int W = c->world;
    *now = false;
    if (c->nccl) {
        if (c->ctl_tail_stream && c->ctl_tail_stream != st && hipStreamWaitEvent(st, c->ctl_tail, 0) != hipSuccess)
            return comm_err(c, err, "hipStreamWaitEvent on the control communicator's last operation failed");
        ncclResult_t r = ncclGroupStart();
        for (int k = 0; k < W && (r == ncclSuccess || r == ncclInProgress); k++) {
            r = ncclSend(d_send + 2 * k, 16, ncclUint8, k, c->ctl, st);
            if (r == ncclSuccess || r == ncclInProgress) r = ncclRecv(d_recv + 2 * k, 16, ncclUint8, k, c->ctl, st);
        }
        const ncclResult_t e = ncclGroupEnd();
        if (r != ncclSuccess && r != ncclInProgress)
            return fail(c, err, std::string("counts all-to-all: ") + ncclGetErrorString(r));
        if (int rc = settle(c, c->ctl, e, "counts all-to-all", err)) return rc;
        if (hipEventRecord(c->ctl_tail, st) != hipSuccess) return comm_err(c, err, "hipEventRecord failed");
        c->ctl_tail_stream = st;
        return BW_OK;
    }
    if (hipStreamSynchronize(st) != hipSuccess || hipMemcpy(h, d_send, 2 * W * 8, hipMemcpyDeviceToHost) != hipSuccess)
        return comm_err(c, err, "counts staging copy (device to host) failed");
    if (int rc = c->host_fn(c->user, h, h + 2 * W, 16)) {
        c->failed = true;
        return comm_err(c, err, "the host all-to-all returned " + std::to_string(rc) + " (communicator failed)");
    }
    *now = true;
    return BW_OK;
}

// One non-blocking look at `ev` (recorded behind this communicator's collectives, enqueued at
// `since_ns` on the steady clock): *ready, or still running within the deadline, or failed.
int bw::comm_poll(bw_comm* c, hipEvent_t ev, uint64_t since_ns, bool* ready, std::string& err) {
    *ready = false;
    if (c->failed) return comm_err(c, err, "the communicator was aborted by an earlier failure");
    const hipError_t q = hipEventQuery(ev);
    if (q == hipSuccess) {
        *ready = true;
        return BW_OK;
    }
    if (q != hipErrorNotReady) return fail(c, err, std::string("hipEventQuery: ") + hipGetErrorString(q));
    if (c->nccl) {
        const ncclResult_t a = async_state(c);
        if (a != ncclSuccess && a != ncclInProgress)
            return fail(c, err, std::string("RCCL async error: ") + ncclGetErrorString(a));
    }
    const uint64_t now = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                             Clock::now().time_since_epoch()).count();
    if (now - since_ns > (uint64_t)c->timeout_ms * 1000000ull)
        return fail(c, err, "an exchange's counts did not arrive within " + std::to_string(c->timeout_ms) +
                                " ms (a peer failed or stalled)");
    return BW_OK;
}

// all[2k, 2k + 1] = rank k's mine[0, 1], now (host-synchronous, deadline-bounded): the settlement
// rounds of a file split across the ranks (bw_chunk_stream_shard).  RCCL: on the control
// communicator and stream, after every counts exchange issued before it; host transport: the
// caller's function.
int bw::comm_allgather2(bw_comm* c, const uint64_t mine[2], uint64_t* all, std::string& err) {
    if (c->failed) return comm_err(c, err, "the communicator was aborted by an earlier failure");
    const int W = c->world;
    std::vector<uint64_t> send(2 * W);
    for (int k = 0; k < W; k++) {
        send[2 * k] = mine[0];
        send[2 * k + 1] = mine[1];
    }
    if (c->nccl) {
        hipStream_t st = c->ctl_st;
        if (c->ctl_tail_stream && c->ctl_tail_stream != st && hipStreamWaitEvent(st, c->ctl_tail, 0) != hipSuccess)
            return comm_err(c, err, "hipStreamWaitEvent on the control communicator's last operation failed");
        uint64_t* ds = c->ctl_buf + 2 * W;
        uint64_t* dr = c->ctl_buf + 4 * W;
        if (hipMemcpyAsync(ds, send.data(), 2 * W * 8, hipMemcpyHostToDevice, st) != hipSuccess)
            return comm_err(c, err, "allgather staging copy failed");
        ncclResult_t r = ncclGroupStart();
        for (int k = 0; k < W && (r == ncclSuccess || r == ncclInProgress); k++) {
            r = ncclSend(ds + 2 * k, 16, ncclUint8, k, c->ctl, st);
            if (r == ncclSuccess || r == ncclInProgress) r = ncclRecv(dr + 2 * k, 16, ncclUint8, k, c->ctl, st);
        }
        const ncclResult_t e = ncclGroupEnd();
        if (r != ncclSuccess && r != ncclInProgress) return fail(c, err, std::string("allgather: ") + ncclGetErrorString(r));
        if (int rc = settle(c, c->ctl, e, "allgather", err)) return rc;
        if (hipEventRecord(c->ctl_tail, st) != hipSuccess) return comm_err(c, err, "hipEventRecord failed");
        c->ctl_tail_stream = st;
        hipEvent_t ev;
        if (hipMemcpyAsync(all, dr, 2 * W * 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess)
            return comm_err(c, err, "allgather staging copy failed");
        hipEventRecord(ev, st);
        const int rc = comm_wait_event(c, ev, err);
        hipEventDestroy(ev);
        return rc;
    }
    if (int rc = c->host_fn(c->user, send.data(), all, 16)) {
        c->failed = true;
        return comm_err(c, err, "the host all-to-all returned " + std::to_string(rc) + " (communicator failed)");
    }
    return BW_OK;
}

uint64_t bw::comm_now_ns() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now().time_since_epoch()).count();
}

// Variable all-to-all: scnt[k] elements of `elem` bytes from d_send (sections back to back in rank
// order) to rank k, rcnt[k] from rank k into d_recv (likewise).  RCCL: one group of send/recv pairs,
// a pair with zero elements skipped on both sides (rcnt at the receiver is the sender's scnt).
// Host transport: equal splits of `pad` elements (>= every section on every rank).  Ordered on st.
int bw::comm_all_to_allv(bw_comm* c, const void* d_send, const uint64_t* scnt, void* d_recv, const uint64_t* rcnt,
                         uint64_t elem, uint64_t pad, hipStream_t st, std::string& err) {
    if (c->failed) return comm_err(c, err, "the communicator was aborted by an earlier failure");
    const int W = c->world;
    uint64_t stot = 0, rtot = 0;
    for (int k = 0; k < W; k++) {
        stot += scnt[k];
        rtot += rcnt[k];
    }
    if (c->nccl) {
        if (!stot && !rtot) return BW_OK;  // per pair, a zero section is skipped on both sides
        if (c->tail_stream && c->tail_stream != st && hipStreamWaitEvent(st, c->tail, 0) != hipSuccess)
            return comm_err(c, err, "hipStreamWaitEvent on the communicator's last collective failed");
        ncclResult_t r = ncclGroupStart();
        uint64_t so = 0, ro = 0;
        for (int k = 0; k < W && (r == ncclSuccess || r == ncclInProgress); k++) {
            if (scnt[k]) r = ncclSend((const uint8_t*)d_send + so * elem, scnt[k] * elem, ncclUint8, k, c->nccl, st);
            if (rcnt[k] && (r == ncclSuccess || r == ncclInProgress))
                r = ncclRecv((uint8_t*)d_recv + ro * elem, rcnt[k] * elem, ncclUint8, k, c->nccl, st);
            so += scnt[k];
            ro += rcnt[k];
        }
        const ncclResult_t e = ncclGroupEnd();
        if (r != ncclSuccess && r != ncclInProgress)
            return fail(c, err, std::string("ncclSend/ncclRecv: ") + ncclGetErrorString(r));
        if (int rc = settle(c, c->nccl, e, "ncclGroupEnd", err)) return rc;
        if (hipEventRecord(c->tail, st) != hipSuccess) return comm_err(c, err, "hipEventRecord failed");
        c->tail_stream = st;
        return BW_OK;
    }
    // host transport: device -> pinned, padded to `pad` per rank -> caller -> unpadded -> device;
    // pad is the same on every rank (the largest section anywhere), so all ranks skip together
    if (!pad) return BW_OK;
    const size_t slot = (size_t)pad * elem, total = slot * W;
    const size_t need = 2 * total + (size_t)(stot + rtot) * elem;
    if (c->pin_cap < need) {
        if (c->pin_send) hipHostFree(c->pin_send);
        c->pin_send = nullptr;
        c->pin_cap = 0;
        if (hipHostMalloc(&c->pin_send, need, hipHostMallocDefault) != hipSuccess)
            return comm_err(c, err, "hipHostMalloc of the exchange staging failed");
        c->pin_cap = need;
    }
    uint8_t* hs = (uint8_t*)c->pin_send;
    uint8_t* hr = hs + total;
    uint8_t* flat_s = hr + total;
    uint8_t* flat_r = flat_s + stot * elem;
    if ((stot && hipMemcpyAsync(flat_s, d_send, stot * elem, hipMemcpyDeviceToHost, st) != hipSuccess) ||
        hipStreamSynchronize(st) != hipSuccess)
        return comm_err(c, err, "exchange staging copy (device to host) failed");
    memset(hs, 0, total);
    uint64_t so = 0, ro = 0;
    for (int k = 0; k < W; k++) {
        if (scnt[k] > pad) return comm_err(c, err, "exchange section larger than the agreed padding (internal error)");
        memcpy(hs + k * slot, flat_s + so * elem, scnt[k] * elem);
        so += scnt[k];
    }
    if (int rc = c->host_fn(c->user, hs, hr, slot)) {
        c->failed = true;  // the caller's transport lost a peer: the ranks no longer agree
        return comm_err(c, err, "the host all-to-all returned " + std::to_string(rc) + " (communicator failed)");
    }
    for (int k = 0; k < W; k++) {
        if (rcnt[k] > pad) return comm_err(c, err, "exchange section larger than the agreed padding (internal error)");
        memcpy(flat_r + ro * elem, hr + k * slot, rcnt[k] * elem);
        ro += rcnt[k];
    }
    if ((rtot && hipMemcpyAsync(d_recv, flat_r, rtot * elem, hipMemcpyHostToDevice, st) != hipSuccess) ||
        hipStreamSynchronize(st) != hipSuccess)
        return comm_err(c, err, "exchange staging copy (host to device) failed");
    return BW_OK;
}

static bool world_ok(int rank, int world) {
    return world >= 1 && world <= 256 && (world & (world - 1)) == 0 && rank >= 0 && rank < world;
}

extern "C" int bw_comm_unique_id(uint8_t id[BW_COMM_ID_BYTES]) {
    if (!id) return BW_EINVAL;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return BW_ECOMM;
    memcpy(id, u.internal, BW_COMM_ID_BYTES);
    return BW_OK;
}

extern "C" int bw_comm_init_timeout(int device, int rank, int world, const uint8_t id[BW_COMM_ID_BYTES],
                                    uint32_t timeout_ms, bw_comm** out) {
    if (!out) return BW_EINVAL;
    *out = nullptr;
    if (!id || !world_ok(rank, world) || !timeout_ms) return BW_EINVAL;
    if (hipSetDevice(device) != hipSuccess) return BW_EHIP;
    bw_comm* c = new bw_comm();
    c->device = device;
    c->rank = rank;
    c->world = world;
    c->timeout_ms = timeout_ms;
    ncclUniqueId u;
    memcpy(u.internal, id, BW_COMM_ID_BYTES);
    std::string err;
    auto bail = [&](int rc) {
        bw_comm_destroy(c);
        return rc;
    };
    if (hipEventCreateWithFlags(&c->tail, hipEventDisableTiming | hipEventReleaseToDevice) != hipSuccess ||
        hipEventCreateWithFlags(&c->ctl_tail, hipEventDisableTiming | hipEventReleaseToDevice) != hipSuccess ||
        hipStreamCreateWithFlags(&c->ctl_st, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&c->ctl_buf, 6 * world * 8) != hipSuccess)
        return bail(BW_EHIP);
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;  // every wait below is ours, with a deadline
    const ncclResult_t r0 = ncclCommInitRankConfig(&c->nccl, world, u, rank, &cfg);
    if (!c->nccl && r0 == ncclSuccess) return bail(BW_ECOMM);
    if (settle(c, c->nccl, r0, "ncclCommInitRankConfig", err)) return bail(BW_ECOMM);
    // the control communicator for the per-exchange counts, split off while every rank is here
    ncclConfig_t cfg2 = NCCL_CONFIG_INITIALIZER;
    cfg2.blocking = 0;
    const ncclResult_t r1 = ncclCommSplit(c->nccl, 0, rank, &c->ctl, &cfg2);
    if (settle(c, c->ctl ? c->ctl : c->nccl, r1, "ncclCommSplit", err)) return bail(BW_ECOMM);
    *out = c;
    return BW_OK;
}

extern "C" int bw_comm_init(int device, int rank, int world, const uint8_t id[BW_COMM_ID_BYTES], bw_comm** out) {
    return bw_comm_init_timeout(device, rank, world, id, BW_COMM_DEFAULT_TIMEOUT_MS, out);
}

extern "C" int bw_comm_init_host(int device, int rank, int world, bw_host_all_to_all fn, void* user, bw_comm** out) {
    if (!out) return BW_EINVAL;
    *out = nullptr;
    if (!fn || !world_ok(rank, world)) return BW_EINVAL;
    bw_comm* c = new bw_comm();
    c->device = device;
    c->rank = rank;
    c->world = world;
    c->host_fn = fn;
    c->user = user;
    *out = c;
    return BW_OK;
}

extern "C" void bw_comm_destroy(bw_comm* c) {
    if (!c) return;
    hipSetDevice(c->device);
    bw::exchange_drain(c);  // exchanges still waiting for their counts are finished (or failed) first
    if (!c->failed && c->tail_stream) {
        std::string err;
        bw::comm_wait_event(c, c->tail, err);  // aborts on a missed deadline instead of hanging
    }
    std::string err;
    for (ncclComm_t* k : {&c->ctl, &c->nccl}) {
        if (!*k) continue;
        if (c->failed) {
            ncclCommAbort(*k);
        } else if (settle(c, *k, ncclCommFinalize(*k), "ncclCommFinalize", err) == BW_OK) {
            ncclCommDestroy(*k);
        }  // else: settle aborted both
        *k = nullptr;
    }
    if (c->tail) hipEventDestroy(c->tail);
    if (c->ctl_tail) hipEventDestroy(c->ctl_tail);
    if (c->ctl_st) hipStreamDestroy(c->ctl_st);
    if (c->ctl_buf) hipFree(c->ctl_buf);
    if (c->pin_send) hipHostFree(c->pin_send);
    if (c->user_free) c->user_free(c->user);
    delete c;
}

// ---------------------------------------------------------------- the ranks of one process
//  The reference packs a backup inside one process (client/src/backup/mod.rs:64):
// these two calls give such a process N ranks, one per context, without one process per GPU.  The
// ranks are then driven from N threads (one per rank, like the tokio tasks that feed the packer):
// each submits its share of the files, calls bw_exchange_dedup with its own context and
// communicator, in the same batch order on every rank.

namespace {

// An all-to-all between the threads of one process: each rank posts its buffers, waits until all
// have, copies its column out of every peer's send buffer, and waits until all have copied (so no
// send buffer is reused under a peer still reading it).  A rank that does not arrive within the
// group's deadline breaks the group: every waiting and later call fails (-> BW_ECOMM).
struct LocalGroup {
    int n = 0;
    uint32_t timeout_ms = BW_COMM_DEFAULT_TIMEOUT_MS;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0, copied = 0;
    uint64_t gen_arrive = 0, gen_copy = 0;
    bool broken = false;
    std::vector<const uint8_t*> send;
    std::vector<uint64_t> bytes;
    std::atomic<int> refs{0};
};
struct LocalMember {
    LocalGroup* g;
    int rank;
};

int local_all_to_all(void* user, const void* send, void* recv, uint64_t bytes) {
    auto* m = (LocalMember*)user;
    LocalGroup& g = *m->g;
    const int r = m->rank;
    std::unique_lock<std::mutex> lk(g.mu);
    const auto dl = Clock::now() + std::chrono::milliseconds(g.timeout_ms);
    auto wait_gen = [&](uint64_t& gen_now, uint64_t gen) {
        if (!g.cv.wait_until(lk, dl, [&] { return gen_now != gen || g.broken; })) g.broken = true;
        g.cv.notify_all();
        return !g.broken;
    };
    if (g.broken) return 1;
    g.send[r] = (const uint8_t*)send;
    g.bytes[r] = bytes;
    const uint64_t ga = g.gen_arrive;
    if (++g.arrived == g.n) {
        g.arrived = 0;
        g.gen_arrive++;
        g.cv.notify_all();
    } else if (!wait_gen(g.gen_arrive, ga)) {
        return 1;
    }
    for (int p = 0; p < g.n; p++)
        if (g.bytes[p] != bytes) {  // the library pads to equal splits: a mismatch is a broken session
            g.broken = true;
            g.cv.notify_all();
            return 1;
        }
    lk.unlock();
    for (int p = 0; p < g.n; p++) memcpy((uint8_t*)recv + (uint64_t)p * bytes, g.send[p] + (uint64_t)r * bytes, bytes);
    lk.lock();
    const uint64_t gc = g.gen_copy;
    if (++g.copied == g.n) {
        g.copied = 0;
        g.gen_copy++;
        g.cv.notify_all();
        return g.broken ? 1 : 0;
    }
    return wait_gen(g.gen_copy, gc) ? 0 : 1;
}

void local_member_free(void* user) {
    auto* m = (LocalMember*)user;
    if (m->g->refs.fetch_sub(1) == 1) delete m->g;
    delete m;
}

}  // namespace

extern "C" int bw_comm_init_local(const int* devices, int n, bw_comm** out) {
    if (!devices || !out || n < 1 || !world_ok(0, n)) return BW_EINVAL;
    for (int r = 0; r < n; r++) out[r] = nullptr;
    auto* g = new LocalGroup();
    g->n = n;
    g->send.assign(n, nullptr);
    g->bytes.assign(n, 0);
    g->refs = n;
    for (int r = 0; r < n; r++) {
        auto* m = new LocalMember{g, r};
        if (int rc = bw_comm_init_host(devices[r], r, n, local_all_to_all, m, &out[r])) {
            delete m;
            g->refs -= n - r;  // the members that were never attached (this one included)
            if (r == 0) delete g;
            for (int k = 0; k < r; k++) {  // the last one out deletes the group
                bw_comm_destroy(out[k]);
                out[k] = nullptr;
            }
            return rc;
        }
        out[r]->user_free = local_member_free;
    }
    return BW_OK;
}

extern "C" int bw_comm_init_all(const int* devices, int n, uint32_t timeout_ms, bw_comm** out) {
    if (!devices || !out || n < 1 || !world_ok(0, n) || !timeout_ms) return BW_EINVAL;
    for (int r = 0; r < n; r++) out[r] = nullptr;
    uint8_t id[BW_COMM_ID_BYTES];
    if (int rc = bw_comm_unique_id(id)) return rc;
    // every rank's initialisation must be in progress at once (RCCL meets the ranks there): one
    // thread per rank, as the ranks of separate processes would be
    std::vector<int> rc(n, BW_OK);
    std::vector<std::thread> th;
    for (int r = 0; r < n; r++)
        th.emplace_back([&, r] { rc[r] = bw_comm_init_timeout(devices[r], r, n, id, timeout_ms, &out[r]); });
    for (auto& t : th) t.join();
    for (int r = 0; r < n; r++)
        if (rc[r] != BW_OK) {
            for (int k = 0; k < n; k++) {
                bw_comm_destroy(out[k]);
                out[k] = nullptr;
            }
            return rc[r];
        }
    return BW_OK;
}

// Kept for the ABI (round 4 sized fixed buckets with it): every transfer is now sized exactly from
// the counts the exchange itself carries, so there is nothing to fix and the value is ignored.
extern "C" int bw_comm_set_capacity(bw_comm* c, uint64_t cap) {
    (void)cap;
    return c ? BW_OK : BW_EINVAL;
}

extern "C" int bw_comm_progress(bw_comm* c) {
    if (!c) return BW_EINVAL;
    hipSetDevice(c->device);
    return bw::exchange_progress(c, nullptr);
}

extern "C" int bw_comm_set_timeout(bw_comm* c, uint32_t timeout_ms) {
    if (!c || !timeout_ms) return BW_EINVAL;
    c->timeout_ms = timeout_ms;
    return BW_OK;
}

extern "C" int bw_comm_status(const bw_comm* c) { return !c ? BW_EINVAL : c->failed ? BW_ECOMM : BW_OK; }

extern "C" const char* bw_comm_last_error(const bw_comm* c) { return c ? c->err.c_str() : "null communicator"; }
