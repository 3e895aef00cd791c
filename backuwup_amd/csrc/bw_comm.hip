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
#include <string.h>

#include <string>

#include <rccl/rccl.h>

#include "bw_internal.h"

static_assert(BW_COMM_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "the C ABI's id size is RCCL's");

struct bw_comm {
    int device = 0, rank = 0, world = 1;
    ncclComm_t nccl = nullptr;            // RCCL transport
    bw_host_all_to_all host_fn = nullptr;  // or the caller's host transport
    void* user = nullptr;
    uint64_t cap = 0;                      // bucket capacity of the session (0 = not agreed yet)
    void* pin_send = nullptr;              // host transport: pinned staging, 2 x pin_cap
    size_t pin_cap = 0;
    // The communicator's collectives run in the order the host issued them, whatever streams they
    // were issued on: every one waits for the previous one's `tail`.  Contexts with batches in
    // flight issue their exchanges on their own streams, and two RCCL operations of one
    // communicator running at once on one GPU can wait on each other forever.
    hipEvent_t tail = nullptr;
    hipStream_t tail_stream = nullptr;
    std::string err;
};

namespace {

int comm_err(bw_comm* c, std::string& err, const std::string& what) {
    err = what;
    if (c) c->err = what;
    return BW_ECOMM;
}

int nccl_chk(bw_comm* c, std::string& err, ncclResult_t r, const char* what) {
    if (r == ncclSuccess) return BW_OK;
    return comm_err(c, err, std::string(what) + ": " + ncclGetErrorString(r));
}

}  // namespace

int bw::comm_rank(const bw_comm* c) { return c->rank; }
int bw::comm_world(const bw_comm* c) { return c->world; }
int bw::comm_device(const bw_comm* c) { return c->device; }
uint64_t& bw::comm_cap(bw_comm* c) { return c->cap; }

// d_recv[r * bytes ..] = rank r's d_send[my_rank * bytes ..], for every rank r; ordered on st.
int bw::comm_all_to_all(bw_comm* c, const void* d_send, void* d_recv, uint64_t bytes, hipStream_t st,
                        std::string& err) {
    if (!bytes) return BW_OK;
    const int W = c->world;
    if (c->nccl) {
        if (c->tail_stream && c->tail_stream != st && hipStreamWaitEvent(st, c->tail, 0) != hipSuccess)
            return comm_err(c, err, "hipStreamWaitEvent on the communicator's last collective failed");
        if (int rc = nccl_chk(c, err, ncclGroupStart(), "ncclGroupStart")) return rc;
        for (int r = 0; r < W; r++) {
            ncclResult_t a = ncclSend((const uint8_t*)d_send + r * bytes, bytes, ncclUint8, r, c->nccl, st);
            ncclResult_t b = ncclRecv((uint8_t*)d_recv + r * bytes, bytes, ncclUint8, r, c->nccl, st);
            if (a != ncclSuccess || b != ncclSuccess) {
                ncclGroupEnd();
                return nccl_chk(c, err, a != ncclSuccess ? a : b, "ncclSend/ncclRecv");
            }
        }
        if (int rc = nccl_chk(c, err, ncclGroupEnd(), "ncclGroupEnd")) return rc;
        if (hipEventRecord(c->tail, st) != hipSuccess) return comm_err(c, err, "hipEventRecord failed");
        c->tail_stream = st;
        return BW_OK;
    }
    // host transport: device -> pinned -> caller -> pinned -> device, synchronous on st
    const size_t total = (size_t)bytes * W;
    if (c->pin_cap < total) {
        if (c->pin_send) hipHostFree(c->pin_send);
        c->pin_send = nullptr;
        c->pin_cap = 0;
        if (hipHostMalloc(&c->pin_send, 2 * total, hipHostMallocDefault) != hipSuccess)
            return comm_err(c, err, "hipHostMalloc of the exchange staging failed");
        c->pin_cap = total;
    }
    uint8_t* hs = (uint8_t*)c->pin_send;
    uint8_t* hr = hs + total;
    if (hipMemcpyAsync(hs, d_send, total, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return comm_err(c, err, "exchange staging copy (device to host) failed");
    if (int rc = c->host_fn(c->user, hs, hr, bytes))
        return comm_err(c, err, "the host all-to-all returned " + std::to_string(rc));
    if (hipMemcpyAsync(d_recv, hr, total, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return comm_err(c, err, "exchange staging copy (host to device) failed");
    return BW_OK;
}

// max of v over the ranks (synchronous): one all-to-all of world x 8 bytes through `scratch`
// (device, >= 2 * world * 8 bytes)
int bw::comm_max(bw_comm* c, uint64_t v, uint64_t* out, void* scratch, hipStream_t st, std::string& err) {
    const int W = c->world;
    std::vector<uint64_t> h(W, v);
    uint64_t* d = (uint64_t*)scratch;
    if (hipMemcpyAsync(d, h.data(), W * 8, hipMemcpyHostToDevice, st) != hipSuccess)
        return comm_err(c, err, "hipMemcpyAsync failed");
    if (int rc = comm_all_to_all(c, d, d + W, 8, st, err)) return rc;
    if (hipMemcpyAsync(h.data(), d + W, W * 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return comm_err(c, err, "hipMemcpyAsync failed");
    uint64_t m = 0;
    for (uint64_t x : h) m = std::max(m, x);
    *out = m;
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

extern "C" int bw_comm_init(int device, int rank, int world, const uint8_t id[BW_COMM_ID_BYTES], bw_comm** out) {
    if (!out) return BW_EINVAL;
    *out = nullptr;
    if (!id || !world_ok(rank, world)) return BW_EINVAL;
    if (hipSetDevice(device) != hipSuccess) return BW_EHIP;
    bw_comm* c = new bw_comm();
    c->device = device;
    c->rank = rank;
    c->world = world;
    ncclUniqueId u;
    memcpy(u.internal, id, BW_COMM_ID_BYTES);
    if (hipEventCreateWithFlags(&c->tail, hipEventDisableTiming | hipEventReleaseToDevice) != hipSuccess) {
        delete c;
        return BW_EHIP;
    }
    if (ncclCommInitRank(&c->nccl, world, u, rank) != ncclSuccess) {  // blocks until every rank joined
        hipEventDestroy(c->tail);
        delete c;
        return BW_ECOMM;
    }
    *out = c;
    return BW_OK;
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
    if (c->tail_stream) hipEventSynchronize(c->tail);
    if (c->nccl) ncclCommDestroy(c->nccl);
    if (c->tail) hipEventDestroy(c->tail);
    if (c->pin_send) hipHostFree(c->pin_send);
    delete c;
}

extern "C" int bw_comm_set_capacity(bw_comm* c, uint64_t cap) {
    if (!c) return BW_EINVAL;
    c->cap = cap;
    return BW_OK;
}

extern "C" const char* bw_comm_last_error(const bw_comm* c) { return c ? c->err.c_str() : "null communicator"; }
