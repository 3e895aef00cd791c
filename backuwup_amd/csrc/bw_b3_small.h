// bw_b3_small.h -- the drop-ins' small-message BLAKE3 (bw_b3_small.hip), driven by bw_dropin.hip.
// Off the batch pipeline's path (backuwup_amd/build.py OFF_PATH).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bw {

// n whole messages of at most 64 KiB each (data + offs[i], lens[i] bytes; all three may be pinned
// host memory, read over PCIe; offsets 16-byte aligned) -> out[32 i ..] (may be pinned host memory):
// one workgroup per message (a quad of lanes per leaf), max_len = the longest (sizes the LDS)
constexpr uint64_t B3_MSG_MAX = 65536;
void launch_b3_msgs(hipStream_t st, const uint8_t* data, const uint64_t* offs, const uint64_t* lens, uint32_t n,
                    uint32_t max_len, uint8_t* out);

// The small-message hash service (bw_dropin.hip drives it): a persistent kernel whose workers take
// messages posted into a ring of request slots and write each digest into a response slot.
//   host -> GPU (B3SvcReq): ptr (the message, 16-byte aligned), then lenseq = len | (ticket + 1) << 32.
//     With a large BAR the requests and the callers' message copies live in HBM (fine-grained,
//     written by the CPU through the BAR: no PCIe read on the GPU's side); otherwise in pinned host
//     memory.
//   GPU -> host (B3SvcResp, pinned): the digest over the ticket's sentinel (b3svc_sentinel; four
//     8-byte stores; the host takes the slot as done once no word equals its sentinel: a digest word
//     matches with probability 2^-64)
struct alignas(64) B3SvcReq {
    uint64_t lenseq;
    uint64_t ptr;
    uint64_t pad[6];
};
static_assert(sizeof(B3SvcReq) == 64, "one cache line per slot");
struct alignas(64) B3SvcResp {
    uint64_t digest[4];
    uint64_t pad[4];
};
static_assert(sizeof(B3SvcResp) == 64, "one cache line per slot");
// bit 31 of lenseq's length word: the host cancelled this ticket (its caller gave up and the slot
// was reclaimed); a worker that reserves it moves on without hashing or writing the response slot
constexpr uint32_t B3SVC_CANCEL = 1u << 31;
__host__ __device__ inline uint64_t b3svc_sentinel(uint32_t seq, int k) {
    return (0x9E3779B97F4A7C15ull * seq) ^ (0xD1B54A32D192ED03ull * (uint64_t)(k + 1));
}
struct B3SvcCtl {            // pinned host memory
    uint32_t stop;           // host: end every instance at once
    uint32_t pad0[15];
    uint32_t dead;           // GPU: the epoch of the last instance whose workers have all exited
    uint32_t pad1[15];
};
struct B3SvcDev {            // device memory, kept across instances
    uint32_t next;           // the next ticket a worker reserves
    uint32_t pad0;
    uint32_t started;        // the epoch whose first wave reset `next` (the workers wait for it)
    uint32_t quit;           // the epoch whose workers are leaving
    uint32_t exited;         // workers that left, over every instance (never reset; mod 2^32)
    uint32_t progress;       // messages hashed (a waiting worker's idle clock restarts when it moves)
    uint32_t pad[2];
};
constexpr uint32_t B3_SVC_RING = 4096;    // slots (tickets in flight at most)
constexpr uint32_t B3_SVC_WORKERS = 64;   // workgroups of 256 (one message each at a time)
// one instance (epoch >= 1) on st, reserving tickets from `start` on; ends when nothing was hashed for
// idle_us, after life_us, or on ctl->stop.  proc: B3_SVC_RING words in device memory (ticket + 1 once
// hashed)
void launch_b3_service(hipStream_t st, B3SvcReq* req, B3SvcResp* resp, B3SvcCtl* ctl, B3SvcDev* dev, uint32_t* proc,
                       uint32_t epoch, uint32_t start, uint32_t idle_us, uint32_t life_us);

}  // namespace bw
