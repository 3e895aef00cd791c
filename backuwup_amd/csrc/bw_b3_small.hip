// bw_b3_small.hip -- BLAKE3 of small whole messages for the drop-in blake3::hash calls (dir_packer.rs
// :286 for a small file, :320 / :353 for tree blobs; crate blake3 1.3.3, spec restated in SURVEY.md
// A.4): the quad-lane compression, a launched batch (k_b3_msgs) and the persistent hash service
// (k_b3_service) that bw_dropin.hip drives.  Off the batch pipeline's path (backuwup_amd/build.py
// OFF_PATH): the chunk pipeline hashes with bw_blake3.hip's k_b3_lines / k_b3_upper.
#include <algorithm>

#include "bw_device.h"
#include "bw_internal.h"
#include "bw_b3_small.h"

namespace bw {

// ---- small whole messages straight from pinned host memory (bw_blake3_hash's coalesced batches:
// the reference's per-file and per-tree blake3::hash calls, dir_packer.rs:286, :320).  Latency, not
// throughput, decides here: a caller waits for its digest, and a few messages are in flight at a
// time.  So a message is spread over as many lanes as BLAKE3 lets it use: a workgroup per message
// of <= 64 leaves (64 KiB), a QUAD of lanes per leaf, lane j of the quad holding column j of the
// 4x4 compression state (v[j], v[4+j], v[8+j], v[12+j]).  The column step is each lane's own G;
// the diagonal step rotates rows 1-3 across the quad (DPP quad permutes) and rotates them back.
// One compression is then ~240 instructions per lane instead of ~700, and a leaf's 16 chained
// compressions take a third of the time of the lane-per-leaf form (which hashes a 16 KiB message in
// ~40 us, k_b3_msgs round 5).  The message words a lane needs in round r are fixed per lane
// (schedule positions 2j, 2j+1, 8+2j, 9+2j), read from LDS with per-lane offsets.
//
// The workgroup first pulls the whole message from the caller-side pinned staging into LDS with
// all its 16-byte loads in flight (over PCIe: one round of latency), leaf c at c * 1040 (a 16-byte
// pad per leaf spreads the quads' reads over the banks).  The leaf chaining values then go to LDS
// and merge into the left-balanced tree level by level (pairs from the left, an odd last node
// carried up), each parent one quad compression whose message block is the two children, adjacent
// in LDS; ROOT on the last merge, or on a single leaf's last block.
constexpr uint32_t B3Q_LEAF_STRIDE = B3_LEAF_BYTES + 16;

// the message schedule: word position p of round r (the spec permutation applied r times)
__device__ __forceinline__ constexpr uint32_t b3q_sched(int r, int p) {
    constexpr uint8_t S[7][16] = {{0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
                                  {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8},
                                  {3, 4, 10, 12, 13, 2, 7, 14, 6, 5, 9, 0, 11, 15, 8, 1},
                                  {10, 7, 12, 9, 14, 3, 13, 15, 4, 0, 11, 2, 5, 8, 1, 6},
                                  {12, 13, 9, 11, 15, 10, 14, 8, 7, 2, 5, 3, 0, 1, 6, 4},
                                  {9, 14, 11, 5, 8, 12, 15, 1, 13, 3, 0, 10, 2, 6, 4, 7},
                                  {11, 15, 5, 0, 1, 9, 8, 6, 14, 10, 2, 12, 3, 4, 7, 13}};
    return S[r][p];
}

// lane j of a quad takes x from lane (j + K) % 4.  As update_dpp with bound_ctrl the compiler folds
// the rotations of c and d into the add / xor that consume them (v_add_u32_dpp, v_xor_b32_dpp).
// Measured on the chip (s_memtime against s_memrealtime in the service): 2.40 GHz, ~7 cycles per
// dependent instruction; a compression is a chain of ~180 of them, so a 1 KiB leaf (16 chained
// compressions) takes ~10 us however many lanes the message has.
template <int K>
__device__ __forceinline__ uint32_t b3q_rot(uint32_t x) {
    constexpr int ctrl = ((0 + K) & 3) | (((1 + K) & 3) << 2) | (((2 + K) & 3) << 4) | (((3 + K) & 3) << 6);
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, ctrl, 0xF, 0xF, true);
}

#define B3Q_G(a, b, c, d, x, y)   \
    do {                          \
        a = a + b + (x);          \
        d = b3_rotr(d ^ a, 16);   \
        c = c + d;                \
        b = b3_rotr(b ^ c, 12);   \
        a = a + b + (y);          \
        d = b3_rotr(d ^ a, 8);    \
        c = c + d;                \
        b = b3_rotr(b ^ c, 7);    \
    } while (0)

// Per-lane byte offsets of the 28 message words lane j reads per compression (4 per round).
struct B3qOffs {
    uint32_t o[7][4];
    __device__ __forceinline__ explicit B3qOffs(uint32_t j) {
#pragma unroll
        for (int r = 0; r < 7; r++)
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int p = (k < 2 ? 0 : 8) + (k & 1);  // positions 2j + p
                const uint32_t i0 = b3q_sched(r, p), i1 = b3q_sched(r, p + 2), i2 = b3q_sched(r, p + 4),
                               i3 = b3q_sched(r, p + 6);
                o[r][k] = 4 * (j == 0 ? i0 : j == 1 ? i1 : j == 2 ? i2 : i3);
            }
    }
};

// One compression by a quad: lane j holds chaining words cv[j] (ca) and cv[4+j] (cb), and gets the
// output's; blk = the 64-byte block in LDS; dj = v[12+j]'s input (counter low / high, length, flags).
__device__ __forceinline__ void b3q_compress(uint32_t& ca, uint32_t& cb, const uint8_t* blk, const B3qOffs& of,
                                             uint32_t cj, uint32_t dj) {
    uint32_t mw[7][4];
#pragma unroll
    for (int r = 0; r < 7; r++)
#pragma unroll
        for (int k = 0; k < 4; k++) mw[r][k] = *(const uint32_t*)(blk + of.o[r][k]);
    // all 28 reads in flight at once, one wait: left to itself the compiler waits for each round's
    // words just before the round, exposing the LDS latency four times per compression
#pragma unroll
    for (int r = 0; r < 7; r++)
#pragma unroll
        for (int k = 0; k < 4; k++) asm volatile("" : "+v"(mw[r][k]));
    uint32_t a = ca, b = cb, c = cj, d = dj;
#pragma unroll
    for (int r = 0; r < 7; r++) {
        B3Q_G(a, b, c, d, mw[r][0], mw[r][1]);
        b = b3q_rot<1>(b);
        c = b3q_rot<2>(c);
        d = b3q_rot<3>(d);
        B3Q_G(a, b, c, d, mw[r][2], mw[r][3]);
        b = b3q_rot<3>(b);
        c = b3q_rot<2>(c);
        d = b3q_rot<1>(d);
    }
    ca = a ^ c;
    cb = b ^ d;
}

__device__ __forceinline__ uint32_t b3q_iv(uint32_t i) {
    return i == 0 ? B3_IV0 : i == 1 ? B3_IV1 : i == 2 ? B3_IV2 : i == 3 ? B3_IV3
         : i == 4 ? B3_IV4 : i == 5 ? B3_IV5 : i == 6 ? B3_IV6 : B3_IV7;
}

// The whole workgroup (nt threads, a multiple of 64, >= 4 * leaves) hashes one message of len <= 64
// KiB at src (16-byte aligned, readable up to len rounded up to 16); returns where in LDS the 32-byte
// digest is (valid after the call's last barrier).  lds: leaves * 1040 + 2048 bytes.  Every thread
// calls it.
__device__ __forceinline__ const uint8_t* b3q_message(const uint8_t* __restrict__ src, uint32_t len, uint8_t* lds,
                                                      uint32_t tid, uint32_t nt) {
    const uint32_t leaves = len == 0 ? 1 : (len + B3_LEAF_BYTES - 1) / B3_LEAF_BYTES;
    uint8_t* nodes = lds + leaves * B3Q_LEAF_STRIDE;  // 64 chaining values of 32 bytes
    const uint32_t nw = len == 0 ? 4 : ((len + 63) & ~63u) / 16;  // 16-byte words incl. the last block's zeros
    const uint4* s16 = (const uint4*)src;
    for (uint32_t i0 = tid; i0 < nw; i0 += 16 * nt) {
        uint4 v[16];
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const uint32_t i = i0 + nt * k;
            v[k] = i < nw && i * 16 < len ? s16[i] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const uint32_t i = i0 + nt * k;
            if (i >= nw) break;
            if (i * 16 + 16 > len && i * 16 < len) {  // the word holding the message's end: zero past it
                uint32_t* w = (uint32_t*)&v[k];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const uint32_t b0 = i * 16 + 4 * q;
                    if (b0 >= len) w[q] = 0;
                    else if (b0 + 4 > len) w[q] &= (1u << (8 * (len - b0))) - 1;
                }
            }
            *(uint4*)(lds + (i >> 6) * B3Q_LEAF_STRIDE + (i & 63) * 16) = v[k];
        }
    }
    __syncthreads();
    const uint32_t q = tid >> 2, j = tid & 3;
    const B3qOffs of(j);
    const uint32_t ivj = b3q_iv(j);
    uint32_t ca = ivj, cb = b3q_iv(4 + j);
    if (q < leaves) {
        const uint32_t ll = len - q * B3_LEAF_BYTES < B3_LEAF_BYTES ? len - q * B3_LEAF_BYTES : B3_LEAF_BYTES;
        const uint32_t nblk = ll == 0 ? 1 : (ll + 63) / 64;
        const uint8_t* leaf = lds + q * B3Q_LEAF_STRIDE;
        for (uint32_t blk = 0; blk < nblk; blk++) {
            const uint32_t left = ll - blk * 64;
            uint32_t flags = blk == 0 ? B3_CHUNK_START : 0;
            if (blk == nblk - 1) flags |= B3_CHUNK_END | (leaves == 1 ? B3_ROOT : 0);
            // v[12..15] = counter (the leaf index: low word, high word 0), block length, flags
            const uint32_t dj = j == 0 ? q : j == 1 ? 0u : j == 2 ? (left < 64 ? left : 64u) : flags;
            b3q_compress(ca, cb, leaf + blk * 64, of, ivj, dj);
        }
        *(uint32_t*)(nodes + q * 32 + 4 * j) = ca;
        *(uint32_t*)(nodes + q * 32 + 16 + 4 * j) = cb;
    }
    // one level: node p <- parent(2p, 2p + 1), the odd last node moved up as it is.  While a level
    // has more than 16 parents its quads span several waves (workgroup barriers); from 32 nodes down
    // wave 0 alone finishes the tree (LDS operations of one wave run in order: no barrier)
    auto level = [&](uint32_t m, bool wave_only) {
        const uint32_t half = m / 2;
        uint32_t na = 0, nb = 0;
        if (q < half) {
            na = ivj;
            nb = b3q_iv(4 + j);
            const uint32_t dj = j < 2 ? 0u : j == 2 ? 64u : (B3_PARENT | (m == 2 ? B3_ROOT : 0));
            b3q_compress(na, nb, nodes + q * 64, of, ivj, dj);
        } else if (q == half && (m & 1)) {
            na = *(const uint32_t*)(nodes + (m - 1) * 32 + 4 * j);
            nb = *(const uint32_t*)(nodes + (m - 1) * 32 + 16 + 4 * j);
        }
        if (wave_only) __builtin_amdgcn_wave_barrier();
        else __syncthreads();
        if (q < half || (q == half && (m & 1))) {
            *(uint32_t*)(nodes + q * 32 + 4 * j) = na;
            *(uint32_t*)(nodes + q * 32 + 16 + 4 * j) = nb;
        }
        if (wave_only) __builtin_amdgcn_wave_barrier();
    };
    uint32_t m = leaves;
    for (; m > 32; m = (m + 1) / 2) {
        __syncthreads();
        level(m, false);
    }
    __syncthreads();
    if (tid < 64)
        for (; m > 1; m = (m + 1) / 2) level(m, true);
    __syncthreads();
    return nodes;  // the root chaining value = the digest: nodes[0, 32)
}

uint32_t b3q_threads(uint32_t max_len) {
    const uint32_t leaves = max_len == 0 ? 1 : (max_len + B3_LEAF_BYTES - 1) / B3_LEAF_BYTES;
    return std::min<uint32_t>(256, (4 * leaves + 63) & ~63u);
}

uint32_t b3q_lds(uint32_t max_len) {
    const uint32_t leaves = max_len == 0 ? 1 : (max_len + B3_LEAF_BYTES - 1) / B3_LEAF_BYTES;
    return leaves * B3Q_LEAF_STRIDE + 64 * 32;
}

__global__ __launch_bounds__(256) void k_b3_msgs(const uint8_t* __restrict__ data, const uint64_t* __restrict__ offs,
                                                 const uint64_t* __restrict__ lens, uint8_t* __restrict__ out) {
    extern __shared__ uint4 s_msg[];
    const uint32_t msg = blockIdx.x;
    // data == nullptr: offs holds absolute addresses (the callers' pinned copies)
    const uint8_t* src = (const uint8_t*)((uintptr_t)data + offs[msg]);
    const uint8_t* dig = b3q_message(src, (uint32_t)lens[msg], (uint8_t*)s_msg, threadIdx.x, blockDim.x);
    if (threadIdx.x < 8) ((uint32_t*)(out + 32ull * msg))[threadIdx.x] = ((const uint32_t*)dig)[threadIdx.x];
}

void launch_b3_msgs(hipStream_t st, const uint8_t* data, const uint64_t* offs, const uint64_t* lens, uint32_t n,
                    uint32_t max_len, uint8_t* out) {
    static const hipError_t attr = hipFuncSetAttribute((const void*)k_b3_msgs, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                       b3q_lds((uint32_t)B3_MSG_MAX));
    (void)attr;
    if (n) hipLaunchKernelGGL(k_b3_msgs, dim3(n), dim3(b3q_threads(max_len)), b3q_lds(max_len), st, data, offs, lens, out);
}

constexpr uint32_t B3Q_SVC_MSG_LDS = (uint32_t)(B3_MSG_MAX / B3_LEAF_BYTES) * B3Q_LEAF_STRIDE + 64 * 32;

// ---- the small-message hash service: one persistent instance per device (bw_dropin.hip).  Callers
// post messages into a ring of request slots (bw_b3_small.h: B3SvcReq; in HBM written through the
// BAR, or in pinned host memory), one ticket
// each.  Every worker workgroup reserves the next ticket (a fetch-add in HBM: no races between the
// workers), polls that ticket's slot over PCIe until the caller has posted it, hashes the message
// (b3q_message) and stores the digest over the slot's sentinel, where the caller spins.  No launch,
// no event, no host thread and no intermediate queue sit between a call and its digest.
//   * A ticket reserved by a worker that leaves unserved is simply reserved again by the next
//     instance: it restarts the reservations at `start`, the host's first ticket not yet returned to
//     its caller, and a worker skips a reserved ticket that was hashed out of order (proc[] in HBM).
//   * Every loop ends.  A worker waiting for its ticket gives up when nothing was hashed anywhere for
//     idle_ticks, after life_ticks, or on ctl->stop, and tells the others (dev->quit); the last worker
//     out publishes the epoch in ctl->dead, and the host starts the next instance when a caller needs
//     one.  Control flow around the barriers is wave-uniform: wave 0 polls with all its lanes (values
//     made uniform by readfirstlane, lane 0 alone reserves), the other waves wait at the barrier.
__global__ __launch_bounds__(256) void k_b3_service(B3SvcReq* req, B3SvcResp* resp, B3SvcCtl* ctl, B3SvcDev* dev,
                                                    uint32_t* proc,
                                                    uint32_t epoch, uint32_t start, uint32_t idle_ticks,
                                                    uint32_t life_ticks) {
    extern __shared__ uint4 s_msg[];
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();  // 100 MHz
    const uint64_t hard_end = (uint64_t)life_ticks + 2000000;    // 20 ms past the instance's limit
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    uint32_t* s_w = (uint32_t*)((uint8_t*)s_msg + B3Q_SVC_MSG_LDS);  // the claimed message (after the message area)
    uint64_t* s_ptr = (uint64_t*)(s_w + 4);
    if (blockIdx.x == 0 && tid < 64) {  // restart the reservations at the first ticket not yet returned
        const uint32_t f = start;
        if (lane == 0) {
            __hip_atomic_store(&dev->next, f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&dev->started, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if (tid < 64) {
        for (;;) {
            const uint32_t st = (uint32_t)__builtin_amdgcn_readfirstlane(
                (int)__hip_atomic_load(&dev->started, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT));
            if (st == epoch || __builtin_amdgcn_s_memrealtime() - t_start > hard_end) break;
            __builtin_amdgcn_s_sleep(1);
        }
    }
    for (;;) {
        if (tid < 64) {
            uint32_t go = 0, ln = 0, t = 0;
            uint64_t pt = 0;
            const bool live = (uint32_t)__builtin_amdgcn_readfirstlane((int)__hip_atomic_load(
                                  &dev->started, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT)) == epoch;
            for (uint32_t attempt = 0; live && !go; attempt++) {
                if ((uint32_t)__builtin_amdgcn_readfirstlane((int)__hip_atomic_load(
                        &dev->quit, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT)) == epoch)
                    break;
                uint32_t r = 0;
                if (lane == 0) r = __hip_atomic_fetch_add(&dev->next, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                t = (uint32_t)__builtin_amdgcn_readfirstlane((int)r);
                if ((uint32_t)__builtin_amdgcn_readfirstlane((int)__hip_atomic_load(
                        &proc[t % B3_SVC_RING], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == t + 1)
                    continue;  // hashed out of order by an earlier instance
                // idle time is measured on this wave's own clock (the XCDs' real-time counters are
                // not comparable to the tick), restarting whenever any worker hashed a message
                uint64_t t_idle = __builtin_amdgcn_s_memrealtime();
                uint32_t seen = __hip_atomic_load(&dev->progress, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                B3SvcReq* sl = req + (t % B3_SVC_RING);
                bool leave = false, skip = false;
                for (uint32_t it = 0;; it++) {
                    const uint64_t h = __hip_atomic_load(&sl->lenseq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    const uint32_t seq = (uint32_t)__builtin_amdgcn_readfirstlane((int)(h >> 32));
                    const uint32_t lw = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)h);
                    // (int)(seq - (t + 1)): 0 = this ticket's request, < 0 = the slot's earlier ticket
                    // (not posted yet), > 0 = a later ticket already holds the slot (this one was
                    // served or abandoned and its slot reclaimed by the host)
                    const int ahead = (int)(seq - (t + 1));
                    if (ahead > 0 || (ahead == 0 && (lw & B3SVC_CANCEL))) {
                        skip = true;  // an abandoned ticket the host cancelled: nobody waits for it
                        break;
                    }
                    if (ahead == 0) {
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // the message is fresh host memory
                        ln = lw;
                        pt = __hip_atomic_load(&sl->ptr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        go = 1;
                        break;
                    }
                    if ((it & 15) == 15) {
                        const uint64_t now = __builtin_amdgcn_s_memrealtime();
                        const uint32_t pr = __hip_atomic_load(&dev->progress, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if (pr != seen) {
                            seen = pr;
                            t_idle = now;
                        }
                        const uint64_t last = t_idle;
                        const uint32_t stop = __hip_atomic_load(&ctl->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        const uint32_t qu = __hip_atomic_load(&dev->quit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        const bool end = (uint32_t)__builtin_amdgcn_readfirstlane(
                                             (int)(stop != 0 || qu == epoch || now - last > idle_ticks ||
                                                   now - t_start > life_ticks)) != 0;
                        if (end) {
                            leave = true;
                            break;
                        }
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
                if (leave) {
                    if (lane == 0) __hip_atomic_store(&dev->quit, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
                (void)skip;  // (go stays 0: reserve the next ticket)
            }
            if (lane == 0) {
                s_w[0] = go;
                s_w[1] = ln;
                s_w[2] = t;
                *s_ptr = pt;
            }
        }
        __syncthreads();
        if (!s_w[0]) break;
        const uint32_t t = s_w[2];
        const uint8_t* dig = b3q_message((const uint8_t*)(uintptr_t)*s_ptr, s_w[1], (uint8_t*)s_msg, tid, 256);
        if (tid < 64) {
            if (lane < 4)  // the digest over the sentinel, 8 bytes per store (each word lands whole)
                __hip_atomic_store(&resp[t % B3_SVC_RING].digest[lane], ((const uint64_t*)dig)[lane], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
            if (lane == 0) {
                __hip_atomic_store(&proc[t % B3_SVC_RING], t + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_fetch_add(&dev->progress, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        __syncthreads();
    }
    if (tid == 0) {  // the last worker out tells the host
        // `exited` counts every worker of every instance since the service was created and is never
        // reset: instances run one after another on one stream, epochs are 1, 2, 3, ..., so the last
        // worker of epoch e is the (gridDim.x * e)-th exit (mod 2^32).  (Round 5 reset the count in
        // block 0: a worker that timed out at hard_end before block 0 ran was then not counted, the
        // end was never published, and the host believed a finished instance was still running.)
        const uint32_t n = __hip_atomic_fetch_add(&dev->exited, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (n + 1 == gridDim.x * epoch) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            __hip_atomic_store(&ctl->dead, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

void launch_b3_service(hipStream_t st, B3SvcReq* req, B3SvcResp* resp, B3SvcCtl* ctl, B3SvcDev* dev, uint32_t* proc,
                       uint32_t epoch, uint32_t start, uint32_t idle_us, uint32_t life_us) {
    static const hipError_t attr = hipFuncSetAttribute((const void*)k_b3_service,
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, B3Q_SVC_MSG_LDS + 32);
    (void)attr;
    hipLaunchKernelGGL(k_b3_service, dim3(B3_SVC_WORKERS), dim3(256), B3Q_SVC_MSG_LDS + 32, st, req, resp, ctl, dev, proc,
                       epoch, start, idle_us * 100u, life_us * 100u);
}

}  // namespace bw
