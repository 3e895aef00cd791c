// tools/collide.hip -- a genuine BLAKE3 collision on the first 8 digest bytes (the key the round-3
// device index merged slots by), found on the GPU with parallel collision search (van Oorschot -
// Wiener distinguished points).  Diagnostic / fixture generator, not part of the product.
//
// f(x) = the first 8 bytes (little endian) of blake3::hash(the 8 bytes of x, little endian): one
// compression of a single-block root chunk.  Every lane walks x, f(x), f(f(x)), ... from random
// starts until a distinguished point (low D bits zero) and records (start, point, length); two
// walks that end at one point merged somewhere, and re-walking both from the same distance to the
// point finds x1 != x2 with f(x1) == f(x2): two 8-byte messages whose digests share 8 bytes.
// About 2^32 evaluations are expected; the GPU does ~5e10 a second.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I backuwup_amd/csrc tools/collide.hip -o build_ab/collide
// Run:   build_ab/collide [out.json] [D=14] [steps per lane=131072] [seed=1]
// The pair lands in tests/golden/blake3_prefix_collision.json (checked on the CPU against the oracle
// by tests/test_oracle.py, and sent through the index and bw_process_files by a GPU test).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <unordered_map>
#include <vector>

#include "bw_device.h"

#define CHECK(x)                                                                                    \
    do {                                                                                            \
        hipError_t e_ = (x);                                                                        \
        if (e_ != hipSuccess) {                                                                     \
            fprintf(stderr, "HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);               \
            exit(1);                                                                                \
        }                                                                                           \
    } while (0)

__device__ __forceinline__ uint64_t f8(uint64_t x, uint32_t out[8]) {
    uint32_t m[16];
#pragma unroll
    for (int i = 0; i < 16; i++) m[i] = 0;
    m[0] = (uint32_t)x;
    m[1] = (uint32_t)(x >> 32);
    b3_iv(out);
    b3_compress(out, m, 8, 0, B3_CHUNK_START | B3_CHUNK_END | B3_ROOT);
    return (uint64_t)out[0] | ((uint64_t)out[1] << 32);
}

__device__ __forceinline__ uint64_t splitmix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

struct Walk {
    uint64_t start, point, len;
};

// Walks from fresh random starts until `budget` evaluations are spent; every finished walk is
// recorded.  A walk longer than 16 x 2^D is abandoned (a cycle without a distinguished point).
__global__ __launch_bounds__(256) void k_walks(uint64_t seed, uint32_t dbits, uint64_t budget, Walk* out,
                                               unsigned long long* n_out, uint64_t cap) {
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t mask = (1ull << dbits) - 1, maxlen = 16ull << dbits;
    uint64_t k = 0, spent = 0;
    uint32_t o[8];
    while (spent < budget) {
        const uint64_t start = splitmix(seed ^ splitmix(gid * 0x100000001B3ull + k++));
        uint64_t x = start, len = 0;
        bool done = false;
        while (spent < budget && len < maxlen) {
            x = f8(x, o);
            len++;
            spent++;
            if ((x & mask) == 0) {
                done = true;
                break;
            }
        }
        if (done) {
            const unsigned long long i = atomicAdd(n_out, 1ull);
            if (i < cap) out[i] = Walk{start, x, len};
        }
    }
}

// Re-walk two walks that end at the same point: advance the longer by the length difference, then
// step both until their images agree.  res = {x1, x2, found}.
__global__ void k_merge(uint64_t a, uint64_t la, uint64_t b, uint64_t lb, uint64_t* res) {
    if (threadIdx.x || blockIdx.x) return;
    uint32_t o[8];
    if (la < lb) {
        uint64_t t = a; a = b; b = t;
        t = la; la = lb; lb = t;
    }
    for (uint64_t i = 0; i < la - lb; i++) a = f8(a, o);
    res[2] = 0;
    if (a == b) return;  // one start lies on the other's path: the walks share a chain, no collision
    for (uint64_t i = 0; i < lb; i++) {
        const uint64_t fa = f8(a, o), fb = f8(b, o);
        if (fa == fb) {
            res[0] = a;
            res[1] = b;
            res[2] = 1;
            return;
        }
        a = fa;
        b = fb;
    }
}

__global__ void k_digest(uint64_t x, uint32_t* d) {
    if (threadIdx.x || blockIdx.x) return;
    uint32_t o[8];
    f8(x, o);
    for (int i = 0; i < 8; i++) d[i] = o[i];
}

int main(int argc, char** argv) {
    const char* path = argc > 1 ? argv[1] : "gpurun_out/blake3_prefix_collision.json";
    const uint32_t D = argc > 2 ? atoi(argv[2]) : 14;
    const uint64_t budget = argc > 3 ? strtoull(argv[3], nullptr, 10) : 131072;
    const uint64_t seed = argc > 4 ? strtoull(argv[4], nullptr, 10) : 1;
    const unsigned blocks = 4096, threads = 256;
    const uint64_t lanes = (uint64_t)blocks * threads;
    const uint64_t cap = lanes * (budget >> D) * 2 + 1024;
    Walk* d_w;
    unsigned long long* d_n;
    uint64_t* d_res;
    uint32_t* d_dig;
    CHECK(hipMalloc(&d_w, cap * sizeof(Walk)));
    CHECK(hipMalloc(&d_n, 8));
    CHECK(hipMalloc(&d_res, 24));
    CHECK(hipMalloc(&d_dig, 32));
    CHECK(hipMemset(d_n, 0, 8));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_walks, dim3(blocks), dim3(threads), 0, 0, seed, D, budget, d_w, d_n, cap);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    unsigned long long n = 0;
    CHECK(hipMemcpy(&n, d_n, 8, hipMemcpyDeviceToHost));
    n = std::min<unsigned long long>(n, cap);
    std::vector<Walk> w(n);
    CHECK(hipMemcpy(w.data(), d_w, n * sizeof(Walk), hipMemcpyDeviceToHost));
    const double evals = (double)lanes * budget;
    printf("walks: %llu distinguished points, %.3g evaluations in %.1f ms (%.3g f/s)\n", n, evals, ms,
           evals / (ms * 1e-3));
    std::unordered_map<uint64_t, size_t> seen;
    seen.reserve(n * 2);
    int found = 0;
    FILE* f = nullptr;
    for (size_t i = 0; i < n && !found; i++) {
        auto it = seen.find(w[i].point);
        if (it == seen.end()) {
            seen.emplace(w[i].point, i);
            continue;
        }
        const Walk& a = w[it->second];
        const Walk& b = w[i];
        if (a.start == b.start) continue;
        hipLaunchKernelGGL(k_merge, dim3(1), dim3(64), 0, 0, a.start, a.len, b.start, b.len, d_res);
        uint64_t res[3];
        CHECK(hipMemcpy(res, d_res, 24, hipMemcpyDeviceToHost));
        if (!res[2]) continue;
        uint32_t d1[8], d2[8];
        hipLaunchKernelGGL(k_digest, dim3(1), dim3(64), 0, 0, res[0], d_dig);
        CHECK(hipMemcpy(d1, d_dig, 32, hipMemcpyDeviceToHost));
        hipLaunchKernelGGL(k_digest, dim3(1), dim3(64), 0, 0, res[1], d_dig);
        CHECK(hipMemcpy(d2, d_dig, 32, hipMemcpyDeviceToHost));
        if (d1[0] != d2[0] || d1[1] != d2[1]) continue;  // cannot happen: f(x1) == f(x2)
        f = fopen(path, "w");
        if (!f) return 3;
        auto hex8 = [&](uint64_t x) {
            for (int k = 0; k < 8; k++) fprintf(f, "%02x", (unsigned)((x >> (8 * k)) & 0xff));
        };
        auto hexd = [&](const uint32_t* d) {
            for (int k = 0; k < 32; k++) fprintf(f, "%02x", (unsigned)((d[k / 4] >> (8 * (k % 4))) & 0xff));
        };
        fprintf(f, "{\"what\": \"two 8-byte messages whose BLAKE3 digests share their first 8 bytes\", \"m1\": \"");
        hex8(res[0]);
        fprintf(f, "\", \"m2\": \"");
        hex8(res[1]);
        fprintf(f, "\", \"digest1\": \"");
        hexd(d1);
        fprintf(f, "\", \"digest2\": \"");
        hexd(d2);
        fprintf(f, "\", \"generator\": \"tools/collide.hip D=%u steps_per_lane=%llu seed=%llu\"}\n", D,
                (unsigned long long)budget, (unsigned long long)seed);
        fclose(f);
        found = 1;
        printf("collision: m1=%016llx m2=%016llx (as u64; messages are their 8 LE bytes) -> %s\n",
               (unsigned long long)res[0], (unsigned long long)res[1], path);
    }
    if (!found) {
        printf("no collision among the distinguished points: rerun with another seed or more steps\n");
        return 2;
    }
    return 0;
}
