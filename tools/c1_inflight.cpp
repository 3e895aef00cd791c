// tools/c1_inflight.cpp -- C1-shaped batches with ONE batch in flight, driven from C++ through the
// C ABI (what a Rust caller of the shim crate does), to separate the library's own per-batch time
// from bench.py's Python between two batches.  Diagnostic, not the bench line.
//
// Build (on the CPU, after the library):
//   hipcc --offload-arch=gfx950 -O2 -std=c++17 -I include tools/c1_inflight.cpp \
//     -L backuwup_amd -lbackuwup_amd -Wl,-rpath,$PWD/backuwup_amd -o build/c1_inflight
// Run: build/c1_inflight [steps=1500] [warmup=20] [table]
//
// The batch: 1 GiB, files log-uniform in 4 KiB..64 MiB (splitmix64 content generated on the GPU),
// 30 % of the bytes whole-file copies of earlier files, like bench.py's C1.  `table` (optional) is
// bench.py's exact C1 file table (u64 n, then n offsets, then n lengths; see tools/gpu_r3p.sh): the
// files are then bench.py's, with random content (copies cost the same as unique files).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "backuwup_gpu.h"

#define CHECK(x)                                                                                  \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) { fprintf(stderr, "HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } \
    } while (0)
#define BW(x)                                                                                     \
    do {                                                                                          \
        int r_ = (x);                                                                             \
        if (r_) { fprintf(stderr, "bw %d (%s) at %d\n", r_, bw_strerror(r_), __LINE__); return 1; } \
    } while (0)

__global__ void k_fill(uint64_t* p, uint64_t n, uint64_t seed) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

static uint64_t rng_state = 0x6261636Bull;
static double urand() {
    rng_state = rng_state * 6364136223846793005ull + 1442695040888963407ull;
    return (double)(rng_state >> 11) / 9007199254740992.0;
}

int main(int argc, char** argv) {
    const int steps = argc > 1 ? atoi(argv[1]) : 1500, warmup = argc > 2 ? atoi(argv[2]) : 20;
    const uint64_t total = 1ull << 30, uniq_target = (uint64_t)(total * 0.7);
    std::vector<uint64_t> off, len;
    uint64_t pos = 0, uniq = 0;
    if (argc > 3) {  // bench.py's table
        FILE* f = fopen(argv[3], "rb");
        uint64_t n = 0;
        if (!f || fread(&n, 8, 1, f) != 1) return 2;
        off.resize(n);
        len.resize(n);
        if (fread(off.data(), 8, n, f) != n || fread(len.data(), 8, n, f) != n) return 2;
        fclose(f);
        for (uint64_t i = 0; i < n; i++) pos = std::max(pos, off[i] + len[i]);
        pos = (pos + 15) & ~15ull;
        uniq = uniq_target;
    }
    const bool own_table = off.empty();
    while (own_table && uniq < uniq_target) {  // unique files, log-uniform sizes
        uint64_t n = (uint64_t)std::exp(std::log(4096.0) + urand() * (std::log(64.0 * 1048576) - std::log(4096.0)));
        n = std::min(n, uniq_target - uniq + 4096);
        off.push_back(pos);
        len.push_back(n);
        pos = (pos + n + 15) & ~15ull;
        uniq += n;
    }
    const size_t n_uniq = off.size();
    std::vector<uint64_t> src;
    while (own_table && pos < total) {  // whole-file copies of earlier files
        const size_t k = (size_t)(urand() * n_uniq);
        if (pos + len[k] > total) break;
        src.push_back(k);
        off.push_back(pos);
        len.push_back(len[k]);
        pos = (pos + len[k] + 15) & ~15ull;
    }
    const uint64_t data_len = pos;
    uint64_t bytes = 0;
    for (uint64_t l : len) bytes += l;

    uint8_t* d = nullptr;
    CHECK(hipMalloc(&d, data_len + 64));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint64_t*)d, (data_len + 7) / 8, 42ull);
    for (size_t i = 0; i < src.size(); i++)
        CHECK(hipMemcpy(d + off[n_uniq + i], d + off[src[i]], len[src[i]], hipMemcpyDeviceToDevice));
    CHECK(hipDeviceSynchronize());

    bw_ctx* c = nullptr;
    BW(bw_create(0, &c));
    bw_params p;
    bw_params_default(&p);
    std::vector<bw_blob> out(bytes / 262144 + 2 * off.size() + 16);
    uint64_t n_out = 0, t = 0, n_blobs = 0;
    BW(bw_index_reset(c, (uint64_t)(warmup + steps + 4) * out.size()));
    for (int i = 0; i < warmup; i++) {
        BW(bw_submit_device(c, d, data_len, off.data(), len.data(), off.size(), &p, &t));
        BW(bw_wait(c, t, out.data(), out.size(), &n_out));
    }
    n_blobs = n_out;
    CHECK(hipDeviceSynchronize());
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < steps; i++) {  // one batch in flight: submit, then wait for its results
        BW(bw_submit_device(c, d, data_len, off.data(), len.data(), off.size(), &p, &t));
        BW(bw_wait(c, t, out.data(), out.size(), &n_out));
    }
    CHECK(hipDeviceSynchronize());
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    BW(bw_index_check(c));
    printf("{\"what\": \"C1-shaped batch, one in flight, C++ caller through the C ABI\", \"files\": %zu, "
           "\"bytes\": %llu, \"blobs\": %llu, \"steps\": %d, \"ms_per_step\": %.4f, \"GBps\": %.1f}\n",
           off.size(), (unsigned long long)bytes, (unsigned long long)n_blobs, steps, s / steps * 1e3,
           (double)bytes * steps / s / 1e9);
    bw_destroy(c);
    hipFree(d);
    return 0;
}
