// tools/slab.hip -- does the BLAKE3 leaf pass gain from reading bytes the gear scan has just brought
// into the 256 MB Infinity Cache (MALL)?  (diagnostic only, not part of the product.)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I backuwup_amd/csrc tools/slab.hip -o build_ab/slab
//
// An 8 GiB random stream is cut into C2-shaped chunks (lengths uniform in [256 KiB, 2.2 MiB], mean
// ~1.2 MiB, arbitrary byte starts).  The shipped kernels run in two arrangements:
//   cold      k_scan over the whole stream, then k_b3_lines (+ k_b3_upper) over every chunk: the
//             product's order, every byte read from HBM twice
//   slab S    the stream in slabs of S MiB on two streams: scan(k) on the first; the hash of the
//             chunks that start in slab k on the second, once scan(k+1) is done (a chunk's boundary
//             needs candidates up to max bytes past it), while scan(k+2) runs: the leaf pass reads
//             bytes scanned one to two slabs earlier, ~2-3 S of them live
// `slab <mode> <S MiB> <G leaves per group> [hold seconds]` prints ms per 8 GiB and GB/s; with a
// hold time it repeats the arrangement that long (socket power is sampled beside it by
// tools/power_sample.py; HBM fetch per kernel by rocprofv3 --pmc FETCH_SIZE).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <string>
#include <vector>

#include "bw_cdc.hip"
#include "bw_blake3.hip"

using namespace bw;

#define CHECK(x)                                                                                                \
    do {                                                                                                        \
        hipError_t e = (x);                                                                                     \
        if (e != hipSuccess) {                                                                                  \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);                                     \
            exit(1);                                                                                            \
        }                                                                                                       \
    } while (0)

__global__ void k_fill(uint64_t* p, uint64_t n8, uint64_t seed) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

struct Part {  // the chunks of one slab (or of the whole stream), device tables
    uint64_t nb = 0, ng = 0, max_len = 0;
    uint64_t *ctr, *bs, *bl, *bg, *fe, *gh;
    uint32_t *bf, *bk, *cv, *cv2;
    uint8_t* dig;
    BlobArrays arr(uint64_t n, uint32_t gshift) const {
        BlobArrays b{bs, bl, bg, bf, bk, fe, gh, nb, n};
        b.gshift = gshift;
        return b;
    }
};

static Part make_part(const std::vector<uint64_t>& st, const std::vector<uint64_t>& ln, uint64_t n, uint32_t gshift) {
    Part p;
    p.nb = st.size();
    std::vector<uint64_t> g(p.nb);
    for (uint64_t i = 0; i < p.nb; i++) {
        g[i] = p.ng;
        p.ng += (ln[i] + (1024u << gshift) - 1) / (1024u << gshift);
        p.max_len = std::max(p.max_len, ln[i]);
    }
    const uint64_t nb = std::max<uint64_t>(p.nb, 1);
    CHECK(hipMalloc(&p.ctr, 16 * 8));
    CHECK(hipMalloc(&p.bs, nb * 8));
    CHECK(hipMalloc(&p.bl, nb * 8));
    CHECK(hipMalloc(&p.bg, nb * 8));
    CHECK(hipMalloc(&p.fe, nb * 8));
    CHECK(hipMalloc(&p.gh, nb * 8));
    CHECK(hipMalloc(&p.bf, nb * 4));
    CHECK(hipMalloc(&p.bk, nb * 4));
    CHECK(hipMalloc(&p.dig, nb * 32));
    CHECK(hipMalloc(&p.cv, (p.ng + 1) * 32));
    CHECK(hipMalloc(&p.cv2, (p.ng + 1) * 32));
    uint64_t hc[16] = {0};
    hc[C_NBLOBS] = p.nb;
    hc[C_NGROUPS] = p.ng;
    CHECK(hipMemcpy(p.ctr, hc, sizeof hc, hipMemcpyHostToDevice));
    if (p.nb) {
        std::vector<uint64_t> fe(p.nb, n);
        std::vector<uint32_t> z(p.nb, 0), one(p.nb, 1);
        CHECK(hipMemcpy(p.bs, st.data(), p.nb * 8, hipMemcpyHostToDevice));
        CHECK(hipMemcpy(p.bl, ln.data(), p.nb * 8, hipMemcpyHostToDevice));
        CHECK(hipMemcpy(p.bg, g.data(), p.nb * 8, hipMemcpyHostToDevice));
        CHECK(hipMemcpy(p.fe, fe.data(), p.nb * 8, hipMemcpyHostToDevice));
        CHECK(hipMemcpy(p.bf, z.data(), p.nb * 4, hipMemcpyHostToDevice));
        CHECK(hipMemcpy(p.bk, one.data(), p.nb * 4, hipMemcpyHostToDevice));
    }
    return p;
}

static void hash_part(hipStream_t st, const uint8_t* d, const Part& p, uint64_t n, uint32_t gshift) {
    if (!p.nb) return;
    launch_blake3(st, d, p.ctr, p.arr(n, gshift), p.nb, p.ng, p.cv, p.cv2, p.dig, (int)((p.max_len + 1023) / 1024),
                  nullptr, B3_LOADS_LINES, st);
}

int main(int argc, char** argv) {
    const std::string mode = argc > 1 ? argv[1] : "cold";
    uint64_t S = (argc > 2 ? atoll(argv[2]) : 64) << 20;
    if (S == 0) S = 64ull << 20;  // cold / scan / hash: the slab tables are built but not used
    const int G = argc > 3 ? atoi(argv[3]) : 4;
    const double hold_s = argc > 4 ? atof(argv[4]) : 0;
    const uint32_t gshift = G == 1 ? 0 : G == 2 ? 1 : 2;
    const uint64_t n = 8ull << 30;
    uint8_t* d;
    CHECK(hipMalloc(&d, n + 4096));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint64_t*)d, (n + 4096) / 8, 42);
    // C2-shaped chunks
    std::vector<uint64_t> st, ln;
    srand(7);
    for (uint64_t p = 0; p < n;) {
        uint64_t l = (256ull << 10) + (uint64_t)(((double)rand() / RAND_MAX) * (1.95 * (1 << 20)));
        l = std::min(l, n - p);
        st.push_back(p);
        ln.push_back(l);
        p += l;
    }
    Masks mk;
    mk.min = 262144; mk.avg = 1048576; mk.max = 3145728; mk.s0 = 262144;
    mk.mask_s = 0x0000d91767537000ull; mk.mask_l = 0x0000d91707537000ull; mk.mask_pre = mk.mask_l;
    mk.pre_shift = 16; mk.pre_hi = (uint32_t)((mk.mask_pre << 16) >> 32);
    const int tile_shift = argc > 5 ? atoi(argv[5]) : SCAN_TILE_SHIFT;
    mk.tile_shift = tile_shift;
    const uint64_t tile = 1ull << tile_shift;
    const uint64_t tiles_all = (n + tile - 1) / tile;
    uint32_t *tc, *ovf;
    uint64_t *ts, *sctr;
    CHECK(hipMalloc(&tc, (tiles_all + 64) * 4));
    CHECK(hipMalloc(&ts, (tiles_all + 64) * SCAN_CAP * 8));
    CHECK(hipMalloc(&ovf, (tiles_all + 64) * 4));
    const uint64_t K = (n + S - 1) / S;
    CHECK(hipMalloc(&sctr, (K + 1) * 16 * 8));
    CHECK(hipMemset(sctr, 0, (K + 1) * 16 * 8));
    hipStream_t s1, s2;
    CHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    std::vector<hipEvent_t> ev(K + 2);
    for (auto& x : ev) CHECK(hipEventCreateWithFlags(&x, hipEventDisableTiming));

    Part all = make_part(st, ln, n, gshift);
    std::vector<Part> parts(K);
    {
        std::vector<std::vector<uint64_t>> ps(K), pl(K);
        for (size_t i = 0; i < st.size(); i++) {
            ps[st[i] / S].push_back(st[i]);
            pl[st[i] / S].push_back(ln[i]);
        }
        for (uint64_t k = 0; k < K; k++) parts[k] = make_part(ps[k], pl[k], n, gshift);
    }
    auto scan = [&](hipStream_t s, uint64_t off, uint64_t len, uint64_t k) {
        const uint64_t t0 = off / tile, nt = (len + tile - 1) / tile;
        launch_scan(s, d + off, len, nt, mk, tc + t0, ts + t0 * SCAN_CAP, ovf + t0, sctr + k * 16, 16);
    };
    auto run = [&]() {
        if (mode == "cold") {
            scan(s1, 0, n, 0);
            hash_part(s1, d, all, n, gshift);
            CHECK(hipStreamSynchronize(s1));
        } else if (mode == "scan") {
            scan(s1, 0, n, 0);
            CHECK(hipStreamSynchronize(s1));
        } else if (mode == "hash") {
            hash_part(s1, d, all, n, gshift);
            CHECK(hipStreamSynchronize(s1));
        } else {  // slab
            for (uint64_t k = 0; k < K; k++) {
                scan(s1, k * S, std::min(S, n - k * S), k);
                CHECK(hipEventRecord(ev[k], s1));
                if (k >= 1) {  // chunks of slab k-1: their boundaries need slab k's candidates
                    CHECK(hipStreamWaitEvent(s2, ev[k], 0));
                    hash_part(s2, d, parts[k - 1], n, gshift);
                }
            }
            CHECK(hipStreamWaitEvent(s2, ev[K - 1], 0));
            hash_part(s2, d, parts[K - 1], n, gshift);
            CHECK(hipStreamSynchronize(s2));
            CHECK(hipStreamSynchronize(s1));
        }
    };
    run();  // warm-up
    CHECK(hipDeviceSynchronize());
    std::vector<uint8_t> ref(all.nb * 32), got(all.nb * 32);
    if (mode == "slab") {  // the slab digests equal the whole-table digests
        hash_part(s1, d, all, n, gshift);
        CHECK(hipStreamSynchronize(s1));
        CHECK(hipMemcpy(ref.data(), all.dig, ref.size(), hipMemcpyDeviceToHost));
        uint64_t i = 0;
        for (uint64_t k = 0; k < K; k++) {
            CHECK(hipMemcpy(got.data() + i * 32, parts[k].dig, parts[k].nb * 32, hipMemcpyDeviceToHost));
            i += parts[k].nb;
        }
        if (ref != got) {
            printf("MISMATCH between slab and whole-table digests\n");
            return 2;
        }
    }
    auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    const int reps = 5;
    double t0 = now();
    for (int r = 0; r < reps; r++) run();
    const double ms = (now() - t0) / reps * 1e3;
    printf("%-5s S=%4llu MiB G=%d tile=2^%d chunks=%zu: %8.3f ms per 8 GiB, %7.1f GB/s\n", mode.c_str(),
           (unsigned long long)(S >> 20), G, tile_shift, st.size(), ms, n / ms / 1e6);
    fflush(stdout);
    if (hold_s > 0) {
        int calls = 0;
        t0 = now();
        printf("HOLD_START %.3f\n", t0);
        fflush(stdout);
        while (now() - t0 < hold_s) {
            run();
            calls++;
        }
        const double el = now() - t0;
        printf("HOLD_END %.3f calls=%d %.3f ms/call %.1f GB/s\n", now(), calls, el / calls * 1e3, n * calls / el / 1e9);
    }
    return 0;
}
