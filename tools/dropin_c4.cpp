// tools/dropin_c4.cpp -- the reference's unchanged call sites on a C4-shaped tree:
// 1 M small files of 4-64 KiB with 30 % whole-file copies (bench.py --workload c4's file table), and
// per file exactly what dir_packer.rs does for a file of at most 1 MiB:
//   fs::read + add_file_blob -> blake3::hash(data)                        (dir_packer.rs:267-271, :286)
//   the file's Tree { File, name, metadata, children: [hash] } -> add_tree_to_blobs
//     -> split_serialize_tree -> bincode::serialize -> blake3::hash(tree)  (:274, :314-320, :366-372)
// through the C ABI the Rust drop-ins bind (bw_blake3_hash_dropin, bw_tree_serialize), on T threads
// pulling files from one queue (tokio's workers running one task per file, dir_packer.rs:166).  The
// threads share a pool of P contexts like the Rust shim (rust/backuwup-gpu: BACKUWUP_GPU_CONTEXTS);
// a small message only names the device, and concurrent calls are coalesced into one launch.
//
// Prints per thread count: files/s, blake3::hash calls/s, GB/s of file bytes, the coalesced
// launches and their mean size, HBM in use; and checks every digest against one batched
// bw_blake3_hash_many over the same messages (a different path through the library: one launch for
// all of them).  The GPU against the oracle: tests/test_gpu_parity.py::test_coalesced_hash_threads.
//
// Build (CPU, after the library):
//   hipcc -O2 -std=c++17 -I include tools/dropin_c4.cpp -L backuwup_amd -lbackuwup_amd \
//     -Wl,-rpath,$PWD/backuwup_amd -lpthread -o build_ab/dropin_c4
// Run: build_ab/dropin_c4 <table.bin> <threads list, e.g. 16,64,256> [contexts=16] [reps=2] [--devices=0,1,...]
//   table.bin = u64 n, u64 unique_bytes, u64 seed, n offsets, n lengths (tools/gpu_dropin.sh writes it)
//   --devices: the Rust pool's policy: thread t hashes on devices[t % n] through
//   bw_blake3_hash_dropin_device (no context; BW_EAGAIN -> a pool context), `contexts` per device.
//   A device may repeat ([0,0] on one GPU).
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "backuwup_gpu.h"

static uint64_t mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int main(int argc, char** argv) {
    std::vector<int> devs;  // --devices=LIST (anywhere on the line)
    {
        int k = 1;
        for (int i = 1; i < argc; i++) {
            if (!strncmp(argv[i], "--devices=", 10)) {
                for (const char* q = argv[i] + 10; *q;) {
                    devs.push_back(atoi(q));
                    while (*q && *q != ',') q++;
                    if (*q) q++;
                }
            } else {
                argv[k++] = argv[i];
            }
        }
        argc = k;
    }
    if (argc < 3) {
        fprintf(stderr, "usage: %s table.bin threads[,threads...] [contexts] [reps]\n", argv[0]);
        return 2;
    }
    FILE* f = fopen(argv[1], "rb");
    uint64_t hdr[3];
    if (!f || fread(hdr, 8, 3, f) != 3) return 2;
    const uint64_t nf = hdr[0], ubytes = hdr[1], seed = hdr[2];
    std::vector<uint64_t> off(nf), len(nf);
    if (fread(off.data(), 8, nf, f) != nf || fread(len.data(), 8, nf, f) != nf) return 2;
    fclose(f);
    std::vector<int> tlist;
    {
        std::stringstream ss(argv[2]);
        for (std::string t; std::getline(ss, t, ',');) tlist.push_back(atoi(t.c_str()));
    }
    const bool pool_devs = !devs.empty();
    if (devs.empty()) devs.push_back(0);
    const int ND = (int)devs.size();
    const int P = (argc > 3 ? atoi(argv[3]) : 16) * (pool_devs ? ND : 1), reps = argc > 4 ? atoi(argv[4]) : 2;
    std::vector<std::mutex> pool_mu(P);
    // the unique bytes: splitmix64 stream `seed` (backuwup_amd/synth.py splitmix_torch), 16 threads
    std::vector<uint8_t> data((ubytes + 7) / 8 * 8);
    {
        const uint64_t nw = data.size() / 8;
        std::vector<std::thread> th;
        for (int t = 0; t < 16; t++)
            th.emplace_back([&, t] {
                uint64_t* w = (uint64_t*)data.data();
                for (uint64_t i = nw * t / 16; i < nw * (t + 1) / 16; i++) w[i] = mix(seed + (i + 1) * 0x9E3779B97F4A7C15ull);
            });
        for (auto& x : th) x.join();
    }
    uint64_t bytes = 0;
    for (uint64_t i = 0; i < nf; i++) bytes += len[i];
    size_t free0 = 0, total_mem = 0;
    hipSetDevice(0);
    hipMemGetInfo(&free0, &total_mem);
    std::vector<bw_ctx*> pool(P);
    for (int j = 0; j < P; j++)
        if (bw_create(devs[j % ND], &pool[j])) return 3;
    printf("corpus: %llu files, %.3f GB of file bytes (%.3f GB unique); contexts %d\n", (unsigned long long)nf,
           bytes / 1e9, ubytes / 1e9, P);
    // one file's Tree (filesystem/mod.rs:63-77) as process_file builds it for a small file
    auto tree_of = [&](uint64_t i, const uint8_t dig[32], uint8_t* buf, uint64_t cap, uint64_t* n) {
        char name[32];
        const int nl = snprintf(name, sizeof name, "file_%07llu.bin", (unsigned long long)i);
        bw_tree t{};
        t.kind = BW_TREE_FILE;
        t.flags = BW_TREE_HAS_SIZE | BW_TREE_HAS_MTIME | BW_TREE_HAS_CTIME;
        t.size = len[i];
        t.mtime = 1700000000ull + i;
        t.ctime = 1700000000ull + i / 2;
        t.name = (const uint8_t*)name;
        t.name_len = (uint64_t)nl;
        t.children = dig;
        t.n_children = 1;
        return bw_tree_serialize(&t, nullptr, buf, cap, n);
    };
    std::vector<uint8_t> fdig(32 * nf), tdig(32 * nf);
    int rc_all = 0;
    for (int T : tlist) {
        double best = 1e30;
        uint64_t b0 = 0, m0 = 0, b1 = 0, m1 = 0;
        size_t tfree = 0, ttot = 0;
        hipMemGetInfo(&tfree, &ttot);  // (the previous sweep's check left a 24 GB batch in pool[0])
        size_t free_min = tfree;
        for (int r = 0; r < reps + 1; r++) {  // the first pass warms the library's buffers
            std::atomic<uint64_t> next{0};
            std::atomic<int> fail{0};
            b0 = m0 = 0;
            for (int d = 0; d < 64; d++) {
                uint64_t b = 0, m = 0;
                bw_blake3_coalesce_stats(d, &b, &m);
                b0 += b;
                m0 += m;
            }
            auto t0 = std::chrono::steady_clock::now();
            std::vector<std::thread> th;
            for (int t = 0; t < T; t++)
                th.emplace_back([&, t] {
                    bw_ctx* ctx = pool[t % P];  // small messages: the context only names the device
                    const int home = devs[t % ND];
                    // the Rust blake3::hash: the home device's service, BW_EAGAIN -> a pool context
                    auto hash = [&](const uint8_t* m, uint64_t n, uint8_t* out) {
                        if (!pool_devs) return bw_blake3_hash_dropin(ctx, m, n, out);
                        int rc = bw_blake3_hash_dropin_device(home, m, n, out);
                        if (rc != BW_EAGAIN) return rc;
                        std::lock_guard<std::mutex> lk(pool_mu[t % P]);
                        const uint64_t o = 0;
                        return bw_blake3_hash_many(pool[t % P], m, n, &o, &n, 1, out);
                    };
                    uint8_t tb[512];
                    for (uint64_t i; (i = next++) < nf && !fail;) {
                        uint8_t* d = &fdig[32 * i];
                        if (int rc = hash(data.data() + off[i], len[i], d)) {
                            fail = rc;
                            break;
                        }
                        uint64_t n = 0;
                        if (int rc = tree_of(i, d, tb, sizeof tb, &n)) {
                            fail = rc;
                            break;
                        }
                        if (int rc = hash(tb, n, &tdig[32 * i])) {
                            fail = rc;
                            break;
                        }
                    }
                });
            for (auto& x : th) x.join();
            const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            b1 = m1 = 0;
            for (int d = 0; d < 64; d++) {
                uint64_t b = 0, m = 0;
                bw_blake3_coalesce_stats(d, &b, &m);
                b1 += b;
                m1 += m;
            }
            size_t fr = 0, tot = 0;
            hipMemGetInfo(&fr, &tot);
            free_min = std::min(free_min, fr);
            if (fail) {
                fprintf(stderr, "threads %d: error %d (%s)\n", T, (int)fail, bw_strerror(fail));
                return 4;
            }
            if (r) best = std::min(best, s);
            printf("threads %4d: pass %d %.3f s\n", T, r, s);  // (a long sweep keeps writing)
            fflush(stdout);
        }
        printf("threads %4d: %8.1f k files/s  %8.1f k calls/s  %7.2f GB/s of file bytes  (%.3f s per pass, best of %d;"
               " last pass %llu launches, %.1f messages each; HBM added by the passes %.2f GiB)\n",
               T, nf / best / 1e3, 2 * nf / best / 1e3, bytes / best / 1e9, best, reps, (unsigned long long)(b1 - b0),
               (double)(m1 - m0) / std::max<uint64_t>(1, b1 - b0), (double)(tfree - free_min) / 1073741824.0);
        fflush(stdout);
        // every digest against one batched launch over the same messages
        std::vector<uint8_t> want(32 * nf);
        if (bw_blake3_hash_many(pool[0], data.data(), data.size(), off.data(), len.data(), nf, want.data())) return 5;
        uint64_t bad = memcmp(want.data(), fdig.data(), want.size()) != 0;
        std::vector<uint8_t> tbytes;
        std::vector<uint64_t> toff(nf), tlen(nf);
        for (uint64_t i = 0; i < nf; i++) {
            uint8_t tb[512];
            uint64_t n = 0;
            tree_of(i, &want[32 * i], tb, sizeof tb, &n);
            toff[i] = tbytes.size();
            tlen[i] = n;
            tbytes.insert(tbytes.end(), tb, tb + n);
        }
        std::vector<uint8_t> twant(32 * nf);
        if (bw_blake3_hash_many(pool[0], tbytes.data(), tbytes.size(), toff.data(), tlen.data(), nf, twant.data())) return 5;
        bad += memcmp(twant.data(), tdig.data(), twant.size()) != 0;
        printf("threads %4d: file and tree digests equal to one batched launch: %s\n", T, bad ? "NO" : "yes");
        if (bad) rc_all = 6;
    }
    for (bw_ctx* c : pool) bw_destroy(c);
    return rc_all;
}
