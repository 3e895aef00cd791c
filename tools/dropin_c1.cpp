// tools/dropin_c1.cpp -- the reference's unchanged call sites, driven from C++ through the C ABI the
// Rust drop-ins bind.  Per file, exactly as dir_packer.rs:246-286 does:
//   len > 1 MiB: FastCDC::new(&mmap, 256 KiB, 1 MiB, 3 MiB), then blake3::hash(&mmap[off..off+len])
//                per chunk;   len <= 1 MiB: blake3::hash(whole file)
// on T threads (one tokio task per file), one context per thread or a pool of P contexts shared
// by the threads (a thread takes the first free one, as the Rust shim does), over C1's files in
// pageable host memory (the mmap'd page cache of the reference).
//   sync  bw_fastcdc_chunks + bw_blake3_hash per chunk: every chunk crosses PCIe twice (the
//         library coalesces concurrent hash calls into shared launches)
//   kept  bw_fastcdc_chunks_hashed (chunks and hashes the file in one submit) + bw_blake3_hash_dropin
//         per chunk answered from the kept digests + bw_fastcdc_release: what the Rust FastCDC
//         drop-in does behind the same signatures
// Prints GB/s of file bytes per mode (best of reps) and checks that both modes give the same
// chunks and digests (the GPU results are checked against the oracle in tests/test_gpu_parity.py).
//
// Build (CPU, after the library):
//   hipcc -O2 -std=c++17 -I include tools/dropin_c1.cpp -L backuwup_amd -lbackuwup_amd \
//     -Wl,-rpath,$PWD/backuwup_amd -lpthread -o build_ab/dropin_c1
// Run: build_ab/dropin_c1 <corpus.bin> [threads=16] [reps=3] [staging chunk MiB=64] [contexts=0: one per thread]
//        [--devices=0,1,...]
//   corpus.bin = u64 n, n offsets, n lengths, then the bytes (tools/gpu_dropin.sh writes bench.py's C1)
//   --devices: the Rust pool's policy over several GPUs (rust/backuwup-gpu Pool): the
//   contexts alternate over the listed devices (`contexts` per device), thread t's home device is
//   devices[t % n] (its small files go to that device's hash service through
//   bw_blake3_hash_dropin_device; BW_EAGAIN -> the context).  A device may repeat ([0,0] on one GPU).
//   BW_DROPIN_REGISTER_MIB=m in the environment page-locks files >= m MiB for their upload (A/B).
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <mutex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "backuwup_gpu.h"

struct Corpus {
    std::vector<uint64_t> off, len;
    std::vector<uint8_t> data;
    std::vector<uint8_t*> file;  // each file in page-aligned memory of its own, as its own mmap would be
};

struct FileOut {
    std::vector<bw_chunk> chunks;
    std::vector<uint8_t> dig;
};

static bool load(const char* path, Corpus& c) {
    FILE* f = fopen(path, "rb");
    uint64_t n = 0;
    if (!f || fread(&n, 8, 1, f) != 1) return false;
    c.off.resize(n);
    c.len.resize(n);
    if (fread(c.off.data(), 8, n, f) != n || fread(c.len.data(), 8, n, f) != n) return false;
    uint64_t total = 0;
    for (uint64_t i = 0; i < n; i++) total = std::max(total, c.off[i] + c.len[i]);
    c.data.resize(total);
    const bool ok = fread(c.data.data(), 1, total, f) == total;
    fclose(f);
    if (!ok) return false;
    // one page-aligned buffer per file (the reference maps each file on its own, dir_packer.rs:252):
    // no page is shared between two files, so page-locking one file in place (BW_DROPIN_REGISTER_MIB)
    // never touches another's pages
    c.file.resize(n);
    for (uint64_t i = 0; i < n; i++) {
        void* p = nullptr;
        if (posix_memalign(&p, 4096, std::max<uint64_t>(c.len[i], 1))) return false;
        memcpy(p, c.data.data() + c.off[i], c.len[i]);
        c.file[i] = (uint8_t*)p;
    }
    std::vector<uint8_t>().swap(c.data);
    return true;
}

static const uint64_t SMALL = 1 << 20;  // dir_packer.rs:246

static int process(bw_ctx* ctx, int home, const uint8_t* p, uint64_t n, bool kept, FileOut& o, std::string& err) {
    o.chunks.clear();
    o.dig.clear();
    uint8_t d[32];
    if (n <= SMALL) {  // fs::read + add_file_blob
        int rc = home >= 0 ? bw_blake3_hash_dropin_device(home, p, n, d) : BW_EAGAIN;
        if (rc == BW_EAGAIN) rc = bw_blake3_hash(ctx, p, n, d);
        if (rc) return err = bw_last_error(ctx), rc;
        o.chunks.push_back({0, 0, n});
        o.dig.insert(o.dig.end(), d, d + 32);
        return 0;
    }
    std::vector<bw_chunk> ch(n / (256 << 10) + 2);
    uint64_t nc = 0, handle = 0;
    int rc = kept ? bw_fastcdc_chunks_hashed(ctx, p, n, 256 << 10, 1 << 20, 3 << 20, ch.data(), ch.size(), &nc, &handle)
                  : bw_fastcdc_chunks(ctx, p, n, 256 << 10, 1 << 20, 3 << 20, ch.data(), ch.size(), &nc);
    if (rc) return err = bw_last_error(ctx), rc;
    ch.resize(nc);
    for (const bw_chunk& c : ch) {  // for chunk in chunker { add_file_blob(&mmap[off..off+len]) }
        if ((rc = kept ? bw_blake3_hash_dropin(ctx, p + c.offset, c.length, d) : bw_blake3_hash(ctx, p + c.offset, c.length, d)))
            break;
        o.dig.insert(o.dig.end(), d, d + 32);
    }
    bw_fastcdc_release(handle);
    if (rc) return err = bw_last_error(ctx), rc;
    o.chunks = std::move(ch);
    return 0;
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
    if (argc < 2) {
        fprintf(stderr, "usage: %s corpus.bin [threads] [reps]\n", argv[0]);
        return 2;
    }
    Corpus c;
    if (!load(argv[1], c)) {
        fprintf(stderr, "cannot read %s\n", argv[1]);
        return 2;
    }
    const int T = argc > 2 ? atoi(argv[2]) : 16, reps = argc > 3 ? atoi(argv[3]) : 3;
    const uint64_t stage_mib = argc > 4 ? strtoull(argv[4], nullptr, 10) : 0;  // BW_OPT_STAGE_CHUNK (0: default)
    const int P0 = argc > 5 && atoi(argv[5]) > 0 ? atoi(argv[5]) : T;             // contexts (0: one per thread)
    const bool pool_devs = !devs.empty();
    if (devs.empty()) devs.push_back(0);
    const int ND = (int)devs.size(), P = pool_devs ? P0 * ND : P0;  // --devices: P0 contexts per listed device
    const uint64_t nf = c.off.size();
    uint64_t bytes = 0, big = 0;
    for (uint64_t i = 0; i < nf; i++) {
        bytes += c.len[i];
        big += c.len[i] > SMALL;
    }
    printf("corpus: %llu files (%llu > 1 MiB), %.3f GB; %d threads, %d contexts; devices", (unsigned long long)nf,
           (unsigned long long)big, bytes / 1e9, T, P);
    for (int d : devs) printf(" %d", d);
    printf("%s\n", pool_devs ? " (home device per thread, small files to its hash service)" : "");
    size_t free0 = 0, tot = 0;
    hipSetDevice(0);
    hipMemGetInfo(&free0, &tot);
    std::vector<bw_ctx*> ctxs(P);
    std::vector<std::mutex> ctx_mu(P);
    for (int t = 0; t < P; t++) {
        if (bw_create(devs[t % ND], &ctxs[t])) return 3;
        if (stage_mib && bw_set_option(ctxs[t], BW_OPT_STAGE_CHUNK, stage_mib << 20)) return 3;
    }
    if (stage_mib) printf("pinned staging chunks of %llu MiB\n", (unsigned long long)stage_mib);
    std::vector<FileOut> ref(nf), got(nf);
    int rc_all = 0;
    for (int mode = 0; mode < 2; mode++) {
        const bool kept = mode == 1;
        std::vector<FileOut>& out = kept ? got : ref;
        double best = 1e30;
        const uint64_t hits0 = bw_blake3_kept_hits();
        for (int r = 0; r < reps + 1; r++) {  // the first pass warms the contexts' buffers
            std::atomic<uint64_t> next{0};
            std::atomic<int> fail{0};
            std::string errs[64];
            auto t0 = std::chrono::steady_clock::now();
            std::vector<std::thread> th;
            for (int t = 0; t < T; t++)
                th.emplace_back([&, t] {
                    for (uint64_t i; (i = next++) < nf && !fail;) {
                        int k = t % P;  // the first free context from this thread's starting point
                        for (int j = 0; j < P; j++)
                            if (ctx_mu[(t + j) % P].try_lock()) {
                                k = (t + j) % P;
                                ctx_mu[k].unlock();
                                break;
                            }
                        std::lock_guard<std::mutex> lk(ctx_mu[k]);
                        if (int rc = process(ctxs[k], pool_devs ? devs[t % ND] : -1, c.file[i], c.len[i],
                                             kept, out[i], errs[t % 64]))
                            fail = rc;
                    }
                });
            for (auto& x : th) x.join();
            const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            if (fail) {
                for (auto& e : errs)
                    if (!e.empty()) fprintf(stderr, "error: %s\n", e.c_str());
                return 4;
            }
            if (r) best = std::min(best, s);
        }
        uint64_t nchunks = 0;
        for (auto& o : out) nchunks += o.chunks.size();
        size_t fr = 0;
        hipMemGetInfo(&fr, &tot);
        printf("HBM in use after the passes: %.2f GiB (%.3f GiB per context)\n", (free0 - fr) / 1073741824.0,
               (free0 - fr) / 1073741824.0 / P);
        printf("%-4s %8.2f GB/s (%.2f ms per pass, best of %d; %llu blobs; kept-digest answers %llu)\n",
               kept ? "kept" : "sync", bytes / best / 1e9, best * 1e3, reps, (unsigned long long)nchunks,
               (unsigned long long)(bw_blake3_kept_hits() - hits0));
        fflush(stdout);
    }
    for (uint64_t i = 0; i < nf; i++) {
        bool same = ref[i].chunks.size() == got[i].chunks.size() && ref[i].dig == got[i].dig;
        for (size_t k = 0; same && k < ref[i].chunks.size(); k++)
            same = ref[i].chunks[k].offset == got[i].chunks[k].offset && ref[i].chunks[k].length == got[i].chunks[k].length &&
                   ref[i].chunks[k].hash == got[i].chunks[k].hash;
        if (!same) {
            fprintf(stderr, "file %llu: sync and kept results differ\n", (unsigned long long)i);
            rc_all = 5;
        }
    }
    printf("sync == kept on every file: %s\n", rc_all ? "NO" : "yes");
    for (bw_ctx* x : ctxs) bw_destroy(x);
    return rc_all;
}
