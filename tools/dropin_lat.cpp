// tools/dropin_lat.cpp -- where a small blake3::hash drop-in call spends its time.
//
// One caller thread (or T) calling bw_blake3_hash_dropin back to back on messages of one size, against
// the bare cost of a GPU round trip on this box: an empty kernel launch + hipEventSynchronize, and the
// same launch followed by a condition-variable hand-off to another thread and back (the coalescer's
// launcher/completer threads).  Run under rocprofv3 --kernel-trace --stats for the kernel's own time.
//
// Build (CPU, after the library):
//   hipcc -O2 -std=c++17 --offload-arch=gfx950 -I include tools/dropin_lat.cpp -L backuwup_amd -lbackuwup_amd \
//     -Wl,-rpath,$PWD/backuwup_amd -lpthread -o build_ab/dropin_lat
// Run: build_ab/dropin_lat <sizes, e.g. 96,4096,16384,65536> [calls=4000] [threads=1]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include <unistd.h>

#include "backuwup_gpu.h"

__global__ void k_empty(int* p) {
    if (p && threadIdx.x == 1024) p[0] = 1;  // never true: keeps the kernel from being elided
}

// a neighbour that keeps every CU busy: each workgroup spins for `ticks` of the 100 MHz clock
__global__ void k_busy(uint64_t ticks, int* p) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
    if (p && threadIdx.x == 1024) p[0] = 1;
}

using clk = std::chrono::steady_clock;

static double us_since(clk::time_point t) { return std::chrono::duration<double, std::micro>(clk::now() - t).count(); }

static void report(const char* what, std::vector<double>& v) {
    std::sort(v.begin(), v.end());
    double s = 0;
    for (double x : v) s += x;
    printf("%-34s mean %8.2f us  p50 %8.2f  p90 %8.2f  p99 %8.2f  (%zu calls)\n", what, s / v.size(), v[v.size() / 2],
           v[v.size() * 9 / 10], v[v.size() * 99 / 100], v.size());
    fflush(stdout);
}

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s sizes [calls] [threads]\n", argv[0]);
        return 2;
    }
    std::vector<uint64_t> sizes;
    {
        std::stringstream ss(argv[1]);
        for (std::string t; std::getline(ss, t, ',');) sizes.push_back(strtoull(t.c_str(), nullptr, 10));
    }
    const int calls = argc > 2 ? atoi(argv[2]) : 4000, T = argc > 3 ? atoi(argv[3]) : 1;
    hipSetDevice(0);
    hipStream_t st;
    hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    hipEvent_t ev;
    hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    // the bare round trip
    {
        std::vector<double> v;
        for (int i = 0; i < calls + 100; i++) {
            auto t = clk::now();
            k_empty<<<1, 64, 0, st>>>(nullptr);
            hipEventRecord(ev, st);
            hipEventSynchronize(ev);
            if (i >= 100) v.push_back(us_since(t));
        }
        report("empty launch + event sync", v);
    }
    // the same with a hand-off to a launching thread and a completing thread, as the coalescer does
    {
        std::mutex mu;
        std::condition_variable cv_l, cv_c, cv_w;
        int stage = 0;  // 1 = request posted, 2 = launched, 3 = done
        bool quit = false;
        std::thread launcher([&] {
            hipSetDevice(0);
            std::unique_lock<std::mutex> lk(mu);
            for (;;) {
                cv_l.wait(lk, [&] { return stage == 1 || quit; });
                if (quit) return;
                k_empty<<<1, 64, 0, st>>>(nullptr);
                hipEventRecord(ev, st);
                stage = 2;
                cv_c.notify_one();
            }
        });
        std::thread completer([&] {
            hipSetDevice(0);
            std::unique_lock<std::mutex> lk(mu);
            for (;;) {
                cv_c.wait(lk, [&] { return stage == 2 || quit; });
                if (quit) return;
                lk.unlock();
                hipEventSynchronize(ev);
                lk.lock();
                stage = 3;
                cv_w.notify_one();
            }
        });
        std::vector<double> v;
        for (int i = 0; i < calls + 100; i++) {
            auto t = clk::now();
            std::unique_lock<std::mutex> lk(mu);
            stage = 1;
            cv_l.notify_one();
            cv_w.wait(lk, [&] { return stage == 3; });
            stage = 0;
            lk.unlock();
            if (i >= 100) v.push_back(us_since(t));
        }
        {
            std::lock_guard<std::mutex> lk(mu);
            quit = true;
        }
        cv_l.notify_all();
        cv_c.notify_all();
        launcher.join();
        completer.join();
        report("launch + event via two threads", v);
    }
    bw_ctx* ctx = nullptr;
    if (bw_create(0, &ctx)) return 3;
    std::vector<uint8_t> msg(1 << 16);
    for (size_t i = 0; i < msg.size(); i++) msg[i] = (uint8_t)(i * 2654435761u >> 13);
    for (uint64_t n : sizes) {
        if (n > msg.size()) msg.resize(n, 7);
        std::vector<std::vector<double>> per(T);
        std::atomic<int> fail{0};
        std::vector<std::thread> th;
        auto t0 = clk::now();
        for (int t = 0; t < T; t++)
            th.emplace_back([&, t] {
                uint8_t d[32];
                for (int i = 0; i < calls / T + 50 && !fail; i++) {
                    auto t1 = clk::now();
                    if (int rc = bw_blake3_hash_dropin(ctx, msg.data(), n, d)) fail = rc;
                    if (i >= 50) per[t].push_back(us_since(t1));
                }
            });
        for (auto& x : th) x.join();
        const double el = us_since(t0);
        if (fail) {
            fprintf(stderr, "size %llu: error %d\n", (unsigned long long)n, (int)fail);
            return 4;
        }
        {  // the digest against the batch pipeline's (another path through the library)
            uint8_t d[32], want[32];
            const uint64_t off = 0;
            if (bw_blake3_hash_dropin(ctx, msg.data(), n, d) || bw_blake3_hash_many(ctx, msg.data(), n, &off, &n, 1, want))
                return 5;
            if (memcmp(d, want, 32)) {
                fprintf(stderr, "size %llu: digest differs from bw_blake3_hash_many\n", (unsigned long long)n);
                return 6;
            }
        }
        std::vector<double> v;
        for (auto& p : per) v.insert(v.end(), p.begin(), p.end());
        char what[96];
        snprintf(what, sizeof what, "dropin %llu B, %d thr", (unsigned long long)n, T);
        report(what, v);
        uint64_t nb = 0, nm = 0;
        bw_blake3_coalesce_stats(0, &nb, &nm);
        printf("   %.1f k calls/s; launches so far %llu (%.2f messages each)\n", v.size() / el * 1e3,
               (unsigned long long)nb, (double)nm / std::max<uint64_t>(1, nb));
    }
    // a neighbour: while T threads keep calling, tiny kernels on 8 streams of their own; a stream that
    // shared a hardware queue with a persistent hash kernel would wait for that kernel to end
    {
        std::atomic<bool> run{true};
        std::vector<std::thread> th;
        for (int t = 0; t < T; t++)
            th.emplace_back([&] {
                uint8_t d[32];
                while (run) bw_blake3_hash_dropin(ctx, msg.data(), 4096, d);
            });
        std::vector<hipStream_t> ss(8);
        for (auto& x : ss) hipStreamCreateWithFlags(&x, hipStreamNonBlocking);
        std::vector<double> v;
        for (int i = 0; i < 400; i++) {
            hipStream_t x = ss[i % 8];
            auto t = clk::now();
            k_empty<<<1, 64, 0, x>>>(nullptr);
            hipStreamSynchronize(x);
            v.push_back(us_since(t));
        }
        // the legacy null stream (PyTorch's default stream, a bare hipMemcpy): it waits for every
        // blocking stream, so a persistent kernel on a blocking stream would hold it up to the
        // kernel's exit
        std::vector<double> vn, vm, vd;
        int* dw = nullptr;
        hipMalloc((void**)&dw, 64);
        int hw = 0;
        for (int i = 0; i < 200; i++) {
            auto t = clk::now();
            k_empty<<<1, 64, 0, 0>>>(nullptr);
            hipStreamSynchronize(0);
            vn.push_back(us_since(t));
            t = clk::now();
            hipMemcpy(&hw, dw, 4, hipMemcpyDeviceToHost);
            vm.push_back(us_since(t));
            if (i % 10 == 0) {  // a device-wide synchronization waits for the running instance
                t = clk::now();
                hipDeviceSynchronize();
                vd.push_back(us_since(t));
            }
        }
        run = false;
        for (auto& x : th) x.join();
        report("neighbour stream launch+sync", v);
        printf("   max %.1f us\n", v.back());
        report("null stream launch+sync", vn);
        printf("   max %.1f us\n", vn.back());
        report("null stream hipMemcpy 4 B", vm);
        printf("   max %.1f us\n", vm.back());
        report("hipDeviceSynchronize", vd);
        printf("   max %.1f us\n", vd.back());
        hipFree(dw);
        for (auto& x : ss) hipStreamDestroy(x);
    }
    // the service beside a neighbour that fills the GPU: back-to-back 1 ms kernels of 4,096
    // workgroups on a normal-priority stream; calls after an idle gap (the instance has ended and a
    // new one must be dispatched beside the neighbour's waves) and back to back
    {
        std::atomic<bool> run{true};
        std::thread busy([&] {
            hipSetDevice(0);
            hipStream_t bs;
            hipStreamCreateWithFlags(&bs, hipStreamNonBlocking);
            while (run) {
                for (int k = 0; k < 8; k++) k_busy<<<4096, 256, 0, bs>>>(100000, nullptr);
                hipStreamSynchronize(bs);
            }
            hipStreamDestroy(bs);
        });
        usleep(20000);
        std::vector<double> vg, vb;
        uint8_t d[32];
        for (int i = 0; i < 40; i++) {
            usleep(12000);  // > the 5 ms idle limit: a fresh instance per call
            auto t = clk::now();
            if (bw_blake3_hash_dropin(ctx, msg.data(), 4096, d)) return 7;
            vg.push_back(us_since(t));
        }
        for (int i = 0; i < 2000; i++) {
            auto t = clk::now();
            if (bw_blake3_hash_dropin(ctx, msg.data(), 4096, d)) return 7;
            vb.push_back(us_since(t));
        }
        run = false;
        busy.join();
        report("busy GPU: 4 KiB after idle gap", vg);
        printf("   max %.1f us\n", vg.back());
        report("busy GPU: 4 KiB back to back", vb);
        printf("   max %.1f us\n", vb.back());
    }
    bw_destroy(ctx);
    return 0;
}
