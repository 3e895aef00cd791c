"""Per-blob zstd level 3 on the GPU (bw_zstd_compress_device) over the CDC
blobs of a compressible corpus, next to the system libzstd on the host cores.

  python tools/zstd_bench.py [--gib 1] [--kind text|mixed|random] [--reps 3]

The corpus is generated on the GPU (backuwup_amd.synth.compressible_corpus_torch), chunked by the
library (FastCDC 256K/1M/3M, like process_file), and every chunk is compressed as the packer's
compress_encrypt_blob does (pack.rs:58-64).  A sample of frames is checked byte for byte against
the oracle's restatement and decoded by libzstd.  CPU baseline: libzstd level 3 with the
reference's settings (tests/zstd_ref.py) over a sample of the same blobs, on 1 and 16 threads.
Prints one JSON line."""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=1.0)
    ap.add_argument("--kind", default="text", choices=["text", "mixed", "random"])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cpu-sample-mib", type=int, default=128)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--check", type=int, default=8, help="frames checked against the oracle")
    ap.add_argument("--slots", type=int, default=None, help="BW_OPT_ZSTD_SLOTS (blobs parsed at once)")
    ap.add_argument("--lanes", type=int, default=0,
                    help="also time the stream through ONE context's asynchronous lanes (bw_zstd_submit_device / "
                         "bw_zstd_wait), this many batches in flight (<= BW_ZSTD_LANES), from one host thread")
    ap.add_argument("--inflight", type=int, default=1,
                    help="also time a stream of batches: this many contexts (own stream and table pool), "
                         "one host thread each, compressing the batch back to back")
    args = ap.parse_args()

    import numpy as np
    import torch
    from backuwup_amd import Context, make_params
    from backuwup_amd.synth import compressible_corpus_torch, splitmix_torch
    import zstd_ref

    dev = torch.device("cuda", 0)
    n = int(args.gib * (1 << 30))
    t0 = time.time()
    if args.kind == "random":
        data = splitmix_torch(42, n, dev)
    else:
        data = compressible_corpus_torch(n, dev, args.kind)
    torch.cuda.synchronize()
    print("corpus %s %.2f GiB generated in %.1f s" % (args.kind, n / 2**30, time.time() - t0), file=sys.stderr)

    ctx = Context(0)
    if args.slots:
        from backuwup_amd._lib import BW_OPT_ZSTD_SLOTS
        ctx.set_option(BW_OPT_ZSTD_SLOTS, args.slots)
    t = ctx.submit_device(data.data_ptr(), n, np.array([0], np.uint64), np.array([n], np.uint64), make_params())
    blobs = ctx.wait(t)
    src_off = blobs["offset"].astype(np.uint64)
    lens = blobs["length"].astype(np.uint64)
    cap = np.array([ctx._L.bw_zstd_store_size(int(x)) for x in lens], dtype=np.uint64)
    dst_off = np.concatenate([[0], np.cumsum(cap)[:-1]]).astype(np.uint64)
    dst = torch.empty(int(cap.sum()), dtype=torch.uint8, device=dev)
    fl = ctx.zstd_compress_device(data.data_ptr(), src_off, lens, dst.data_ptr(), dst_off)  # warm-up
    torch.cuda.synchronize()
    times = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        fl = ctx.zstd_compress_device(data.data_ptr(), src_off, lens, dst.data_ptr(), dst_off)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    best = min(times)
    raw = int(lens.sum())
    stream = None
    if args.inflight > 1:
        # The parse is one wave per blob, serial within a blob, so one call lasts as long as its
        # largest blob (3 MiB against a 1.25 MiB mean on text): the chip idles through the tail.
        # Calls on more contexts fill it, as a packer's consecutive batches would.
        ctxs = [ctx] + [Context(0) for _ in range(args.inflight - 1)]
        dsts = [dst] + [torch.empty_like(dst) for _ in range(args.inflight - 1)]
        for c, d in zip(ctxs[1:], dsts[1:]):
            c.zstd_compress_device(data.data_ptr(), src_off, lens, d.data_ptr(), dst_off)  # warm-up
        torch.cuda.synchronize()
        per = max(args.reps, 2)

        def run(i):
            out = []
            for _ in range(per):
                out.append(ctxs[i].zstd_compress_device(data.data_ptr(), src_off, lens, dsts[i].data_ptr(), dst_off))
            return out

        with ThreadPoolExecutor(args.inflight) as ex:
            t0 = time.perf_counter()
            res = list(ex.map(run, range(args.inflight)))
            torch.cuda.synchronize()
            wall = time.perf_counter() - t0
        frames = lambda d: torch.cat([d[int(o):int(o + n)] for o, n in zip(dst_off, fl)])
        same = all(np.array_equal(f, fl) for r in res for f in r) and all(
            torch.equal(frames(d), frames(dst)) for d in dsts[1:])
        stream = {"inflight": args.inflight, "calls": args.inflight * per, "bytes": raw * args.inflight * per,
                  "ms": round(wall * 1e3, 2), "GBps": round(raw * args.inflight * per / wall / 1e9, 2),
                  "frames_equal_across_contexts": bool(same)}
        for c in ctxs[1:]:
            c.close()
    comp = int(fl.sum())

    lanes = None
    if args.lanes:
        from backuwup_amd import _lib
        k = min(args.lanes, _lib.BW_ZSTD_LANES)
        ldst = [dst] + [torch.empty_like(dst) for _ in range(k - 1)]
        for d in ldst:  # warm-up: every lane's tables and scratch allocated
            ctx.zstd_wait(ctx.zstd_submit_device(data.data_ptr(), src_off, lens, d.data_ptr(), dst_off))
        calls = k * max(args.reps, 2)
        torch.cuda.synchronize()
        pending, same = [], True
        t0 = time.perf_counter()
        for i in range(calls):
            if len(pending) == k:
                same &= bool(np.array_equal(ctx.zstd_wait(pending.pop(0)), fl))
            pending.append(ctx.zstd_submit_device(data.data_ptr(), src_off, lens, ldst[i % k].data_ptr(), dst_off))
        for t in pending:
            same &= bool(np.array_equal(ctx.zstd_wait(t), fl))
        wall = time.perf_counter() - t0
        lanes = {"lanes": k, "calls": calls, "bytes": raw * calls, "ms": round(wall * 1e3, 2),
                 "GBps": round(raw * calls / wall / 1e9, 2), "frame_lengths_equal": same}

    from oracle import oracle
    rng = np.random.default_rng(3)
    ok = True
    picks = rng.choice(len(lens), size=min(args.check, len(lens)), replace=False)
    for i in picks:
        blob = data[int(src_off[i]):int(src_off[i] + lens[i])].cpu().numpy().tobytes()
        frame = dst[int(dst_off[i]):int(dst_off[i] + fl[i])].cpu().numpy().tobytes()
        ok = ok and frame == oracle.zstd3_compress(blob) and zstd_ref.decompress(frame) == blob

    # CPU: libzstd level 3 (the reference's compressor is the same C library, zstd-sys) over the
    # first blobs up to the sample size
    k = int(np.searchsorted(np.cumsum(lens), args.cpu_sample_mib << 20)) + 1
    k = min(k, len(lens))
    sample = [data[int(src_off[i]):int(src_off[i] + lens[i])].cpu().numpy().tobytes() for i in range(k)]
    sb = sum(len(s) for s in sample)
    t0 = time.perf_counter()
    for s in sample:
        zstd_ref.compress(s)
    one = time.perf_counter() - t0
    with ThreadPoolExecutor(args.threads) as ex:
        list(ex.map(zstd_ref.compress, sample[:args.threads]))
        t0 = time.perf_counter()
        list(ex.map(zstd_ref.compress, sample))
        many = time.perf_counter() - t0
    line = {"what": "per-blob zstd level 3 (pack.rs:58-64) on the GPU", "corpus": args.kind,
            "blobs": int(len(lens)), "raw_bytes": raw, "frame_bytes": comp, "ratio": round(raw / max(comp, 1), 3),
            "ms": round(best * 1e3, 3), "GBps": round(raw / best / 1e9, 2), "reps_ms": [round(x * 1e3, 2) for x in times],
            "bit_exact_sample": bool(ok), "checked": int(len(picks)), "stream": stream, "lanes": lanes,
            "cpu_libzstd": {"version": zstd_ref.lib().ZSTD_versionNumber(), "sample_bytes": sb, "blobs": k,
                            "one_thread_GBps": round(sb / one / 1e9, 3),
                            "threads": args.threads, "all_threads_GBps": round(sb / many / 1e9, 3)}}
    print(json.dumps(line), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
