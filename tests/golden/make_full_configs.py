#!/usr/bin/env python3
"""Whole-result fixtures of the full-size BASELINE.json configurations, computed by the CPU oracle.

Test infrastructure (build container only; the GPU box reads the JSON it writes).  For each
configuration the oracle (oracle/bw_oracle.c: fastcdc 3.0.3 v2020 `cut`, blake3 1.3.3 `hash`, the
dedup gate of blob_index.rs:130-148 in canonical order) produces every blob of the batch, and the
fixture records the blob count, the duplicate count / bytes and sha256 over the canonical records
`(file, offset, length, gear_hash, digest, is_dup)` (backuwup_amd/synth.py CANON_DTYPE).  The GPU
tests (tests/test_gpu_full_configs.py) and bench.py's parity check hash the HIP path's whole result
the same way and compare.

  c2  the 16 GiB splitmix64 stream, seed 42 (bench.py's default line, rank 0), one file: chunked in
      windows that always restart at a true cut (a cut depends on at most `max` bytes after its
      chunk's start), every chunk hashed, one fresh index
  c3  the VM-image family of bench.py --workload c3 (rank 0): a 4 GiB base (seed 1) + 15 variants
      with 32 byte indels and 16 x 4 KiB overwrites each = 64 GiB, 16 files, one index across them
  c4  1,000,000 small files of 4-64 KiB with 30 % whole-file copies (seed 3; copies alias their
      source's bytes, synth.small_files_table), one blob per file (dir_packer.rs:246), one index

  c1  bench.py --workload c1 (rank 0): the 1 GiB directory tree (log-uniform sizes, 30 % copies)
  c5  bench.py --workload c5 (rank 0): C3's family, files 0-7 (32 GiB), as rank 0 holds them
  edge  synth.edge_corpus: the content and size edges (no candidates, dense candidates, periodic,
      compressible text, threshold sizes, cross-file duplicates), 1.4 GB

Usage: python tests/golden/make_full_configs.py [c1] [c2] [c3] [c4] [c5]   (all by default; ~10 min)
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from backuwup_amd import synth  # noqa: E402
from oracle import oracle  # noqa: E402

BK = (262144, 1048576, 3145728)
OUT = os.path.dirname(os.path.abspath(__file__))


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def c2(seed=42, n=16 << 30, window=512 << 20):
    ix = oracle.Index()
    rd = synth.ResultDigest()
    pos, t0 = 0, time.time()
    while pos < n:
        end = min(n, pos + window)
        win = synth.splitmix_bytes(seed, end - pos, offset=pos)
        chunks = oracle.fastcdc(win, *BK)
        rows, nxt = [], end
        for h, o, ln in chunks:
            if end < n and o + BK[2] > len(win):  # its cut may depend on bytes past the window
                nxt = pos + o
                break
            d = oracle.blake3_fast(win[o:o + ln])
            dup = ix.is_blob_duplicate(d)
            if not dup:
                ix.insert(d)
            rows.append((0, pos + o, ln, h, np.frombuffer(d, np.uint8), int(dup)))
        blobs = np.zeros(len(rows), dtype=synth.CANON_DTYPE)
        for i, r in enumerate(rows):
            blobs[i] = r
        rd.update(blobs)
        pos = nxt
        log("c2: %.1f / %.1f GiB, %d blobs, %.0f s" % (pos / 2**30, n / 2**30, rd.n, time.time() - t0))
    return rd.summary()


def c3(seed=1, base_bytes=4 << 30, n_images=16):
    ix = oracle.Index()
    rd = synth.ResultDigest()
    base = synth.splitmix_bytes(seed, base_bytes)
    t0 = time.time()
    for v in range(n_images):
        if v == 0:
            img = base
        else:
            over, parts = synth._variant_plan(base_bytes, v, seed, 32, 16, 64)
            tmp = base.copy()
            for at, b in over:
                tmp[at:at + b.size] = b[:tmp.size - at]
            img = np.concatenate([tmp[p[1]:p[2]] if p[0] == "keep" else p[1] for p in parts])
            del tmp
        res = oracle.process_files(img, [0], [img.size], index=ix, threads=1)
        rd.update(res, file_base=v)
        log("c3: image %d (%d B): %d blobs, %.0f s" % (v, img.size, rd.n, time.time() - t0))
        del img, res
    return rd.summary()


def c4(seed=3, n_files=1_000_000, window=1 << 30):
    u, offs, lens = synth.small_files_table(n_files, seed=seed)
    uo, first = np.unique(offs, return_index=True)  # the distinct files, ascending offsets
    ul = lens[first]
    udig = np.zeros((len(uo), 32), dtype=np.uint8)
    t0 = time.time()
    i = 0
    while i < len(uo):
        lo = int(uo[i])
        j = int(np.searchsorted(uo, lo + window, side="left"))
        j = max(j, i + 1)
        hi = int(uo[j - 1] + ul[j - 1])
        win = synth.splitmix_bytes(seed, hi - lo, offset=lo)
        res = oracle.process_files(win, uo[i:j] - np.uint64(lo), ul[i:j], threads=os.cpu_count() or 8)
        assert len(res) == j - i  # every file <= 1 MiB is one blob (dir_packer.rs:246)
        udig[i:j] = res["digest"]
        i = j
        log("c4: %d / %d distinct files hashed, %.0f s" % (i, len(uo), time.time() - t0))
    k = np.searchsorted(uo, offs)
    ix = oracle.Index()
    blobs = np.zeros(n_files, dtype=synth.CANON_DTYPE)
    blobs["file"] = np.arange(n_files, dtype=np.uint64)
    blobs["length"] = lens
    blobs["digest"] = udig[k]
    for f in range(n_files):
        d = bytes(udig[k[f]])
        if ix.is_blob_duplicate(d):
            blobs["is_dup"][f] = 1
        else:
            ix.insert(d)
    log("c4: dedup in canonical order, %.0f s" % (time.time() - t0))
    return synth.result_digest(blobs)


def c1(seed=0x6261636B, total=1 << 30):
    data, offs, lens = synth.tree_corpus(total, seed=seed)
    return synth.result_digest(oracle.process_files(data, offs, lens, threads=os.cpu_count() or 8))


def c5(seed=1, base_bytes=4 << 30):
    # rank 0 of bench.py --workload c5: family 0 (= C3's corpus, seed 1), its files 0-7, one index
    return c3(seed=seed, base_bytes=base_bytes, n_images=8)


def edge():
    data, offs, lens = synth.edge_corpus()
    return synth.result_digest(oracle.process_files(data, offs, lens, threads=os.cpu_count() or 8))


CONFIGS = {
    "edge": (edge, {"workload": "synth.edge_corpus(seed=11): threshold sizes, empty/tiny files, zeros, periodic, "
                                "two-symbol, text and mixed compressible content, zero runs, copies",
                    "seed": 11, "files": 24}),
    "c1": (c1, {"workload": "bench.py --workload c1 rank 0: tree_corpus(1 GiB, seed 0x6261636B), 30 % whole-file "
                            "copies", "seed": 0x6261636B, "total_bytes": 1 << 30}),
    "c5": (c5, {"workload": "bench.py --workload c5 rank 0: VM-image family 0 (vm_image_variants(4 GiB, 16, seed=1)), "
                            "its files 0-7, from pinned host memory", "seed": 1, "base_bytes": 4 << 30, "files": 8}),
    "c2": (c2, {"workload": "bench.py --workload c2 rank 0: splitmix64 seed 42, 16 GiB, one file",
                "seed": 42, "bytes": 16 << 30, "files": 1}),
    "c3": (c3, {"workload": "bench.py --workload c3 rank 0: vm_image_variants(4 GiB, 16, seed=1), 32 indels "
                            "(1-64 B) + 16 x 4 KiB overwrites per variant", "seed": 1, "base_bytes": 4 << 30,
                "files": 16}),
    "c4": (c4, {"workload": "bench.py --workload c4 rank 0: small_files_table(1,000,000, seed=3), file bytes "
                            "splitmix64 seed 3, copies alias their source", "seed": 3, "files": 1_000_000}),
}


def main():
    want = sys.argv[1:] or ["c1", "c2", "c3", "c4", "c5", "edge"]
    oracle.set_blake3_simd(True)
    for name in want:
        fn, meta = CONFIGS[name]
        t0 = time.time()
        summary = fn()
        doc = {"config": name, **meta, "params": {"min": BK[0], "avg": BK[1], "max": BK[2]},
               "index": "one fresh index for the whole batch (canonical order: files in order, chunks by offset)",
               "record": "file u64, offset u64, length u64, gear_hash u64, digest 32 B, is_dup u8 "
                         "(little endian, packed: backuwup_amd/synth.py CANON_DTYPE)",
               "source": "CPU oracle (oracle/bw_oracle.c), tests/golden/make_full_configs.py",
               "oracle_seconds": round(time.time() - t0, 1), **summary}
        path = os.path.join(OUT, "%s_full.json" % name)
        with open(path, "w") as f:
            json.dump(doc, f, indent=1)
            f.write("\n")
        log("%s -> %s: %s" % (name, path, summary))


if __name__ == "__main__":
    main()
