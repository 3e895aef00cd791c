#!/usr/bin/env python3
"""Run the hot path once through the BW_DEBUG build (libbackuwup_amd_debug.so: device bounds asserts
in walk_next, unit_blobs, k_b3_groups and k_b3_lines) over the inputs that stress those paths, checked against
the oracle.  A failed device assert traps the kernel, so this runs as its own step of the GPU
session (tools/gpu_r2.sh debug), never inside the pytest process."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["BW_LIB"] = os.path.join(ROOT, "backuwup_amd", "libbackuwup_amd_debug.so")

import numpy as np  # noqa: E402

from backuwup_amd import Context, make_params  # noqa: E402
from backuwup_amd._lib import BW_OPT_CAND_CAP, BW_OPT_SCAN_SMALL_BYTES  # noqa: E402
from backuwup_amd.synth import small_files, splitmix_bytes, tree_corpus  # noqa: E402
from oracle import oracle  # noqa: E402

SMALL, MID, BK = (64, 256, 1024), (4096, 16384, 65536), (262144, 1048576, 3145728)


def same(a, b):
    return a.shape == b.shape and all(np.array_equal(a[f], b[f]) for f in ("file", "offset", "length", "gear_hash",
                                                                           "is_dup", "digest"))


def main():
    from backuwup_amd import _lib
    assert _lib.LIB_PATH.endswith("_debug.so")
    checks = 0
    with Context(0) as c:
        for n, p in [((3 << 20) + 11, SMALL), ((40 << 20) + 7, BK), ((9 << 20) + 1, MID)]:
            d = splitmix_bytes(n, n)
            assert c.fastcdc_chunks(d, *p) == oracle.fastcdc(d, *p), n
            checks += 1
        z = np.concatenate([splitmix_bytes(9, 300_000), np.zeros(2_000_000, np.uint8)])
        assert c.fastcdc_chunks(z, *MID) == oracle.fastcdc(z, *MID)
        c.set_option(BW_OPT_CAND_CAP, 100)  # the direct-scan path of walk_next
        d = splitmix_bytes(5, (12 << 20) + 3)
        assert c.fastcdc_chunks(d, *MID) == oracle.fastcdc(d, *MID)
        c.set_option(BW_OPT_CAND_CAP, 0)
        for small_bytes in (0, 2**64 - 1):
            c.set_option(BW_OPT_SCAN_SMALL_BYTES, small_bytes)
            data, offs, lens = tree_corpus(64 << 20, seed=3, max_file=9 << 20)
            c.index_reset()
            assert same(c.process_files(data, offs, lens), oracle.process_files(data, offs, lens, threads=8))
            checks += 1
        # round 3: every BLAKE3 group size, and the upper levels fused into the leaf pass
        from backuwup_amd._lib import BW_OPT_B3_GROUP, BW_OPT_B3_UPPER
        data, offs, lens = tree_corpus(48 << 20, seed=5, max_file=9 << 20)
        want = oracle.process_files(data, offs, lens, threads=8)
        for grp, upper in ((1, 0), (2, 0), (4, 0), (2, 1)):
            c.set_option(BW_OPT_B3_GROUP, grp)
            c.set_option(BW_OPT_B3_UPPER, upper)
            c.index_reset()
            assert same(c.process_files(data, offs, lens), want), (grp, upper)
            checks += 1
        c.set_option(BW_OPT_B3_GROUP, 0)
        c.set_option(BW_OPT_B3_UPPER, 0)
        data, offs, lens = small_files(20000, seed=4)
        c.index_reset()
        assert same(c.process_files(data, offs, lens), oracle.process_files(data, offs, lens, threads=8))
        rng = np.random.default_rng(7)
        lens = rng.integers(0, 200_000, 300).astype(np.uint64)
        data = splitmix_bytes(8, int(lens.sum()) + 9)
        offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
        c.index_reset()
        assert same(c.process_files(data, offs, lens, make_params(*SMALL)),
                    oracle.process_files(data, offs, lens, *SMALL))
        checks += 3
        # round 4: the variants pruned from the product library (BW_DIAG) stay parity-checked here
        from backuwup_amd._lib import (BW_OPT_B3_LOADS, BW_OPT_LATENCY_STREAM, BW_OPT_ORDER_HASH, BW_OPT_SCAN_WAVES,
                                       BW_OPT_SPLIT)
        data, offs, lens = tree_corpus(96 << 20, seed=9, max_file=20 << 20)
        want = oracle.process_files(data, offs, lens, threads=8)
        for opt, v in ((BW_OPT_B3_LOADS, 0), (BW_OPT_B3_LOADS, 1), (BW_OPT_SCAN_WAVES, 8), (BW_OPT_LATENCY_STREAM, 1),
                       (BW_OPT_ORDER_HASH, 1), (BW_OPT_SPLIT, 2)):
            with Context(0) as v_ctx:
                v_ctx.set_option(opt, v)
                v_ctx.index_reset()
                assert same(v_ctx.process_files(data, offs, lens), want), (opt, v)
                checks += 1
    print("BW_DEBUG build: %d parity checks passed, no device assert fired" % checks)


if __name__ == "__main__":
    main()
