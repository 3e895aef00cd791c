"""Experiment: does the byte alignment of blob starts change k_b3_groups' time?

Batches of 1 MiB files (one blob each: files <= 1 MiB are not chunked, dir_packer.rs:246) are
placed at offsets that are 128-byte aligned plus a fixed skew, over 8 GiB of random data already
in HBM.  The BLAKE3 leaf stage's time (HIP events, bw_profile_read) per skew tells whether the
misaligned-line re-fetch (PMC: 1.42x) costs time.  Usage: python tools/b3_align.py [gib]
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from backuwup_amd import Context  # noqa: E402
from backuwup_amd.synth import splitmix_torch  # noqa: E402


def main():
    gib = float(sys.argv[1]) if len(sys.argv) > 1 else 8.0
    n = int(gib * (1 << 30))
    dev = splitmix_torch(7, n + (1 << 20), "cuda:0")
    torch.cuda.synchronize()
    flen = 1 << 20
    stride = flen + 256
    nf = (n - 256) // stride
    out = {}
    with Context(0) as ctx:
        for skew in (0, 4, 16, 64, 100):
            off = np.arange(nf, dtype=np.uint64) * stride + skew
            ln = np.full(nf, flen, dtype=np.uint64)
            runs = []
            for r in range(6):
                ctx.index_reset()
                ctx.profile_enable(True)
                t = ctx.submit_device(dev.data_ptr(), n, off, ln)
                ctx.wait(t)
                ms, nb = ctx.profile_read()
                ctx.profile_enable(False)
                if r:
                    runs.append(ms["b3_leaf"] / max(nb, 1))
            out[skew] = {"b3_leaf_ms": round(float(np.median(runs)), 4),
                         "GBps": round(nf * flen / (np.median(runs) * 1e6), 1)}
            print(skew, out[skew], flush=True)
    print(json.dumps({"files": int(nf), "file_bytes": flen, "by_skew": out}))


if __name__ == "__main__":
    main()
