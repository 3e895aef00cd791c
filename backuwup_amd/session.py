"""One backup session over every GPU of the node from ONE process.

The reference packs a backup inside one client process (client/src/backup/mod.rs:64): its tokio
tasks feed one packer whose `BlobIndex` decides duplicates (pack.rs:37, blob_index.rs:130-148).
`NodeSession` gives such a process N ranks (one context each, on devices[r]; a device may repeat)
whose dedup index is partitioned by digest prefix (owner = digest[0] >> (8 - log2 N)) and
exchanged through the C ABI (bw_exchange_dedup), exactly as the one-process-per-GPU path does, but
with the ranks as threads of this process and their communicators from bw_comm_init_local (an
in-process host transport: any devices, several ranks per device included) or bw_comm_init_all
(RCCL over xGMI, one device per rank).

A batch of files is sharded rank-major: rank r takes a contiguous run of files (balanced by bytes),
so the canonical order (files in batch order, chunks by offset) is rank order and "first
occurrence" at a digest's owner is the reference's first occurrence.  Each rank chunks + hashes its
files with BW_F_NO_DEDUP and sends its digests to their owners; the verdicts come back into its
results.  The Rust crate's `NodeSession` (rust/backuwup-gpu/src/lib.rs) is the same sequence.
"""
import threading

import numpy as np

from . import _lib
from .comm import Comm
from .context import Context, make_params


def shard_rank_major(file_len, n):
    """[lo_r, hi_r) file ranges, contiguous in order, balanced by bytes (a rank may get none)."""
    fl = np.asarray(file_len, dtype=np.uint64)
    if len(fl) == 0:
        return [(0, 0)] * n
    cum = np.cumsum(fl.astype(np.float64) + 1.0)  # (+1: empty files still count)
    cuts = [0] + [int(np.searchsorted(cum, cum[-1] * r / n, side="right")) for r in range(1, n)] + [len(fl)]
    cuts = [min(max(c, 0), len(fl)) for c in cuts]
    for r in range(1, n + 1):
        cuts[r] = max(cuts[r], cuts[r - 1])
    return [(cuts[r], cuts[r + 1]) for r in range(n)]


class NodeSession:
    def __init__(self, devices, transport="local", index_hint=1 << 16, params=None):
        self.devices = list(devices)
        n = len(self.devices)
        if n < 1 or n & (n - 1):
            raise ValueError("NodeSession: the number of ranks must be a power of two (digest-prefix owners)")
        self.comms = Comm.local(self.devices) if transport == "local" else Comm.all(self.devices)
        self.ctxs = [Context(d) for d in self.devices]  # rank r's private index = its shard of the BlobIndex
        for c in self.ctxs:
            c.index_reset(index_hint)
        p = params or make_params()
        self.params = make_params(min_size=p.min_size, avg_size=p.avg_size, max_size=p.max_size,
                                  flags=p.flags | _lib.BW_F_NO_DEDUP, small_file_threshold=p.small_file_threshold)

    def process_files(self, data, file_off, file_len):
        """The whole batch through every rank -> BLOB_DTYPE results in canonical order (file indices
        of the batch).  Like Context.process_files, with the dedup gate spread over the ranks."""
        data = np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)
        fo = np.ascontiguousarray(file_off, dtype=np.uint64)
        fl = np.ascontiguousarray(file_len, dtype=np.uint64)
        ranges = shard_rank_major(fl, len(self.devices))
        out, errors = [None] * len(ranges), []

        def rank(r):
            lo, hi = ranges[r]
            c, comm = self.ctxs[r], self.comms[r]
            try:
                if hi > lo:
                    a, b = int(fo[lo:hi].min()), int((fo[lo:hi] + fl[lo:hi]).max())
                else:
                    a = b = 0
                t = c.submit_host(data[a:b], fo[lo:hi] - np.uint64(a), fl[lo:hi], self.params)
                c.exchange_dedup(comm, t)
                res = c.wait(t)
                res["file"] += np.uint64(lo)
                out[r] = res
            except Exception as e:  # reported below (a rank that fails breaks the others' exchange)
                errors.append((r, repr(e)))

        th = [threading.Thread(target=rank, args=(r,)) for r in range(len(ranges))]
        for x in th:
            x.start()
        for x in th:
            x.join()
        if errors:
            raise RuntimeError("NodeSession: rank failures %s" % errors)
        return np.concatenate(out)

    def close(self):
        # the communicators first: destroying one finishes any exchange still queued on it, which
        # uses its context
        for m in self.comms:
            m.close()
        for c in self.ctxs:
            c.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()
