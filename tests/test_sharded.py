"""World-size-2 (and 4) gloo run of the multi-GPU dedup exchange (backuwup_amd/sharded.py).

The collective sequence is the product code; the three local steps run through a CPU stand-in
(this file only) so the exchange logic is covered without a GPU.  The GPU implementation of
those steps is covered by the -m gpu tests."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from backuwup_amd.sharded import exchange_dedup, owner_of


class CpuShardOps:
    """Test stand-in: numpy partition / a Python set as this rank's index shard."""

    def __init__(self):
        self.shard = set()

    def partition(self, digests, n, world):
        d = digests.numpy().reshape(-1, 32)[:n]
        owners = np.array([owner_of(int(x[0]), world) for x in d], dtype=np.int64)
        perm = np.argsort(owners, kind="stable")
        counts = [int((owners == o).sum()) for o in range(world)]
        out = torch.from_numpy(np.ascontiguousarray(d[perm]).reshape(-1).copy())
        return out, torch.from_numpy(perm.astype(np.int64)), counts

    def decide(self, recv, n):
        d = recv.numpy().reshape(-1, 32)[:n]
        v = np.zeros(max(n, 1), dtype=np.uint8)
        for i, x in enumerate(d):
            k = x.tobytes()
            v[i] = k in self.shard
            self.shard.add(k)
        return torch.from_numpy(v)

    def scatter(self, back, perm, n, is_dup):
        is_dup[perm[:n]] = back[:n]


def make_digests(rank, batch, n):
    rng = np.random.default_rng(1000 * batch + rank)
    pool = np.random.default_rng(7).integers(0, 256, (300, 32), dtype=np.uint8)  # shared pool: cross-rank dups
    return pool[rng.integers(0, 300, n)]


def worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ops = CpuShardOps()
    results = []
    for batch in range(3):
        n = 100 + 37 * rank + batch
        d = make_digests(rank, batch, n)
        is_dup = torch.zeros(n, dtype=torch.uint8)
        exchange_dedup(ops, torch.from_numpy(d.reshape(-1).copy()), n, is_dup, world, "cpu")
        results.append(is_dup.numpy().tolist())
    q.put((rank, results))
    dist.destroy_process_group()


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 4])
def test_exchange_matches_single_index(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # canonical order: batch-major, then rank-major, then local position
    seen = set()
    for batch in range(3):
        for r in range(world):
            n = 100 + 37 * r + batch
            want = []
            for x in make_digests(r, batch, n):
                k = x.tobytes()
                want.append(int(k in seen))
                seen.add(k)
            assert got[r][batch] == want, (r, batch)
