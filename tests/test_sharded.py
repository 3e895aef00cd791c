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

from backuwup_amd.sharded import exchange_dedup, owner_of, session_capacity


class CpuShardOps:
    """Test stand-in: numpy buckets / a Python set as this rank's index shard.  A batch is
    (n, digests tensor, is_dup tensor, max_n), mirroring Context.batch_views."""

    def __init__(self):
        self.shard = set()

    def partition(self, batch, cap, world):
        n, digests, _, _ = batch
        d = digests.numpy().reshape(-1, 32)[:n]
        owners = np.array([owner_of(int(x[0]), world) for x in d], dtype=np.int64)
        buckets = np.zeros((world, cap, 32), dtype=np.uint8)
        perm = np.zeros((world, cap), dtype=np.int64)
        counts = np.zeros(world, dtype=np.int64)
        for i, o in enumerate(owners):  # stable: canonical order inside each bucket
            buckets[o, counts[o]] = d[i]
            perm[o, counts[o]] = i
            counts[o] += 1
        return torch.from_numpy(buckets.reshape(-1)), torch.from_numpy(perm.reshape(-1)), torch.from_numpy(counts)

    def decide(self, recv, recv_counts, world, cap):
        b = recv.numpy().reshape(world, cap, 32)
        v = np.zeros((world, cap), dtype=np.uint8)
        for s in range(world):  # source-major = canonical
            for i in range(int(recv_counts[s])):
                k = b[s, i].tobytes()
                v[s, i] = k in self.shard
                self.shard.add(k)
        return torch.from_numpy(v.reshape(-1))

    def scatter(self, back, perm, counts, world, cap, batch):
        is_dup = batch[2]
        b, p = back.numpy().reshape(world, cap), perm.numpy().reshape(world, cap)
        for o in range(world):
            for i in range(int(counts[o])):
                is_dup[int(p[o, i])] = int(b[o, i])


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
        cap = session_capacity(100 + 37 * (world - 1) + 2, "cpu")
        exchange_dedup(ops, (n, torch.from_numpy(d.reshape(-1).copy()), is_dup, n), world, cap)
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


# ------------------------------------------------------------------ ranks as threads of one process
# backuwup_amd/session.py (NodeSession) drives N ranks from N threads of ONE process.
# The same sequence on the CPU: rank-major shards of one batch, the oracle as each rank's chunk +
# hash stand-in, the exchange of sharded.py over an in-process all-to-all between the threads.

class ThreadAllToAll:
    """all_to_all_single between the threads of one process (the role of bw_comm_init_local)."""

    def __init__(self, n):
        import threading
        self.n, self.bar, self.slots = n, threading.Barrier(n, timeout=60), [None] * n

    def __call__(self, out, inp, rank):
        self.slots[rank] = inp
        self.bar.wait()
        k = inp.numel() // self.n
        for p in range(self.n):
            out[p * k:(p + 1) * k] = self.slots[p][rank * k:(rank + 1) * k]
        self.bar.wait()


def test_shard_rank_major_contiguous_and_balanced():
    from backuwup_amd.session import shard_rank_major
    for n in (1, 2, 4, 8):
        for fl in ([], [5], [0, 0, 0], [1 << 20] * 10, list(np.random.default_rng(n).integers(0, 1 << 16, 333))):
            r = shard_rank_major(fl, n)
            assert len(r) == n and r[0][0] == 0 and r[-1][1] == len(fl)
            assert all(r[k][1] == r[k + 1][0] and r[k][0] <= r[k][1] for k in range(n - 1))
    r = shard_rank_major([1 << 20] * 16, 4)
    assert [b - a for a, b in r] == [4, 4, 4, 4]


@pytest.mark.parametrize("world", [2, 4])
def test_node_session_threads_match_one_index(world, oracle):
    import threading
    from backuwup_amd.session import shard_rank_major
    from backuwup_amd.synth import small_files
    data, offs, lens = small_files(900, seed=58)
    batches = [(0, 300), (300, 302), (0, 300), (200, 900)]  # a batch of 2 files: ranks without files
    a2a = ThreadAllToAll(world)
    shards = [CpuShardOps() for _ in range(world)]
    got = [[None] * world for _ in batches]

    def rank(r):
        for b, (blo, bhi) in enumerate(batches):
            lo, hi = shard_rank_major(lens[blo:bhi], world)[r]
            lo, hi = blo + lo, blo + hi
            res = oracle.process_files(data, offs[lo:hi], lens[lo:hi]) if hi > lo else None
            d = res["digest"] if res is not None else np.zeros((0, 32), np.uint8)
            n = len(d)
            is_dup = torch.zeros(max(n, 1), dtype=torch.uint8)
            cap = 900  # the session's largest batch bound
            exchange_dedup(shards[r], (n, torch.from_numpy(d.reshape(-1).copy()), is_dup, n), world, cap,
                           group=r, all_to_all=a2a)
            got[b][r] = is_dup.numpy()[:n].tolist()

    th = [threading.Thread(target=rank, args=(r,)) for r in range(world)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=120)
    ix = oracle.Index()
    for b, (blo, bhi) in enumerate(batches):
        want = oracle.process_files(data, offs[blo:bhi], lens[blo:bhi], index=ix)["is_dup"].tolist()
        assert sum(got[b], []) == want, b
