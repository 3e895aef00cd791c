"""One long file split across ranks (backuwup_amd/stream_split.py): the boundary
settlement must give exactly the chunks of chunking the whole file serially
(FastCDC::new(file).collect(), dir_packer.rs:254-266), with the straddling chunks hashed once.

CPU: the settlement over gloo at world size 2 and 4 with the oracle's chunker standing in for the
device (test infrastructure), on random data (resync within the halo), zeros (no content-defined
cut: every rank's speculative chain is out of phase, so the entries settle rank by rank), a
periodic pattern, and files so small that ranks own less than one chunk.  GPU: the same with
device_chunk_fn (bw_process_files_device over each rank's window in HBM), ranks driven from one
process, digests checked against the oracle."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from backuwup_amd import stream_split as ss
from backuwup_amd.synth import splitmix_bytes

SMALL = (256, 1024, 4096)  # min, avg, max: many chunks per rank in small files


def make_file(kind, n):
    if kind == "random":
        return splitmix_bytes(91, n)
    if kind == "zeros":
        return np.zeros(n, dtype=np.uint8)
    if kind == "periodic":
        return np.resize(splitmix_bytes(5, 1500), n)
    raise ValueError(kind)


def oracle_chunk_fn(data, params):
    from oracle import oracle

    def fn(start, end):
        ch = oracle.fastcdc(data[start:end], *params)
        return np.array([start + o + l for _, o, l in ch], dtype=np.int64), None

    return fn


CASES = [("random", 300000, SMALL), ("zeros", 300000, SMALL), ("periodic", 200000, SMALL),
         ("random", 9000, SMALL), ("random", 40 << 20, (262144, 1048576, 3145728))]


def worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def allgather(x):
        out = [None] * world
        dist.all_gather_object(out, x)
        return out

    got = []
    for kind, n, params in CASES:
        data = make_file(kind, n)
        r = ss.SplitResolver(oracle_chunk_fn(data, params), n, rank, world, params[2])
        ss.settle(r, allgather)
        first, count, starts, lens = r.emitted()
        got.append((starts.tolist(), lens.tolist(), r.rounds, r.rechunks))
    q.put((rank, got))
    dist.destroy_process_group()


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 4])
def test_split_settlement_matches_serial_chunking(world, oracle):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for c, (kind, n, params) in enumerate(CASES):
        want = oracle.fastcdc(make_file(kind, n), *params)
        starts = sum((got[r][c][0] for r in range(world)), [])
        lens = sum((got[r][c][1] for r in range(world)), [])
        assert starts == [o for _, o, _ in want] and lens == [l for _, _, l in want], (kind, n, world)
        rounds = [got[r][c][2] for r in range(world)]
        if kind == "zeros":
            # no resync is possible: the true phase travels one rank per round
            assert max(rounds) >= world - 1
        if kind == "random" and n > 100000:
            assert max(rounds) == 1  # every speculative chain resynchronised inside its halo


def test_windows_cover_every_chunk_they_keep():
    for n in (1, 4095, 4096, 4097, 10 ** 6):
        for world in (1, 2, 3, 8):
            s = ss.split_bounds(n, world)
            assert s[0] == 0 and s[-1] == n
            for r in range(world):
                lo, hi = ss.window(n, r, world, 4096)
                assert lo <= max(0, s[r] - 4096) and hi >= min(n, s[r + 1] + 4096)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,n,world", [("random", 64 << 20, 4), ("zeros", 40 << 20, 3), ("random", 5 << 20, 8)])
def test_split_on_device_matches_serial(ctx, oracle, kind, n, world):
    import torch
    from backuwup_amd import make_params
    data = make_file(kind, n)
    params = make_params()
    wins = []
    for r in range(world):
        lo, hi = ss.window(n, r, world, params.max_size)
        wins.append((lo, torch.from_numpy(data[lo:hi].copy()).cuda()))  # each rank's HBM window
    torch.cuda.synchronize()
    rs = [ss.SplitResolver(ss.device_chunk_fn(ctx, w.data_ptr(), lo, params), n, r, world, params.max_size)
          for r, (lo, w) in enumerate(wins)]
    ss.settle(rs)
    want = oracle.fastcdc(data, 262144, 1048576, 3145728)
    got = []
    for r in rs:
        first, count, starts, lens = r.emitted()
        blobs = r.payload[first:first + count]
        assert (r.start + blobs["offset"].astype(np.int64) == starts).all()
        for s, l, d in zip(starts, lens, blobs["digest"]):
            got.append((int(s), int(l), bytes(d)))
    assert [(s, l) for s, l, _ in got] == [(o, l) for _, o, l in want]
    for s, l, d in got[:: max(1, len(got) // 12)]:
        assert d == oracle.blake3(data[s:s + l])


# ------------------------------------------------------------------ bw_chunk_stream_shard (C ABI)
# the settlement behind the C ABI, over a communicator (the caller's host transport
# here: two processes share the one GPU, which RCCL refuses), followed by bw_exchange_dedup of the
# emitted range.  Every rank's emitted chunks, in rank order, equal the serial oracle's chunks of the
# whole file (boundaries, Chunk.hash, digests), and the verdicts equal one global index.
BK = (262144, 1048576, 3145728)
SHARD_CASES = [("random", 24 << 20, BK), ("zeros", 14 << 20, BK), ("periodic", 9 << 20, BK),
               ("random", 300 << 10, BK),  # shorter than one chunk per rank
               ("random", 300000, SMALL), ("zeros", 200000, SMALL), ("random", 0, BK)]


def _shard_worker(rank, world, port, q):
    import torch
    from backuwup_amd import Context, make_params
    from backuwup_amd.comm import Comm, gloo_all_to_all
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = []
        with Context(0) as c, Comm.host(0, rank, world, gloo_all_to_all()) as comm:
            c.index_reset(1 << 14)
            for kind, n, params in SHARD_CASES:
                data = make_file(kind, n)
                lo, hi = ss.window(n, rank, world, params[2])
                win = torch.from_numpy(data[lo:hi].copy()).cuda() if hi > lo else None
                torch.cuda.synchronize()
                p = make_params(*params)
                sh = c.chunk_stream_shard(comm, win.data_ptr() + 0 if win is not None else 0, n, p)
                if sh["ticket"]:
                    c.exchange_dedup(comm, sh["ticket"])
                    res = c.wait(sh["ticket"])
                    mine = res[sh["first_blob"]:sh["first_blob"] + sh["n_blobs"]]
                    out.append([(int(sh["chain_start"] + b["offset"]), int(b["length"]), int(b["gear_hash"]),
                                 bytes(b["digest"]), int(b["is_dup"])) for b in mine] + [("rounds", sh["rounds"])])
                else:
                    out.append([("rounds", sh["rounds"])])
            c.index_check()
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_stream_shard_c_abi_two_ranks_one_gpu(world, oracle):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_shard_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ix = oracle.Index()  # one backup session: the files in order, each in offset order
    for c, (kind, n, params) in enumerate(SHARD_CASES):
        data = make_file(kind, n)
        chunks = [b for r in range(world) for b in got[r][c] if b[0] != "rounds"]
        rounds = max(dict([b for b in got[r][c] if b[0] == "rounds"])["rounds"] for r in range(world))
        if n == 0:
            assert chunks == []
            continue
        want = oracle.process_files(data, [0], [n], *params, small_threshold=0, index=ix)
        assert [(s, l) for s, l, _, _, _ in chunks] == [(int(o), int(l)) for o, l in zip(want["offset"], want["length"])], (kind, n)
        assert [g for _, _, g, _, _ in chunks] == [int(x) for x in want["gear_hash"]], (kind, n)
        assert [d for _, _, _, d, _ in chunks] == [bytes(x) for x in want["digest"]], (kind, n)
        assert [v for _, _, _, _, v in chunks] == [int(x) for x in want["is_dup"]], (kind, n)
        if kind == "random" and n > (1 << 20):
            assert rounds == 1
        if kind == "zeros":
            assert rounds >= 2  # the true phase travels from rank 0


@pytest.mark.gpu
def test_stream_shard_c_abi_rccl_world1(ctx, oracle):
    """World size 1 over RCCL: the settlement is one round, the emitted chunks are the whole file."""
    import torch
    from backuwup_amd import make_params
    from backuwup_amd.comm import Comm, unique_id
    data = make_file("random", 7 << 20)
    win = torch.from_numpy(data).cuda()
    torch.cuda.synchronize()
    with Comm.rccl(0, 0, 1, unique_id()) as comm:
        ctx.index_reset(1 << 12)
        from backuwup_amd._lib import BW_EINVAL, BwError
        with pytest.raises(BwError) as e:  # min > max: refused (the windows rest on chunks <= max)
            ctx.chunk_stream_shard(comm, win.data_ptr(), data.size, make_params(8192, 2048, 4096))
        assert e.value.rc == BW_EINVAL
        sh = ctx.chunk_stream_shard(comm, win.data_ptr(), data.size, make_params())
        ctx.exchange_dedup(comm, sh["ticket"])
        res = ctx.wait(sh["ticket"])
    want = oracle.process_files(data, [0], [data.size], small_threshold=0)
    assert sh["rounds"] == 1 and sh["first_blob"] == 0 and sh["n_blobs"] == len(want) == len(res)
    assert np.array_equal(res["offset"], want["offset"]) and np.array_equal(res["digest"], want["digest"])


def rand_file(seed, kind, n):
    """Content for the random shard cases: random, zeros, a short period, two-symbol bytes."""
    if kind == "random":
        return splitmix_bytes(seed, n)
    if kind == "zeros":
        return np.zeros(n, dtype=np.uint8)
    if kind == "period":
        return np.resize(splitmix_bytes(seed, 1 + seed % 5000), n)
    return (splitmix_bytes(seed, n) & 1).astype(np.uint8)


def random_shard_cases(seed, k):
    """k random (kind, n, params, seed) cases: min <= max and avg <= max (the shard's domain), files
    from empty to 24 MiB (most of them several max long), parameters log-uniform in the crate's
    ranges."""
    rng = np.random.default_rng(seed)
    lu = lambda lo, hi: int(np.exp(rng.uniform(np.log(lo), np.log(hi + 1))))  # noqa: E731
    out = []
    for i in range(k):
        mx = min(lu(1024, 4 << 20), 16 << 20)
        mn = min(lu(64, 1 << 20), mx)
        av = min(lu(256, 4 << 20), mx)
        r = rng.random()
        n = 0 if r < 0.08 else int(rng.integers(mx, 8 * mx + 2)) if r < 0.6 else lu(1, 12 << 20)
        n = min(n, 24 << 20)
        out.append((["random", "zeros", "period", "two"][i % 4], n, (mn, av, mx), seed * 100 + i))
    return out


def _rand_shard_worker(rank, world, port, q, cases):
    import torch
    from backuwup_amd import Context, make_params
    from backuwup_amd.comm import Comm, gloo_all_to_all
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = []
        with Context(0) as c, Comm.host(0, rank, world, gloo_all_to_all()) as comm:
            c.index_reset(1 << 14)
            for kind, n, params, seed in cases:
                data = rand_file(seed, kind, n)
                lo, hi = ss.window(n, rank, world, params[2])
                win = torch.from_numpy(data[lo:hi].copy()).cuda() if hi > lo else None
                torch.cuda.synchronize()
                sh = c.chunk_stream_shard(comm, win.data_ptr() if win is not None else 0, n, make_params(*params))
                if sh["ticket"]:
                    c.exchange_dedup(comm, sh["ticket"])
                    res = c.wait(sh["ticket"])
                    mine = res[sh["first_blob"]:sh["first_blob"] + sh["n_blobs"]]
                    out.append([(int(sh["chain_start"] + b["offset"]), int(b["length"]), int(b["gear_hash"]),
                                 bytes(b["digest"]), int(b["is_dup"])) for b in mine])
                else:
                    out.append([])
            c.index_check()
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4, 8])
def test_stream_shard_c_abi_random(world, oracle):
    """bw_chunk_stream_shard at random parameters, sizes and contents (round 6 fuzz), `world`
    processes sharing the one GPU over the host transport, one backup session across the files:
    every chunk, Chunk.hash, digest and verdict equal to serial chunking and one oracle.Index."""
    # (BW_SHARD_RANDOM_CASES / BW_SHARD_RANDOM_SEED widen it into a soak)
    cases = random_shard_cases(int(os.environ.get("BW_SHARD_RANDOM_SEED", 23000)) + world,
                               int(os.environ.get("BW_SHARD_RANDOM_CASES", 6)))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_rand_shard_worker, args=(r, world, port, q, cases)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=max(300, 3 * len(cases))) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ix = oracle.Index()
    for c, (kind, n, params, seed) in enumerate(cases):
        chunks = [b for r in range(world) for b in got[r][c]]
        if n == 0:
            assert chunks == []
            continue
        data = rand_file(seed, kind, n)
        want = oracle.process_files(data, [0], [n], *params, small_threshold=0, index=ix)
        assert [(s, l) for s, l, _, _, _ in chunks] == [(int(o), int(l)) for o, l in zip(want["offset"], want["length"])], \
            (kind, n, params)
        assert [g for _, _, g, _, _ in chunks] == [int(x) for x in want["gear_hash"]], (kind, n, params)
        assert [d for _, _, _, d, _ in chunks] == [bytes(x) for x in want["digest"]], (kind, n, params)
        assert [v for _, _, _, _, v in chunks] == [int(x) for x in want["is_dup"]], (kind, n, params)
