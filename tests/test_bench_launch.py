"""bench.py's multi-GPU launch contract without a GPU, and the host transport of the C exchange.

  * `bench.py --gpus 2` started without a torchrun environment launches 2 ranks itself (one
    process per GPU), which rendezvous and report n_gpus = 2 (dry run: gloo, a CPU stand-in step);
  * a WORLD_SIZE that contradicts --gpus is refused (no 1-GPU line passed off as N GPUs);
  * backuwup_amd.comm.gloo_all_to_all, the host all-to-all handed to bw_comm_init_host in the
    multi-process GPU tests, delivers send[r] of every rank to rank r (world 2 and 4, gloo).
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                           "MASTER_PORT")}
    env.update(kw)
    return env


@pytest.mark.parametrize("n", [2, 4])
def test_bench_gpus_n_launches_n_ranks(n):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--dry-run", "--no-power",
                          "--steps", "2", "--warmup", "1"], env=_env(), capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout  # rank 0 prints the one line
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == n and rec["dry_run"] is True and rec["value"] is None
    assert rec["config"]["parallelism"] == "dp%d" % n


def test_bench_rank_failure_exits_nonzero():
    """one rank of `bench.py --gpus 2` dies after warmup while its peer waits in the
    timing barrier; the launcher tears the survivor down and exits non-zero (no hang, no line)."""
    import time
    t0 = time.time()
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run", "--no-power",
                          "--steps", "2", "--warmup", "1", "--dry-run-fail-rank", "1"], env=_env(),
                         capture_output=True, text=True, timeout=240)
    assert out.returncode != 0, out.stderr[-3000:]
    assert not [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert time.time() - t0 < 200


def test_bench_refuses_world_mismatch():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run", "--no-power"],
                         env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True,
                         timeout=120)
    assert out.returncode != 0
    assert "refusing" in out.stderr


def _a2a_worker(rank, world, port, q):
    import torch.distributed as dist
    from backuwup_amd.comm import gloo_all_to_all
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        b = 40
        send = np.zeros(world * b, dtype=np.uint8)
        for r in range(world):
            send[r * b:(r + 1) * b] = (rank * 16 + r) + np.arange(b, dtype=np.uint8)
        recv = np.zeros_like(send)
        gloo_all_to_all()(send, recv, b)
        q.put((rank, recv.tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_host_all_to_all(world):
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_a2a_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    b = 40
    for r in range(world):
        recv = np.array(got[r], dtype=np.uint8)
        for src in range(world):
            assert recv[src * b:(src + 1) * b].tolist() == ((src * 16 + r) + np.arange(b, dtype=np.uint8)).tolist()
