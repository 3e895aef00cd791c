"""One process, N ranks: backuwup_amd/session.py NodeSession drives the digest-prefix
exchange from N threads of one process, one context and one communicator per rank
(bw_comm_init_local: an in-process host transport; bw_comm_init_all: RCCL, one device per rank).
On the one GPU of a test box the four ranks share device 0 (the local transport allows it; RCCL
refuses two ranks on one device, so its one-process path runs at world 1 here)."""
import numpy as np
import pytest

from backuwup_amd.synth import small_files, splitmix_bytes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _corpus():
    """Small files plus CDC files (> 1 MiB) between them, 30 % whole-file copies."""
    data, offs, lens = small_files(3000, seed=71)
    big = [splitmix_bytes(710 + k, (1 << 20) + 1 + 777 * k) for k in range(6)]
    parts = [data] + big + [big[0]]
    fo = list(offs) + [0] * 7
    fl = list(lens) + [b.size for b in big] + [big[0].size]
    pos = data.size
    for k, b in enumerate(big + [big[0]]):
        fo[len(offs) + k] = pos
        pos += b.size
    order = np.random.default_rng(72).permutation(len(fl))
    return np.concatenate(parts), np.asarray(fo, np.uint64)[order], np.asarray(fl, np.uint64)[order]


@pytest.mark.parametrize("world", [2, 4, 8])
def test_node_session_local_transport_matches_one_index(gpu, oracle, world):
    from backuwup_amd.session import NodeSession
    data, offs, lens = _corpus()
    n = len(lens)
    batches = [(0, n // 2), (n // 2, n // 2 + 3), (0, n // 2), (n // 3, n)]  # 3 files: ranks without any
    ix = oracle.Index()
    with NodeSession([0] * world, transport="local") as s:
        for lo, hi in batches:
            got = s.process_files(data, offs[lo:hi], lens[lo:hi])
            want = oracle.process_files(data, offs[lo:hi], lens[lo:hi], index=ix, threads=8)
            for f in ("file", "offset", "length", "gear_hash", "is_dup"):
                assert np.array_equal(got[f], want[f]), (lo, hi, f)
            assert np.array_equal(got["digest"], want["digest"]), (lo, hi)
    assert want["is_dup"].sum() > 0


def test_node_session_rccl_one_process(gpu, oracle):
    """bw_comm_init_all: the ranks' RCCL communicators from one call (one thread per rank inside);
    world 1 on a one-GPU box, the 8-GPU node runs one rank per device."""
    import torch
    from backuwup_amd.session import NodeSession
    data, offs, lens = _corpus()
    ndev = torch.cuda.device_count()
    world = 1 << (min(ndev, 8).bit_length() - 1)
    ix = oracle.Index()
    with NodeSession(list(range(world)), transport="rccl") as s:
        for lo, hi in [(0, 1000), (0, 1000), (500, len(lens))]:
            got = s.process_files(data, offs[lo:hi], lens[lo:hi])
            want = oracle.process_files(data, offs[lo:hi], lens[lo:hi], index=ix, threads=8)
            assert np.array_equal(got["digest"], want["digest"]) and np.array_equal(got["is_dup"], want["is_dup"])
