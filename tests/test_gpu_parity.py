"""GPU parity: the HIP path (through the C ABI) against the CPU oracle, bit for bit.

Integer/byte work only, so every comparison is exact.  Inputs are seeded; sizes stay where the
oracle finishes in seconds.  Edge cases follow SURVEY.md §4 item 4: odd tails, lengths at
min/avg/max +-1, all-zero data (every chunk = max), byte-shifted copies, empty inputs.
"""
import ctypes

import numpy as np
import pytest

from backuwup_amd import make_params
from backuwup_amd._lib import BW_F_NO_DEDUP, BW_F_SERIAL_RESOLVE, BW_OPT_B3_GROUP, BwError
from backuwup_amd.synth import splitmix_bytes

pytestmark = pytest.mark.gpu

BK = (262144, 1048576, 3145728)  # backuwup: defaults.rs:61-68
SMALL = (64, 256, 1024)           # tiny sizes: thousands of chunks in a few MiB
MID = (4096, 16384, 65536)


def chunks_oracle(oracle, data, p):
    return oracle.fastcdc(data, *p)


# ------------------------------------------------------------------ BLAKE3

KAT = {
    b"": "af1349b9f5f9a1a6a0404dea36dcc9499bcb25c9adc112b7cc9a93cae41f3262",
    b"abc": "6437b3ac38465133ffb63b75273a8db548c558465d79db03fd359c6cd5bd9d85",
    b"\x00": "2d3adedff11b61f14c886e35afa036736dcd87a74d27b5c1510225d0f592e213",
}


# every BLAKE3 test runs with each shipped leaf-pass grouping: the leaf kernel k_b3_lines (aligned
# 128-byte lines through registers) with 4, 2 or 1 leaves per lane (BW_OPT_B3_GROUP; 0 = the
# automatic choice).  The loaders and the fused upper levels measured slower live in the diagnostic
# build only (BW_DIAG, tools/debug_check.py).
@pytest.fixture(params=[0, 4, 2, 1], ids=["lines", "lines-g4", "lines-g2", "lines-g1"])
def b3ctx(ctx, request):
    ctx.set_option(BW_OPT_B3_GROUP, request.param)
    yield ctx
    ctx.set_option(BW_OPT_B3_GROUP, 0)  # the context default


def test_blake3_kat(b3ctx):
    for msg, hexd in KAT.items():
        assert b3ctx.blake3(msg).hex() == hexd


# the official test-vector lengths (input byte i = i % 251) plus the tree-shape edges
TV_LENS = [0, 1, 63, 64, 65, 127, 128, 1023, 1024, 1025, 2048, 2049, 3072, 3073, 4096, 4097, 5120, 5121,
           6144, 6145, 7168, 7169, 8192, 8193, 16384, 31744, 102400, 12288, 12289, 65536, 65537, 1048575,
           1048576, 1048577, 3145728]


def test_blake3_lengths(b3ctx, oracle):
    ctx = b3ctx
    for n in TV_LENS:
        msg = (np.arange(n) % 251).astype(np.uint8)
        assert ctx.blake3(msg) == oracle.blake3(msg), n


def test_blake3_tree_shapes_batched(b3ctx, oracle):
    ctx = b3ctx
    # every leaf count around the group (4 leaves), lane-per-blob (<= 64 leaves) and wave-per-blob
    # tree paths, ragged and exact, hashed in one batch
    lens = [k * 1024 + d for k in range(1, 140) for d in (-1, 0, 1)]
    data = splitmix_bytes(17, sum(lens) + 64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64) + 3
    got = ctx.blake3_many(data, offs, lens)
    for i, l in enumerate(lens):
        o = int(offs[i])
        assert bytes(got[i]) == oracle.blake3(data[o:o + l]), l


def test_blake3_upper_tree_levels(b3ctx, oracle):
    ctx = b3ctx
    # wave-per-blob upper tree: leaf counts around its global passes (more than 64 level-2 nodes,
    # i.e. > 259 leaves) and the register levels below them, every spine-bit pattern near powers
    # of two, next to lane-per-blob blobs in the same launch
    leaves = [65, 66, 67, 68, 127, 128, 129, 255, 256, 257, 258, 259, 260, 261, 263, 264, 511, 512, 513, 515,
              516, 517, 1000, 1023, 1024, 1025, 2047, 2048, 2049, 3071, 3072, 4095, 4096, 4097, 5000, 8191, 8193]
    lens = [k * 1024 + d for k in leaves for d in (-1, 0, 1)] + [5 * 1024, 64 * 1024 + 7, 9000]
    data = splitmix_bytes(23, sum(lens) + 64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64) + 1
    got = ctx.blake3_many(data, offs, lens)
    for i, l in enumerate(lens):
        o = int(offs[i])
        assert bytes(got[i]) == oracle.blake3(data[o:o + l]), l


def test_blake3_many_unaligned(b3ctx, oracle):
    ctx = b3ctx
    rng = np.random.default_rng(7)
    data = splitmix_bytes(11, 6 << 20)
    n = 400
    lens = rng.integers(0, 70000, n)
    lens[:40] = rng.integers(0, 9000, 40)
    offs = np.array([rng.integers(0, data.size - l) for l in lens], dtype=np.uint64)
    got = ctx.blake3_many(data, offs, lens)
    for i in range(n):
        o, l = int(offs[i]), int(lens[i])
        assert bytes(got[i]) == oracle.blake3(data[o:o + l]), (o, l)


def test_blake3_message_at_buffer_end(b3ctx, oracle):
    ctx = b3ctx
    # last message ends exactly at the caller's buffer end (bounds-safe tail loads)
    for n in [1, 3, 67, 1021, 4099, 70001]:
        data = splitmix_bytes(n, n + 5)
        got = ctx.blake3_many(data, [5], [n])
        assert bytes(got[0]) == oracle.blake3(data[5:]), n


def test_blake3_line_ring_offsets(b3ctx, oracle):
    """k_b3_lines' two paths: whole waves inside one blob at each of the 128 start offsets of a
    128-byte line (the ring, one switch case per offset and block half), and waves across blobs
    (the per-lane fallback).  Blob lengths end at every position of the last block and leaf."""
    ctx = b3ctx
    rng = np.random.default_rng(128)
    lens, offs, pos = [], [], 7
    for o in range(128):
        n = 64 * 4096 + int(rng.integers(0, 70000))  # >= 64 groups: whole waves in the blob
        pos += (o - pos) % 128
        offs.append(pos)
        lens.append(n)
        pos += n + int(rng.integers(1, 300))
    for k in range(200):  # small blobs packed tightly: waves straddle blobs with mixed offsets
        n = int(rng.integers(0, 20000))
        offs.append(pos)
        lens.append(n)
        pos += n + int(rng.integers(0, 5))
    data = splitmix_bytes(129, pos + 16)
    got = ctx.blake3_many(data, np.array(offs, dtype=np.uint64), np.array(lens, dtype=np.uint64))
    for i, (o, l) in enumerate(zip(offs, lens)):
        assert bytes(got[i]) == oracle.blake3(data[o:o + l]), (i, o % 128, l)


# ------------------------------------------------------------------ FastCDC


@pytest.mark.parametrize("p", [SMALL, MID])
def test_fastcdc_random_small_params(ctx, oracle, p):
    for seed, n in [(1, 100_000), (2, 1_000_003), (3, 4_000_001), (4, p[0]), (5, p[0] + 1), (6, p[1] - 1),
                    (7, p[1] + 1), (8, p[2] - 1), (9, p[2]), (10, p[2] + 1), (11, 2 * p[2] + 17), (12, 1)]:
        data = splitmix_bytes(seed, n)
        assert ctx.fastcdc_chunks(data, *p) == chunks_oracle(oracle, data, p), (seed, n)


def test_fastcdc_backuwup_params(ctx, oracle):
    for seed, n in [(0, 8_400_953), (21, 40 << 20), (22, (17 << 20) + 3), (23, BK[2] + 1), (24, BK[0] + 1),
                    (25, BK[1] - 1), (26, BK[1] + 1)]:
        data = splitmix_bytes(seed, n)
        assert ctx.fastcdc_chunks(data, *BK) == chunks_oracle(oracle, data, BK), (seed, n)


def test_fastcdc_a5_vector(ctx):
    data = splitmix_bytes(0, 8_400_953)
    lens = [c[2] for c in ctx.fastcdc_chunks(data, *BK)]
    assert lens == [1560056, 791747, 1444242, 1177622, 806036, 2266142, 355108]


def test_fastcdc_zeros_and_patterns(ctx, oracle):
    cases = [np.zeros((8 << 20) + 5, dtype=np.uint8), np.full(5 << 20, 0xAB, dtype=np.uint8),
             np.tile(np.arange(256, dtype=np.uint8), 20000), np.tile(splitmix_bytes(3, 4096), 1200)]
    for data in cases:
        for p in (BK, SMALL, MID):
            assert ctx.fastcdc_chunks(data, *p) == chunks_oracle(oracle, data, p)
    z = ctx.fastcdc_chunks(np.zeros((8 << 20) + 5, dtype=np.uint8), *BK)
    assert [c[2] for c in z] == [3145728, 3145728, 2097157]


def test_fastcdc_odd_params(ctx, oracle):
    data = splitmix_bytes(44, 3_000_001)
    for p in [(65, 300, 1100), (1001, 4000, 9999), (64, 256, 1024), (4095, 4096, 4097), (8191, 2048, 4096)]:
        assert ctx.fastcdc_chunks(data, *p) == chunks_oracle(oracle, data, p), p


def test_fastcdc_shifted_copies_resync(ctx, oracle):
    base = splitmix_bytes(31, 6 << 20)
    for shift in [1, 7, 63, 4097]:
        data = np.concatenate([splitmix_bytes(32, shift), base])
        assert ctx.fastcdc_chunks(data, *MID) == chunks_oracle(oracle, data, MID)


def test_fastcdc_empty_and_invalid(ctx):
    assert ctx.fastcdc_chunks(b"", *BK) == []
    for bad in [(63, 256, 1024), (64, 255, 1024), (64, 256, 1023), (64, 256, 16777217), (1048577, 4096, 8192),
                (64, 4096, 1024)]:  # avg > max: the crate's cut() reads past max (oracle CratePanic)
        with pytest.raises(BwError):
            ctx.fastcdc_chunks(b"x" * 5000, *bad)


def test_serial_resolve_matches_parallel(ctx, oracle):
    data = splitmix_bytes(77, 12 << 20)
    for p in (SMALL, MID, BK):
        par = make_params(*p, small_file_threshold=0, flags=BW_F_NO_DEDUP)
        ser = make_params(*p, small_file_threshold=0, flags=BW_F_NO_DEDUP | BW_F_SERIAL_RESOLVE)
        a = ctx.process_files(data, [0], [data.size], par)
        b = ctx.process_files(data, [0], [data.size], ser)
        assert np.array_equal(a, b)
        assert [(int(x["gear_hash"]), int(x["offset"]), int(x["length"])) for x in a] == \
            chunks_oracle(oracle, data, p)


# ------------------------------------------------------------------ whole front end


def blobs_equal(a, b):
    assert a.shape == b.shape, (a.shape, b.shape)
    for f in ("file", "offset", "length", "gear_hash", "is_dup"):
        assert np.array_equal(a[f], b[f]), f
    assert np.array_equal(a["digest"], b["digest"])


def test_process_files_mixed(ctx, oracle):
    from backuwup_amd.synth import tree_corpus
    data, offs, lens = tree_corpus(48 << 20, seed=5, max_file=12 << 20)
    lens[3] = 0  # an empty file is one empty blob
    ctx.index_reset()
    got = ctx.process_files(data, offs, lens)
    want = oracle.process_files(data, offs, lens)
    blobs_equal(got, want)
    assert got["is_dup"].sum() > 0


def test_process_files_threshold_edges(ctx, oracle):
    # dir_packer.rs:246: CDC only when file_len > 1 MiB; lengths around that threshold and around
    # the chunker's min / max (a file is chunked from its own start), plus empty files
    mib = 1 << 20
    lens = np.array([0, 1, mib - 1, mib, mib + 1, mib + 2, 262144 + 1, 3145728 - 1, 3145728, 3145728 + 1,
                     2 * 3145728 + 262144, 2 * 3145728 + 262145, 0, mib], dtype=np.uint64)
    data = splitmix_bytes(33, int(lens.sum()) + 64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    data[int(offs[-1]):int(offs[-1] + lens[-1])] = data[int(offs[3]):int(offs[3] + lens[3])]  # copy of file 3
    ctx.index_reset()
    got = ctx.process_files(data, offs, lens)
    want = oracle.process_files(data, offs, lens)
    blobs_equal(got, want)
    per_file = np.bincount(got["file"].astype(np.int64), minlength=len(lens))
    assert list(per_file[:4]) == [1, 1, 1, 1]  # <= 1 MiB: one blob each
    assert bool(got["is_dup"][-1]) and int(got["file"][-1]) == len(lens) - 1


def test_process_files_small_params_many_files(ctx, oracle):
    rng = np.random.default_rng(9)
    lens = rng.integers(0, 300_000, 120).astype(np.uint64)
    data = splitmix_bytes(90, int(lens.sum()) + 100)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    ctx.index_reset()
    got = ctx.process_files(data, offs, lens, make_params(*SMALL))
    want = oracle.process_files(data, offs, lens, *SMALL)
    blobs_equal(got, want)


def test_dedup_seeded_and_cross_batch(ctx, oracle):
    from backuwup_amd.synth import small_files
    data, offs, lens = small_files(3000, seed=4)
    seed_digests = np.array(sorted(oracle.blake3(data[int(offs[i]):int(offs[i] + lens[i])]) for i in range(0, 3000, 7)))
    seed_arr = np.frombuffer(b"".join(seed_digests), dtype=np.uint8).reshape(-1, 32)
    ctx.index_reset()
    ctx.index_seed(seed_arr)
    half = 1500
    got1 = ctx.process_files(data, offs[:half], lens[:half])
    got2 = ctx.process_files(data, offs[half:], lens[half:])
    ix = oracle.Index(b"".join(seed_digests))
    want = oracle.process_files(data, offs, lens, index=ix)
    assert np.array_equal(np.concatenate([got1["is_dup"], got2["is_dup"]]), want["is_dup"])
    assert ctx.index_size() == len(set(bytes(d) for d in want["digest"]) | set(seed_digests))


def test_index_check_insert_random(ctx, oracle):
    rng = np.random.default_rng(3)
    pool = rng.integers(0, 256, (5000, 32), dtype=np.uint8)
    seq = pool[rng.integers(0, 5000, 20000)]
    ctx.index_reset()
    got = ctx.index_check_insert(seq)
    ix = oracle.Index()
    want = []
    for d in seq:
        dup = ix.is_blob_duplicate(d.tobytes())
        if not dup:
            ix.insert(d.tobytes())
        want.append(int(dup))
    assert got.tolist() == want
    assert ctx.index_size() == len({d.tobytes() for d in seq})


def test_index_growth(ctx):
    rng = np.random.default_rng(5)
    ctx.index_reset(16)
    a = rng.integers(0, 256, (200_000, 32), dtype=np.uint8)
    assert ctx.index_check_insert(a).sum() == 0
    assert ctx.index_check_insert(a[::3]).all()
    assert ctx.index_size() == 200_000


def test_device_resident_batch(ctx, oracle):
    import torch
    from backuwup_amd.synth import splitmix_torch
    n = (64 << 20) + 12345
    t = splitmix_torch(123, n, "cuda")
    torch.cuda.synchronize()
    ctx.index_reset()
    ctx.submit_device(t.data_ptr(), n, [0, 1000, 20 << 20], [1000, (20 << 20) - 1000, n - (20 << 20)])
    got = ctx.results()
    host = t.cpu().numpy()
    want = oracle.process_files(host, [0, 1000, 20 << 20], [1000, (20 << 20) - 1000, n - (20 << 20)])
    blobs_equal(got, want)


def test_unmerged_chains_fall_back_exactly(ctx, oracle):
    """Random prefix then zeros: the true chain's max-size phase differs from every speculative
    chain's, so chains never merge and the serial walker must take over -- exactly."""
    for pre, zeros, p in [(5000, 200_000, SMALL), (300_000, 2_000_000, MID), (3 << 20, 40 << 20, BK)]:
        data = np.concatenate([splitmix_bytes(pre, pre), np.zeros(zeros, dtype=np.uint8)])
        assert ctx.fastcdc_chunks(data, *p) == chunks_oracle(oracle, data, p), (pre, zeros)


def test_candidate_dense_input(ctx, oracle):
    """A period whose every window passes the prefilter: tiles overflow their slots and the exact
    rescan + candidate-capacity retry paths run."""
    data = _dense_input()
    assert ctx.fastcdc_chunks(data, *SMALL) == chunks_oracle(oracle, data, SMALL)


def _dense_input():
    from oracle import oracle as o
    g = [int(x) for x in o.gear_table()]
    # find a byte b whose constant window hash -GEAR[b]*(2^64-1)... passes mask_l for SMALL params
    ms, ml = o.masks(*SMALL)
    for b in range(256):
        h = 0
        for _ in range(64):
            h = ((h << 1) + g[b]) & ((1 << 64) - 1)
        if h & ml == 0:
            break
    else:
        pytest.skip("no constant byte passes the mask")
    data = np.full(3 << 20, b, dtype=np.uint8)
    data[:1000] = splitmix_bytes(1, 1000)
    return data


def _dense_input_bk(n=8 << 20):
    """A 64-byte period one of whose windows is an exact MaskL candidate at backuwup's parameters:
    a candidate every 64 bytes, so every scan tile overflows while the parameters keep the rescan
    inside k_tile_partial / k_compact (the sparse-parameter path; SMALL takes the spread k_rescan)."""
    from oracle import oracle as o
    gear = np.array([int(x) for x in o.gear_table()], dtype=np.uint64)
    _, ml = o.masks(*BK)
    rng = np.random.default_rng(2024)
    for _ in range(64):
        pat = rng.integers(0, 256, (4096, 64), dtype=np.uint8)
        g = gear[pat]
        for r in range(64):  # window hash ending at period position r: sum_k GEAR[pat[r - k]] << k
            h = np.zeros(len(pat), dtype=np.uint64)
            for k in range(64):
                h += g[:, (r - k) % 64] << np.uint64(k)
            hit = np.nonzero((h & np.uint64(ml)) == 0)[0]
            if hit.size:
                body = np.tile(pat[hit[0]], n // 64 + 1)[:n]
                body[:1000] = splitmix_bytes(3, 1000)
                return body
    pytest.skip("no periodic MaskL candidate found")


def test_candidate_dense_backuwup_params(ctx, oracle):
    """candidate-dense data at backuwup's own parameters (every tile overflows, exact
    rescans inside the compaction kernels) and at small parameters (the rescans spread over a grid
    of their own): boundaries, Chunk.hash and digests equal the oracle."""
    data = _dense_input_bk()
    assert ctx.fastcdc_chunks(data, *BK) == chunks_oracle(oracle, data, BK)
    offs = np.array([0, 3 << 20, 5 << 20], dtype=np.uint64)
    lens = np.array([3 << 20, 2 << 20, data.size - (5 << 20)], dtype=np.uint64)
    ctx.index_reset()
    blobs_equal(ctx.process_files(data, offs, lens), oracle.process_files(data, offs, lens))
    small = _dense_input()
    assert ctx.fastcdc_chunks(small, *SMALL) == chunks_oracle(oracle, small, SMALL)


@pytest.mark.parametrize("small_bytes", [0, 2**64 - 1])
def test_scan_tile_sizes(oracle, small_bytes):
    """Batches below 4 GiB scan half-size tiles (bw_capi.hip submit): force each tile size
    (BW_OPT_SCAN_SMALL_BYTES) on the same inputs -- ragged ends, the candidate-dense
    overflow/rescan path, many small-parameter files and a multi-file corpus -- and compare with
    the oracle."""
    from backuwup_amd import Context
    from backuwup_amd._lib import BW_OPT_SCAN_SMALL_BYTES
    with Context(0) as ctx:
        ctx.set_option(BW_OPT_SCAN_SMALL_BYTES, small_bytes)
        _scan_tile_sizes(ctx, oracle)


def _scan_tile_sizes(ctx, oracle):
    from backuwup_amd.synth import tree_corpus
    for n, p in [(1, SMALL), (64 * 1024 + 1, SMALL), ((3 << 20) + 12345, MID), ((40 << 20) + 7, BK)]:
        data = splitmix_bytes(n, n)
        assert ctx.fastcdc_chunks(data, *p) == chunks_oracle(oracle, data, p), n
    data = _dense_input()
    assert ctx.fastcdc_chunks(data, *SMALL) == chunks_oracle(oracle, data, SMALL)
    rng = np.random.default_rng(21)
    lens = rng.integers(0, 400_000, 80).astype(np.uint64)
    data = splitmix_bytes(91, int(lens.sum()) + 100)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    ctx.index_reset()
    blobs_equal(ctx.process_files(data, offs, lens, make_params(*SMALL)), oracle.process_files(data, offs, lens, *SMALL))
    data, offs, lens = tree_corpus(40 << 20, seed=12, max_file=9 << 20)
    ctx.index_reset()
    blobs_equal(ctx.process_files(data, offs, lens), oracle.process_files(data, offs, lens))


def test_exchange_dedup_rccl_world1(ctx, oracle):
    """The multi-GPU exchange (partition -> RCCL all-to-all -> owner decides -> all-to-all back ->
    scatter) on one rank equals the inline index."""
    import os
    import socket
    import torch
    import torch.distributed as dist
    from backuwup_amd.sharded import DeviceShardOps, exchange_dedup
    from backuwup_amd.synth import small_files
    owned = not dist.is_initialized()
    if owned:
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        with torch.cuda.stream(torch.cuda.Stream()):
            _exchange_world1(ctx, torch, DeviceShardOps, exchange_dedup, small_files)
    finally:
        if owned:
            dist.destroy_process_group()


def _exchange_world1(ctx, torch, DeviceShardOps, exchange_dedup, small_files):
    data, offs, lens = small_files(4000, seed=8)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    ctx.index_reset()
    want = ctx.process_files(data, offs, lens)
    ctx.index_reset()
    dev = torch.from_numpy(data).cuda()
    torch.cuda.synchronize()
    t = ctx.submit_device(dev.data_ptr(), data.size, offs, lens, make_params(flags=BW_F_NO_DEDUP))
    d_n, d_dig, _, max_n = ctx.batch_views(t)
    is_dup = torch.zeros(max_n, dtype=torch.uint8, device="cuda")
    exchange_dedup(DeviceShardOps(ctx, torch.device("cuda", 0)), (d_n, d_dig, is_dup.data_ptr(), max_n), 1, max_n)
    nb = int(ctx.wait(t).shape[0])
    host = is_dup[:nb].cpu().numpy()
    ctx.set_stream(0)  # back to the context's own stream
    assert np.array_equal(host, want["is_dup"])
    assert host.sum() > 0


# ------------------------------------------------------------------ the reference's per-file call pattern

def test_dropin_call_sites_kept_digests(ctx, oracle):
    """dir_packer.rs:254-266 chunks a file, then :286 hashes each chunk slice of it.
    bw_fastcdc_chunks_hashed chunks and hashes in one submit; bw_blake3_hash_dropin of exactly one of
    its chunk slices returns the kept digest (counted by bw_blake3_kept_hits), anything else is
    hashed on the GPU, the generic bw_blake3_hash never answers from them, and after the
    release nothing is answered from them.  Every digest equals the oracle's, and so do the Python
    drop-ins (fastcdc.FastCDC + blake3.hash on memoryview slices of immutable bytes)."""
    from backuwup_amd import _lib
    from backuwup_amd import blake3 as b3
    from backuwup_amd import fastcdc as fc
    L = _lib.load()
    data = splitmix_bytes(77, (20 << 20) + 333)
    want = oracle.fastcdc(data, *BK)
    chunks, h = ctx.fastcdc_chunks_hashed(data, *BK)
    assert chunks == want and h != 0
    hits0 = L.bw_blake3_kept_hits()
    for _, off, ln in chunks:
        assert ctx.blake3_at(data, off, ln, kept=True) == oracle.blake3(data[off:off + ln])
    assert L.bw_blake3_kept_hits() - hits0 == len(chunks)
    # the generic entry always hashes
    assert ctx.blake3_at(data, chunks[0][1], chunks[0][2]) == oracle.blake3(data[:chunks[0][2]])
    assert L.bw_blake3_kept_hits() - hits0 == len(chunks)
    # not a chunk of it: hashed on the GPU (same pointer, other length; other pointer, same length)
    n0 = chunks[0][2]
    assert ctx.blake3_at(data, 0, n0 - 1, kept=True) == oracle.blake3(data[:n0 - 1])
    assert ctx.blake3_at(data, 1, n0, kept=True) == oracle.blake3(data[1:n0 + 1])
    assert L.bw_blake3_kept_hits() - hits0 == len(chunks)
    ctx.fastcdc_release(h)
    assert ctx.blake3_at(data, 0, n0, kept=True) == oracle.blake3(data[:n0])
    assert L.bw_blake3_kept_hits() - hits0 == len(chunks)
    # the Python drop-ins, written exactly like the reference's loop, over immutable bytes
    mv = memoryview(data.tobytes())
    hits1 = L.bw_blake3_kept_hits()
    chunker = fc.FastCDC(mv, *BK, ctx=ctx)
    got = [b3.hash(mv[c.offset:c.offset + c.length], ctx=ctx) for c in chunker]
    assert got == [oracle.blake3(data[o:o + n]) for _, o, n in want]
    assert L.bw_blake3_kept_hits() - hits1 == len(want)
    del chunker
    # a writable source is chunked without keeping digests, so rewriting it in place
    # while the FastCDC lives gives the new bytes' digest, never the one taken at chunking time
    buf = bytearray(data.tobytes())
    mvw = memoryview(buf)
    hits2 = L.bw_blake3_kept_hits()
    chunker = fc.FastCDC(mvw, *BK, ctx=ctx)
    cuts = [(c.offset, c.length) for c in chunker]
    assert cuts == [(o, n) for _, o, n in want]
    o1, n1 = cuts[1]
    buf[o1:o1 + 64] = bytes(64)  # a reused read buffer: the chunk's bytes change
    assert b3.hash(mvw[o1:o1 + n1], ctx=ctx) == oracle.blake3(bytes(buf[o1:o1 + n1]))
    assert L.bw_blake3_kept_hits() == hits2
    del chunker
    # empty source: no chunks, nothing kept
    assert ctx.fastcdc_chunks_hashed(np.zeros(0, np.uint8), *BK) == ([], 0)


def test_dropin_call_sites_many_threads(oracle):
    """The reference runs process_file as one tokio task per file (dir_packer.rs:166): four threads,
    one context each, chunk + hash their own files through the kept-digest drop-ins at the same
    time (the kept digests are one process-wide registry); every chunk and digest equals the
    oracle's and every per-chunk hash is answered from the kept digests."""
    import threading
    from backuwup_amd import Context, _lib
    L = _lib.load()
    files = [splitmix_bytes(900 + k, (3 << 20) + 7919 * k) for k in range(8)]
    want = [[(o, n, oracle.blake3(f[o:o + n])) for _, o, n in oracle.fastcdc(f, *BK)] for f in files]
    got = [None] * len(files)
    errors = []
    hits0 = L.bw_blake3_kept_hits()

    def worker(t):
        try:
            with Context(0) as c:
                for k in range(t, len(files), 4):
                    chunks, h = c.fastcdc_chunks_hashed(files[k], *BK)
                    got[k] = [(o, n, c.blake3_at(files[k], o, n, kept=True)) for _, o, n in chunks]
                    c.fastcdc_release(h)
        except Exception as e:  # reported below
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=120)
    assert not errors, errors
    assert got == want
    assert L.bw_blake3_kept_hits() - hits0 == sum(len(w) for w in want)


def test_hash_service_instances_and_ring_wrap(oracle):
    """The hash service's persistent instance ends by itself when idle (5 ms) and the next call
    starts another; tickets wrap the 4,096-slot ring many times over; every digest equals the
    oracle's, across instance boundaries and from several threads (bw_b3_small.hip k_b3_service)."""
    import threading
    import time
    from backuwup_amd import Context, _lib
    L = _lib.load()
    rng = np.random.default_rng(9)
    blob = splitmix_bytes(77, 1 << 20)
    b0, m0 = ctypes.c_uint64(), ctypes.c_uint64()
    L.bw_blake3_coalesce_stats(0, ctypes.byref(b0), ctypes.byref(m0))
    with Context(0) as c:
        for rep in range(3):  # idle gaps: each burst finds the last instance ended
            o, n = int(rng.integers(0, 1 << 19)), int(rng.integers(0, 65536))
            assert c.blake3_at(blob, o, n) == oracle.blake3(blob[o:o + n]), (rep, n)
            time.sleep(0.03)
        offs = rng.integers(0, (1 << 20) - 2048, 12000)
        lens = rng.integers(0, 2048, 12000)
        want = [oracle.blake3(blob[o:o + n]) for o, n in zip(offs, lens)]
        got = [None] * len(offs)
        errors = []

        def worker(t):
            try:
                for i in range(t, len(offs), 8):
                    got[i] = c.blake3_at(blob, int(offs[i]), int(lens[i]))
                    if i % 3001 == 0:
                        time.sleep(0.012)  # some instances end mid-run
            except Exception as e:  # reported below
                errors.append(repr(e))

        th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
        for x in th:
            x.start()
        for x in th:
            x.join(timeout=240)
    assert not errors, errors
    assert got == want
    b1, m1 = ctypes.c_uint64(), ctypes.c_uint64()
    L.bw_blake3_coalesce_stats(0, ctypes.byref(b1), ctypes.byref(m1))
    assert m1.value - m0.value == 12003
    assert b1.value - b0.value >= 3  # at least one instance per idle-separated burst


def test_hash_service_leaves_null_stream_free(oracle):
    """While callers keep the hash service's persistent instance running, work on the legacy null
    stream (a bare hipMemcpy, PyTorch's default stream) is not held up until the instance ends: the
    service's stream is a non-blocking one (bw_dropin.hip service(); a CU-masked stream, a blocking
    one, held such calls up to the instance's 500 ms life, profiles/r05/s25_svc_stream)."""
    import threading
    import time
    import torch
    from backuwup_amd import Context
    hip = ctypes.CDLL("libamdhip64.so.7")  # the runtime already loaded (torch's and the library's)
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    blob = splitmix_bytes(78, 1 << 16)
    x = torch.arange(16, dtype=torch.int32, device="cuda:0")
    assert int(torch.ones(4, device="cuda:0").sum()) == 4  # (first-use code loading, before the timing)
    host = (ctypes.c_int32 * 16)()
    stop = threading.Event()
    errors = []
    with Context(0) as c:
        want = oracle.blake3(blob[:4096])

        def caller():
            try:
                while not stop.is_set():
                    if c.blake3_at(blob, 0, 4096) != want:
                        errors.append("digest")
                        return
            except Exception as e:  # reported below
                errors.append(repr(e))

        th = threading.Thread(target=caller)
        th.start()
        try:
            time.sleep(0.05)  # an instance is running
            worst = 0.0
            for _ in range(40):
                t = time.perf_counter()
                assert hip.hipMemcpy(host, ctypes.c_void_p(x.data_ptr()), 64, 2) == 0  # device to host
                assert int(torch.ones(4, device="cuda:0").sum()) == 4  # the default stream
                worst = max(worst, time.perf_counter() - t)
        finally:
            stop.set()
            th.join(timeout=60)
    assert not errors, errors
    assert list(host) == list(range(16))
    assert worst < 0.1, f"a null-stream call waited {worst * 1e3:.1f} ms behind the hash service"


_ALT_PATH = """
import sys, threading
sys.path.insert(0, %r)
import numpy as np
from backuwup_amd import Context
from backuwup_amd.synth import splitmix_bytes
blob = splitmix_bytes(79, 1 << 20)
rng = np.random.default_rng(11)
offs = rng.integers(0, (1 << 20) - 70000, 600)
lens = rng.integers(0, 65537, 600)
lens[:6] = [0, 1, 64, 1024, 65535, 65536]
got = [None] * len(offs)
with Context(0) as c:
    def worker(t):
        for i in range(t, len(offs), 4):
            got[i] = c.blake3_at(blob, int(offs[i]), int(lens[i])).hex()
    th = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    [x.start() for x in th]
    [x.join() for x in th]
print("@@", ",".join("%%d:%%d:%%s" %% (o, n, g) for o, n, g in zip(offs, lens, got)))
"""


@pytest.mark.parametrize("env", [{"BW_SVC_HOST_RING": "1"}, {"BW_DROPIN_SERVICE": "0"}])
def test_small_hash_alternative_paths(oracle, env):
    """The hash service with its requests in pinned host memory (the path of a host without a large
    BAR), and the launched-batch coalescer (BW_DROPIN_SERVICE=0): each in a child process (the
    library reads the choice once per process), 600 messages from 4 threads, equal to the oracle."""
    import os
    import subprocess
    import sys
    from backuwup_amd.synth import splitmix_bytes
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", _ALT_PATH % root], capture_output=True, text=True, timeout=120,
                         env=dict(os.environ, **env))
    line = [l for l in out.stdout.splitlines() if l.startswith("@@ ")]
    assert line, (out.stdout[-2000:], out.stderr[-2000:])
    blob = splitmix_bytes(79, 1 << 20)
    for item in line[0][3:].split(","):
        o, n, g = item.split(":")
        o, n = int(o), int(n)
        assert bytes.fromhex(g) == oracle.blake3(blob[o:o + n]), (env, o, n)


def test_coalesced_hash_many_threads(oracle):
    """the reference calls blake3::hash once per small file and once per tree blob,
    from every tokio worker at once (dir_packer.rs:166, :286, :320).  Sixteen threads hash thousands
    of small messages (0 B - 70 KiB, trees' ~100 B included) through bw_blake3_hash at the same time:
    the library's hash service (one persistent kernel serving every caller) answers them, and every
    digest equals the oracle's."""
    import threading
    from backuwup_amd import Context, _lib
    L = _lib.load()
    rng = np.random.default_rng(5)
    lens = rng.integers(0, 64 << 10, 4000)  # the one-wave-per-message kernel (<= 64 KiB)
    lens[::7] = rng.integers(60, 140, len(lens[::7]))  # tree-blob sized
    lens[::97] = rng.integers(64 << 10, 200 << 10, len(lens[::97]))  # above 64 KiB: through the caller's context
    edges = [0, 1, 63, 64, 65, 1023, 1024, 1025, 2048, 3071, 3072, 4097, 32768, 65535, 65536, 65537]
    lens[:len(edges)] = edges
    blob = splitmix_bytes(31, int(lens.sum()) + 64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]])
    want = [oracle.blake3(blob[o:o + n]) for o, n in zip(offs, lens)]
    got = [None] * len(lens)
    errors = []
    b0, m0 = ctypes.c_uint64(), ctypes.c_uint64()
    L.bw_blake3_coalesce_stats(0, ctypes.byref(b0), ctypes.byref(m0))
    ctxs = [Context(0) for _ in range(4)]  # 16 threads over 4 contexts: small messages only name the device
    for i in range(len(edges)):  # alone: a batch of one message each, either path
        assert ctxs[0].blake3_at(blob, int(offs[i]), int(lens[i])) == want[i], lens[i]

    locks = [threading.Lock() for _ in ctxs]

    def worker(t):
        # a larger message runs on the caller's context, which one thread uses at a time (the Rust
        # shim's pool locks it the same way); a small one takes no context lock
        try:
            for i in range(t, len(lens), 16):
                if lens[i] > 65536:
                    with locks[t % 4]:
                        got[i] = ctxs[t % 4].blake3_at(blob, int(offs[i]), int(lens[i]))
                else:
                    got[i] = ctxs[t % 4].blake3_at(blob, int(offs[i]), int(lens[i]))
        except Exception as e:  # reported below
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=240)
    for c in ctxs:
        c.close()
    assert not errors, errors
    assert got == want
    b1, m1 = ctypes.c_uint64(), ctypes.c_uint64()
    L.bw_blake3_coalesce_stats(0, ctypes.byref(b1), ctypes.byref(m1))
    small = int(np.sum(lens <= 65536)) + sum(1 for e in edges if e <= 65536)  # larger: the caller's context
    assert m1.value - m0.value == small
    assert b1.value - b0.value < len(lens)  # launches: a persistent instance serves many calls
