"""Per-blob zstd level 3 (pack.rs:58-64).

CPU part: the oracle's restatement (oracle/bw_oracle_zstd.c) against the system libzstd
(tests/zstd_ref.py, the reference's Compressor settings) byte for byte, and its level-3
parameters against ZSTD_getCParams.  The image's libzstd is 1.4.8; the reference links 1.5.5
(zstd-sys, Cargo.lock:2760), which is absent: equality with 1.5.5 output is "parity unpinned".
GPU part: bw_zstd_compress(_device) against the oracle on the same corpus, and every frame
decoded by libzstd (the reference reader's Decompressor, unpack.rs:66-68).
"""
import ctypes

import numpy as np
import pytest

import zstd_corpus

SIZES_CPU = [0, 1, 6, 7, 63, 64, 200, 1000, 4096, 16384, 16385, 70000, 131072, 131073,
             262144, 262145, 700000, 2 * 1024 * 1024 + 4096, 3 * 1024 * 1024]


def _zstd():
    import zstd_ref
    if not zstd_ref.available():
        pytest.skip("libzstd not available")
    return zstd_ref


def test_level3_params_match_libzstd(oracle):
    z = _zstd()
    L = z.lib()

    class CP(ctypes.Structure):
        _fields_ = [(f, ctypes.c_uint) for f in
                    ("windowLog", "chainLog", "hashLog", "searchLog", "minMatch", "targetLength", "strategy")]
    L.ZSTD_getCParams.restype = CP
    L.ZSTD_getCParams.argtypes = [ctypes.c_int, ctypes.c_ulonglong, ctypes.c_size_t]
    sizes = set(range(1, 200)) | {(1 << k) + d for k in range(6, 23) for d in (-1, 0, 1)} | {3 << 20}
    for n in sorted(sizes):
        c = L.ZSTD_getCParams(3, n, 0)
        assert c.strategy == 2  # ZSTD_dfast
        assert oracle.zstd3_params(n) == (c.windowLog, c.chainLog, c.hashLog, c.minMatch), n


@pytest.mark.parametrize("kind", zstd_corpus.KINDS)
def test_oracle_equals_libzstd_level3(oracle, kind):
    z = _zstd()
    for i, n in enumerate(SIZES_CPU):
        data = zstd_corpus.blob(kind, n, i)
        frame = oracle.zstd3_compress(data)
        assert frame == z.compress(data), (kind, n)
        assert z.decompress(frame) == data


def test_oracle_random_sizes_equal_libzstd(oracle):
    z = _zstd()
    rng = np.random.default_rng(5)
    for i in range(60):
        kind = zstd_corpus.KINDS[i % len(zstd_corpus.KINDS)]
        n = int(rng.integers(0, 400000)) if i % 3 else int(rng.integers(0, 3000))
        data = zstd_corpus.blob(kind, n, 100 + i)
        assert oracle.zstd3_compress(data) == z.compress(data), (kind, n)


def test_random_data_gives_the_store_frame(oracle):
    """Incompressible blobs: level 3 writes raw blocks, i.e. the store frame the packer's fused
    path emits (oracle/pack_oracle.py zstd_store)."""
    from oracle import pack_oracle as po
    for n in (0, 1, 100, 131072, 131073, 1 << 20, 3 << 20):
        data = zstd_corpus.blob("random", n, n)
        assert oracle.zstd3_compress(data) == po.zstd_store(data)


# ------------------------------------------------------------------ GPU (bw_zstd.hip) vs the oracle
SIZES_GPU = [0, 1, 6, 7, 8, 63, 64, 65, 200, 255, 256, 1000, 1023, 1024, 4096, 16383, 16384, 16385, 70000,
             131071, 131072, 131073, 262144, 262145, 700000, 2 * 1024 * 1024 + 4096, 3 * 1024 * 1024]


def _check_frames(oracle, blobs, frames, z=None):
    for i, (d, f) in enumerate(zip(blobs, frames)):
        want = oracle.zstd3_compress(d)
        assert f == want, (i, len(d), len(f), len(want))
        if z is not None:
            assert z.decompress(f) == bytes(d)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", zstd_corpus.KINDS)
def test_gpu_zstd_equals_oracle(ctx, oracle, kind):
    blobs = [zstd_corpus.blob(kind, n, i) for i, n in enumerate(SIZES_GPU)]
    frames = ctx.zstd_compress(blobs)
    import zstd_ref
    _check_frames(oracle, blobs, frames, zstd_ref if zstd_ref.available() else None)


@pytest.mark.gpu
def test_gpu_zstd_many_mixed_blobs_small_batches(oracle):
    """Hundreds of blobs of every kind in one call, split into internal batches of at most 7 blobs
    / 1 MiB (hash-table slots reused across batches through their index bases)."""
    from backuwup_amd import Context, _lib
    rng = np.random.default_rng(11)
    blobs = []
    for i in range(240):
        kind = zstd_corpus.KINDS[int(rng.integers(len(zstd_corpus.KINDS)))]
        n = int(rng.choice([rng.integers(0, 300), rng.integers(300, 20000), rng.integers(20000, 300000)]))
        blobs.append(zstd_corpus.blob(kind, n, 1000 + i))
    with Context(0) as c:
        c.set_option(_lib.BW_OPT_ZSTD_SLOTS, 7)
        c.set_option(_lib.BW_OPT_ZSTD_BATCH_BYTES, 1 << 20)
        f1 = c.zstd_compress(blobs)
        f2 = c.zstd_compress(blobs[::-1])  # the same slots again, at higher index bases
    _check_frames(oracle, blobs, f1)
    _check_frames(oracle, blobs[::-1], f2)


@pytest.mark.gpu
def test_gpu_zstd_device_buffers(ctx, oracle):
    import torch
    blobs = [zstd_corpus.blob(k, 3 * 1024 * 1024 - 5 * i, 77 + i) for i, k in enumerate(zstd_corpus.KINDS)]
    lens = np.array([len(b) for b in blobs], dtype=np.uint64)
    so = np.concatenate([[0], np.cumsum(lens + 16)[:-1]]).astype(np.uint64)
    host = np.zeros(int(so[-1] + lens[-1]), dtype=np.uint8)
    for o, b in zip(so, blobs):
        host[int(o):int(o) + len(b)] = np.frombuffer(b, np.uint8)
    d_src = torch.from_numpy(host).cuda()
    cap = np.array([ctx._L.bw_zstd_store_size(int(x)) for x in lens], dtype=np.uint64)
    do = np.concatenate([[0], np.cumsum(cap)[:-1]]).astype(np.uint64)
    d_dst = torch.zeros(int(cap.sum()), dtype=torch.uint8, device="cuda")
    fl = ctx.zstd_compress_device(d_src.data_ptr(), so, lens, d_dst.data_ptr(), do)
    out = d_dst.cpu().numpy()
    frames = [out[int(do[i]):int(do[i] + fl[i])].tobytes() for i in range(len(blobs))]
    _check_frames(oracle, blobs, frames)


@pytest.mark.gpu
def test_gpu_zstd_rejects_blob_over_3mib(ctx):
    from backuwup_amd._lib import BwError
    with pytest.raises(BwError):
        ctx.zstd_compress([bytes(3 * 1024 * 1024 + 1)])


@pytest.mark.gpu
def test_gpu_zstd_async_lanes_equal_oracle(oracle):
    """bw_zstd_submit_device / bw_zstd_wait: BW_ZSTD_LANES batches in flight on one context (each
    lane its own stream and hash tables, one with small slot limits so its tables are reused),
    waited out of order; every frame equals the oracle's; a submit with every lane busy and a
    wait on an unknown ticket are BW_ESTATE."""
    import torch
    from backuwup_amd import Context, _lib
    from backuwup_amd._lib import BwError
    rng = np.random.default_rng(23)
    batches = []
    for b in range(_lib.BW_ZSTD_LANES):
        blobs = [zstd_corpus.blob(zstd_corpus.KINDS[(b + i) % len(zstd_corpus.KINDS)],
                                  int(rng.choice([rng.integers(0, 500), rng.integers(500, 200000)])), 3000 + 100 * b + i)
                 for i in range(40)]
        lens = np.array([len(x) for x in blobs], dtype=np.uint64)
        so = np.concatenate([[0], np.cumsum(lens + 16)[:-1]]).astype(np.uint64)
        host = np.zeros(int(so[-1] + lens[-1]) + 16, dtype=np.uint8)
        for o, x in zip(so, blobs):
            host[int(o):int(o) + len(x)] = np.frombuffer(x, np.uint8)
        cap = np.array([_lib.load().bw_zstd_store_size(int(x)) for x in lens], dtype=np.uint64)
        do = np.concatenate([[0], np.cumsum(cap)[:-1]]).astype(np.uint64)
        batches.append((blobs, so, lens, do, torch.from_numpy(host).cuda(),
                        torch.zeros(int(cap.sum()), dtype=torch.uint8, device="cuda")))
    with Context(0) as c:
        c.set_option(_lib.BW_OPT_ZSTD_SLOTS, 5)  # copied to the lanes: internal batches of 5 blobs
        tickets = [c.zstd_submit_device(src.data_ptr(), so, lens, dst.data_ptr(), do)
                   for blobs, so, lens, do, src, dst in batches]
        with pytest.raises(BwError):
            c.zstd_submit_device(batches[0][4].data_ptr(), batches[0][1], batches[0][2], batches[0][5].data_ptr(),
                                 batches[0][3])
        fls = {t: c.zstd_wait(t) for t in reversed(tickets)}
        with pytest.raises(BwError):
            c.zstd_wait(tickets[0])
        again = c.zstd_submit_device(batches[1][4].data_ptr(), batches[1][1], batches[1][2], batches[1][5].data_ptr(),
                                     batches[1][3])  # a lane is free again
        fl_again = c.zstd_wait(again)
    for t, (blobs, so, lens, do, src, dst) in zip(tickets, batches):
        out = dst.cpu().numpy()
        frames = [out[int(do[i]):int(do[i] + fls[t][i])].tobytes() for i in range(len(blobs))]
        _check_frames(oracle, blobs, frames)
    assert np.array_equal(fl_again, fls[tickets[1]])


@pytest.mark.gpu
def test_gpu_zstd_table_layouts_and_switches(oracle):
    """Sub-batches of more than 2,048 blobs parse with narrow (libzstd u32) tables, smaller ones with
    wide entries that carry their bytes; a slot that changes layout is cleared first.  One context:
    narrow, wide, narrow again over the same slots; every frame equals the oracle's."""
    from backuwup_amd import Context
    rng = np.random.default_rng(29)
    many = [zstd_corpus.blob(zstd_corpus.KINDS[i % len(zstd_corpus.KINDS)], int(rng.integers(0, 3000)), 5000 + i)
            for i in range(2100)]
    few = [zstd_corpus.blob(zstd_corpus.KINDS[i % len(zstd_corpus.KINDS)], int(rng.integers(1000, 300000)), 9000 + i)
           for i in range(30)]
    with Context(0) as c:
        f_many = c.zstd_compress(many)
        f_few = c.zstd_compress(few)
        f_many2 = c.zstd_compress(many[::-1])
    _check_frames(oracle, many, f_many)
    _check_frames(oracle, few, f_few)
    _check_frames(oracle, many[::-1], f_many2)
