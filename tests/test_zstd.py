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
