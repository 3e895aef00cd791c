"""The CPU oracle (oracle/bw_oracle.c) pinned against everything available offline:
published BLAKE3 known answers, the GEAR derivation rule and its sha256, the MASKS popcount
identity, the SURVEY.md A.5 cross-check vector, and tests/golden/vectors.json produced by an
independent pure-Python restatement (tests/golden/make_golden.py).  Parity is otherwise
unpinned by the reference (its tests cover none of this path)."""
import hashlib
import json
import os
import re

import numpy as np
import pytest

from backuwup_amd.synth import splitmix_bytes

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
VEC = json.load(open(os.path.join(HERE, "golden", "vectors.json")))
GEAR_SHA256 = "9df0a720752a7d211fdebaf39bed01610983756fc340a1cfef41052b7356ae73"

KAT = {b"": "af1349b9f5f9a1a6a0404dea36dcc9499bcb25c9adc112b7cc9a93cae41f3262",
       b"abc": "6437b3ac38465133ffb63b75273a8db548c558465d79db03fd359c6cd5bd9d85",
       b"\x00": "2d3adedff11b61f14c886e35afa036736dcd87a74d27b5c1510225d0f592e213"}


def test_blake3_known_answers(oracle):
    for m, d in KAT.items():
        assert oracle.blake3(m).hex() == d
        assert VEC["blake3_kat"][m.hex()] == d


def test_blake3_golden_lengths(oracle):
    for v in VEC["blake3"]:
        msg = (np.arange(v["len"]) % 251).astype(np.uint8)
        assert oracle.blake3(msg).hex() == v["digest"], v["len"]


def test_gear_table_rule_and_sha(oracle):
    g = oracle.gear_table()
    rule = [int.from_bytes(hashlib.md5(bytes([i]) * 64).digest()[:8], "big") for i in range(256)]
    assert [int(x) for x in g] == rule
    assert hashlib.sha256(b"".join(int(x).to_bytes(8, "big") for x in g)).hexdigest() == GEAR_SHA256
    assert VEC["gear_sha256"] == GEAR_SHA256


def test_product_tables_match_rule():
    """The HIP path's generated constants (backuwup_amd/csrc/bw_tables.inc) equal the rule."""
    txt = open(os.path.join(ROOT, "backuwup_amd", "csrc", "bw_tables.inc")).read()
    gear_txt = txt[txt.index("BW_GEAR_INIT"):txt.index("BW_MASKS_INIT")]
    masks_txt = txt[txt.index("BW_MASKS_INIT"):]
    gear = [int(x, 16) for x in re.findall(r"0x([0-9a-f]{16})ULL", gear_txt)]
    masks = [int(x, 16) for x in re.findall(r"0x([0-9a-f]{16})ULL", masks_txt)]
    rule = [int.from_bytes(hashlib.md5(bytes([i]) * 64).digest()[:8], "big") for i in range(256)]
    assert gear == rule
    assert len(masks) == 26
    for i, m in enumerate(masks):
        if i >= 5:
            assert bin(m).count("1") == i


def test_masks_backuwup(oracle):
    ms, ml = oracle.masks(262144, 1048576, 3145728)
    assert ms == 0x0000d91767537000 and ml == 0x0000d91707537000
    assert ms & ml == ml  # mask_l is a subset of mask_s
    with pytest.raises(ValueError):
        oracle.masks(63, 256, 1024)
    with pytest.raises(ValueError):
        oracle.masks(64, 256, 16777217)


def test_a5_cross_check_vector(oracle):
    d = splitmix_bytes(0, 8_400_953)
    assert hashlib.sha256(d.tobytes()).hexdigest() == "a3a2fa7930e9d9abd798e344b87815732eba55302b1a6770fea5bb7034ec3010"
    ch = oracle.fastcdc(d, 262144, 1048576, 3145728)
    assert [c[2] for c in ch] == [1560056, 791747, 1444242, 1177622, 806036, 2266142, 355108]
    assert oracle.blake3(d[:ch[0][2]]).hex() == "288bba07c57e7334145f6905c58d864d9ce21618c6dadef35a7a25bb48c1c3a7"


def test_fastcdc_golden(oracle):
    for v in VEC["fastcdc"]:
        d = splitmix_bytes(v["seed"], v["len"])
        assert hashlib.sha256(d.tobytes()).hexdigest() == v["sha256"]
        got = oracle.fastcdc(d, v["min"], v["avg"], v["max"])
        assert [list(c) for c in got] == v["chunks"], (v["seed"], v["len"])
        if v["first_chunk_blake3"]:
            o, l = got[0][1], got[0][2]
            assert oracle.blake3(d[o:o + l]).hex() == v["first_chunk_blake3"]


def test_fastcdc_zeros(oracle):
    z = np.zeros(VEC["zeros"]["len"], dtype=np.uint8)
    assert [list(c) for c in oracle.fastcdc(z, 262144, 1048576, 3145728)] == VEC["zeros"]["chunks"]
    assert VEC["zeros"]["chunks"][0][0] == (-0x3b5d3c7d207e37dc) % (1 << 64)  # -GEAR[0]


def test_fastcdc_invariants(oracle):
    rng = np.random.default_rng(0)
    for trial in range(20):
        n = int(rng.integers(1, 200_000))
        d = splitmix_bytes(100 + trial, n)
        mn, av, mx = 64, 256, 1024
        ch = oracle.fastcdc(d, mn, av, mx)
        assert sum(c[2] for c in ch) == n
        assert all(ch[i][1] + ch[i][2] == ch[i + 1][1] for i in range(len(ch) - 1))
        assert all(mn <= c[2] <= mx for c in ch[:-1])


def test_process_file_policy(oracle):
    """dir_packer.rs:246: len > 1 MiB -> CDC; else one blob (an empty file too)."""
    sizes = [0, 1, 4096, 1 << 20, (1 << 20) + 1, 5 << 20]
    data = splitmix_bytes(9, sum(sizes))
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
    b = oracle.process_files(data, offs, sizes)
    per_file = [int((b["file"] == f).sum()) for f in range(len(sizes))]
    assert per_file[:4] == [1, 1, 1, 1]
    assert per_file[4] >= 1 and per_file[5] >= 2
    assert bytes(b["digest"][0]).hex() == KAT[b""]
    assert b["length"][0] == 0 and b["gear_hash"][0] == 0


def test_dedup_canonical_order(oracle):
    """blob_index.rs:130-148 + :109: dup iff seeded or seen at an earlier canonical position."""
    rng = np.random.default_rng(1)
    pool = [bytes(rng.integers(0, 256, 32, dtype=np.uint8)) for _ in range(50)]
    seed = sorted(pool[:10])
    ix = oracle.Index(b"".join(seed))
    seen = set(seed)
    for k in rng.integers(0, 50, 400):
        d = pool[int(k)]
        dup = ix.is_blob_duplicate(d)
        assert dup == (d in seen)
        if not dup:
            assert ix.insert(d) == 0
            seen.add(d)
        else:
            assert d in seen
    assert ix.insert(pool[20]) == -1 or pool[20] not in seen  # DuplicateBlob on a second insert


def test_process_files_dedup_copies(oracle):
    from backuwup_amd.synth import tree_corpus
    data, offs, lens = tree_corpus(24 << 20, seed=3, max_file=6 << 20)
    b = oracle.process_files(data, offs, lens)
    digests = [bytes(x) for x in b["digest"]]
    first = {}
    for i, d in enumerate(digests):
        first.setdefault(d, i)
    assert [int(x) for x in b["is_dup"]] == [int(first[d] != i) for i, d in enumerate(digests)]
    assert b["is_dup"].sum() > 0


def test_golden_generator_agrees_on_small_cases():
    """Re-run the pure-Python restatement on a few cheap fixtures (the generator is test code)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(HERE, "golden", "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    for v in VEC["fastcdc"][:6]:
        d = mg.splitmix(v["seed"], v["len"])
        assert [list(c) for c in mg.fastcdc_py(d, v["min"], v["avg"], v["max"])] == v["chunks"]
    for v in VEC["blake3"][:12]:
        assert mg.blake3_py(bytes(i % 251 for i in range(v["len"]))).hex() == v["digest"]



def test_blake3_simd_baseline_is_bit_exact(oracle):
    """The CPU baseline's 16-way BLAKE3 (bw_oracle_simd.c: the crate's hash_many strategy) equals
    the scalar restatement at every tree shape: 16-chunk groups, leftover chunks, odd parent
    levels, the 16-parent SIMD groups, counters past one group."""
    from backuwup_amd.synth import splitmix_bytes
    if not oracle.simd_available():
        pytest.skip("no AVX-512 on this host (the baseline falls back to the scalar restatement)")
    data = splitmix_bytes(99, (40 << 20) + 777)
    lens = [0, 1, 1023, 1024, 1025, 2047, 2048, 2049, 15 * 1024, 16 * 1024, 16 * 1024 + 1, 17 * 1024,
            31 * 1024 + 5, 32 * 1024, 33 * 1024, 64 * 1024 - 1, 257 * 1024, 262144, 1 << 20, (1 << 20) + 1,
            3 << 20, (3 << 20) - 1, 1000 * 1024 + 3, 40 << 20]
    for n in lens:
        for off in (0, 3):
            m = data[off:off + n]
            assert oracle.blake3_fast(m) == oracle.blake3(m), (n, off)
    # and through the batch driver, as the bench runs it
    offs = np.array([0, 5, 5000000, 9000001], dtype=np.uint64)
    lensb = np.array([5, 4999995, 4000001, 31 << 20], dtype=np.uint64)
    a = oracle.process_files(data, offs, lensb)
    try:
        assert oracle.set_blake3_simd(True)
        b = oracle.process_files(data, offs, lensb)
    finally:
        oracle.set_blake3_simd(False)
    assert np.array_equal(a, b)


def _prefix_collision():
    import json
    import os
    p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "blake3_prefix_collision.json")
    if not os.path.exists(p):
        pytest.skip("tests/golden/blake3_prefix_collision.json not generated (tools/collide.hip)")
    return json.load(open(p))


def test_blake3_prefix_collision_fixture(oracle):
    """A genuine collision of BLAKE3 on the first 8 digest bytes (found on the GPU by tools/collide.hip,
    parallel collision search): two distinct 8-byte messages whose digests share the 64-bit key the
    round-3 device index merged slots by.  The oracle's BLAKE3 confirms both digests."""
    fx = _prefix_collision()
    m1, m2 = bytes.fromhex(fx["m1"]), bytes.fromhex(fx["m2"])
    d1, d2 = oracle.blake3(m1), oracle.blake3(m2)
    assert m1 != m2 and len(m1) == len(m2) == 8
    assert d1.hex() == fx["digest1"] and d2.hex() == fx["digest2"]
    assert d1[:8] == d2[:8] and d1 != d2
    ix = oracle.Index()  # the reference's BlobIndex keeps both
    assert not ix.is_blob_duplicate(d1) and ix.insert(d1) == 0
    assert not ix.is_blob_duplicate(d2) and ix.insert(d2) == 0


def test_avg_above_max_follows_the_crate(oracle):
    """avg > max passes FastCDC::with_level's asserts, but cut() then keeps center = avg past
    remaining = max: its first loop reads beyond max, so a chunk can be longer than max, and where the
    source ends first it indexes out of bounds (a panic in the crate).  The oracle restates both; the
    GPU ABI refuses such sizes with BW_EINVAL (tests/test_gpu_fuzz.py)."""
    from backuwup_amd.synth import splitmix_bytes
    c = oracle.fastcdc(splitmix_bytes(3, 6000), 64, 4096, 1024)
    assert [l for _, _, l in c] == [1024, 3961, 360, 655]  # the second chunk is longer than max
    with pytest.raises(oracle.CratePanic):
        oracle.fastcdc(splitmix_bytes(0, 6000), 64, 4096, 1024)
