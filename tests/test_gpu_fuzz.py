"""Seeded random sweep of the whole front end against the oracle (round 6): FastCDC parameters drawn
anywhere in the crate's asserted ranges (fastcdc 3.0.3 v2020 FastCDC::new: 64 <= min <= 1 MiB, 256 <=
avg <= 4 MiB, 1 KiB <= max <= 16 MiB, in any order; avg > max is refused with BW_EINVAL, where the
crate's cut() reads past max and mostly panics -- oracle.CratePanic), content of every kind the chunker treats
differently (random, zeros, one-byte and short periodic patterns, two-symbol bytes with dense
candidates, compressible text, random with zero runs), ragged batches of many files with the
small-file threshold anywhere, and a seeded index.  Every blob -- boundaries, Chunk.hash, digest,
verdict -- must equal the oracle's.  The cases are fixed by the seed; each is small enough for the
oracle to finish in well under a second."""
import numpy as np
import pytest

from backuwup_amd import make_params, make_tree
from backuwup_amd._lib import BW_EINVAL, BwError
from backuwup_amd.synth import compressible_corpus, splitmix_bytes

pytestmark = pytest.mark.gpu

MiB = 1 << 20


def _content(rng, kind, n):
    if kind == "random":
        return splitmix_bytes(int(rng.integers(1 << 30)), n)
    if kind == "zeros":
        return np.zeros(n, np.uint8)
    if kind == "byte":
        return np.full(n, int(rng.integers(256)), np.uint8)
    if kind == "period":
        p = int(rng.integers(2, 9000))
        return np.resize(splitmix_bytes(int(rng.integers(1 << 30)), p), n)
    if kind == "two":
        return (splitmix_bytes(int(rng.integers(1 << 30)), n) & 1).astype(np.uint8)
    if kind == "text":
        return compressible_corpus(n, "text", seed=int(rng.integers(1 << 30)), piece=4 * MiB)
    r = splitmix_bytes(int(rng.integers(1 << 30)), n)  # random with zero runs
    for at in rng.integers(0, max(1, n), 8):
        r[int(at):int(at) + int(rng.integers(1, 1 << 18))] = 0
    return r


KINDS = ["random", "zeros", "byte", "period", "two", "text", "runs"]


def _params(rng):
    # log-uniform inside each asserted range, independently (max < min and avg outside [min, max] allowed)
    lu = lambda lo, hi: int(np.exp(rng.uniform(np.log(lo), np.log(hi + 1))))  # noqa: E731
    return min(lu(64, MiB), MiB), min(lu(256, 4 * MiB), 4 * MiB), min(lu(1024, 16 * MiB), 16 * MiB)


def _blobs_equal(a, b):
    assert a.shape == b.shape, (a.shape, b.shape)
    for f in ("file", "offset", "length", "gear_hash", "is_dup", "digest"):
        assert np.array_equal(a[f], b[f]), f


@pytest.mark.parametrize("case", range(48))
def test_fastcdc_random_params_and_content(ctx, oracle, case):
    rng = np.random.default_rng(1000 + case)
    mn, av, mx = _params(rng)
    kind = KINDS[case % len(KINDS)]
    # enough bytes for tens of chunks at the drawn sizes, at most 24 MiB
    n = int(min(24 * MiB, max(1, rng.integers(1, 40) * max(mn, min(av, mx)) + rng.integers(0, 4096))))
    data = _content(rng, kind, n)
    if av > mx:  # the crate reads past max and mostly panics; the ABI refuses (oracle CratePanic)
        with pytest.raises(BwError) as e:
            ctx.fastcdc_chunks(data, mn, av, mx)
        assert e.value.rc == BW_EINVAL
        return
    assert ctx.fastcdc_chunks(data, mn, av, mx) == oracle.fastcdc(data, mn, av, mx), (kind, n, mn, av, mx)


def _valid_params(rng, case):
    mn, av, mx = _params(rng) if case % 3 else (262144, 1048576, 3145728)
    if av > mx:  # (refused: test_fastcdc_random_params_and_content)
        av = max(256, mx)
    return mn, av, mx


def _batch(rng, nf_max=400, pool=()):
    """A ragged batch: empty and tiny files up to 3 MiB, every content kind, whole-file copies within
    the batch and of `pool` (files of earlier batches: prior backups' blobs)."""
    nf = int(rng.integers(1, nf_max))
    lens = np.where(rng.random(nf) < 0.1, 0, rng.integers(0, 3 * MiB, nf) >> rng.integers(0, 12, nf)).astype(np.uint64)
    files = [_content(rng, KINDS[int(rng.integers(len(KINDS)))] if rng.random() < 0.3 else "random", int(m))
             for m in lens]
    for k in range(1, nf):  # whole-file copies: duplicates across the batch
        if rng.random() < 0.15:
            files[k] = files[int(rng.integers(k))].copy()
    for k in range(nf):
        if pool and rng.random() < 0.1:
            files[k] = pool[int(rng.integers(len(pool)))].copy()
    lens = np.array([f.size for f in files], np.uint64)
    offs = np.zeros(nf, np.uint64)
    offs[1:] = np.cumsum((lens[:-1] + 15) // 16 * 16)
    data = np.zeros(int(offs[-1] + lens[-1]) + 16, np.uint8)
    for o, f in zip(offs, files):
        data[int(o):int(o) + f.size] = f
    return data, offs, lens, files


@pytest.mark.parametrize("case", range(24))
def test_process_files_random_batches(ctx, oracle, case):
    rng = np.random.default_rng(5000 + case)
    mn, av, mx = _valid_params(rng, case)
    thr = int(rng.choice([0, 1, 4096, MiB, 8 * MiB]))  # the small-file threshold (dir_packer.rs:246 = 1 MiB)
    data, offs, lens, files = _batch(rng)
    nf = len(files)
    # a seeded index: the digests of a few of the batch's own files (prior backups, BlobIndex::load)
    seed_files = rng.choice(nf, size=min(nf, 5), replace=False)
    seeded = sorted({oracle.blake3(files[int(k)]) for k in seed_files})
    ctx.index_reset()
    ctx.index_seed(np.frombuffer(b"".join(seeded), np.uint8).reshape(-1, 32))
    got = ctx.process_files(data, offs, lens, make_params(mn, av, mx, small_file_threshold=thr))
    want = oracle.process_files(data, offs, lens, mn, av, mx, small_threshold=thr, index=oracle.Index(b"".join(seeded)),
                                threads=8)
    _blobs_equal(got, want)


def test_min_above_max_hashes_whole_remainders(ctx, oracle):
    """min > max (the crate allows it): cut() returns a remainder <= min whole, so chunks run up to min,
    past max -- the leaf pass and the upper levels are sized for max(min, max) (fuzz case 23 above
    found a 70,325 B chunk hashed as if it were <= max = 1,520)."""
    p = (496561, 1520, 1520)
    files = [splitmix_bytes(90 + k, n) for k, n in enumerate([70325, 1520, 1521, 496561, 496562, 3 << 20, 0])]
    lens = np.array([f.size for f in files], np.uint64)
    offs = np.zeros(len(files), np.uint64)
    offs[1:] = np.cumsum((lens[:-1] + 15) // 16 * 16)
    data = np.zeros(int(offs[-1] + lens[-1]) + 16, np.uint8)
    for o, f in zip(offs, files):
        data[int(o):int(o) + f.size] = f
    ctx.index_reset()
    got = ctx.process_files(data, offs, lens, make_params(*p, small_file_threshold=0))
    want = oracle.process_files(data, offs, lens, *p, small_threshold=0)
    assert int(want["length"].max()) == 496561 > p[2]
    _blobs_equal(got, want)


@pytest.mark.parametrize("case", range(8))
def test_host_batches_in_flight_random(oracle, case):
    """bw_submit_host (row N1): random batches in flight on one context up to its ring depth
    (BW_OPT_DEPTH 2-4), pageable, one backup session's index across them -- every blob equal to the
    oracle's with one Index over the batches in submit order."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from backuwup_amd import Context
    from backuwup_amd._lib import BW_OPT_DEPTH
    rng = np.random.default_rng(7000 + case)
    mn, av, mx = _valid_params(rng, case)
    thr = int(rng.choice([0, 4096, MiB]))
    depth = int(rng.integers(2, 5))
    p = make_params(mn, av, mx, small_file_threshold=thr)
    ix, pool, pending = oracle.Index(), [], []
    with Context(0) as c:
        c.set_option(BW_OPT_DEPTH, depth)
        c.index_reset()
        for _ in range(int(rng.integers(2, 7))):
            data, offs, lens, files = _batch(rng, 120, pool)
            pool += files
            pending.append((c.submit_host(data, offs, lens, p), data, offs, lens))
            if len(pending) == depth or rng.random() < 0.3:
                t, d, o, l = pending.pop(0)
                _blobs_equal(c.wait(t), oracle.process_files(d, o, l, mn, av, mx, small_threshold=thr, index=ix,
                                                             threads=8))
        for t, d, o, l in pending:
            _blobs_equal(c.wait(t), oracle.process_files(d, o, l, mn, av, mx, small_threshold=thr, index=ix, threads=8))


@pytest.mark.parametrize("case", range(6))
def test_node_session_random_batches(oracle, case):
    """NodeSession (row e, one process, N ranks on the local transport): random batches, parameters
    and world sizes, files repeated across batches -- the digest-prefix-partitioned index decides
    exactly as one oracle.Index over the batches in order."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from backuwup_amd.session import NodeSession
    rng = np.random.default_rng(9000 + case)
    world = [2, 4, 8][case % 3]
    mn, av, mx = _valid_params(rng, case)
    thr = int(rng.choice([0, 4096, MiB]))
    ix, pool = oracle.Index(), []
    with NodeSession([0] * world, transport="local", params=make_params(mn, av, mx, small_file_threshold=thr)) as s:
        for _ in range(3):
            data, offs, lens, files = _batch(rng, 200, pool)
            pool += files
            got = s.process_files(data, offs, lens)
            _blobs_equal(got, oracle.process_files(data, offs, lens, mn, av, mx, small_threshold=thr, index=ix,
                                                   threads=8))


@pytest.mark.parametrize("case", range(12))
def test_dropin_kept_digests_random(ctx, oracle, case):
    """The drop-in call sites (dir_packer.rs:254-266, :286) at random parameters: FastCDC over the
    whole source with digests kept, then blake3::hash of every chunk slice answered from them, and of
    slices that are not chunks (hashed afresh) -- all against the oracle."""
    rng = np.random.default_rng(11000 + case)
    mn, av, mx = _valid_params(rng, case)
    n = int(min(16 * MiB, rng.integers(1, 30) * max(mn, mx) + rng.integers(0, 4096)))
    buf = _content(rng, KINDS[case % len(KINDS)], n)
    buf.flags.writeable = False
    cuts, h = ctx.fastcdc_chunks_hashed(buf, mn, av, mx)
    try:
        want = oracle.fastcdc(buf, mn, av, mx)
        assert cuts == want
        for _, o, ln in cuts:
            assert ctx.blake3_at(buf, o, ln, kept=True) == oracle.blake3(buf[o:o + ln]), (o, ln)
        for _ in range(8):  # not chunks: a shifted start, a shorter length
            o = int(rng.integers(0, n))
            ln = int(rng.integers(0, min(n - o, 70000) + 1))
            assert ctx.blake3_at(buf, o, ln, kept=True) == oracle.blake3(buf[o:o + ln]), (o, ln)
    finally:
        ctx.fastcdc_release(h)


@pytest.mark.parametrize("case", range(12))
def test_random_options_random_batches(oracle, case):
    """The product's free context options drawn at random on a fresh context -- the small-batch tile
    size threshold, a candidate array forced too small (the walkers' direct path), BLAKE3 leaves per
    lane, when the scan is enqueued, the pinned staging chunk -- under random batches through
    process_files, submit_host (pageable) and submit_device, one index across them."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from backuwup_amd import Context
    from backuwup_amd._lib import BW_OPT_B3_GROUP, BW_OPT_CAND_CAP, BW_OPT_SCAN_FIRST, BW_OPT_SCAN_SMALL_BYTES, \
        BW_OPT_STAGE_CHUNK
    rng = np.random.default_rng(13000 + case)
    mn, av, mx = _valid_params(rng, case)
    thr = int(rng.choice([0, 4096, MiB]))
    p = make_params(mn, av, mx, small_file_threshold=thr)
    opts = {BW_OPT_SCAN_SMALL_BYTES: int(rng.choice([0, 1 << 40, int(rng.integers(1, 64 * MiB))])),
            BW_OPT_CAND_CAP: int(rng.choice([0, 0, 0, 16, 1000, int(rng.integers(1, 50000))])),
            BW_OPT_B3_GROUP: int(rng.choice([0, 1, 2, 4])),
            BW_OPT_SCAN_FIRST: int(rng.integers(0, 3)),
            BW_OPT_STAGE_CHUNK: int(rng.choice([(1 << 20) + 13, (3 << 20) + 4097, 64 * MiB]))}
    ix, pool = oracle.Index(), []
    with Context(0) as c:
        for k, v in opts.items():
            c.set_option(k, v)
        c.index_reset()
        for _ in range(3):
            data, offs, lens, files = _batch(rng, 150, pool)
            pool += files
            how = int(rng.integers(0, 3))
            if how == 0:
                got = c.process_files(data, offs, lens, p)
            elif how == 1:
                got = c.wait(c.submit_host(data, offs, lens, p))
            else:
                dev = torch.from_numpy(data).cuda()
                torch.cuda.synchronize()
                got = c.wait(c.submit_device(dev.data_ptr(), data.size, offs, lens, p))
            want = oracle.process_files(data, offs, lens, mn, av, mx, small_threshold=thr, index=ix, threads=8)
            _blobs_equal(got, want)


@pytest.mark.parametrize("case", range(6))
def test_zstd_random_blobs(ctx, oracle, case):
    """Per-blob zstd level 3 (§8f row 2, pack.rs:58-64) on the chunker fuzz's content kinds --
    periods of 2 to 9,000 bytes, two-symbol bytes, one-byte fills, zeros, zero runs in random data,
    text -- at log-uniform sizes up to the 3 MiB blob limit, many per call: every frame equal to the
    oracle's (and to the image's libzstd through it, tests/test_zstd.py)."""
    rng = np.random.default_rng(15000 + case)
    blobs = []
    for _ in range(int(rng.integers(10, 40))):
        n = min(3 * MiB, int(np.exp(rng.uniform(0, np.log(3 * MiB)))) - 1)
        blobs.append(_content(rng, KINDS[int(rng.integers(len(KINDS)))], max(n, 0)).tobytes())
    frames = ctx.zstd_compress(blobs)
    for i, (b, f) in enumerate(zip(blobs, frames)):
        assert f == oracle.zstd3_compress(b), (i, len(b))


@pytest.mark.parametrize("case", range(6))
def test_tree_blobs_random(ctx, oracle, case):
    """Tree blobs (§8f row 1, dir_packer.rs:314-390) on random trees: names of any bytes up to 3,000
    long, metadata absent or at the u64 extremes, child counts at and around the 10,000-per-piece
    split (pieces over 64 KiB hash through the context's launch path), repeated trees, and an index
    seeded with some pieces of earlier backups -- every piece's bytes, hash and verdict against the
    oracle's split_serialize_tree and Index."""
    rng = np.random.default_rng(17000 + case)
    specs = []
    for i in range(int(rng.integers(40, 200))):
        if specs and rng.random() < 0.1:
            specs.append(specs[int(rng.integers(len(specs)))])
            continue
        nl = int(rng.choice([0, 1, int(rng.integers(2, 64)), int(rng.integers(64, 3000))]))
        name = rng.integers(0, 256, nl, dtype=np.uint8).tobytes()
        meta = [None if rng.random() < 0.25 else [0, 2**64 - 1, int(rng.integers(0, 2**63))][int(rng.integers(3))]
                for _ in range(3)]
        nch = int(rng.choice([0, 1, 2, int(rng.integers(3, 2000)), 9999, 10000, 10001, 20000, 25001]))
        ch = rng.integers(0, 256, nch * 32, dtype=np.uint8).tobytes()
        specs.append((int(rng.integers(2)), name, *meta, ch))
    dedup = bool(case % 3)
    pieces = [oracle.split_serialize_tree(*s) for s in specs]
    prior = sorted({h for ps in pieces for _, h in ps if rng.random() < 0.1})
    ctx.index_reset()
    if prior:
        ctx.index_seed(np.frombuffer(b"".join(prior), np.uint8).reshape(-1, 32))
    hashes, blobs = ctx.tree_blobs([make_tree(*s) for s in specs], dedup=dedup)
    ix = oracle.Index(b"".join(prior))
    k = 0
    for i, ps in enumerate(pieces):
        assert bytes(hashes[i]) == ps[0][1], i
        for p, (data, h) in enumerate(ps):
            b = blobs[k]
            assert (int(b["tree"]), int(b["piece"]), int(b["length"])) == (i, p, len(data)), (i, p)
            assert bytes(b["hash"]) == h, (i, p)
            if dedup:
                dup = ix.is_blob_duplicate(h)
                if not dup:
                    ix.insert(h)
                assert int(b["is_dup"]) == int(dup), (i, p)
            k += 1
    assert k == len(blobs)


@pytest.mark.parametrize("case", range(6))
def test_seal_open_random(ctx, oracle, case):
    """Per-blob sealing (§8f row 3: derive_backup_key + Aes256Gcm, pack.rs:70-80) and opening
    (unpack.rs:58-63) on random items: log-uniform lengths up to 3 MiB, unaligned sources and
    destinations, info lengths 0-54 bytes -- every sealed item equal to the oracle's, and opened back
    to the plaintext with every tag accepted."""
    rng = np.random.default_rng(19000 + case)
    n = int(rng.integers(1, 120))
    lens = np.array([min(3 * MiB, int(np.exp(rng.uniform(0, np.log(3 * MiB)))) - 1) for _ in range(n)], np.uint64)
    gaps = rng.integers(0, 40, n)
    off = np.zeros(n, np.uint64)
    dst = np.zeros(n, np.uint64)
    pos = dpos = 0
    for i in range(n):
        pos += int(gaps[i])
        off[i] = pos
        pos += int(lens[i])
        dpos += int(rng.integers(0, 24))
        dst[i] = dpos
        dpos += int(lens[i]) + 16
    data = splitmix_bytes(int(rng.integers(1 << 30)), max(pos, 1))
    info_len = int(rng.integers(0, 55))
    infos = rng.integers(0, 256, (n, info_len), dtype=np.uint8)
    nonces = rng.integers(0, 256, (n, 12), dtype=np.uint8)
    prk = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    sealed = ctx.seal(prk, data, off, lens, infos, nonces, dst, dpos)
    for i in range(n):
        pt = data[int(off[i]):int(off[i] + lens[i])]
        want = oracle.seal_blob(prk, bytes(infos[i]), bytes(nonces[i]), pt)
        assert sealed[int(dst[i]):int(dst[i]) + int(lens[i]) + 16].tobytes() == want, (i, int(lens[i]), info_len)
    plain, ok = ctx.seal(prk, sealed, dst, lens + np.uint64(16), infos, nonces, off, pos, open_=True)
    assert ok.all()
    for i in range(n):
        assert np.array_equal(plain[int(off[i]):int(off[i] + lens[i])], data[int(off[i]):int(off[i] + lens[i])]), i


@pytest.mark.parametrize("case", range(4))
def test_packfiles_and_index_files_random(ctx, oracle, case):
    """Packfiles (§8f row 4: write_packfiles + serialize_packfile, pack.rs:115-227) of random blob
    queues -- many tiny blobs, some up to 3 MiB, ragged source offsets, store frames (flags default)
    -- equal byte for byte to the format oracle's; then the index files of the same entries
    (BlobIndex::push/flush, blob_index.rs:151-240) built, loaded back and gating new digests."""
    from oracle import pack_oracle as po
    rng = np.random.default_rng(21000 + case)
    prk = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    n = int(rng.integers(1, 300))
    sizes = [int(rng.integers(0, 64)) if rng.random() < 0.5 else
             min(3 * MiB, int(np.exp(rng.uniform(0, np.log(3 * MiB))))) for _ in range(n)]
    while sum(sizes) > 24 * MiB:
        sizes[int(np.argmax(sizes))] //= 4
    datas = [splitmix_bytes(int(rng.integers(1 << 30)), s).tobytes() for s in sizes]
    align = int(rng.integers(1, 17))
    offs, cur = [], 0
    for d in datas:
        offs.append(cur)
        cur += len(d) + (-len(d)) % align
    src = np.zeros(max(cur, 1), np.uint8)
    for o, d in zip(offs, datas):
        src[o:o + len(d)] = np.frombuffer(d, np.uint8)
    offs = np.asarray(offs, np.uint64)
    lens = np.asarray(sizes, np.uint64)
    hashes = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    kinds = rng.integers(0, 2, n).astype(np.uint8)
    nonces = rng.integers(0, 256, (n, 12), dtype=np.uint8)
    plan, total = ctx.pack_plan(lens)
    ids = rng.integers(0, 256, (len(plan), 12), dtype=np.uint8)
    got = ctx.pack_build(prk, src, offs, lens, hashes, kinds, nonces, plan, total, ids)
    blobs = [(bytes(hashes[i]), int(kinds[i]), bytes(nonces[i]),
              po.seal_blob_payload(prk, hashes[i], nonces[i], po.zstd_store(d))) for i, d in enumerate(datas)]
    want = po.write_packfiles(prk, blobs, [bytes(x) for x in ids])
    assert len(want) == len(plan)
    for p, (_, buf) in zip(plan, want):
        assert got[int(p["offset"]):int(p["offset"] + p["size"])].tobytes() == buf
    ents = np.concatenate([hashes, rng.integers(0, 256, (n, 12), dtype=np.uint8)], axis=1)
    last = int(rng.integers(0, 1000))
    files = ctx.index_files_build(prk, ents, last_file_num=last)
    assert [(f, b) for f, b in files] == po.push_and_flush(prk, last, [(bytes(e[:32]), bytes(e[32:])) for e in ents])
    ctx.index_reset()
    assert ctx.index_load_files(prk, files).tobytes() == ents.tobytes()
    probe = np.concatenate([hashes[::3], rng.integers(0, 256, (7, 32), dtype=np.uint8)])
    assert ctx.index_check_insert(probe).tolist() == [1] * len(hashes[::3]) + [0] * 7
