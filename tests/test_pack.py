"""Packfiles and index files: Manager::write_packfiles / serialize_packfile
(pack.rs:115-227), the reader Manager::get_blob (unpack.rs:22-78), BlobIndex::push / flush / load
(blob_index.rs:151-240), and the zstd store frames that stand in for level-3 zstd on
incompressible blobs (pack.rs:58-64).

CPU tests pin the format oracle (oracle/pack_oracle.py) to hand-derived bincode literals, the
reference's own size test (pack.rs:239-265 `validate_size_constraints`) and the system libzstd
(tests/zstd_ref.py), and check the C ABI's host-only planner against the oracle's grouping.  GPU
tests compare the packfiles and index files built through the C ABI with the oracle byte for
byte, read every blob back through the oracle's get_blob + libzstd, and seed the device index
from index files.
"""
import os
import struct

import numpy as np
import pytest

from backuwup_amd.synth import splitmix_bytes as _smb  # noqa: E402


def splitmix_bytes(seed, n):
    return _smb(seed, n).tobytes()

PRK = bytes.fromhex("5c" * 32)


@pytest.fixture(scope="module")
def po(oracle):
    from oracle import pack_oracle
    return pack_oracle


def _zstd():
    import zstd_ref
    if not zstd_ref.available():
        pytest.skip("libzstd not available")
    return zstd_ref


# ------------------------------------------------------------------ CPU: bincode + formats

def test_varint_literals(po):
    assert po.varint(0) == b"\x00" and po.varint(250) == b"\xfa"
    assert po.varint(251) == b"\xfb\xfb\x00" and po.varint(65535) == b"\xfb\xff\xff"
    assert po.varint(65536) == b"\xfc\x00\x00\x01\x00"
    assert po.varint(1 << 32) == b"\xfd" + struct.pack("<Q", 1 << 32)
    for v in (0, 250, 251, 65535, 65536, (1 << 32) - 1, 1 << 32, (1 << 64) - 1):
        assert po.read_varint(po.varint(v), 0) == (v, len(po.varint(v)))
    with pytest.raises(po.FormatError):
        po.read_varint(b"\xfe", 0)


def test_header_entry_matches_reference_size_test(po):
    """pack.rs:239-265: the entry {hash [0;32], FileChunk, Zstd, offset 0, length 0} and the
    packfile size bound it asserts."""
    e = po.header_entry(bytes(32), po.KIND_FILE_CHUNK, po.COMPRESSION_ZSTD, 0, 0)
    assert e == bytes(32) + b"\x00\x01\x00\x00" and len(e) == 36
    assert (po.PACKFILE_TARGET_SIZE + po.BLOB_MAX_UNCOMPRESSED_SIZE + len(e) * po.PACKFILE_MAX_BLOBS
            + po.BLOB_NONCE_SIZE <= po.PACKFILE_MAX_SIZE)
    # field order hash, kind, compression, length, offset (filesystem/mod.rs:36-43)
    e = po.header_entry(b"\x11" * 32, po.KIND_TREE, po.COMPRESSION_ZSTD, 300, 7)
    assert e == b"\x11" * 32 + b"\x01\x01\xfb\x2c\x01\x07"
    hdr = po.serialize_header([(b"\x11" * 32, 1, 1, 300, 7)])
    assert hdr[0] == 1 and po.deserialize_header(hdr) == [(b"\x11" * 32, 1, 1, 300, 7)]
    with pytest.raises(po.FormatError):
        po.deserialize_header(hdr + b"\x00")  # DefaultOptions reject trailing bytes
    with pytest.raises(po.FormatError):
        po.deserialize_header(hdr[:-1])


def test_index_plaintext_literals(po):
    h, p = b"\xaa" * 32, b"\xbb" * 12
    assert po.index_plaintext([]) == b"\x00"
    assert po.index_plaintext([(h, p)]) == b"\x01" + h + p
    assert po.index_plaintext([(h, p)] * 251)[:3] == b"\xfb\xfb\x00"
    assert po.counter_to_nonce(0x01020304) == b"\x04\x03\x02\x01" + bytes(8)
    with pytest.raises(po.FormatError):
        po.parse_index_plaintext(po.index_plaintext([(h, p)]) + b"\x00")


@pytest.mark.parametrize("n", [0, 1, 63, 64, 100, 1023, 1025, 65536, 131071, 131072, 131073, 262145,
                               1048576, 1048577, 3145728])
def test_zstd_store_frame_is_level3_output_for_incompressible_data(po, n):
    z = _zstd()
    data = splitmix_bytes(0x5eed + n, n)
    frame = po.zstd_store(data)
    assert len(frame) == po.zstd_store_size(n)
    assert frame == z.compress(data)       # what the reference's Compressor emits (pack.rs:58-64)
    assert z.decompress(frame) == data     # what its Decompressor reads back (unpack.rs:66-68)


def test_zstd_store_frame_is_valid_for_compressible_data(po):
    z = _zstd()
    data = bytes(200000) + b"abc" * 1000
    frame = po.zstd_store(data)
    assert z.decompress(frame) == data and len(z.compress(data)) < len(frame)


def test_plan_matches_oracle_grouping(po):
    from backuwup_amd import _lib
    from backuwup_amd.context import Context
    ctx = object.__new__(Context)
    ctx._L = _lib.load()
    rng = np.random.default_rng(11)
    cases = [
        [],
        [0],
        [3 * 1024 * 1024],
        [po.PACKFILE_TARGET_SIZE - 12 - 16 - 5],  # frame + tag + nonce lands exactly on the target
        list(rng.integers(0, 3 << 20, 40)),
        list(rng.integers(0, 70000, 300)),
    ]
    for lens in cases:
        plan, total = ctx.pack_plan(np.asarray(lens, dtype=np.uint64))
        sealed = [po.zstd_store_size(int(x)) + 16 for x in lens]
        groups = po.plan_packfiles(sealed)
        assert [(int(p["first_blob"]), int(p["n_blobs"])) for p in plan] == groups
        off = 0
        for p, (f, c) in zip(plan, groups):
            hdr = len(po.varint(c)) + sum(36 - 2 + len(po.varint(sealed[i])) +
                                          len(po.varint(sum(sealed[j] + 12 for j in range(f, i))))
                                          for i in range(f, f + c)) if c < 1000 else None
            if hdr is not None:
                assert int(p["header_len"]) == hdr + 16
            assert int(p["offset"]) == off
            off += int(p["size"])
        assert total == off
    # store frames are >= 5 bytes, so 3 MiB is always reached before PACKFILE_MAX_BLOBS (33 B per blob);
    # the count limit needs caller payloads under 4 bytes
    assert ctx.pack_plan([0] * (po.PACKFILE_MAX_BLOBS + 3))[0]["n_blobs"].tolist() == [95326, 4677]
    lens = [0, 1, 2, 3] * 25001
    plan, total = ctx.pack_plan(lens, flags=0)
    assert plan["n_blobs"].tolist() == [po.PACKFILE_MAX_BLOBS, 4]
    assert [(int(p["first_blob"]), int(p["n_blobs"])) for p in plan] == po.plan_packfiles([x + 16 for x in lens])


def test_oracle_packfile_round_trip(po):
    z = _zstd()
    rng = np.random.default_rng(3)
    blobs, raw = [], {}
    for i, n in enumerate([0, 1, 4096, 131072, 131073, 1 << 20, 3 << 20]):
        data = splitmix_bytes(100 + i, n)
        h = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
        nonce = bytes(rng.integers(0, 256, 12, dtype=np.uint8))
        raw[h] = data
        blobs.append((h, i & 1, nonce, po.seal_blob_payload(PRK, h, nonce, po.zstd_store(data))))
    ids = [bytes(rng.integers(0, 256, 12, dtype=np.uint8)) for _ in blobs]
    packs = po.write_packfiles(PRK, blobs, ids)
    assert len(packs) == len(po.plan_packfiles([len(b[3]) for b in blobs]))
    found = 0
    for pid, buf in packs:
        hl = struct.unpack_from("<Q", buf)[0]
        hdr = po.deserialize_header(po.oracle.open_blob(PRK, b"header", pid, buf[8:8 + hl]))
        for h, kind, comp, length, offset in hdr:
            k, payload = po.get_blob(PRK, pid, buf, h)
            assert z.decompress(payload) == raw[h] and comp == po.COMPRESSION_ZSTD
            found += 1
    assert found == len(blobs)
    # a flipped ciphertext byte of the packfile's last blob fails its tag
    pid, buf = packs[0]
    hl = struct.unpack_from("<Q", buf)[0]
    last = po.deserialize_header(po.oracle.open_blob(PRK, b"header", pid, buf[8:8 + hl]))[-1][0]
    bad = bytearray(buf)
    bad[-1] ^= 1
    with pytest.raises(po.CryptoError):
        po.get_blob(PRK, pid, bytes(bad), last)
    with pytest.raises(po.FormatError):
        po.get_blob(PRK, pid, buf, b"\x00" * 32)  # IndexHeaderMismatch


def test_oracle_index_round_trip(po):
    rng = np.random.default_rng(4)
    ents = [(bytes(rng.integers(0, 256, 32, dtype=np.uint8)), bytes(rng.integers(0, 256, 12, dtype=np.uint8)))
            for _ in range(120)]
    files = po.push_and_flush(PRK, 7, ents)
    assert [n for n, _ in files] == [8] and len(files[0][1]) == 1 + 44 * 120 + 16
    assert po.load_index(PRK, files) == sorted(ents)
    empty = po.push_and_flush(PRK, 0, [])
    assert empty[0][0] == 1 and len(empty[0][1]) == 17 and po.load_index(PRK, empty) == []
    with pytest.raises(po.CryptoError):
        po.load_index(PRK, [(9, files[0][1])])  # wrong file number = wrong nonce


# ------------------------------------------------------------------ GPU

def _blob_set(n_sizes, seed):
    rng = np.random.default_rng(seed)
    datas = [splitmix_bytes(seed * 1000 + i, int(n)) for i, n in enumerate(n_sizes)]
    hashes = rng.integers(0, 256, (len(datas), 32), dtype=np.uint8)
    kinds = rng.integers(0, 2, len(datas)).astype(np.uint8)
    nonces = rng.integers(0, 256, (len(datas), 12), dtype=np.uint8)
    return datas, hashes, kinds, nonces


def _concat(datas, align=1):
    offs, cur = [], 0
    for d in datas:
        offs.append(cur)
        cur += len(d) + (-(len(d)) % align)
    buf = np.zeros(max(cur, 1), dtype=np.uint8)
    for o, d in zip(offs, datas):
        buf[o:o + len(d)] = np.frombuffer(d, dtype=np.uint8)
    return buf, np.asarray(offs, dtype=np.uint64), np.asarray([len(d) for d in datas], dtype=np.uint64)


def _oracle_packs(po, datas, hashes, kinds, nonces, ids, store=True):
    blobs = [(bytes(hashes[i]), int(kinds[i]), bytes(nonces[i]),
              po.seal_blob_payload(PRK, hashes[i], nonces[i], po.zstd_store(d) if store else d))
             for i, d in enumerate(datas)]
    return po.write_packfiles(PRK, blobs, [bytes(x) for x in ids])


@pytest.mark.gpu
@pytest.mark.parametrize("seed,sizes", [
    (1, [0, 1, 15, 16, 17, 131071, 131072, 131073, 262147, 1 << 20, 3 << 20, 5, 3 << 20, 77]),
    (2, list(np.random.default_rng(9).integers(0, 3 << 20, 24))),
])
def test_pack_build_matches_oracle(ctx, po, seed, sizes):
    z = _zstd()
    datas, hashes, kinds, nonces = _blob_set(sizes, seed)
    src, offs, lens = _concat(datas, align=1 + seed)  # ragged source offsets
    plan, total = ctx.pack_plan(lens)
    ids = np.random.default_rng(seed + 50).integers(0, 256, (len(plan), 12), dtype=np.uint8)
    got = ctx.pack_build(PRK, src, offs, lens, hashes, kinds, nonces, plan, total, ids)
    want = _oracle_packs(po, datas, hashes, kinds, nonces, ids)
    assert len(want) == len(plan)
    for p, (pid, buf) in zip(plan, want):
        assert got[int(p["offset"]):int(p["offset"] + p["size"])].tobytes() == buf
    # and every blob reads back through the reference's reader path + zstd
    for i, d in enumerate(datas):
        p = plan[np.searchsorted(plan["first_blob"], i, side="right") - 1]
        buf = got[int(p["offset"]):int(p["offset"] + p["size"])].tobytes()
        pid = bytes(ids[list(plan["first_blob"]).index(p["first_blob"])])
        kind, payload = po.get_blob(PRK, pid, buf, bytes(hashes[i]))
        assert kind == kinds[i] and z.decompress(payload) == d


@pytest.mark.gpu
def test_pack_build_device_precompressed(ctx, po):
    """Caller-made zstd frames (libzstd level 3 on compressible data), device buffers."""
    import torch
    z = _zstd()
    raw = [bytes(5000) + splitmix_bytes(i, 3000) * 3 for i in range(9)] + [b"x" * 100000]
    datas = [z.compress(d) for d in raw]
    _, hashes, kinds, nonces = _blob_set([len(d) for d in datas], 7)
    src, offs, lens = _concat(datas)
    plan, total = ctx.pack_plan(lens, flags=0)
    ids = np.random.default_rng(8).integers(0, 256, (len(plan), 12), dtype=np.uint8)
    d_src = torch.from_numpy(src).cuda()
    d_out = torch.zeros(total, dtype=torch.uint8, device="cuda")
    ctx.pack_build_device(PRK, d_src.data_ptr(), offs, lens, hashes, kinds, nonces, plan, ids, d_out.data_ptr(),
                          flags=0)
    torch.cuda.synchronize()
    got = d_out.cpu().numpy().tobytes()
    want = b"".join(b for _, b in _oracle_packs(po, datas, hashes, kinds, nonces, ids, store=False))
    assert got == want
    for i, d in enumerate(raw):
        pid, buf = [(bytes(ids[k]), got[int(p["offset"]):int(p["offset"] + p["size"])]) for k, p in enumerate(plan)
                    if p["first_blob"] <= i < p["first_blob"] + p["n_blobs"]][0]
        assert z.decompress(po.get_blob(PRK, pid, buf, bytes(hashes[i]))[1]) == d


@pytest.mark.gpu
def test_pack_compressed_chain_matches_oracle(ctx, po, oracle):
    """compress_encrypt_blob + write_packfiles end to end on the device (pack.rs:58-80, 115-227):
    level-3 frames of a queue of mixed blobs (text, repeats, runs, random, tiny) staged by
    bw_pack_compress_device, the reference's grouping over the frame sizes, and the sealed
    packfiles from bw_pack_build_compressed -- equal byte for byte to the oracle chain (the zstd
    restatement, pinned to libzstd level 3, then seal + serialize) and read back through get_blob
    + libzstd.  The queue sits at ragged device offsets and spans several packfiles."""
    import torch
    import zstd_corpus
    z = _zstd()
    rng = np.random.default_rng(31)
    kinds_c = ["text", "repeats", "runs", "random", "tokens", "mixed"]
    raw = [zstd_corpus.blob(kinds_c[i % 6], int(n), i) for i, n in
           enumerate(list(rng.integers(0, 3 << 20, 18)) + [0, 1, 5, 3 << 20, 131072, 131073])]
    src, offs, lens = _concat(raw, align=3)
    _, hashes, kinds, nonces = _blob_set([len(d) for d in raw], 41)
    d_src = torch.from_numpy(src).cuda()
    fl = ctx.pack_compress_device(d_src.data_ptr(), offs, lens)
    frames = [oracle.zstd3_compress(d) for d in raw]
    assert [int(x) for x in fl] == [len(f) for f in frames]
    plan, total = ctx.pack_plan(fl, flags=0)
    assert len(plan) > 2
    ids = rng.integers(0, 256, (len(plan), 12), dtype=np.uint8)
    d_out = torch.zeros(total, dtype=torch.uint8, device="cuda")
    ctx.pack_build_compressed(PRK, hashes, kinds, nonces, plan, ids, d_out.data_ptr())
    torch.cuda.synchronize()
    got = d_out.cpu().numpy().tobytes()
    want = b"".join(b for _, b in _oracle_packs(po, frames, hashes, kinds, nonces, ids, store=False))
    assert got == want
    for i, d in enumerate(raw):
        k = int(np.searchsorted(plan["first_blob"], i, side="right") - 1)
        p = plan[k]
        buf = got[int(p["offset"]):int(p["offset"] + p["size"])]
        assert z.decompress(po.get_blob(PRK, bytes(ids[k]), buf, bytes(hashes[i]))[1]) == d
    # the host forms give the same packfiles
    fl2 = ctx.pack_compress(raw)
    assert np.array_equal(fl2, fl)
    assert ctx.pack_build_compressed_host(PRK, hashes, kinds, nonces, plan, total, ids).tobytes() == want
    # an empty queue stages nothing and builds nothing
    assert ctx.pack_compress_device(d_src.data_ptr(), [], []).size == 0
    plan0, total0 = ctx.pack_plan(np.zeros(0, np.uint64), flags=0)
    assert len(plan0) == 0 and total0 == 0
    ctx.pack_build_compressed(PRK, np.zeros((0, 32), np.uint8), [], np.zeros((0, 12), np.uint8), plan0,
                              np.zeros((0, 12), np.uint8), d_out.data_ptr())
    torch.cuda.synchronize()
    # a plan that does not cover the staged queue is refused
    fl = ctx.pack_compress_device(d_src.data_ptr(), offs, lens)
    from backuwup_amd._lib import BwError
    with pytest.raises(BwError):
        ctx.pack_build_compressed(PRK, hashes, kinds, nonces, plan[:1], ids, d_out.data_ptr())


@pytest.mark.gpu
def test_pack_build_blob_count_limit(ctx, po):
    """100 003 tiny caller payloads: the first packfile closes at PACKFILE_MAX_BLOBS (a 5-byte Vec
    length).  Store frames never get there (>= 33 bytes per blob reach 3 MiB first)."""
    n = po.PACKFILE_MAX_BLOBS + 3
    rng = np.random.default_rng(12)
    lens = rng.integers(0, 4, n).astype(np.uint64)
    src = rng.integers(0, 256, int(lens.sum()) + 1, dtype=np.uint8)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    hashes = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    kinds = np.zeros(n, dtype=np.uint8)
    nonces = rng.integers(0, 256, (n, 12), dtype=np.uint8)
    plan, total = ctx.pack_plan(lens, flags=0)
    assert plan["n_blobs"].tolist() == [po.PACKFILE_MAX_BLOBS, 3]
    ids = rng.integers(0, 256, (2, 12), dtype=np.uint8)
    got = ctx.pack_build(PRK, src, offs, lens, hashes, kinds, nonces, plan, total, ids, flags=0)
    # the second packfile in full, and the first one's header, against the oracle
    datas = [src[int(o):int(o + l)].tobytes() for o, l in zip(offs, lens)]
    tail = _oracle_packs(po, datas[-3:], hashes[-3:], kinds[-3:], nonces[-3:], ids[1:], store=False)
    assert got[int(plan[1]["offset"]):].tobytes() == tail[0][1]
    hl = int(plan[0]["header_len"])
    hdr = po.oracle.open_blob(PRK, b"header", bytes(ids[0]), got[8:8 + hl].tobytes())
    assert hdr[:5] == b"\xfc\xa0\x86\x01\x00"
    ents = po.deserialize_header(hdr)
    assert len(ents) == po.PACKFILE_MAX_BLOBS
    off = 0
    for i in (0, 1, 99999):
        h, kind, comp, length, offset = ents[i]
        assert h == bytes(hashes[i]) and length == int(lens[i]) + 16
    for i in range(len(ents)):
        assert ents[i][4] == off
        off += ents[i][3] + 12


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 1, 50000, 50001])
def test_index_files_build_and_load(ctx, po, n):
    rng = np.random.default_rng(n + 1)
    ents = rng.integers(0, 256, (n, 44), dtype=np.uint8)
    files = ctx.index_files_build(PRK, ents, last_file_num=41)
    want = po.push_and_flush(PRK, 41, [(bytes(e[:32]), bytes(e[32:])) for e in ents])
    assert [f for f, _ in files] == [f for f, _ in want] == list(range(42, 42 + n // 50000 + 1))
    assert [b for _, b in files] == [b for _, b in want]
    ctx.index_reset()
    got = ctx.index_load_files(PRK, files)
    assert got.tobytes() == ents.tobytes()
    # the loaded digests now gate the next backup: all of them are duplicates, new ones are not
    if n:
        probe = np.concatenate([ents[:1000, :32], rng.integers(0, 256, (10, 32), dtype=np.uint8)])
        assert ctx.index_check_insert(probe).tolist() == [1] * min(n, 1000) + [0] * 10


@pytest.mark.gpu
def test_index_load_errors(ctx, po):
    from backuwup_amd._lib import BW_ECRYPTO, BW_EFORMAT, BwError
    ents = [(bytes([i]) * 32, bytes([i]) * 12) for i in range(5)]
    good = po.push_and_flush(PRK, 0, ents)
    bad = bytearray(good[0][1])
    bad[3] ^= 0x40
    for files, rc in [([good[0], (2, bytes(bad))], BW_ECRYPTO),
                      ([(5, good[0][1])], BW_ECRYPTO),  # the nonce is the file number
                      ([(1, b"\x00" * 10)], BW_ECRYPTO),  # shorter than the tag
                      ([(3, po.oracle.seal_blob(PRK, b"index", po.counter_to_nonce(3),
                                                po.index_plaintext(ents) + b"\x00"))], BW_EFORMAT),
                      ([(3, po.oracle.seal_blob(PRK, b"index", po.counter_to_nonce(3), b"\x02" + bytes(44)))],
                       BW_EFORMAT),
                      ([(3, po.oracle.seal_blob(PRK, b"index", po.counter_to_nonce(3), b"\xff"))], BW_EFORMAT)]:
        ctx.index_reset()
        with pytest.raises(BwError) as e:
            ctx.index_load_files(PRK, files)
        assert e.value.rc == rc
        assert ctx.index_size() == 0  # nothing seeded
    assert ctx.index_load_files(PRK, good).shape == (5, 44)


@pytest.mark.gpu
def test_two_backups_through_index_files(ctx, po):
    """The reference's flow across two backups (BlobIndex::new -> load, add_blob gate, write_packfiles,
    flush): backup 1 chunks, hashes and gates a corpus, packs its unique blobs and writes index files;
    backup 2 starts from a fresh context seeded only by those files and sees every unchanged chunk
    as a duplicate -- only the chunks around an edit are new -- and its new blobs pack and read back."""
    import torch
    from backuwup_amd import Context
    z = _zstd()
    files = [_smb(700 + i, n) for i, n in enumerate([5 << 20, 3 << 20, 700000, 9 << 20, 4096, 0])]
    lens = np.array([len(f) for f in files], dtype=np.uint64)
    offs = np.concatenate([[0], np.cumsum((lens + 15) // 16 * 16)[:-1]]).astype(np.uint64)
    buf = np.zeros(int(offs[-1] + lens[-1]) + 16, dtype=np.uint8)
    for o, f in zip(offs, files):
        buf[int(o):int(o) + len(f)] = f
    rng = np.random.default_rng(77)

    def backup(c, data, seed_files):
        c.index_reset()
        if seed_files:
            c.index_load_files(PRK, seed_files, want_entries=False)
        res = c.process_files(data, offs, lens)
        u = res[res["is_dup"] == 0]
        plan, total = c.pack_plan(u["length"].astype(np.uint64))
        ids = rng.integers(0, 256, (len(plan), 12), dtype=np.uint8)
        nonces = rng.integers(0, 256, (len(u), 12), dtype=np.uint8)
        src_off = offs[u["file"].astype(np.int64)] + u["offset"]
        packs = c.pack_build(PRK, data, src_off, u["length"], u["digest"], np.zeros(len(u), np.uint8), nonces, plan,
                             total, ids) if len(u) else np.zeros(0, np.uint8)
        ents = []
        for k, p in enumerate(plan):
            for i in range(int(p["first_blob"]), int(p["first_blob"] + p["n_blobs"])):
                ents.append(np.concatenate([u["digest"][i], ids[k]]))
        return res, u, plan, ids, packs, np.array(ents, dtype=np.uint8).reshape(-1, 44), src_off

    c2 = Context(0)
    try:
        res1, u1, plan1, ids1, packs1, ents1, _ = backup(ctx, buf, None)
        assert len(u1) == len(res1)  # distinct random files: nothing repeats within backup 1
        index_files = ctx.index_files_build(PRK, ents1, last_file_num=0)
        # backup 2: same corpus with 100 bytes inserted into file 3 (a shift that CDC resyncs after)
        edited = buf.copy()
        o3 = int(offs[3])
        edited[o3 + 4000000:o3 + int(lens[3])] = buf[o3 + 3999900:o3 + int(lens[3]) - 100]
        res2, u2, plan2, ids2, packs2, ents2, src2 = backup(c2, edited, index_files)
        new = set(map(bytes, u2["digest"]))
        old = set(map(bytes, u1["digest"]))
        assert new.isdisjoint(old) and 0 < len(u2) <= 4  # the edited chunk(s) and the file's new tail
        assert set(u2["file"].tolist()) == {3}
        # the new blobs read back from backup 2's packfiles
        for k, p in enumerate(plan2):
            pf = packs2[int(p["offset"]):int(p["offset"] + p["size"])].tobytes()
            for i in range(int(p["first_blob"]), int(p["first_blob"] + p["n_blobs"])):
                kind, payload = po.get_blob(PRK, bytes(ids2[k]), pf, bytes(u2["digest"][i]))
                want = edited[int(src2[i]):int(src2[i] + u2["length"][i])].tobytes()
                assert z.decompress(payload) == want
    finally:
        c2.close()


# ------------------------------------------------------------------ the reference's write cadence

def _session_case(seed, n, n_distinct, p_seeded, size_hi, flags_store=True):
    rng = np.random.default_rng(seed)
    pool = rng.integers(0, 256, (n_distinct, 32), dtype=np.uint8)
    plen = rng.integers(0, size_hi, n_distinct).astype(np.uint64)
    pick = rng.integers(0, n_distinct, n) if n_distinct < n else np.arange(n)
    seeded = {bytes(pool[i]) for i in range(n_distinct) if rng.random() < p_seeded}
    return pool, plen, pick, seeded


@pytest.mark.parametrize("seed,n,nd,ps,hi,store", [
    (1, 3000, 2000, 0.1, 300_000, True),     # many drains, pending duplicates, seeded blobs
    (2, 500, 60, 0.0, 2 << 20, True),        # big blobs: nearly every add triggers a drain
    (3, 4000, 4000, 0.2, 5000, True),        # small blobs: long drains, one remainder per drain
    (4, 250_000, 250_000, 0.05, 1, False),   # caller frames of 0 B: the blob-count trigger fires
])
def test_session_cadence_matches_reference(po, seed, n, nd, ps, hi, store):
    """bw_pack_plan_session vs a literal restatement of add_blob / trigger_write_if_desired /
    write_packfiles / flush (oracle/pack_oracle.py session_packfiles), given the gate verdicts
    the device produces (first occurrence in canonical order, seeded digests duplicates)."""
    from backuwup_amd import Context
    from backuwup_amd._lib import BW_PACK_ZSTD_STORE
    pool, plen, pick, seeded = _session_case(seed, n, nd, ps, hi)
    digests = pool[pick]
    seen, is_dup = set(seeded), np.zeros(n, np.uint8)
    for i, d in enumerate(digests):
        k = d.tobytes()
        is_dup[i] = k in seen
        seen.add(k)
    payload = plen[pick]
    flags = BW_PACK_ZSTD_STORE if store else 0
    sealed = [(po.zstd_store_size(int(x)) if store else int(x)) + 16 for x in payload]
    want = po.session_packfiles([(digests[i].tobytes(), sealed[i]) for i in range(n)], seeded)
    plan, total = Context.pack_plan_session(digests, is_dup, payload, flags)
    uniq = [digests[i].tobytes() for i in range(n) if not is_dup[i]]
    got = [uniq[int(p["first_blob"]):int(p["first_blob"] + p["n_blobs"])] for p in plan]
    assert got == want
    assert sum(len(g) for g in got) == len(uniq)
    if not store:
        assert any(len(g) == 100_000 for g in got)
    # sizes/offsets are write_packfiles' (the same per-packfile layout as bw_pack_plan's)
    assert total == sum(int(p["size"]) for p in plan)


@pytest.mark.gpu
def test_session_cadence_packfiles_on_gpu(ctx, po):
    """A session's blobs gated on the GPU, packed with the reference's cadence: every packfile,
    remainders included, is byte-identical to the format oracle's serialization of the group the
    literal cadence restatement assigns."""
    from backuwup_amd.synth import small_files
    data, offs, lens = small_files(1200, seed=19, lo=1000, hi=400_000)
    ctx.index_reset()
    res = ctx.process_files(data, offs, lens)
    plan, total = ctx.pack_plan_session(res["digest"], res["is_dup"], res["length"])
    u = res[res["is_dup"] == 0]
    want = po.session_packfiles([(bytes(r["digest"]), po.zstd_store_size(int(r["length"])) + 16) for r in res])
    assert len(plan) == len(want) and any(int(p["n_blobs"]) < 10 for p in plan)  # remainders exist
    rng = np.random.default_rng(5)
    nonces = rng.integers(0, 256, (len(u), 12), dtype=np.uint8)
    ids = rng.integers(0, 256, (len(plan), 12), dtype=np.uint8)
    src_off = offs[u["file"].astype(np.int64)] + u["offset"]
    out = ctx.pack_build(PRK, data, src_off, u["length"], u["digest"], np.zeros(len(u), np.uint8), nonces, plan,
                         total, ids)
    for k, p in enumerate(plan):
        f, c = int(p["first_blob"]), int(p["n_blobs"])
        assert [bytes(d) for d in u["digest"][f:f + c]] == want[k]
        blobs = [(bytes(u["digest"][i]), 0, bytes(nonces[i]),
                  po.seal_blob_payload(PRK, u["digest"][i], nonces[i],
                                       po.zstd_store(data[int(src_off[i]):int(src_off[i] + u["length"][i])])))
                 for i in range(f, f + c)]
        assert out[int(p["offset"]):int(p["offset"] + p["size"])].tobytes() == po.serialize_packfile(PRK, bytes(ids[k]), blobs)
