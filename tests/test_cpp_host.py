"""The C++ host mirror (backuwup_amd/host/backuwup.hpp) compiled against the C ABI and run on
the GPU, checked against the oracle."""
import os
import subprocess

import pytest

from backuwup_amd.synth import splitmix_bytes

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def build(tmp_path):
    exe = tmp_path / "host_parity"
    libdir = os.path.join(ROOT, "backuwup_amd")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-I", os.path.join(ROOT, "include"),
                           os.path.join(HERE, "cpp", "host_parity.cpp"), "-L", libdir, "-lbackuwup_amd",
                           "-Wl,-rpath," + libdir, "-o", str(exe)])
    return exe


def test_cpp_mirror_compiles(tmp_path):
    assert build(tmp_path).exists()


@pytest.mark.gpu
def test_cpp_mirror_parity(tmp_path, oracle):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    out = subprocess.check_output([str(build(tmp_path))], timeout=300).decode().splitlines()
    data = splitmix_bytes(0, 8400953)
    want = oracle.fastcdc(data, 262144, 1048576, 3145728)
    chunks = [l.split() for l in out if l.startswith("chunk ")]
    assert len(chunks) == len(want)
    for (_, h, o, l, d), (wh, wo, wl) in zip(chunks, want):
        assert (int(h), int(o), int(l)) == (wh, wo, wl)
        assert d == oracle.blake3(data[wo:wo + wl]).hex()
    assert "invalid-params rc=-1" in out
    # a seeded -> duplicate; b new then duplicate; index holds 2
    assert "gate 0 1 0 2" in out
    assert "too-large ok" in out
    tb = bytes.fromhex([l.split()[1] for l in out if l.startswith("tree-bytes ")][0])
    children = b"".join(oracle.blake3(data[wo:wo + wl]) for _, wo, wl in want)
    assert tb == oracle.tree_serialize(0, "a5.bin", len(data), 1700000000, None, children)
    th = [l.split()[1] for l in out if l.startswith("tree-hash ")][0]
    assert th == oracle.blake3(tb).hex()
    # packfiles and index files (pack.rs:115-227, blob_index.rs:151-240) against the format oracle
    from oracle import pack_oracle as po
    prk = bytes(range(0x40, 0x60))
    sizes = [0, 1000, 3 << 20, 70000]
    blobs = []
    for i, n in enumerate(sizes):
        d = data[5 * i:5 * i + n].tobytes()
        h = oracle.blake3(d)
        nonce = bytes(7 * i + k for k in range(12))
        blobs.append((h, 1 if i == 3 else 0, nonce, po.seal_blob_payload(prk, h, nonce, po.zstd_store(d))))
    groups = po.plan_packfiles([len(b[3]) for b in blobs])
    ids = [bytes(0xa0 + 16 * p + k for k in range(12)) for p in range(len(groups))]
    want = po.write_packfiles(prk, blobs, ids)
    got = [bytes.fromhex(l.split()[2]) for l in out if l.startswith("packfile ")]
    assert got == [b for _, b in want] and len(got) == 2
    ents = [(b[0], ids[0 if i < 3 else 1]) for i, b in enumerate(blobs)]
    files = [(int(l.split()[1]), bytes.fromhex(l.split()[2])) for l in out if l.startswith("index ")]
    assert files == po.push_and_flush(prk, 9, ents)
    assert "index-load 4 1" in out
    # the level-3 chain (write_packfiles_zstd) against the oracle chain: zstd restatement (pinned
    # to libzstd level 3) -> seal -> packfile layout
    zb = []
    for j, n in enumerate([0, 5000, 200000, (1 << 20) + 17]):
        d = bytes(ord("a") + ((i * (j + 3)) // 7) % 26 for i in range(n))
        h = oracle.blake3(d)
        nonce = bytes(3 * j + k + 1 for k in range(12))
        zb.append((h, 0, nonce, po.seal_blob_payload(prk, h, nonce, oracle.zstd3_compress(d))))
    zgroups = po.plan_packfiles([len(b[3]) for b in zb])
    zids = [bytes(0x30 + 16 * p + k for k in range(12)) for p in range(len(zgroups))]
    zwant = po.write_packfiles(prk, zb, zids)
    zgot = [bytes.fromhex(l.split()[2]) for l in out if l.startswith("packfile-zstd ")]
    assert zgot == [b for _, b in zwant] and len(zgot) >= 1
    # all-empty queue (one empty file): one packfile holding one empty level-3 frame
    e = (oracle.blake3(b""), 0, zb[0][2], po.seal_blob_payload(prk, oracle.blake3(b""), zb[0][2],
                                                             oracle.zstd3_compress(b"")))
    ewant = po.write_packfiles(prk, [e], zids[:1])
    egot = [bytes.fromhex(l.split()[2]) for l in out if l.startswith("packfile-zstd-empty ")]
    assert egot == [b for _, b in ewant]

    # NodeSession: four ranks of one process on device 0 (bw_comm_init_local), against one oracle
    # index over the canonical order of the three batches
    import numpy as np
    sizes, srcs, parts = [], [], []
    for i in range(603):
        src = i - 3 if (i < 600 and i % 10 == 3) else i
        sizes.append(4096 + (src * 7919) % 61440 if src < 600 else (1 << 20) + 1 + src * 12345)
        srcs.append(src)
    corpus = np.concatenate([splitmix_bytes(1000 + s, n) for s, n in zip(srcs, sizes)])
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
    lens = np.asarray(sizes, np.uint64)
    ns = [l.split() for l in out if l.startswith("ns ")]
    ix = oracle.Index()
    k = 0
    for bi, (lo, hi) in enumerate([(0, 301), (600, 603), (0, 301)]):
        want = oracle.process_files(corpus, offs[lo:hi], lens[lo:hi], index=ix, threads=8)
        for w in want:
            _, b, f, o, ln, gh, d, dup = ns[k]
            assert (int(b), int(f), int(o), int(ln), int(gh), d, int(dup)) == \
                (bi, lo + int(w["file"]), int(w["offset"]), int(w["length"]), int(w["gear_hash"]),
                 bytes(w["digest"]).hex(), int(w["is_dup"])), (bi, k)
            k += 1
    assert k == len(ns) and sum(int(x[-1]) for x in ns) > 0
    # the drop-in pool over [0, 0]: every digest equal to the oracle's
    ph = [l.split() for l in out if l.startswith("ph ")]
    assert len(ph) == 400
    for _, o, n, d in ph:
        assert d == oracle.blake3(corpus[int(o):int(o) + int(n)]).hex(), (o, n)
    # FastCDC on the pool (kept digests) + Pool::hash per chunk: the Rust drop-ins' loop
    pf = [l.split() for l in out if l.startswith("pf ")]
    nk = 0
    for f in (600, 601, 602):
        got = [(int(h), int(o), int(n), d) for _, ff, h, o, n, d in pf if int(ff) == f]
        fb = corpus[int(offs[f]):int(offs[f] + lens[f])]
        want = [(h, o, n, oracle.blake3(fb[o:o + n]).hex()) for h, o, n in oracle.fastcdc(fb, 262144, 1048576, 3145728)]
        assert got == want, f
        nk += len(want)
    assert [l for l in out if l.startswith("pf-kept ")] == ["pf-kept %d" % nk]
