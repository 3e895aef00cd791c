"""Tree blobs (§8f row 1): split_serialize_tree + add_tree_to_blobs (dir_packer.rs:314-390).

The bincode layout is pinned three ways: a hand-derived literal from the bincode 1.3.3 legacy
format (fixint little endian, u32 enum tags, u64 lengths, one-byte Option tags, [u8; 32] raw),
the pure-Python oracle restatement, and the library's host serializer.  The GPU test hashes and
dedups split and unsplit trees through the library and compares with the oracle.
"""
import struct

import numpy as np
import pytest

from backuwup_amd import make_tree, tree_serialize
from backuwup_amd._lib import BW_EINVAL


def test_tree_bincode_layout_literal():
    # Tree { kind: File, name: "a", metadata: { size: Some(3), mtime: None, ctime: Some(5) },
    #        children: [00 01 .. 1f], next_sibling: None }
    want = bytes.fromhex(
        "00000000"              # TreeKind::File (u32 variant index)
        "0100000000000000" "61"  # String: u64 length + UTF-8
        "01" "0300000000000000"  # size: Some(3)
        "00"                     # mtime: None
        "01" "0500000000000000"  # ctime: Some(5)
        "0100000000000000") + bytes(range(32)) + b"\x00"  # Vec<BlobHash> + next_sibling: None
    assert tree_serialize(make_tree(0, "a", 3, None, 5, bytes(range(32)))) == want
    # Dir with a sibling and no children
    sib = bytes(range(100, 132))
    want = struct.pack("<IQ", 1, 3) + b"dir" + b"\x00\x00\x00" + struct.pack("<Q", 0) + b"\x01" + sib
    assert tree_serialize(make_tree(1, "dir"), next_sibling=sib) == want


def test_tree_serialize_matches_oracle(oracle):
    rng = np.random.default_rng(12)
    names = ["", "a", "photo.jpg", "été — 日本.txt", "x" * 300, "\U0001f600"]
    for i in range(200):
        kind = int(rng.integers(2))
        name = names[i % len(names)]
        meta = [None if rng.integers(3) == 0 else int(rng.integers(0, 2**63)) for _ in range(3)]
        nch = int(rng.choice([0, 1, 2, 17, 300]))
        ch = rng.integers(0, 256, nch * 32, dtype=np.uint8).tobytes()
        sib = rng.integers(0, 256, 32, dtype=np.uint8).tobytes() if rng.integers(2) else None
        got = tree_serialize(make_tree(kind, name, *meta, ch), next_sibling=sib)
        assert got == oracle.tree_serialize(kind, name, *meta, ch, sib), i


def test_tree_serialize_rejects_bad_kind():
    t, keep = make_tree(0, "f")
    t.kind = 2
    with pytest.raises(RuntimeError) as e:  # BwError (compared by rc: test_capi reloads _lib)
        tree_serialize((t, keep))
    assert e.value.rc == BW_EINVAL


def test_split_tree_sibling_chain(oracle):
    ch = np.random.default_rng(3).integers(0, 256, 25001 * 32, dtype=np.uint8).tobytes()
    pieces = oracle.split_serialize_tree(1, "big", 1, 2, 3, ch)
    assert len(pieces) == 3
    for k, (data, h) in enumerate(pieces):
        assert h == oracle.blake3(data)
        n = struct.unpack_from("<Q", data, 4 + 8 + 3 + 27)[0]
        assert n == (10000 if k < 2 else 5001)
        if k < 2:
            assert data[-33] == 1 and data[-32:] == pieces[k + 1][1]
        else:
            assert data[-1] == 0


@pytest.mark.gpu
def test_tree_blobs_match_oracle(ctx, oracle):
    rng = np.random.default_rng(5)
    specs = []
    for i in range(300):
        nch = int(rng.choice([0, 1, 3, 40, 1000]))
        specs.append((int(rng.integers(2)), "f%05d" % i, 1000 + i, 1700000000 + i, None,
                      rng.integers(0, 256, nch * 32, dtype=np.uint8).tobytes()))
    specs.append((1, "huge", None, None, None, rng.integers(0, 256, 23456 * 32, dtype=np.uint8).tobytes()))
    specs += specs[:20]  # identical trees later in the batch: duplicates at the gate
    ctx.index_reset()
    hashes, blobs = ctx.tree_blobs([make_tree(*s) for s in specs])
    ix = oracle.Index()
    k = 0
    for i, s in enumerate(specs):
        pieces = oracle.split_serialize_tree(*s)
        assert bytes(hashes[i]) == pieces[0][1], i
        for p, (data, h) in enumerate(pieces):
            b = blobs[k]
            assert (int(b["tree"]), int(b["piece"]), int(b["length"])) == (i, p, len(data))
            assert bytes(b["hash"]) == h
            dup = ix.is_blob_duplicate(h)
            if not dup:
                ix.insert(h)
            assert int(b["is_dup"]) == int(dup), (i, p)
            k += 1
    assert k == len(blobs)
    assert blobs["is_dup"][-20:].all() and not blobs["is_dup"][:301].any()
