"""Pipelined batches on the GPU, all through the C ABI and compared bit for bit with the oracle:

  * tickets: several batches queued on one context before any is read (ring of result slots)
  * bw_submit_host (BASELINE C5): batches copied from pinned host memory on
    the copy stream while the previous batch computes; pageable memory through pinned staging
  * one index shared by two contexts on two streams: one backup session with batches in flight,
    gated in submission order (BlobIndex behind the packer mutex, packfile/mod.rs:77,
    blob_index.rs:130-148)
  * an undersized candidate array: the walkers test the bytes past its end, no re-run
  * index errors of the device-side gate, and the ADVICE r1 staging regression
The dedup oracle over several batches is one oracle.Index fed the batches in order: the canonical
order of a session is batch order, then file order, then chunk offset.
"""
import numpy as np
import pytest

from backuwup_amd import Context, Index, make_params, make_tree
from backuwup_amd._lib import (BW_ESTATE, BW_F_NO_DEDUP, BW_OPT_CAND_CAP, BW_OPT_DEPTH,
                               BW_OPT_STAGE_CHUNK, BwError)
from backuwup_amd.synth import small_files, splitmix_bytes, tree_corpus, vm_image_variants

pytestmark = pytest.mark.gpu

BK = (262144, 1048576, 3145728)
SMALL = (64, 256, 1024)
MID = (4096, 16384, 65536)


def blobs_equal(a, b, what=""):
    assert a.shape == b.shape, (what, a.shape, b.shape)
    for f in ("file", "offset", "length", "gear_hash", "is_dup"):
        assert np.array_equal(a[f], b[f]), (what, f)
    assert np.array_equal(a["digest"], b["digest"]), what


def oracle_session(oracle, batches, seed_digests=b"", params=BK):
    """The oracle over consecutive batches gated by one index."""
    ix = oracle.Index(seed_digests)
    return [oracle.process_files(d, o, l, *params, index=ix, threads=8) for d, o, l in batches]


def _slices(data, offs, lens, bounds):
    """Batches of files [a, b) as (bytes, file_off relative to the batch, file_len)."""
    out = []
    for a, b in bounds:
        lo, hi = int(offs[a]), int(offs[b - 1] + lens[b - 1])
        out.append((np.ascontiguousarray(data[lo:hi]), (offs[a:b] - np.uint64(lo)).astype(np.uint64),
                    lens[a:b].astype(np.uint64)))
    return out


def test_tickets_ring(oracle):
    import torch
    data, offs, lens = small_files(4000, seed=31)
    batches = _slices(data, offs, lens, [(0, 1000), (1000, 2000), (2000, 3000), (3000, 4000)])
    want = oracle_session(oracle, batches)
    devs = [torch.from_numpy(d).cuda() for d, _, _ in batches]
    torch.cuda.synchronize()
    with Context(0) as c:
        c.set_option(BW_OPT_DEPTH, 3)
        c.index_reset()
        tickets = [c.submit_device(t.data_ptr(), d.size, o, l) for t, (d, o, l) in zip(devs, batches)]
        assert tickets == sorted(tickets) and len(set(tickets)) == 4
        with pytest.raises(BwError) as e:  # the ring holds 3: the first batch was dropped
            c.wait(tickets[0])
        assert e.value.rc == BW_ESTATE
        for k in (3, 1, 2, 3):  # any order, repeatable
            blobs_equal(c.wait(tickets[k]), want[k], k)
        blobs_equal(c.results(), want[3])  # bw_results = the most recent batch
        with pytest.raises(BwError):
            c.wait(tickets[3] + 1)


def _diag_lib():
    """True when the loaded library is the diagnostic build (BW_DIAG variants compiled in)."""
    from backuwup_amd import _lib
    return _lib.LIB_PATH.endswith("_debug.so")


def test_split_batches_match_unsplit(oracle):
    """Four batches of a tree corpus over two contexts sharing an index, depth 3 rings: the blobs
    (file indices in the batch's numbering), digests and verdicts equal the oracle, also from pinned
    host memory.  With the diagnostic build (BW_LIB = the BW_DIAG library) also with BW_OPT_SPLIT 2:
    multi-file batches of 64 MiB - 4 GiB as a head and a tail part (helper context), whose batches
    have no single device view; the product library refuses that variant (measured slower)."""
    import torch
    from backuwup_amd._lib import BW_OPT_SPLIT
    data, offs, lens = tree_corpus(320 << 20, seed=91, max_file=40 << 20)
    nf, cum = len(lens), np.cumsum(lens)
    b1 = int(np.searchsorted(cum, cum[-1] / 3)) + 1
    b2 = int(np.searchsorted(cum, 2 * cum[-1] / 3)) + 1
    bounds = [(0, b1), (b1, b2), (b2, nf), (0, b1)]  # about a third of the bytes each
    batches = _slices(data, offs, lens, bounds)
    assert all(int(l.sum()) >= (64 << 20) and len(l) >= 2 for _, _, l in batches)
    want = oracle_session(oracle, batches)
    devs = [torch.from_numpy(d).cuda() for d, _, _ in batches]
    torch.cuda.synchronize()
    if not _diag_lib():
        with Context(0) as c, pytest.raises(BwError):
            c.set_option(BW_OPT_SPLIT, 2)
    for split in ((2, 1) if _diag_lib() else (1,)):
        ix = Index(0)
        cs = [Context(0), Context(0)]
        try:
            for c in cs:
                c.set_stream(torch.cuda.Stream().cuda_stream)
                c.attach_index(ix)
                c.set_option(BW_OPT_SPLIT, split)
                c.set_option(BW_OPT_DEPTH, 3)
            cs[0].index_reset(1 << 16)
            tickets = [cs[k % 2].submit_device(t.data_ptr(), d.size, o, l) for k, (t, (d, o, l)) in
                       enumerate(zip(devs, batches))]
            for k, t in enumerate(tickets):
                blobs_equal(cs[k % 2].wait(t), want[k], (split, k))
            blobs_equal(cs[1].results(), want[3], (split, "results"))
            if split == 2:
                with pytest.raises(BwError) as e:
                    cs[1].batch_views(tickets[3])
                assert e.value.rc == BW_ESTATE
            cs[0].index_check()
        finally:
            for c in cs:
                c.close()
            ix.close()
    # the same batches from pinned host memory on one context
    pinned = []
    for d, _, _ in batches:
        t = torch.empty(d.size, dtype=torch.uint8, pin_memory=True)
        t.numpy()[:] = d
        pinned.append(t)
    with Context(0) as c:
        c.index_reset(1 << 16)
        tickets = [c.submit_host(t.data_ptr(), o, l, data_len=d.size) for t, (d, o, l) in zip(pinned[:2], batches)]
        got = [c.wait(tickets[0])]
        tickets.append(c.submit_host(pinned[2].data_ptr(), batches[2][1], batches[2][2], data_len=batches[2][0].size))
        got.append(c.wait(tickets[1]))
        tickets.append(c.submit_host(pinned[3].data_ptr(), batches[3][1], batches[3][2], data_len=batches[3][0].size))
        got += [c.wait(tickets[2]), c.wait(tickets[3])]
        for k in range(4):
            blobs_equal(got[k], want[k], ("pinned", k))


def test_sync_helpers_leave_held_tickets_alone(oracle):
    """the synchronous helpers (tree blobs, blake3.hash, process_files, fastcdc_chunks)
    run outside the ticket ring.  With the default depth of 2, two submitted batches stay readable
    after them, and bw_results still names the most recent submitted batch."""
    import torch
    data, offs, lens = small_files(2000, seed=61)
    batches = _slices(data, offs, lens, [(0, 1000), (1000, 2000)])
    want = oracle_session(oracle, batches)
    devs = [torch.from_numpy(d).cuda() for d, _, _ in batches]
    torch.cuda.synchronize()
    with Context(0) as c:
        c.index_reset()
        tickets = [c.submit_device(t.data_ptr(), d.size, o, l) for t, (d, o, l) in zip(devs, batches)]
        spec = (0, "f", 5, 1700000000, None, bytes(range(64)))
        hashes, _ = c.tree_blobs([make_tree(*spec)], dedup=False)
        assert bytes(hashes[0]) == oracle.split_serialize_tree(*spec)[0][1]
        m = splitmix_bytes(8, 5000)
        assert c.blake3(m) == oracle.blake3(m)
        assert c.fastcdc_chunks(splitmix_bytes(9, 20000), *SMALL) == oracle.fastcdc(splitmix_bytes(9, 20000), *SMALL)
        sm, so, sl = small_files(50, seed=62)
        pf = c.process_files(sm, so, sl, make_params(flags=BW_F_NO_DEDUP))
        assert np.array_equal(pf["digest"], oracle.process_files(sm, so, sl)["digest"])
        for k in (0, 1):
            blobs_equal(c.wait(tickets[k]), want[k], k)
        blobs_equal(c.results(), want[1])


@pytest.mark.parametrize("nctx,order", [(2, 0), (3, 0), (3, 1)])
def test_shared_index_two_contexts_six_batches(oracle, nctx, order):
    """One session, two (three) contexts on their own streams, one index: six batches of C1 (tree
    corpus) and C4 (small files) data with duplicates across batches and contexts, submitted back
    to back (one batch per context in flight); verdicts equal the oracle over the concatenated
    batches.  order = BW_OPT_ORDER_HASH (scans and leaf passes serialized across the contexts; the
    diagnostic build only)."""
    from backuwup_amd._lib import BW_OPT_ORDER_HASH
    if order and not _diag_lib():
        pytest.skip("BW_OPT_ORDER_HASH is a diagnostic variant (BW_DIAG build)")
    import torch
    t_data, t_offs, t_lens = tree_corpus(48 << 20, seed=77, max_file=6 << 20)
    s_data, s_offs, s_lens = small_files(3000, seed=78)
    nt, ns = len(t_lens), len(s_lens)
    b = _slices(t_data, t_offs, t_lens, [(0, nt // 2), (nt // 2, nt)]) + \
        _slices(s_data, s_offs, s_lens, [(0, ns // 2), (ns // 2, ns)])
    batches = [b[0], b[2], b[1], b[3], b[2], b[0]]  # the last two repeat batches first run by the other context
    seed = b"".join(sorted(bytes(x) for x in oracle.process_files(*b[3])["digest"][::5]))
    want = oracle_session(oracle, batches, seed)
    devs = [torch.from_numpy(d).cuda() for d, _, _ in batches]
    torch.cuda.synchronize()
    ix = Index(0)
    cs = [Context(0) for _ in range(nctx)]
    ss = [torch.cuda.Stream() for _ in range(nctx)]
    ca, cb = cs[0], cs[1]
    try:
        for c, st in zip(cs, ss):
            c.set_stream(st.cuda_stream)
            c.attach_index(ix)
            c.set_option(BW_OPT_ORDER_HASH, order)
        ca.index_reset(1 << 16)
        cb.index_seed(np.frombuffer(seed, dtype=np.uint8).reshape(-1, 32))
        got, pending = [None] * len(batches), []
        for k, (t, (d, o, l)) in enumerate(zip(devs, batches)):
            c = cs[k % nctx]
            pending.append((k, c, c.submit_device(t.data_ptr(), d.size, o, l)))
            if len(pending) >= nctx:
                j, cj, tj = pending.pop(0)
                got[j] = cj.wait(tj)
        for j, cj, tj in pending:
            got[j] = cj.wait(tj)
        for k in range(len(batches)):
            blobs_equal(got[k], want[k], k)
        assert got[4]["is_dup"].all() and got[5]["is_dup"].all()
        uniq = {bytes(x) for w in want for x in w["digest"]} | {seed[i:i + 32] for i in range(0, len(seed), 32)}
        assert ca.index_size() == cb.index_size() == len(uniq)
        ca.index_check()
    finally:
        for c in cs:
            c.close()
        ix.close()


def test_submit_host_c5_shaped(oracle):
    """C5's layout at a size the oracle covers: one VM-image family (64 MiB base + 15 variants),
    files 0-7 on rank 2f and 8-15 on rank 2f+1; here both ranks' files go through one context as
    four batches from pinned host memory, each queued while the previous one computes.  Then the
    same batches from pageable memory through small, odd-sized staging chunks."""
    import torch
    # C3's edit density per byte would touch nearly every chunk of a 64 MiB image: fewer edits
    data, offs, lens = vm_image_variants(64 << 20, 16, seed=5, n_indels=4, n_overwrites=2)
    batches = _slices(data, offs, lens, [(0, 4), (4, 8), (8, 12), (12, 16)])
    want = oracle_session(oracle, batches)
    assert sum(int(w["is_dup"].sum()) for w in want) > 0.5 * sum(len(w) for w in want)
    pinned = []
    for d, _, _ in batches:
        t = torch.empty(d.size, dtype=torch.uint8, pin_memory=True)
        t.numpy()[:] = d
        pinned.append(t)
    with Context(0) as c:
        c.index_reset(1 << 14)
        tickets = [c.submit_host(t.data_ptr(), o, l, data_len=d.size) for t, (d, o, l) in zip(pinned[:2], batches)]
        got = [c.wait(tickets[0])]
        tickets.append(c.submit_host(pinned[2].data_ptr(), batches[2][1], batches[2][2], data_len=batches[2][0].size))
        got.append(c.wait(tickets[1]))
        tickets.append(c.submit_host(pinned[3].data_ptr(), batches[3][1], batches[3][2], data_len=batches[3][0].size))
        got += [c.wait(tickets[2]), c.wait(tickets[3])]
        for k in range(4):
            blobs_equal(got[k], want[k], ("pinned", k))
    with Context(0) as c:
        c.set_option(BW_OPT_STAGE_CHUNK, (3 << 20) + 4097)
        c.index_reset(1 << 14)
        tickets = [c.submit_host(d, o, l) for d, o, l in batches]
        for k, t in enumerate(tickets[-2:], start=2):
            blobs_equal(c.wait(t), want[k], ("pageable", k))


def test_submit_host_registered_and_small_params(oracle):
    """A page-locked (bw_host_register) numpy buffer is DMA'd in place; small parameters."""
    import ctypes
    from backuwup_amd import host_register, host_unregister
    rng = np.random.default_rng(41)
    lens = rng.integers(0, 200_000, 60).astype(np.uint64)
    data = splitmix_bytes(42, int(lens.sum()) + 4096)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    want = oracle.process_files(data, offs, lens, *SMALL)
    host_register(data.ctypes.data, data.nbytes)
    try:
        with Context(0) as c:
            c.index_reset()
            t = c.submit_host(data.ctypes.data, offs, lens, make_params(*SMALL), data_len=data.size)
            blobs_equal(c.wait(t), want)
    finally:
        host_unregister(data.ctypes.data)


@pytest.mark.parametrize("cap", [16, 1000, 20000])
def test_candidate_array_truncation(oracle, cap):
    """BW_OPT_CAND_CAP forces a candidate array far too small: every position past the first
    truncated tile is tested by the walkers directly (C_TRUNC), and boundaries stay exact."""
    with Context(0) as c:
        c.set_option(BW_OPT_CAND_CAP, cap)
        for n, p in [((3 << 20) + 11, SMALL), ((8 << 20) + 5, MID), ((40 << 20) + 7, BK)]:
            d = splitmix_bytes(n + cap, n)
            assert c.fastcdc_chunks(d, *p) == oracle.fastcdc(d, *p), (n, p)
        z = np.concatenate([splitmix_bytes(9, 300_000), np.zeros(2_000_000, np.uint8)])
        assert c.fastcdc_chunks(z, *MID) == oracle.fastcdc(z, *MID)
        data, offs, lens = tree_corpus(40 << 20, seed=13, max_file=9 << 20)
        c.index_reset()
        blobs_equal(c.process_files(data, offs, lens, make_params(*MID)),
                    oracle.process_files(data, offs, lens, *MID, threads=8))


def _colliding_digests(seed):
    """Digests built to collide in the index's 64-bit key: 40 groups of 2-12 distinct digests
    that share their first 8 bytes (one group with key 0, one with key 1 -- the old table mapped
    key 0 onto key 1), some sharing 16, 24 or 31 bytes, plus random singletons."""
    rng = np.random.default_rng(seed)
    groups = []
    for g in range(40):
        k = int(rng.integers(2, 13))
        a = rng.integers(0, 256, (k, 32), dtype=np.uint8)
        a[:, :8] = a[0, :8]
        if g == 0:
            a[:, :8] = 0
        elif g == 1:
            a[:, :8] = 0
            a[:, 0] = 1
        elif g % 5 == 2:
            n = int(rng.choice([16, 24, 31]))
            a[:, :n] = a[0, :n]
            a[:, 31] = np.arange(k, dtype=np.uint8) + a[0, 31]  # keep the rows distinct
        groups.append(a)
    a = np.concatenate(groups + [rng.integers(0, 256, (200, 32), dtype=np.uint8)])
    # a group sharing 31 of 32 bytes
    t = np.repeat(rng.integers(0, 256, (1, 32), dtype=np.uint8), 6, axis=0)
    t[:, 31] = np.arange(6, dtype=np.uint8)
    a = np.concatenate([a, t])
    assert len({bytes(x) for x in a}) == len(a)
    return a


def _oracle_verdicts(oracle, seq, seed=b""):
    ix = oracle.Index(seed)
    out = []
    for d in seq:
        dup = ix.is_blob_duplicate(d.tobytes())
        if not dup:
            ix.insert(d.tobytes())
        out.append(int(dup))
    return out


def test_index_key_collisions_bit_exact(oracle):
    """distinct digests that share the table's 64-bit key (and longer prefixes)
    are distinct entries, as in the reference's full-digest HashSet / binary search
    (blob_index.rs:109,130-148).  Host gate, device gate, the exchange owner's bucket gate, a
    seeded index and table growth (rehash) are all bit-exact against oracle.Index, and no call
    reports an error."""
    import torch
    pool = _colliding_digests(7)
    rng = np.random.default_rng(8)
    seed_rows = pool[rng.choice(len(pool), 60, replace=False)]
    seed = np.array(sorted(seed_rows.tolist()), dtype=np.uint8)
    batches = [pool[rng.integers(0, len(pool), n)] for n in (500, 1, 777, 3000)]
    want = _oracle_verdicts(oracle, np.concatenate(batches), b"".join(bytes(x) for x in seed))
    with Context(0) as c:
        # host path, seeded, tiny table hint so the batches force growth + rehash
        c.index_reset(16)
        c.index_seed(seed)
        got = np.concatenate([c.index_check_insert(b) for b in batches])
        assert got.tolist() == want
        c.index_check()
        distinct = {bytes(x) for x in np.concatenate(batches + [seed])}
        assert c.index_size() == len(distinct)
        # device path (the gate of a submitted batch and of bw_index_check_insert_device)
        c.index_reset(16)
        c.index_seed(seed)
        got = []
        for b in batches:
            d = torch.from_numpy(np.ascontiguousarray(b).reshape(-1)).cuda()
            v = torch.full((len(b),), 7, dtype=torch.uint8, device="cuda")
            c.index_check_insert_device(d.data_ptr(), len(b), v.data_ptr())
            torch.cuda.synchronize()
            got.append(v.cpu().numpy())
        assert np.concatenate(got).tolist() == want
        c.index_check()
        # the exchange owner's gate: two source buckets of cap slots, source-major order
        c.index_reset()
        cap = 2000
        src = [pool[rng.integers(0, len(pool), 1500)], pool[rng.integers(0, len(pool), 900)]]
        bk = np.zeros((2, cap, 32), np.uint8)
        for j, s in enumerate(src):
            bk[j, :len(s)] = s
        d_bk = torch.from_numpy(bk.reshape(-1)).cuda()
        d_cnt = torch.tensor([len(s) for s in src], dtype=torch.int64, device="cuda")
        d_v = torch.full((2 * cap,), 7, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        c.index_check_insert_buckets(d_bk.data_ptr(), d_cnt.data_ptr(), 2, cap, d_v.data_ptr())
        torch.cuda.synchronize()
        v = d_v.cpu().numpy().reshape(2, cap)
        assert np.concatenate([v[0, :1500], v[1, :900]]).tolist() == _oracle_verdicts(oracle, np.concatenate(src))
        c.index_check()


def test_genuine_blake3_prefix_collision_end_to_end(oracle):
    """VERDICT r3 #1 (optional part): two real 8-byte files whose BLAKE3 digests share their first 8
    bytes (tests/golden/blake3_prefix_collision.json, found by tools/collide.hip) go through
    bw_process_files as small files, with repeats and random neighbours: both are stored, the
    repeats are duplicates, exactly as oracle.Index decides, and no call reports an error."""
    import json
    import os
    p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "blake3_prefix_collision.json")
    if not os.path.exists(p):
        pytest.skip("collision fixture not generated")
    fx = json.load(open(p))
    m1, m2 = bytes.fromhex(fx["m1"]), bytes.fromhex(fx["m2"])
    rng = np.random.default_rng(12)
    files = [m1, rng.bytes(8), m2, m1, rng.bytes(3000), m2, m2, m1]
    data = np.frombuffer(b"".join(files), dtype=np.uint8).copy()
    lens = np.array([len(f) for f in files], dtype=np.uint64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    want = oracle.process_files(data, offs, lens)
    assert bytes(want["digest"][0][:8]) == bytes(want["digest"][2][:8])
    assert want["is_dup"].tolist() == [0, 0, 0, 1, 0, 1, 1, 1]
    with Context(0) as c:
        c.index_reset()
        blobs_equal(c.process_files(data, offs, lens), want)
        c.index_check()
        assert c.index_size() == 4
        # and as one-call-per-file drop-ins: blake3.hash, then the gate
        d = np.array([np.frombuffer(c.blake3(f), np.uint8) for f in files])
        c.index_reset()
        assert c.index_check_insert(d).tolist() == want["is_dup"].tolist()


def test_tree_pack_tree_on_one_context(oracle):
    """tree blobs, then sealing/packing, then tree blobs again on one context, then
    destroy (the pinned message staging used to be freed by the sealing path)."""
    from oracle import pack_oracle as po
    rng = np.random.default_rng(6)
    specs = [(0, "f%d" % i, 100 + i, 1700000000, None, rng.integers(0, 256, 32 * (i % 5), dtype=np.uint8).tobytes())
             for i in range(3000)]
    prk = bytes(range(32))
    c = Context(0)
    try:
        for rnd in range(2):
            c.index_reset()
            hashes, _ = c.tree_blobs([make_tree(*s) for s in specs], dedup=False)
            for i in (0, 1, 1234, 2999):
                assert bytes(hashes[i]) == oracle.split_serialize_tree(*specs[i])[0][1], (rnd, i)
            blobs = [splitmix_bytes(50 + k + 100 * rnd, 70000 + 999 * k) for k in range(40)]
            lens = np.array([b.size for b in blobs], dtype=np.uint64)
            offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
            hs = np.array([np.frombuffer(oracle.blake3(b), np.uint8) for b in blobs])
            nonces = rng.integers(0, 256, (40, 12), dtype=np.uint8)
            plan, total = c.pack_plan(lens)
            ids = rng.integers(0, 256, (len(plan), 12), dtype=np.uint8)
            out = c.pack_build(prk, np.concatenate(blobs), offs, lens, hs, np.zeros(40, np.uint8), nonces, plan,
                               total, ids)
            p = plan[0]
            want = po.serialize_packfile(prk, bytes(ids[0]), [
                (bytes(hs[i]), 0, bytes(nonces[i]), po.seal_blob_payload(prk, hs[i], nonces[i], po.zstd_store(blobs[i])))
                for i in range(int(p["first_blob"]), int(p["first_blob"] + p["n_blobs"]))])
            assert out[int(p["offset"]):int(p["offset"] + p["size"])].tobytes() == want
    finally:
        c.close()


def test_pack_rejects_blob_over_3mib():
    from backuwup_amd._lib import BW_EINVAL
    with Context(0) as c:
        n = (3 << 20) + 1
        plan, total = c.pack_plan([n])
        with pytest.raises(BwError) as e:
            c.pack_build(bytes(32), np.zeros(n, np.uint8), [0], [n], np.zeros((1, 32), np.uint8), [0],
                         np.zeros((1, 12), np.uint8), plan, total, np.zeros((1, 12), np.uint8))
        assert e.value.rc == BW_EINVAL


def test_no_dedup_batches_leave_shared_index_alone(oracle):
    """BW_F_NO_DEDUP batches (the sharded path's local pass) append nothing to the shared index."""
    import torch
    data, offs, lens = small_files(500, seed=90)
    t = torch.from_numpy(data).cuda()
    torch.cuda.synchronize()
    ix = Index(0)
    try:
        with Context(0) as c:
            c.attach_index(ix)
            c.index_reset()
            tk = c.submit_device(t.data_ptr(), data.size, offs, lens, make_params(flags=BW_F_NO_DEDUP))
            r = c.wait(tk)
            assert not r["is_dup"].any() and c.index_size() == 0
            want = oracle.process_files(data, offs, lens)
            assert np.array_equal(r["digest"], want["digest"])
    finally:
        ix.close()


def _two_rank_worker(rank, world, port, q):
    """One rank of a 2-process exchange on the single GPU: its own context chunks + hashes its
    share of the files (BW_F_NO_DEDUP), then the device shard ops (bucket partition, owner gate,
    verdict scatter kernels) run with the collectives staged through host memory over gloo."""
    import os
    import torch
    import torch.distributed as dist
    from backuwup_amd.sharded import DeviceShardOps, exchange_dedup, session_capacity, staged_all_to_all
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        data, offs, lens = small_files(6000, seed=55)
        per = len(lens) // world
        out = []
        with Context(0) as c, torch.cuda.stream(torch.cuda.Stream()):
            ops = DeviceShardOps(c, torch.device("cuda", 0))
            c.index_reset(1 << 16)
            for batch in range(2):  # two batches per rank: batch-major, then rank-major canonical order
                lo = (batch * world + rank) * per // 2
                hi = lo + per // 2
                b = _slices(data, offs, lens, [(lo, hi)])[0]
                t_dev = torch.from_numpy(b[0]).cuda()
                tk = c.submit_device(t_dev.data_ptr(), b[0].size, b[1], b[2], make_params(flags=BW_F_NO_DEDUP))
                d_n, d_dig, _, max_n = c.batch_views(tk)
                cap = session_capacity(max_n, "cpu")
                is_dup = torch.zeros(max_n, dtype=torch.uint8, device="cuda")
                exchange_dedup(ops, (d_n, d_dig, is_dup.data_ptr(), max_n), world, cap, all_to_all=staged_all_to_all)
                res = c.wait(tk)
                out.append((lo, hi, res["digest"].copy(), is_dup[:len(res)].cpu().numpy()))
            c.index_check()
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_device_shard_ops_two_ranks_one_gpu(oracle):
    """Unmeasured on xGMI: two processes share the one GPU, gloo carries the collectives, and the
    device kernels of the sharded exchange decide every blob exactly as one global index would."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_two_rank_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    data, offs, lens = small_files(6000, seed=55)
    ix = oracle.Index()
    n_checked = 0
    for batch in range(2):
        for r in range(2):
            lo, hi, dig, dup = got[r][batch]
            b = _slices(data, offs, lens, [(lo, hi)])[0]
            want = oracle.process_files(*b, index=ix)
            assert np.array_equal(dig, want["digest"]) and np.array_equal(dup, want["is_dup"]), (batch, r)
            n_checked += int(want["is_dup"].sum())
    assert n_checked > 0


def test_exchange_dedup_rccl_world1_c_abi(oracle):
    """bw_comm_init (RCCL, world size 1) + bw_exchange_dedup per batch: four NO_DEDUP batches on
    two contexts sharing one index, each sent through the exchange (partition, RCCL all-to-alls,
    owner gate, verdicts back); bw_wait returns the verdicts of one global index."""
    import torch
    from backuwup_amd.comm import Comm, unique_id
    data, offs, lens = small_files(4000, seed=71)
    batches = _slices(data, offs, lens, [(0, 1000), (1000, 2000), (0, 1000), (2000, 4000)])
    want = oracle_session(oracle, batches)
    devs = [torch.from_numpy(d).cuda() for d, _, _ in batches]
    torch.cuda.synchronize()
    ix = Index(0)
    cs = [Context(0), Context(0)]
    comm = Comm.rccl(0, 0, 1, unique_id())
    comm2 = None
    try:
        for c in cs:
            c.set_stream(torch.cuda.Stream().cuda_stream)
            c.attach_index(ix)
        cs[0].index_reset(1 << 16)
        p = make_params(flags=BW_F_NO_DEDUP)
        tickets = []
        for k, (t, (d, o, l)) in enumerate(zip(devs, batches)):
            tk = cs[k % 2].submit_device(t.data_ptr(), d.size, o, l, p)
            cs[k % 2].exchange_dedup(comm, tk)
            tickets.append(tk)
        for k, tk in enumerate(tickets):
            blobs_equal(cs[k % 2].wait(tk), want[k], k)
        assert cs[0].wait(tickets[2])["is_dup"].all()
        cs[0].index_check()
        # a batch gated locally already cannot go through the exchange again
        tk = cs[0].submit_device(devs[0].data_ptr(), batches[0][0].size, batches[0][1], batches[0][2])
        with pytest.raises(BwError) as e:
            cs[0].exchange_dedup(comm, tk)
        assert e.value.rc == BW_ESTATE
        # a batch hashed with BW_F_NO_HASH has no digests to exchange
        from backuwup_amd._lib import BW_ENOSPC, BW_F_NO_HASH
        tk = cs[0].submit_device(devs[0].data_ptr(), batches[0][0].size, batches[0][1], batches[0][2],
                                 make_params(flags=BW_F_NO_DEDUP | BW_F_NO_HASH))
        with pytest.raises(BwError) as e:
            cs[0].exchange_dedup(comm, tk)
        assert e.value.rc == BW_ESTATE
        # round 5: no capacity at all -- every transfer is sized from the exchange's own counts, so
        # batches that grow and shrink on one communicator (and a set_capacity, now ignored) need
        # nothing from the caller; several exchanges queue before any wait, and progress() finishes
        # whatever has its counts without waiting
        cs[0].index_reset(1 << 16)
        comm2 = Comm.rccl(0, 0, 1, unique_id())
        comm2.set_capacity(1000)
        order = (0, 3, 1, 0, 2)
        want2 = oracle_session(oracle, [batches[k] for k in order])
        tks = []
        for j, k in enumerate(order):
            d, o, l = batches[k]
            c = cs[j % 2]
            tk = c.submit_device(devs[k].data_ptr(), d.size, o, l, p)
            c.exchange_dedup(comm2, tk)
            comm2.progress()
            tks.append((c, tk))
            if len(tks) > 2:  # two exchanged batches in flight, the oldest read
                c0, t0 = tks[j - 2]
                blobs_equal(c0.wait(t0), want2[j - 2], ("grow/shrink", j - 2))
        for j in (len(order) - 2, len(order) - 1):
            blobs_equal(tks[j][0].wait(tks[j][1]), want2[j], ("grow/shrink", j))
        cs[0].index_check()
    finally:
        for c in cs:
            c.close()
        comm.close()
        if comm2 is not None:
            comm2.close()
        ix.close()


def _two_rank_c_worker(rank, world, port, q):
    """One rank of the exchange through the C entry point (bw_exchange_dedup) with the caller's
    host transport (bw_comm_init_host over gloo): two ranks share the one GPU, which RCCL refuses."""
    import os
    import torch
    import torch.distributed as dist
    from backuwup_amd.comm import Comm, gloo_all_to_all
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        data, offs, lens = small_files(6000, seed=56)
        per = len(lens) // world
        out = []
        with Context(0) as c, Comm.host(0, rank, world, gloo_all_to_all()) as comm:
            c.index_reset(1 << 16)
            for batch in range(4):  # batch-major, then rank-major canonical order
                lo = ((batch % 2) * world + rank) * per // 4
                hi = lo + per // 4 - 7 * rank * (batch == 1)  # ragged: the ranks' batch sizes differ
                if batch == 2 and rank == 1:  # 4x the size of its first batch
                    lo, hi = 2 * per // 2, 2 * per // 2 + per
                if batch == 3:  # then small again (partly repeats: duplicates across the ranks)
                    lo, hi = (rank * 37, rank * 37 + 50)
                b = _slices(data, offs, lens, [(lo, hi)])[0]
                t_dev = torch.from_numpy(b[0]).cuda()
                tk = c.submit_device(t_dev.data_ptr(), b[0].size, b[1], b[2], make_params(flags=BW_F_NO_DEDUP))
                c.exchange_dedup(comm, tk)
                res = c.wait(tk)
                out.append((lo, hi, res["digest"].copy(), res["is_dup"].copy()))
            c.index_check()
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_exchange_dedup_c_abi_two_ranks_one_gpu(oracle, world):
    """bw_exchange_dedup with two (four) processes on the one GPU: every verdict equals one global
    index over the canonical order (batch, rank, position), including a repeated batch (all
    duplicates) and batches whose sizes differ between the ranks and grow and shrink."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_two_rank_c_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    data, offs, lens = small_files(6000, seed=56)
    ix = oracle.Index()
    for batch in range(4):
        for r in range(world):
            lo, hi, dig, dup = got[r][batch]
            want = oracle.process_files(*_slices(data, offs, lens, [(lo, hi)])[0], index=ix)
            assert np.array_equal(dig, want["digest"]) and np.array_equal(dup, want["is_dup"]), (batch, r)
    assert got[0][2][3].all()  # batch 2 repeats batch 0 on rank 0


def _dying_peer_worker(rank, world, port, q):
    """Rank 1 leaves after the first exchange (os._exit, no goodbye); rank 0's next exchange must
    fail with BW_ECOMM within the deadline instead of hanging."""
    import datetime
    import os
    import time
    import torch
    import torch.distributed as dist
    from backuwup_amd._lib import BW_ECOMM
    from backuwup_amd.comm import Comm, gloo_all_to_all
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=20))
    data, offs, lens = small_files(800, seed=57)
    with Context(0) as c, Comm.host(0, rank, world, gloo_all_to_all()) as comm:
        c.index_reset(1 << 14)
        res = []
        for batch in range(2):
            b = _slices(data, offs, lens, [((2 * batch + rank) * 200, (2 * batch + rank + 1) * 200)])[0]
            t_dev = torch.from_numpy(b[0]).cuda()
            tk = c.submit_device(t_dev.data_ptr(), b[0].size, b[1], b[2], make_params(flags=BW_F_NO_DEDUP))
            if batch == 1 and rank == 1:
                q.put((rank, "left"))
                q.close()
                q.join_thread()  # flush the queue's feeder before leaving without teardown
                os._exit(0)
            t0 = time.time()
            try:
                c.exchange_dedup(comm, tk)
                c.wait(tk)
                res.append("ok")
            except BwError as e:
                res.append((e.rc, round(time.time() - t0, 1), comm.status()))
                # every later call on the failed communicator fails at once
                t1 = time.time()
                with pytest.raises(BwError) as e2:
                    c.exchange_dedup(comm, tk)
                res.append((e2.value.rc, round(time.time() - t1, 1)))
        q.put((rank, res))
    q.close()
    q.join_thread()
    os._exit(0)  # the process group lost a member: skip its teardown


def test_exchange_peer_failure_returns_ecomm():
    """Host transport (gloo) with two ranks on the one GPU: the survivor of a peer that dies gets
    BW_ECOMM from bw_exchange_dedup well within the transport's 20 s deadline, the communicator
    reports itself failed, and later calls fail immediately."""
    import socket
    import torch.multiprocessing as mp
    from backuwup_amd._lib import BW_ECOMM
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dying_peer_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=180) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    assert got[1] == "left"
    first, (rc, dt, status), (rc2, dt2) = got[0]
    assert first == "ok"
    assert rc == BW_ECOMM and status == BW_ECOMM and dt < 30, got[0]
    assert rc2 == BW_ECOMM and dt2 < 1, got[0]


def _dying_rccl_peer_worker(rank, world, uid, q):
    """One GPU per rank over RCCL: rank 1 leaves after the first exchange (os._exit, no goodbye);
    rank 0's next exchange (the control communicator's counts, then the data all-to-all) must fail
    with BW_ECOMM within the deadline, and bw_comm_destroy must return."""
    import os
    import time
    import torch
    from backuwup_amd._lib import BW_ECOMM
    from backuwup_amd.comm import Comm
    torch.cuda.set_device(rank)
    data, offs, lens = small_files(800, seed=58)
    res = []
    with Context(rank) as c:
        comm = Comm.rccl(rank, rank, world, uid, timeout_ms=8000)
        c.index_reset(1 << 14)
        for batch in range(2):
            b = _slices(data, offs, lens, [((2 * batch + rank) * 200, (2 * batch + rank + 1) * 200)])[0]
            t_dev = torch.from_numpy(b[0]).cuda()
            tk = c.submit_device(t_dev.data_ptr(), b[0].size, b[1], b[2], make_params(flags=BW_F_NO_DEDUP))
            if batch == 1 and rank == 1:
                q.put((rank, "left"))
                q.close()
                q.join_thread()
                os._exit(0)
            t0 = time.time()
            try:
                c.exchange_dedup(comm, tk)
                c.wait(tk)
                res.append("ok")
            except BwError as e:
                res.append((e.rc, round(time.time() - t0, 1), comm.status()))
        t1 = time.time()
        comm.close()
        res.append(round(time.time() - t1, 1))
    q.put((rank, res))
    q.close()
    q.join_thread()
    os._exit(0)


def test_rccl_peer_failure_mid_session_returns_ecomm():
    """RCCL with two ranks on two GPUs (skipped with fewer): a peer that dies after the first
    exchange makes the survivor's next bw_exchange_dedup / bw_wait return BW_ECOMM within the 8 s
    deadline (non-blocking communicators, the polled waits, ncclCommAbort), and destroying the failed
    communicator returns promptly."""
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs (RCCL refuses two ranks on one device)")
    import torch.multiprocessing as mp
    from backuwup_amd._lib import BW_ECOMM
    from backuwup_amd.comm import unique_id
    uid = unique_id()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dying_rccl_peer_worker, args=(r, 2, uid, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=180) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    assert got[1] == "left"
    first, (rc, dt, status), t_close = got[0]
    assert first == "ok"
    assert rc == BW_ECOMM and status == BW_ECOMM and dt < 30, got[0]
    assert t_close < 10, got[0]


_NEVER_JOINED = """
import sys, time
sys.path.insert(0, %r)
from backuwup_amd.comm import Comm, unique_id
from backuwup_amd._lib import BwError
t0 = time.time()
try:
    Comm.rccl(0, 0, 2, unique_id(), timeout_ms=4000)
    print("@@JOINED")
except BwError as e:
    print("@@RC", e.rc, round(time.time() - t0, 1))
"""


def test_rccl_init_deadline_when_a_rank_never_joins():
    """bw_comm_init_timeout with world 2 and no rank 1: the non-blocking RCCL initialisation is
    aborted at the deadline and returns BW_ECOMM (it used to block forever).  Run in a child with
    its own time limit so a regression cannot stall the suite."""
    import subprocess
    import sys
    from backuwup_amd._lib import BW_ECOMM
    root = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", _NEVER_JOINED % root], capture_output=True, text=True, timeout=90)
    line = [l for l in out.stdout.splitlines() if l.startswith(("@@RC", "@@JOINED"))]
    assert line and line[0].startswith("@@RC"), (out.stdout[-2000:], out.stderr[-2000:])
    _, rc, dt = line[0].split()
    assert int(rc) == BW_ECOMM and 3.5 < float(dt) < 30, line


# the shipped kernels: one scan per tile size, k_b3_lines with 4 / 2 / 1 leaves per lane.  The
# diagnostic variants (8-wave scan blocks, the latency stream, the other leaf loaders, the fused
# upper levels) run only with the BW_DIAG library (BW_LIB=...libbackuwup_amd_debug.so).
_VARIANTS = [(16, 0, 2, 0, 4), (16, 0, 2, 0, 2), (16, 0, 2, 0, 1)]
_DIAG_VARIANTS = [(8, 0, 1, 0, 4), (16, 1, 1, 0, 4), (8, 1, 0, 0, 4), (16, 0, 0, 0, 4), (16, 0, 2, 1, 4),
                  (8, 1, 2, 1, 2), (8, 0, 2, 0, 1)]


@pytest.mark.parametrize("scan_waves,latency,loads,upper,group", _VARIANTS + (_DIAG_VARIANTS if _diag_lib() else []))
def test_kernel_variants_bit_exact(oracle, scan_waves, latency, loads, upper, group):
    """Two batches in flight on two contexts that share an index, four batches of a tree corpus,
    for each leaf grouping (and, with the diagnostic build, each scheduling variant): results equal
    the oracle."""
    import torch
    from backuwup_amd._lib import BW_OPT_B3_GROUP, BW_OPT_B3_LOADS, BW_OPT_B3_UPPER, BW_OPT_LATENCY_STREAM, BW_OPT_SCAN_WAVES
    data, offs, lens = tree_corpus(80 << 20, seed=21, max_file=20 << 20)
    batches = _slices(data, offs, lens, [(0, len(lens) // 2), (len(lens) // 2, len(lens))]) * 2
    want = oracle_session(oracle, batches)
    devs = [torch.from_numpy(d).cuda() for d, _, _ in batches[:2]] * 2
    torch.cuda.synchronize()
    ix = Index(0)
    cs = [Context(0), Context(0)]
    try:
        for c in cs:
            c.set_stream(torch.cuda.Stream().cuda_stream)
            c.attach_index(ix)
            if (scan_waves, latency, loads, upper) != (16, 0, 2, 0):
                c.set_option(BW_OPT_SCAN_WAVES, scan_waves)
                c.set_option(BW_OPT_LATENCY_STREAM, latency)
                c.set_option(BW_OPT_B3_LOADS, loads)
                c.set_option(BW_OPT_B3_UPPER, upper)
            c.set_option(BW_OPT_B3_GROUP, group)
        cs[0].index_reset()
        tickets = [cs[k % 2].submit_device(t.data_ptr(), d.size, o, l) for k, (t, (d, o, l)) in enumerate(zip(devs, batches))]
        for k, t in enumerate(tickets):
            blobs_equal(cs[k % 2].wait(t), want[k], k)
    finally:
        for c in cs:
            c.close()
        ix.close()


@pytest.mark.parametrize("scan_first", [0, 1])
def test_scan_first_and_profile_mask(oracle, scan_first):
    """BW_OPT_SCAN_FIRST moves the gear scan ahead of the host's batch tables and
    BW_OPT_PROFILE_MASK thins the stage marks: neither changes a result (two contexts sharing an
    index, profiled, four batches), and only the marked stages accumulate time."""
    import torch
    from backuwup_amd._lib import BW_OPT_PROFILE_MASK, BW_OPT_SCAN_FIRST, STAGES
    data, offs, lens = tree_corpus(48 << 20, seed=23, max_file=12 << 20)
    batches = _slices(data, offs, lens, [(0, len(lens) // 2), (len(lens) // 2, len(lens))]) * 2
    want = oracle_session(oracle, batches)
    devs = [torch.from_numpy(d).cuda() for d, _, _ in batches[:2]] * 2
    torch.cuda.synchronize()
    mask = (1 << 0) | (1 << 4) | (1 << 5) | (1 << len(STAGES))  # scan, b3_leaf, b3_tree, batch end
    ix = Index(0)
    cs = [Context(0), Context(0)]
    try:
        for c in cs:
            c.set_stream(torch.cuda.Stream().cuda_stream)
            c.attach_index(ix)
            c.set_option(BW_OPT_SCAN_FIRST, scan_first)
            c.set_option(BW_OPT_PROFILE_MASK, mask)
            c.profile_enable(True)
        for bad in (0, 1 << 4, 2 << len(STAGES)):  # fewer than two marks, or past the batch end
            with pytest.raises(BwError):
                cs[0].set_option(BW_OPT_PROFILE_MASK, bad)
        with pytest.raises(BwError):
            cs[0].set_option(BW_OPT_SCAN_FIRST, 3)
        cs[0].index_reset()
        tickets = [cs[k % 2].submit_device(t.data_ptr(), d.size, o, l) for k, (t, (d, o, l)) in enumerate(zip(devs, batches))]
        for k, t in enumerate(tickets):
            blobs_equal(cs[k % 2].wait(t), want[k], k)
        ms, n = cs[0].profile_read()
        assert n == 2
        for i, s in enumerate(STAGES):
            assert (ms[s] > 0) == bool((mask >> i) & 1), (s, ms[s])
        # the leaf pass alone, the batch closed by the b3_tree mark
        for c in cs:
            c.set_option(BW_OPT_PROFILE_MASK, (1 << 4) | (1 << 5))
            c.profile_enable(True)
        t = cs[0].submit_device(devs[0].data_ptr(), batches[0][0].size, batches[0][1], batches[0][2])
        cs[0].wait(t)
        ms, n = cs[0].profile_read()
        assert n == 1 and ms["b3_leaf"] > 0 and sum(ms.values()) == ms["b3_leaf"], ms
    finally:
        for c in cs:
            c.close()
        ix.close()


def test_calibrate_b3():
    """bw_calibrate_b3: the leaf pass's compression from registers, timed on the device."""
    with Context(0) as c:
        cal = c.calibrate_b3(20.0)
        assert 100 < cal["gbs"] < 20000, cal
        assert 0.3 < cal["ghz"] < 3.5, cal
        assert cal["launch_ms"] > 2, cal
        n_cu = cal["gbs"] / cal["ghz"] / cal["bytes_per_clk_cu"]
        assert 200 < n_cu < 320, cal
        with pytest.raises(BwError):
            c.calibrate_b3(0.0)
