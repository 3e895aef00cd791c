"""Soak run of the seeded fuzz (round 6): the generators of tests/test_gpu_fuzz.py at many more seeds,
for as long as BW_SOAK_SECONDS says (skipped when it is unset, so the driver's `pytest -m gpu` does
not run it).  By default it alternates the chunker case (parameters anywhere in the crate's ranges,
every content kind) and the batch case (ragged batches, the small-file threshold anywhere, a seeded
index); BW_SOAK_KINDS=all adds the fuzz's options, in-flight, NodeSession, drop-in, zstd and tree
generators.  Every result against the oracle.  Failing seeds are collected and reported together;
the counts go to gpurun_out/soak.json when that directory exists."""
import json
import os
import time

import numpy as np
import pytest

import test_gpu_fuzz as F
from backuwup_amd import make_params
from backuwup_amd._lib import BW_EINVAL, BwError

pytestmark = pytest.mark.gpu


def _chunker_case(ctx, oracle, seed):
    rng = np.random.default_rng(seed)
    mn, av, mx = F._params(rng)
    kind = F.KINDS[seed % len(F.KINDS)]
    n = int(min(24 * F.MiB, max(1, rng.integers(1, 40) * max(mn, min(av, mx)) + rng.integers(0, 4096))))
    data = F._content(rng, kind, n)
    if av > mx:
        try:
            ctx.fastcdc_chunks(data, mn, av, mx)
        except BwError as e:
            return e.rc == BW_EINVAL
        return False
    return ctx.fastcdc_chunks(data, mn, av, mx) == oracle.fastcdc(data, mn, av, mx)


def _batch_case(ctx, oracle, seed):
    rng = np.random.default_rng(seed)
    mn, av, mx = F._valid_params(rng, seed)
    thr = int(rng.choice([0, 1, 4096, F.MiB, 8 * F.MiB]))
    data, offs, lens, files = F._batch(rng)
    seed_files = rng.choice(len(files), size=min(len(files), 5), replace=False)
    seeded = sorted({oracle.blake3(files[int(k)]) for k in seed_files})
    ctx.index_reset()
    ctx.index_seed(np.frombuffer(b"".join(seeded), np.uint8).reshape(-1, 32))
    got = ctx.process_files(data, offs, lens, make_params(mn, av, mx, small_file_threshold=thr))
    want = oracle.process_files(data, offs, lens, mn, av, mx, small_threshold=thr,
                                index=oracle.Index(b"".join(seeded)), threads=8)
    if got.shape != want.shape:
        return False
    return all(np.array_equal(got[f], want[f]) for f in ("file", "offset", "length", "gear_hash", "is_dup", "digest"))


def _wrap(fn):
    def run(ctx, oracle, seed):
        try:
            fn(ctx, oracle, seed)
            return True
        except AssertionError:
            return False
    return run


# BW_SOAK_KINDS picks the rotation (default: the chunker and batch cases); "all" adds the fuzz's other
# generators, each called with the seed as its case number
KINDS = {
    "chunker": _chunker_case,
    "batch": _batch_case,
    "options": _wrap(lambda c, o, s: F.test_random_options_random_batches(o, s)),
    "inflight": _wrap(lambda c, o, s: F.test_host_batches_in_flight_random(o, s)),
    "nodes": _wrap(lambda c, o, s: F.test_node_session_random_batches(o, s)),
    "dropin": _wrap(lambda c, o, s: F.test_dropin_kept_digests_random(c, o, s)),
    "zstd": _wrap(lambda c, o, s: F.test_zstd_random_blobs(c, o, s)),
    "trees": _wrap(lambda c, o, s: F.test_tree_blobs_random(c, o, s)),
}


def test_soak(ctx, oracle):
    seconds = float(os.environ.get("BW_SOAK_SECONDS", "0"))
    if seconds <= 0:
        pytest.skip("set BW_SOAK_SECONDS to run the soak")
    base = int(os.environ.get("BW_SOAK_SEED", "100000"))
    t_end = time.time() + seconds
    sel = os.environ.get("BW_SOAK_KINDS", "chunker,batch")
    rot = list(KINDS) if sel == "all" else sel.split(",")
    done = {k: 0 for k in rot}
    failed = []
    k = 0
    last = time.time()
    while time.time() < t_end:
        seed = base + k
        kind = rot[k % len(rot)]
        ok = KINDS[kind](ctx, oracle, seed)
        done[kind] += 1
        if not ok:
            failed.append((kind, seed))
        k += 1
        if time.time() - last > 30:  # (progress for gpurun's silence watchdog)
            print("soak: %d cases, %d failed" % (k, len(failed)), flush=True)
            last = time.time()
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
    if os.path.isdir(out):
        with open(os.path.join(out, "soak.json"), "w") as f:
            json.dump({"seconds": seconds, "first_seed": base, "kinds": rot, "cases": done, "failed": failed}, f)
    assert not failed, failed[:10]
