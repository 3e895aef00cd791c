"""The whole-result fixtures of the full-size configurations (tests/golden/c{2,3,4}_full.json) and
the generator that made them, on the CPU: the generator's windowed / per-image / per-file-table
forms equal the oracle over the laid-out corpus at small sizes, and the committed fixtures describe
bench.py's rank-0 corpora.  The GPU side is tests/test_gpu_full_configs.py."""
import importlib.util
import json
import os

import numpy as np

from backuwup_amd import synth

HERE = os.path.dirname(os.path.abspath(__file__))


def _gen():
    spec = importlib.util.spec_from_file_location("make_full_configs", os.path.join(HERE, "golden", "make_full_configs.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_windowed_c2_equals_whole_stream(oracle):
    m = _gen()
    n = 40 << 20
    a = m.c2(seed=5, n=n, window=7 << 20)  # windows restart at cuts decided entirely inside them
    b = synth.result_digest(oracle.process_files(synth.splitmix_bytes(5, n), [0], [n]))
    assert a == b and a["blobs"] > 20


def test_per_image_c3_equals_laid_out_corpus(oracle):
    m = _gen()
    a = m.c3(seed=1, base_bytes=12 << 20, n_images=3)
    d, o, l = synth.vm_image_variants(12 << 20, 3, seed=1)
    b = synth.result_digest(oracle.process_files(d, o, l, threads=3))
    assert a == b and a["dup_blobs"] > 0


def test_file_table_c4_equals_laid_out_corpus(oracle):
    m = _gen()
    a = m.c4(seed=3, n_files=2000, window=8 << 20)
    d, o, l = synth.small_files(2000, seed=3)
    b = synth.result_digest(oracle.process_files(d, o, l, threads=4))
    assert a == b and a["dup_blobs"] == 600


def test_result_digest_is_order_and_field_sensitive():
    blobs = np.zeros(3, dtype=synth.CANON_DTYPE)
    blobs["length"] = [5, 6, 7]
    base = synth.result_digest(blobs)
    for f in ("file", "offset", "length", "gear_hash", "is_dup"):
        b = blobs.copy()
        b[f][1] ^= 1
        assert synth.result_digest(b)["sha256_records"] != base["sha256_records"], f
    b = blobs.copy()
    b["digest"][2, 31] = 1
    assert synth.result_digest(b)["sha256_digests"] != base["sha256_digests"]
    assert synth.result_digest(blobs[::-1].copy())["sha256_records"] != base["sha256_records"]


def test_committed_fixtures_describe_the_bench_corpora():
    fx = {k: json.load(open(os.path.join(HERE, "golden", "%s_full.json" % k))) for k in ("c1", "c2", "c3", "c4", "c5",
                                                                                         "edge")}
    assert fx["edge"]["files"] == 24 and fx["edge"]["dup_blobs"] > 0
    assert fx["c1"]["total_bytes"] == 1 << 30 and fx["c1"]["dup_bytes"] > 0.2 * fx["c1"]["bytes"]
    # C5's rank 0 holds C3's first 8 images: its blobs are a prefix of C3's
    assert fx["c5"]["files"] == 8 and fx["c5"]["blobs"] < fx["c3"]["blobs"] and fx["c5"]["base_bytes"] == 4 << 30
    assert fx["c2"]["bytes"] == 16 << 30 and fx["c2"]["seed"] == 42 and fx["c2"]["dup_blobs"] == 0
    assert 12000 < fx["c2"]["blobs"] < 15500
    assert fx["c3"]["files"] == 16 and fx["c3"]["base_bytes"] == 4 << 30 and fx["c3"]["seed"] == 1
    assert fx["c3"]["dup_bytes"] > 0.9 * fx["c3"]["bytes"]  # ~92 % dedup
    assert fx["c4"]["blobs"] == fx["c4"]["files"] == 1_000_000 and fx["c4"]["dup_blobs"] == 300_000
    u, offs, lens = synth.small_files_table(fx["c4"]["files"], seed=fx["c4"]["seed"])
    assert int(np.sum(lens)) == fx["c4"]["bytes"]
    for f in fx.values():
        assert len(f["sha256_records"]) == 64 and f["params"] == {"min": 262144, "avg": 1048576, "max": 3145728}
