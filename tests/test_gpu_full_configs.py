"""Whole-result parity on the full-size configurations.

Each test runs one BASELINE.json configuration at its full size through the C ABI
(bw_submit_device + bw_results, bytes generated in HBM exactly as bench.py's rank 0 does) and
compares the WHOLE result -- every blob's (file, offset, length, gear_hash, digest, is_dup) in
canonical order -- with the fixture the CPU oracle computed over the same bytes
(tests/golden/c{2,3,4}_full.json, tests/golden/make_full_configs.py): blob count, duplicate
count and bytes, and sha256 over the packed records (backuwup_amd/synth.py CANON_DTYPE).

  C2  16 GiB splitmix64 stream (seed 42), one file: 13.6 k chunks, none duplicate
  C3  4 GiB base + 15 byte-shifted variants (seed 1) = 64 GiB, 16 files, one index
  C4  1,000,000 files of 4-64 KiB with 30 % copies (seed 3), one blob per file
  C1  the 1 GiB directory tree (seed 0x6261636B), 122 files, 30 % whole-file copies
  C5  rank 0's share of C5: VM-image family 0, files 0-7 (32 GiB), from pinned host memory
      (bw_submit_host: the H2D copy overlapped with the processing)
  edge  synth.edge_corpus: threshold sizes, empty files, zeros (no candidates), periodic and
      two-symbol data (dense candidates), compressible text, zero runs, copies; both scan tile sizes
"""
import json
import os

import numpy as np
import pytest
import torch

from backuwup_amd import synth

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def fixture(name):
    with open(os.path.join(GOLDEN, "%s_full.json" % name)) as f:
        return json.load(f)


def compare(got, want):
    have = synth.result_digest(got)
    keys = ("blobs", "dup_blobs", "bytes", "dup_bytes", "sha256_digests", "sha256_records")
    assert {k: have[k] for k in keys} == {k: want[k] for k in keys}


@pytest.fixture
def fresh_ctx():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from backuwup_amd import Context
    c = Context(0)
    yield c
    c.close()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def test_c2_full_16gib_whole_result(fresh_ctx):
    want = fixture("c2")
    n = want["bytes"]
    dev = synth.splitmix_torch(want["seed"], n, "cuda")
    torch.cuda.synchronize()  # (generated on torch's stream; the context runs on its own)
    fresh_ctx.index_reset(want["blobs"] + 1024)
    fresh_ctx.submit_device(dev.data_ptr(), n, [0], [n])
    compare(fresh_ctx.results(), want)
    del dev


def test_c3_full_64gib_whole_result(fresh_ctx):
    want = fixture("c3")
    data, offs, lens = synth.vm_image_variants_torch(want["base_bytes"], want["files"], "cuda", seed=want["seed"])
    torch.cuda.synchronize()
    assert int(np.sum(lens)) == want["bytes"]
    fresh_ctx.index_reset(want["blobs"] + 1024)
    fresh_ctx.submit_device(data.data_ptr(), data.numel(), offs, lens)
    compare(fresh_ctx.results(), want)
    del data


def test_c4_full_1m_files_whole_result(fresh_ctx):
    want = fixture("c4")
    u, offs, lens = synth.small_files_table(want["files"], seed=want["seed"])
    dev = synth.splitmix_torch(want["seed"], u, "cuda")
    torch.cuda.synchronize()
    fresh_ctx.index_reset(want["blobs"] + 1024)
    fresh_ctx.submit_device(dev.data_ptr(), u, offs, lens)
    got = fresh_ctx.results()
    assert len(got) == want["files"]  # dir_packer.rs:246: one blob per file <= 1 MiB
    compare(got, want)
    del dev


def test_c1_full_1gib_whole_result(fresh_ctx):
    want = fixture("c1")
    data, offs, lens = synth.tree_corpus(want["total_bytes"], seed=want["seed"])
    fresh_ctx.index_reset(want["blobs"] + 1024)
    got = fresh_ctx.process_files(data, offs, lens)
    compare(got, want)


def test_c5_rank0_32gib_from_pinned_host_whole_result(fresh_ctx):
    want = fixture("c5")
    full, offs, lens = synth.vm_image_variants_torch(want["base_bytes"], 16, "cuda", seed=want["seed"])
    hi = int(offs[7] + lens[7])
    host = torch.empty(hi, dtype=torch.uint8, pin_memory=True)
    host.copy_(full[:hi])
    torch.cuda.synchronize()
    del full
    torch.cuda.empty_cache()
    fresh_ctx.index_reset(want["blobs"] + 1024)
    t = fresh_ctx.submit_host(host.data_ptr(), offs[:8], lens[:8], data_len=hi)
    compare(fresh_ctx.wait(t), want)
    del host


@pytest.fixture(scope="module")
def edge_data():
    return synth.edge_corpus()


@pytest.mark.parametrize("small_bytes", [0, 1 << 40])  # full-size scan tiles, half-size tiles
def test_edge_corpus_whole_result(fresh_ctx, edge_data, small_bytes):
    from backuwup_amd._lib import BW_OPT_SCAN_SMALL_BYTES
    want = fixture("edge")
    data, offs, lens = edge_data
    fresh_ctx.set_option(BW_OPT_SCAN_SMALL_BYTES, small_bytes)
    fresh_ctx.index_reset(want["blobs"] + 1024)
    compare(fresh_ctx.process_files(data, offs, lens), want)
