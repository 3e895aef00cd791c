"""Deterministic synthetic corpora for the BASELINE.json configurations.

All byte streams are counter-based splitmix64: word i of stream `seed` is
mix(seed + (i + 1) * 0x9E3779B97F4A7C15), emitted little-endian.  The same stream is produced
by numpy on the host and by torch on the GPU (`splitmix_torch`), so a device-resident corpus can
be checked slice by slice on the CPU.
"""
import numpy as np

GOLDEN = 0x9E3779B97F4A7C15
M1 = 0xBF58476D1CE4E5B9
M2 = 0x94D049BB133111EB


def splitmix_words(seed, first_word, n_words):
    with np.errstate(over="ignore"):
        i = np.arange(first_word + 1, first_word + 1 + n_words, dtype=np.uint64)
        z = np.uint64(seed) + i * np.uint64(GOLDEN)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(M1)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(M2)
        z = z ^ (z >> np.uint64(31))
    return z


def splitmix_bytes(seed, nbytes, offset=0):
    """bytes [offset, offset + nbytes) of stream `seed`."""
    w0 = offset // 8
    w1 = (offset + nbytes + 7) // 8
    words = splitmix_words(seed, w0, w1 - w0)
    b = words.view(np.uint8)
    s = offset - w0 * 8
    return b[s:s + nbytes].copy()


def _to_i64(x):
    x &= (1 << 64) - 1
    return x - (1 << 64) if x >= 1 << 63 else x


def splitmix_torch(seed, nbytes, device, out=None, chunk_words=1 << 27):
    """The same stream generated on the GPU with torch int64 arithmetic (wrapping multiply,
    logical shifts via masks).  Returns a uint8 tensor of nbytes (16-byte aligned storage)."""
    import torch
    n_words = (nbytes + 7) // 8
    if out is None:
        out = torch.empty(n_words * 8, dtype=torch.uint8, device=device)
    ow = out.view(torch.int64) if out.numel() % 8 == 0 else None
    g, m1, m2, sd = _to_i64(GOLDEN), _to_i64(M1), _to_i64(M2), _to_i64(seed)

    def lsr(z, k):
        return (z >> k) & ((1 << (64 - k)) - 1)

    for w0 in range(0, n_words, chunk_words):
        w1 = min(n_words, w0 + chunk_words)
        z = torch.arange(w0 + 1, w1 + 1, dtype=torch.int64, device=device)
        z.mul_(g).add_(sd)
        z = (z ^ lsr(z, 30)).mul_(m1)
        z = (z ^ lsr(z, 27)).mul_(m2)
        z = z ^ lsr(z, 31)
        ow[w0:w1] = z
    return out[:nbytes]


# ------------------------------------------------------------------ corpora

def tree_corpus(total_bytes, seed=0x6261636B, dup_fraction=0.30, min_file=4096, max_file=64 << 20):
    """C1: log-uniform file sizes, unique PRNG content, plus `dup_fraction` of the bytes as
    whole-file copies of earlier files.  Returns (data uint8, file_off, file_len)."""
    rng = np.random.default_rng(seed)
    uniq_target = int(total_bytes * (1 - dup_fraction))
    sizes = []
    acc = 0
    while acc < uniq_target:
        s = int(np.exp(rng.uniform(np.log(min_file), np.log(max_file))))
        s = min(s, uniq_target - acc) if uniq_target - acc > min_file else s
        sizes.append(s)
        acc += s
    files = [(i, s) for i, s in enumerate(sizes)]
    copies = []
    dup_acc = 0
    while dup_acc < total_bytes - acc and files:
        i = int(rng.integers(len(files)))
        copies.append(i)
        dup_acc += sizes[i]
    order = list(range(len(sizes))) + [("copy", c) for c in copies]
    rng.shuffle(order)
    lens = [sizes[o[1]] if isinstance(o, tuple) else sizes[o] for o in order]
    total = sum(lens)
    data = np.empty(total, dtype=np.uint8)
    offs = np.zeros(len(order), dtype=np.uint64)
    pos = 0
    for k, o in enumerate(order):
        src = o[1] if isinstance(o, tuple) else o
        n = sizes[src]
        data[pos:pos + n] = splitmix_bytes(seed * 1000 + src, n)
        offs[k] = pos
        pos += n
    return data, offs, np.array(lens, dtype=np.uint64)


def _variant_plan(base_size, v, seed, n_indels, n_overwrites, max_indel):
    """Edits of C3 variant v: 4 KiB overwrites [(at, bytes)] applied first, then the image is
    re-assembled from parts: ("keep", start, end) ranges of the overwritten image and ("ins",
    bytes) insertions (a deletion is a skipped range)."""
    r = np.random.default_rng(seed * 7919 + v)
    over = []
    for _ in range(n_overwrites):
        at = int(r.integers(0, max(1, base_size - 4096)))
        over.append((at, r.integers(0, 256, 4096, dtype=np.uint8)))
    edits = sorted(int(x) for x in r.integers(0, base_size, n_indels))
    parts = []
    prev = 0
    for at in edits:
        if at > prev:
            parts.append(("keep", prev, at))
        k = int(r.integers(1, max_indel + 1))
        if r.integers(2):
            parts.append(("ins", r.integers(0, 256, k, dtype=np.uint8)))
            prev = max(prev, at)
        else:
            prev = max(prev, min(base_size, at + k))
    if prev < base_size:
        parts.append(("keep", prev, base_size))
    return over, parts


def _part_len(p):
    return p[2] - p[1] if p[0] == "keep" else p[1].size


def vm_image_variants(base_bytes, n_variants, seed=1, n_indels=32, n_overwrites=16, max_indel=64):
    """C3: a random base image plus variants with small insertions/deletions (byte shifts) and
    4 KiB overwrites.  Returns (data, file_off, file_len) with the base as file 0."""
    base = splitmix_bytes(seed, base_bytes)
    images = [base]
    for v in range(1, n_variants):
        over, parts = _variant_plan(base_bytes, v, seed, n_indels, n_overwrites, max_indel)
        img = base.copy()
        for at, b in over:
            img[at:at + b.size] = b[:img.size - at]
        images.append(np.concatenate([img[p[1]:p[2]] if p[0] == "keep" else p[1] for p in parts]))
    offs = np.cumsum([0] + [im.size for im in images[:-1]]).astype(np.uint64)
    lens = np.array([im.size for im in images], dtype=np.uint64)
    return np.concatenate(images), offs, lens


def vm_image_variants_torch(base_bytes, n_variants, device, seed=1, n_indels=32, n_overwrites=16, max_indel=64):
    """The same corpus as vm_image_variants, assembled in HBM with device copies (C3 at 4 GiB x
    16 = 64 GiB never touches the host).  Returns (uint8 tensor, file_off, file_len)."""
    import torch
    plans = [_variant_plan(base_bytes, v, seed, n_indels, n_overwrites, max_indel) for v in range(1, n_variants)]
    lens = [base_bytes] + [sum(_part_len(p) for p in parts) for _, parts in plans]
    offs = np.cumsum([0] + lens[:-1]).astype(np.uint64)
    total = int(sum(lens))
    out = torch.empty(total + 16, dtype=torch.uint8, device=device)
    base = out[:base_bytes]
    base.copy_(splitmix_torch(seed, base_bytes, device))
    img = torch.empty(base_bytes, dtype=torch.uint8, device=device)
    for v, (over, parts) in enumerate(plans, start=1):
        img.copy_(base)
        for at, b in over:
            n = min(b.size, base_bytes - at)
            img[at:at + n] = torch.from_numpy(b[:n]).to(device)
        pos = int(offs[v])
        for p in parts:
            if p[0] == "keep":
                out[pos:pos + p[2] - p[1]] = img[p[1]:p[2]]
            else:
                out[pos:pos + p[1].size] = torch.from_numpy(p[1]).to(device)
            pos += _part_len(p)
    del img
    return out[:total], offs, np.array(lens, dtype=np.uint64)


def small_files(n_files, seed=3, lo=4096, hi=65536, dup_fraction=0.30):
    """C4: n_files with sizes uniform in [lo, hi] plus whole-file copies."""
    rng = np.random.default_rng(seed)
    n_uniq = int(round(n_files * (1 - dup_fraction)))
    sizes = rng.integers(lo, hi + 1, n_uniq)
    src = list(range(n_uniq)) + [int(x) for x in rng.integers(0, n_uniq, n_files - n_uniq)]
    rng.shuffle(src)
    uniq_off = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
    blob = splitmix_bytes(seed, int(sizes.sum()))
    lens = np.array([sizes[s] for s in src], dtype=np.uint64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    data = np.empty(int(lens.sum()), dtype=np.uint8)
    for k, s in enumerate(src):
        data[int(offs[k]):int(offs[k]) + int(lens[k])] = blob[int(uniq_off[s]):int(uniq_off[s]) + int(sizes[s])]
    return data, offs, lens


def small_files_table(n_files, seed=3, lo=4096, hi=65536, dup_fraction=0.30):
    """C4's file table over a buffer holding only the distinct files back to back: copies alias
    the bytes of their source (same content, hence same digest and dedup verdict as the laid-out
    corpus of small_files).  Returns (unique_bytes, file_off, file_len)."""
    rng = np.random.default_rng(seed)
    n_uniq = int(round(n_files * (1 - dup_fraction)))
    sizes = rng.integers(lo, hi + 1, n_uniq)
    src = np.array(list(range(n_uniq)) + [int(x) for x in rng.integers(0, n_uniq, n_files - n_uniq)])
    rng.shuffle(src)
    uniq_off = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
    return int(sizes.sum()), uniq_off[src], sizes[src].astype(np.uint64)


def edge_corpus(seed=11, text_bytes=384 << 20):
    """A corpus of the content and size edges of process_file + FastCDC at full scale (the whole-result
    fixture tests/golden/edge_full.json): files at the small-file threshold (dir_packer.rs:246: 1 MiB
    and one byte either side), empty and tiny files, odd and even tails, content with no cut candidates
    (zeros: every chunk `max`), one-byte and 4 KiB periodic patterns, two-symbol bytes (dense
    candidates), compressible text and mixed segments, random data with zero runs, and whole-file
    copies and a concatenation of two files (cross-file duplicate chunks).  Returns (data, file_off,
    file_len), files 16-byte aligned."""
    rng = np.random.default_rng(seed)
    MiB = 1 << 20
    files = []
    for n in (0, 1, 63, 64, 65, 4095, 4096, MiB - 1, MiB, MiB + 1, MiB + 2, 3 * MiB, 3 * MiB + 1, 6 * MiB + 5):
        files.append(splitmix_bytes(seed * 100 + len(files), n))
    files.append(np.zeros(32 * MiB + 7, np.uint8))                                   # no candidates
    files.append(np.full(24 * MiB + 3, 0xAB, np.uint8))                               # 1-byte period
    files.append(np.tile(splitmix_bytes(seed + 1, 4096), 16 * 1024)[:64 * MiB + 1])   # 4 KiB period
    files.append((splitmix_bytes(seed + 2, 48 * MiB) & 1).astype(np.uint8))           # two symbols
    files.append(compressible_corpus(text_bytes, "text", seed=seed + 3))
    files.append(compressible_corpus(text_bytes // 2, "mixed", seed=seed + 4))
    r = splitmix_bytes(seed + 5, 256 * MiB + 13)
    for at in rng.integers(0, r.size - MiB, 64):                                       # zero runs
        r[int(at):int(at) + int(rng.integers(1, MiB))] = 0
    files.append(r)
    files.append(files[-1].copy())                                                     # whole-file copy
    files.append(np.concatenate([files[20][:40 * MiB], files[18][:8 * MiB + 9]]))      # zero-run random + text
    files.append(files[7].copy())                                                      # 1 MiB - 1 copy
    lens = np.array([f.size for f in files], dtype=np.uint64)
    offs = np.zeros(len(files), dtype=np.uint64)
    offs[1:] = np.cumsum((lens[:-1] + 15) // 16 * 16)
    data = np.zeros(int(offs[-1] + lens[-1]) + 16, dtype=np.uint8)
    for o, f in zip(offs, files):
        data[int(o):int(o) + f.size] = f
    return data, offs, lens


# ------------------------------------------------------------------ whole-result fingerprints
# The canonical record of one blob, packed little-endian with no padding: the fields the reference's
# path decides (dir_packer.rs:246-286 boundaries and digests, blob_index.rs:130-148 verdicts).  The
# sha256 over a batch's records in canonical order pins the WHOLE result of a configuration
# (tests/golden/c{2,3,4}_full.json, made on the CPU by tests/golden/make_full_configs.py).
CANON_DTYPE = np.dtype([("file", "<u8"), ("offset", "<u8"), ("length", "<u8"), ("gear_hash", "<u8"),
                        ("digest", "u1", (32,)), ("is_dup", "u1")], align=False)
assert CANON_DTYPE.itemsize == 65


class ResultDigest:
    """Incremental fingerprint of a result array (any dtype with the CANON_DTYPE fields): blob
    count, duplicate count and bytes, and sha256 over the canonical records (plus one over the
    digests alone, which localises a mismatch to hashing or to boundaries/verdicts)."""

    def __init__(self):
        import hashlib
        self.records, self.digests = hashlib.sha256(), hashlib.sha256()
        self.n = self.n_dup = self.bytes = self.dup_bytes = 0

    def update(self, blobs, file_base=0):
        rec = np.zeros(len(blobs), dtype=CANON_DTYPE)
        for f in ("offset", "length", "gear_hash", "digest", "is_dup"):
            rec[f] = blobs[f]
        rec["file"] = np.asarray(blobs["file"], dtype=np.uint64) + np.uint64(file_base)
        self.records.update(rec.tobytes())
        self.digests.update(np.ascontiguousarray(rec["digest"]).tobytes())
        lens = rec["length"].astype(np.uint64)
        dup = rec["is_dup"] != 0
        self.n += len(rec)
        self.n_dup += int(dup.sum())
        self.bytes += int(lens.sum())
        self.dup_bytes += int(lens[dup].sum())
        return self

    def summary(self):
        return {"blobs": self.n, "dup_blobs": self.n_dup, "bytes": self.bytes, "dup_bytes": self.dup_bytes,
                "sha256_records": self.records.hexdigest(), "sha256_digests": self.digests.hexdigest()}


def result_digest(blobs):
    return ResultDigest().update(blobs).summary()


def _text_piece(rng, nbytes, vocab, ws, wl1, pw):
    """nbytes of words drawn from a Zipf-weighted vocabulary (vectorized gather)."""
    nw = int(nbytes / float(wl1 @ pw) * 1.05) + 16
    ids = np.minimum(np.searchsorted(np.cumsum(pw), rng.random(nw)), len(wl1) - 1)
    lens = wl1[ids]
    ends = np.cumsum(lens)
    k = int(np.searchsorted(ends, nbytes)) + 1
    ids, lens, ends = ids[:k], lens[:k], ends[:k]
    gather = np.repeat(ws[ids] - (ends - lens), lens) + np.arange(int(ends[-1]))
    return vocab[gather[:nbytes]]


def compressible_corpus(nbytes, kind="text", seed=7, piece=64 << 20):
    """Compressible synthetic bytes for the zstd level-3 measurements (§8f row 2; the benchmark
    configurations themselves are incompressible splitmix64).  Test/benchmark data only.
      text   words of 1-8 symbols from a skewed 48-letter alphabet, Zipf word frequencies
             (Huffman-coded literals plus many short repeat matches: ratio ~3)
      mixed  segments of 64 KiB - 4 MiB: half text, a quarter random (already-compressed media),
             a quarter long byte runs with sparse noise (sparse VM-image regions)"""
    rng = np.random.default_rng(seed)
    p = rng.dirichlet(np.ones(48) * 0.35)
    V = 4096
    wl = rng.integers(1, 9, V)
    wl1 = wl + 1
    ws = np.concatenate([[0], np.cumsum(wl1)[:-1]])
    vocab = np.full(int(wl1.sum()), 32, dtype=np.uint8)
    letters = (rng.choice(48, size=int(wl.sum()), p=p) + 40).astype(np.uint8)
    wstart = np.concatenate([[0], np.cumsum(wl)[:-1]])
    vocab[np.repeat(ws, wl) + (np.arange(int(wl.sum())) - np.repeat(wstart, wl))] = letters
    pw = 1.0 / (np.arange(V) + 2.0) ** 1.05
    pw /= pw.sum()
    out = np.empty(nbytes, dtype=np.uint8)
    pos = 0
    while pos < nbytes:
        if kind == "text":
            n = min(piece, nbytes - pos)
            out[pos:pos + n] = _text_piece(rng, n, vocab, ws, wl1, pw)
        else:
            n = min(int(rng.integers(64 << 10, 4 << 20)), nbytes - pos)
            r = rng.random()
            if r < 0.5:
                out[pos:pos + n] = _text_piece(rng, n, vocab, ws, wl1, pw)
            elif r < 0.75:
                out[pos:pos + n] = rng.integers(0, 256, n, dtype=np.uint8)
            else:
                seg = np.full(n, int(rng.integers(0, 3)), dtype=np.uint8)
                k = max(1, n // 4096)
                seg[rng.integers(0, n, k)] = rng.integers(0, 256, k, dtype=np.uint8)
                out[pos:pos + n] = seg
        pos += n
    return out


def compressible_corpus_torch(nbytes, device, kind="text", seed=7, piece=256 << 20):
    """compressible_corpus's distributions generated on the GPU with torch (same recipe, its own
    random stream): seconds for GiBs instead of a minute of numpy.  Checks read the bytes back
    from the device, so nothing needs to regenerate them on the host."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    rng = np.random.default_rng(seed)
    p = rng.dirichlet(np.ones(48) * 0.35)
    V = 4096
    wl = rng.integers(1, 9, V)
    wl1 = wl + 1
    ws = np.concatenate([[0], np.cumsum(wl1)[:-1]])
    vocab = np.full(int(wl1.sum()), 32, dtype=np.uint8)
    letters = (rng.choice(48, size=int(wl.sum()), p=p) + 40).astype(np.uint8)
    wstart = np.concatenate([[0], np.cumsum(wl)[:-1]])
    vocab[np.repeat(ws, wl) + (np.arange(int(wl.sum())) - np.repeat(wstart, wl))] = letters
    pw = 1.0 / (np.arange(V) + 2.0) ** 1.05
    pw /= pw.sum()
    t_vocab = torch.from_numpy(vocab).to(device)
    t_ws = torch.from_numpy(ws.astype(np.int64)).to(device)
    t_wl1 = torch.from_numpy(wl1.astype(np.int64)).to(device)
    t_cdf = torch.from_numpy(np.cumsum(pw)).to(device)
    mean = float(wl1 @ pw)

    def text(n):
        nw = int(n / mean * 1.05) + 16
        ids = torch.searchsorted(t_cdf, torch.rand(nw, generator=g, device=device, dtype=torch.float64))
        ids.clamp_(max=V - 1)
        lens = t_wl1[ids]
        ends = torch.cumsum(lens, 0)
        k = int(torch.searchsorted(ends, torch.tensor([n], device=device)).item()) + 1
        ids, lens, ends = ids[:k], lens[:k], ends[:k]
        base = torch.repeat_interleave(t_ws[ids] - (ends - lens), lens)
        return t_vocab[base[:n] + torch.arange(n, device=device)]

    out = torch.empty(nbytes, dtype=torch.uint8, device=device)
    pos = 0
    while pos < nbytes:
        if kind == "text":
            n = min(piece, nbytes - pos)
            out[pos:pos + n] = text(n)
        else:
            n = min(int(rng.integers(64 << 10, 4 << 20)), nbytes - pos)
            r = rng.random()
            if r < 0.5:
                out[pos:pos + n] = text(n)
            elif r < 0.75:
                out[pos:pos + n] = torch.randint(0, 256, (n,), generator=g, device=device, dtype=torch.uint8)
            else:
                seg = torch.full((n,), int(rng.integers(0, 3)), dtype=torch.uint8, device=device)
                k = max(1, n // 4096)
                idx = torch.randint(0, n, (k,), generator=g, device=device)
                seg[idx] = torch.randint(0, 256, (k,), generator=g, device=device, dtype=torch.uint8)
                out[pos:pos + n] = seg
        pos += n
    return out
