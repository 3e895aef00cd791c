"""Deterministic blob corpus for the zstd level-3 tests (test data, generated; no reference
content).  Each kind exercises a different part of the compressor: Huffman literals of skewed
text, dense short matches (thousands of sequences per block, FSE tables with low-probability
symbols), long-distance repeats across a window larger than 2 MiB, long runs (match lengths over
64 KiB, RLE blocks), random bytes (raw blocks) and tiny blobs."""
import random

import numpy as np

KINDS = ("text", "tokens", "repeats", "runs", "random", "mixed")


def blob(kind, n, seed):
    r = random.Random(seed * 1000003 + KINDS.index(kind))
    g = np.random.default_rng(seed * 7 + KINDS.index(kind))
    if kind == "text":
        p = g.dirichlet(np.ones(48) * 0.35)
        words = [bytes((g.choice(48, size=int(g.integers(1, 9)), p=p) + 40).astype(np.uint8))
                 for _ in range(int(g.integers(8, 600)))]
        b = bytearray()
        while len(b) < n:
            b += words[int(g.integers(len(words)))] + b" "
        return bytes(b[:n])
    if kind == "tokens":
        toks = [r.randbytes(r.randrange(4, 7)) for _ in range(r.randrange(2, 64))]
        parts, size = [], 0
        while size < n:
            t = toks[r.randrange(len(toks))]
            if r.random() < 0.3:
                t += bytes([r.randrange(256)])
            parts.append(t)
            size += len(t)
        return b"".join(parts)[:n]
    if kind == "repeats":
        base = r.randbytes(r.randrange(1000, 300000))
        b = bytearray()
        while len(b) < n:
            s = r.randrange(len(base))
            b += base[s:s + r.randrange(100, 200000)]
            if r.random() < 0.3:
                b += r.randbytes(r.randrange(1, 50))
        return bytes(b[:n])
    if kind == "runs":
        b = bytearray()
        while len(b) < n:
            b += bytes([r.randrange(3)]) * r.randrange(1, 400000)
            b += r.randbytes(r.randrange(0, 100))
        return bytes(b[:n])
    if kind == "random":
        return r.randbytes(n)
    b = bytearray()
    while len(b) < n:
        k = r.randrange(3)
        if k == 0:
            b += r.randbytes(r.randrange(1, 3000))
        elif k == 1 and b:
            s = r.randrange(len(b))
            b += b[s:s + r.randrange(4, 5000)]
        else:
            b += bytes([r.randrange(256)]) * r.randrange(1, 2000)
    return bytes(b[:n])


def corpus(sizes, seed=0):
    """[(kind, n, bytes)] for every kind at every size."""
    return [(k, n, blob(k, n, seed + i)) for i, n in enumerate(sizes) for k in KINDS]
