#!/usr/bin/env python3
"""Generate tests/golden/vectors.json with an independent pure-Python restatement.

Why: the reference's hot-path arithmetic lives in the Rust crates fastcdc 3.0.3 and blake3 1.3.3,
which are absent from /root/reference and cannot be built here (no cargo/rustc, no network),
and the reference's own tests pin none of this path.  So the fixtures are
produced by a SECOND restatement written in a different style from oracle/bw_oracle.c:

  * BLAKE3: the spec's incremental hasher (chunk state + lazily merged CV stack), versus the
    C oracle's recursive subtree split;
  * FastCDC v2020: the per-byte recurrence h_p = (h_{p-1} << 1) + GEAR[b] with explicit
    mask regions, versus the C oracle's two-bytes-per-step loop (SURVEY.md A.1 equivalence);
  * GEAR regenerated from its MD5 rule with hashlib; MASKS restated from SURVEY.md A.3.

Both restatements must agree with the published BLAKE3 known answers and the
A.5 cross-check vector.  Inputs are splitmix64 streams (seed, length), stored with their sha256.
Run:  python tests/golden/make_golden.py   (~30 s)
"""
import hashlib
import json
import os
import sys

M64 = (1 << 64) - 1
M32 = (1 << 32) - 1

# ------------------------------------------------------------------ FastCDC v2020 constants
GEAR = [int.from_bytes(hashlib.md5(bytes([i]) * 64).digest()[:8], "big") for i in range(256)]
MASKS = [0, 0, 0, 0, 0, 0x0000000001804110, 0x0000000001803110, 0x0000000018035100, 0x0000001800035300,
         0x0000019000353000, 0x0000590003530000, 0x0000d90003530000, 0x0000d90103530000, 0x0000d90303530000,
         0x0000d90313530000, 0x0000d90f03530000, 0x0000d90303537000, 0x0000d90703537000, 0x0000d90707537000,
         0x0000d91707537000, 0x0000d91747537000, 0x0000d91767537000, 0x0000d93767537000, 0x0000d93777537000,
         0x0000d93777577000, 0x0000db3777577000]


def masks_for(avg):
    import math
    bits = int(round(math.log2(avg)))
    return MASKS[bits + 1], MASKS[bits - 1]


def cut_per_byte(src, start, end, mn, av, mx, ms, ml):
    n = end - start
    if n <= mn:
        return 0, n
    center, remaining = av, n
    if remaining > mx:
        remaining = mx
    elif remaining < center:
        center = remaining
    s0, c2, r2 = 2 * (mn // 2), 2 * (center // 2), 2 * (remaining // 2)
    h = 0
    for p in range(s0, r2):
        h = ((h << 1) + GEAR[src[start + p]]) & M64
        if h & (ms if p < c2 else ml) == 0:
            return ((h << 1) & M64 if p % 2 == 0 else h), p
    return (h if r2 > s0 else 0), remaining


def fastcdc_py(src, mn, av, mx):
    ms, ml = masks_for(av)
    out, off = [], 0
    while off < len(src):
        h, c = cut_per_byte(src, off, len(src), mn, av, mx, ms, ml)
        out.append((h, off, c))
        off += c
    return out


# ------------------------------------------------------------------ BLAKE3 (incremental form)
IV = [0x6A09E667, 0xBB67AE85, 0x3C6EF372, 0xA54FF53A, 0x510E527F, 0x9B05688C, 0x1F83D9AB, 0x5BE0CD19]
PERM = [2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8]
CHUNK_START, CHUNK_END, PARENT, ROOT = 1, 2, 4, 8


def _g(s, a, b, c, d, x, y):
    s[a] = (s[a] + s[b] + x) & M32
    s[d] = ((s[d] ^ s[a]) >> 16 | (s[d] ^ s[a]) << 16) & M32
    s[c] = (s[c] + s[d]) & M32
    s[b] = ((s[b] ^ s[c]) >> 12 | (s[b] ^ s[c]) << 20) & M32
    s[a] = (s[a] + s[b] + y) & M32
    s[d] = ((s[d] ^ s[a]) >> 8 | (s[d] ^ s[a]) << 24) & M32
    s[c] = (s[c] + s[d]) & M32
    s[b] = ((s[b] ^ s[c]) >> 7 | (s[b] ^ s[c]) << 25) & M32


def compress(cv, words, counter, blen, flags):
    s = list(cv) + IV[:4] + [counter & M32, counter >> 32, blen, flags]
    m = list(words)
    for _ in range(7):
        _g(s, 0, 4, 8, 12, m[0], m[1]); _g(s, 1, 5, 9, 13, m[2], m[3])
        _g(s, 2, 6, 10, 14, m[4], m[5]); _g(s, 3, 7, 11, 15, m[6], m[7])
        _g(s, 0, 5, 10, 15, m[8], m[9]); _g(s, 1, 6, 11, 12, m[10], m[11])
        _g(s, 2, 7, 8, 13, m[12], m[13]); _g(s, 3, 4, 9, 14, m[14], m[15])
        m = [m[i] for i in PERM]
    return [s[i] ^ s[i + 8] for i in range(8)]


def words_of(block):
    block = block + bytes(64 - len(block))
    return [int.from_bytes(block[4 * i:4 * i + 4], "little") for i in range(16)]


class _Chunk:
    def __init__(self, counter):
        self.cv, self.counter, self.buf, self.blocks = list(IV), counter, b"", 0

    def size(self):
        return 64 * self.blocks + len(self.buf)

    def update(self, data):
        while data:
            if len(self.buf) == 64:
                self.cv = compress(self.cv, words_of(self.buf), self.counter, 64,
                                   CHUNK_START if self.blocks == 0 else 0)
                self.blocks += 1
                self.buf = b""
            take = min(64 - len(self.buf), len(data))
            self.buf += data[:take]
            data = data[take:]

    def output(self):  # (cv, words, counter, blen, flags) of the final block
        return (self.cv, words_of(self.buf), self.counter, len(self.buf),
                (CHUNK_START if self.blocks == 0 else 0) | CHUNK_END)


def blake3_py(data):
    stack, chunk = [], _Chunk(0)
    while data:
        if chunk.size() == 1024:
            cv = compress(*chunk.output())
            total = chunk.counter + 1
            while total & 1 == 0:
                cv = compress(IV, stack.pop() + cv, 0, 64, PARENT)
                total >>= 1
            stack.append(cv)
            chunk = _Chunk(chunk.counter + 1)
        take = min(1024 - chunk.size(), len(data))
        chunk.update(data[:take])
        data = data[take:]
    out = chunk.output()
    while stack:
        out = (IV, stack.pop() + compress(*out), 0, 64, PARENT)
    cv, words, counter, blen, flags = out
    root = compress(cv, words, counter, blen, flags | ROOT)
    return b"".join(w.to_bytes(4, "little") for w in root)


# ------------------------------------------------------------------ inputs
def splitmix(seed, n):
    out, x = bytearray(), seed
    while len(out) < n:
        x = (x + 0x9E3779B97F4A7C15) & M64
        z = x
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
        z ^= z >> 31
        out += z.to_bytes(8, "little")
    return bytes(out[:n])


BLAKE3_LENS = [0, 1, 63, 64, 65, 1023, 1024, 1025, 2048, 2049, 3072, 3073, 4096, 4097, 5120, 5121, 6144, 6145,
               7168, 7169, 8192, 8193, 16384, 31744, 102400]

FASTCDC_CASES = [  # (seed, length, min, avg, max)
    (1, 20000, 64, 256, 1024), (2, 50001, 64, 256, 1024), (3, 1, 64, 256, 1024), (4, 64, 64, 256, 1024),
    (5, 65, 64, 256, 1024), (6, 1023, 64, 256, 1024), (7, 1025, 64, 256, 1024), (8, 30000, 65, 300, 1100),
    (9, 120000, 4096, 16384, 65536), (10, 65537, 4096, 16384, 65536), (11, 65535, 4096, 16384, 65535),
    (12, 40000, 8191, 2048, 4096), (13, 300000, 1001, 4000, 9999),
    (0, 8400953, 262144, 1048576, 3145728),
]


def main():
    out = {"generator": "tests/golden/make_golden.py (pure-Python restatement, independent of oracle/)",
           "gear_sha256": hashlib.sha256(b"".join(g.to_bytes(8, "big") for g in GEAR)).hexdigest(),
           "blake3": [], "blake3_kat": {}, "fastcdc": [], "zeros": None}
    for msg in [b"", b"abc", b"\x00"]:
        out["blake3_kat"][msg.hex()] = blake3_py(msg).hex()
    for n in BLAKE3_LENS:
        msg = bytes(i % 251 for i in range(n))
        out["blake3"].append({"input": "i%251", "len": n, "digest": blake3_py(msg).hex()})
    for (seed, n, mn, av, mx) in FASTCDC_CASES:
        data = splitmix(seed, n)
        chunks = fastcdc_py(data, mn, av, mx)
        first = chunks[0]
        out["fastcdc"].append({"seed": seed, "len": n, "min": mn, "avg": av, "max": mx,
                               "sha256": hashlib.sha256(data).hexdigest(),
                               "chunks": [[h, o, l] for (h, o, l) in chunks],
                               "first_chunk_blake3": blake3_py(data[first[1]:first[1] + first[2]]).hex()
                               if first[2] <= 300000 else None})
        print("fastcdc", seed, n, len(chunks), file=sys.stderr)
    z = bytes((8 << 20) + 5)
    out["zeros"] = {"len": len(z), "chunks": [[h, o, l] for (h, o, l) in fastcdc_py(z, 262144, 1048576, 3145728)]}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "vectors.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", path, file=sys.stderr)


if __name__ == "__main__":
    main()
