"""ctypes loader for the CPU oracle (oracle/_build/liboracle.so).

TEST INFRASTRUCTURE ONLY -- import from tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never from the product package (backuwup_amd/).  Parity status: see
oracle/bw_oracle.h (unpinned by the reference; pinned by spec KATs and derived constants).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "liboracle.so")


class OrcBlob(ctypes.Structure):
    _fields_ = [("file", ctypes.c_uint64), ("offset", ctypes.c_uint64),
                ("length", ctypes.c_uint64), ("gear_hash", ctypes.c_uint64),
                ("digest", ctypes.c_uint8 * 32), ("is_dup", ctypes.c_uint8),
                ("pad", ctypes.c_uint8 * 7)]


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        u64p = ctypes.POINTER(ctypes.c_uint64)
        L.orc_gear_table.argtypes = [u64p]
        L.orc_fastcdc_masks.argtypes = [ctypes.c_uint32] * 3 + [u64p, u64p]
        L.orc_fastcdc_chunks.argtypes = [ctypes.c_void_p, ctypes.c_size_t] + [ctypes.c_uint32] * 3 + \
            [u64p, u64p, u64p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]
        L.orc_blake3.argtypes = [ctypes.c_void_p, ctypes.c_size_t, u8p]
        L.orc_blake3_fast.argtypes = [ctypes.c_void_p, ctypes.c_size_t, u8p]
        L.orc_set_blake3_simd.argtypes = [ctypes.c_int]
        L.orc_index_new.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        L.orc_index_new.restype = ctypes.c_void_p
        L.orc_index_free.argtypes = [ctypes.c_void_p]
        L.orc_index_is_duplicate.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.orc_index_insert.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        vp = ctypes.c_void_p
        L.orc_sha256.argtypes = [vp, ctypes.c_size_t, vp]
        L.orc_hmac_sha256.argtypes = [vp, ctypes.c_size_t, vp, ctypes.c_size_t, vp]
        L.orc_hkdf_expand32.argtypes = [vp, vp, ctypes.c_size_t, vp]
        L.orc_aes256_encrypt_block.argtypes = [vp, vp, vp]
        L.orc_aes256_gcm_seal.argtypes = [vp, vp, vp, ctypes.c_size_t, vp]
        L.orc_aes256_gcm_open.argtypes = [vp, vp, vp, ctypes.c_size_t, vp]
        L.orc_seal_blob.argtypes = [vp, vp, ctypes.c_size_t, vp, vp, ctypes.c_size_t, vp]
        L.orc_open_blob.argtypes = [vp, vp, ctypes.c_size_t, vp, vp, ctypes.c_size_t, vp]
        L.orc_process_files.argtypes = [ctypes.c_void_p, u64p, u64p, ctypes.c_size_t,
                                        ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                        ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int,
                                        ctypes.POINTER(OrcBlob), ctypes.c_size_t,
                                        ctypes.POINTER(ctypes.c_size_t)]
        L.bwo_zstd3_params.argtypes = [ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint)]
        L.bwo_zstd3_bound.argtypes = [ctypes.c_size_t]
        L.bwo_zstd3_bound.restype = ctypes.c_size_t
        L.bwo_zstd3_compress.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        L.bwo_zstd3_compress.restype = ctypes.c_size_t
        _lib = L
    return _lib


def _u64p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))


def _buf(data):
    if isinstance(data, np.ndarray):
        return data.ctypes.data, data.nbytes, data
    b = bytes(data)
    return ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p).value, len(b), b


def gear_table():
    out = np.zeros(256, dtype=np.uint64)
    lib().orc_gear_table(_u64p(out))
    return out


def masks(min_size, avg_size, max_size):
    s, l = ctypes.c_uint64(), ctypes.c_uint64()
    if lib().orc_fastcdc_masks(min_size, avg_size, max_size, ctypes.byref(s), ctypes.byref(l)):
        raise ValueError("fastcdc parameter out of range")
    return s.value, l.value


class CratePanic(ValueError):
    """The crate would panic here (index out of bounds in cut(), only with avg > max)."""


def fastcdc(data, min_size, avg_size, max_size):
    """FastCDC::new(data, min, avg, max).collect() -> list of (hash, offset, length)."""
    ptr, n, keep = _buf(data)
    cap = n // max(min(2 * (min_size // 2), max_size), 1) + 2
    h, o, l = (np.zeros(cap, dtype=np.uint64) for _ in range(3))
    cnt = ctypes.c_size_t()
    rc = lib().orc_fastcdc_chunks(ptr, n, min_size, avg_size, max_size, _u64p(h), _u64p(o),
                                  _u64p(l), cap, ctypes.byref(cnt))
    if rc == -3:
        raise CratePanic("fastcdc 3.0.3 cut() indexes past the source (avg %d > max %d)" % (avg_size, max_size))
    if rc:
        raise ValueError("orc_fastcdc_chunks rc=%d" % rc)
    k = cnt.value
    return [(int(h[i]), int(o[i]), int(l[i])) for i in range(k)]


def blake3(data):
    ptr, n, keep = _buf(data)
    out = (ctypes.c_uint8 * 32)()
    lib().orc_blake3(ptr, n, out)
    return bytes(out)


def blake3_fast(data):
    """The 16-way SIMD restatement of the crate's hash_many strategy (bit-identical to blake3)."""
    ptr, n, keep = _buf(data)
    out = (ctypes.c_uint8 * 32)()
    lib().orc_blake3_fast(ptr, n, out)
    return bytes(out)


def simd_available():
    return bool(lib().orc_blake3_simd_available())


def set_blake3_simd(on):
    """process_files hashes with the SIMD restatement (True) or the scalar one; returns the mode."""
    return bool(lib().orc_set_blake3_simd(1 if on else 0))


class Index:
    """BlobIndex restatement: sorted prior items + blobs_queued set (blob_index.rs:44-148)."""

    def __init__(self, sorted_digests=b""):
        arr = np.frombuffer(bytes(sorted_digests), dtype=np.uint8)
        self._keep = arr
        self.h = lib().orc_index_new(arr.ctypes.data if arr.size else None, arr.size // 32)

    def is_blob_duplicate(self, d):
        return bool(lib().orc_index_is_duplicate(self.h, bytes(d)))

    def insert(self, d):
        return lib().orc_index_insert(self.h, bytes(d))

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_index_free(self.h)
            self.h = None


def process_files(data, file_off, file_len, min_size=262144, avg_size=1048576,
                  max_size=3145728, small_threshold=None, index=None, threads=1):
    """Batch front end -> structured numpy array of blobs (file, offset, length, gear_hash,
    digest, is_dup) in canonical order."""
    if small_threshold is None:
        small_threshold = avg_size
    ptr, n, keep = _buf(data)
    fo = np.ascontiguousarray(file_off, dtype=np.uint64)
    fl = np.ascontiguousarray(file_len, dtype=np.uint64)
    cap = int(sum(int(x) // max(min(2 * (min_size // 2), max_size), 1) + 2 for x in fl)) + 1
    out = (OrcBlob * cap)()
    cnt = ctypes.c_size_t()
    rc = lib().orc_process_files(ptr, _u64p(fo), _u64p(fl), len(fo), min_size, avg_size, max_size,
                                 small_threshold, index.h if index else None, threads, out, cap,
                                 ctypes.byref(cnt))
    if rc:
        raise RuntimeError("orc_process_files rc=%d" % rc)
    arr = np.frombuffer(out, dtype=BLOB_DTYPE, count=cnt.value).copy()
    return arr


BLOB_DTYPE = np.dtype([("file", "<u8"), ("offset", "<u8"), ("length", "<u8"),
                       ("gear_hash", "<u8"), ("digest", "u1", (32,)), ("is_dup", "u1"),
                       ("pad", "u1", (7,))])
assert BLOB_DTYPE.itemsize == ctypes.sizeof(OrcBlob) == 72


# ------------------------------------------------------------------ tree blobs (pure Python)
# dir_packer.rs:314-363 split_serialize_tree; mod.rs:63-77 Tree / TreeMetadata; bincode 1.3.3
# `bincode::serialize` (Cargo.lock:117-119): fixint little endian, enum = u32 variant index,
# String / Vec = u64 length + items, Option = u8 tag + value, [u8; 32] = 32 raw bytes.
TREE_BLOB_MAX_CHILDREN = 10000  # dir_packer.rs:35


def tree_serialize(kind, name, size, mtime, ctime, children, next_sibling=None):
    import struct
    nm = name.encode("utf-8") if isinstance(name, str) else bytes(name)
    out = struct.pack("<I", kind) + struct.pack("<Q", len(nm)) + nm
    for v in (size, mtime, ctime):
        out += b"\x00" if v is None else b"\x01" + struct.pack("<Q", v)
    ch = bytes(children)
    assert len(ch) % 32 == 0
    out += struct.pack("<Q", len(ch) // 32) + ch
    out += b"\x00" if next_sibling is None else b"\x01" + bytes(next_sibling)
    return out


def split_serialize_tree(kind, name, size, mtime, ctime, children):
    """-> [(serialized piece, blake3 hash)] in the order add_tree_to_blobs adds them."""
    ch = bytes(children)
    n = len(ch) // 32
    if n <= TREE_BLOB_MAX_CHILDREN:
        d = tree_serialize(kind, name, size, mtime, ctime, ch)
        return [(d, blake3(d))]
    pieces = [ch[i * 32:(i + TREE_BLOB_MAX_CHILDREN) * 32] for i in range(0, n, TREE_BLOB_MAX_CHILDREN)]
    out = []
    for idx, part in enumerate(reversed(pieces)):
        sib = None if idx == 0 else out[0][1]
        d = tree_serialize(kind, name, size, mtime, ctime, part, sib)
        out.insert(0, (d, blake3(d)))
    return out


# ------------------------------------------------------------------ sealing (bw_oracle_seal.c)
# pack.rs:58-80 compress_encrypt_blob (after zstd), key_manager.rs:80-86 derive_backup_key.


def _out(n):
    return (ctypes.c_uint8 * max(n, 1))()


def sha256(data):
    ptr, n, keep = _buf(data)
    o = _out(32)
    lib().orc_sha256(ptr, n, o)
    return bytes(o)


def hmac_sha256(key, msg):
    o = _out(32)
    key, msg = bytes(key), bytes(msg)
    lib().orc_hmac_sha256(key, len(key), msg, len(msg), o)
    return bytes(o)


def hkdf_expand32(prk, info):
    """Hkdf::<Sha256>::from_prk(prk).expand(info, [0u8; 32])"""
    o = _out(32)
    info = bytes(info)
    lib().orc_hkdf_expand32(bytes(prk), info, len(info), o)
    return bytes(o)


def aes256_block(key, block):
    o = _out(16)
    lib().orc_aes256_encrypt_block(bytes(key), bytes(block), o)
    return bytes(o)


def gcm_seal(key, nonce, pt):
    """Aes256Gcm::new(key).encrypt_in_place(nonce, b"", pt) -> ciphertext || tag"""
    ptr, n, keep = _buf(pt)
    o = _out(n + 16)
    lib().orc_aes256_gcm_seal(bytes(key), bytes(nonce), ptr, n, o)
    return bytes(o)[:n + 16]


def gcm_open(key, nonce, ct):
    """decrypt_in_place: plaintext, or None when the tag does not verify"""
    ptr, n, keep = _buf(ct)
    o = _out(n)
    if lib().orc_aes256_gcm_open(bytes(key), bytes(nonce), ptr, n, o):
        return None
    return bytes(o)[:max(n - 16, 0)]


def seal_blob(prk, info, nonce, payload):
    return gcm_seal(hkdf_expand32(prk, info), nonce, payload)


def open_blob(prk, info, nonce, sealed):
    return gcm_open(hkdf_expand32(prk, info), nonce, sealed)


# ---- zstd level 3 (bw_oracle_zstd.c; pack.rs:58-64) ----
def zstd3_params(n):
    """(window log, small-hash log, long-hash log, min match) of level 3 for an n-byte blob."""
    out = (ctypes.c_uint * 4)()
    lib().bwo_zstd3_params(n, out)
    return tuple(out)


def zstd3_compress(data):
    """The magicless level-3 frame the reference's Compressor writes for one blob."""
    data = bytes(data)
    L = lib()
    out = ctypes.create_string_buffer(L.bwo_zstd3_bound(len(data)))
    n = L.bwo_zstd3_compress(data, len(data), out)
    return out.raw[:n]
