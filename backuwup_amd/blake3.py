"""Drop-in for `blake3::hash` as backuwup uses it (crate blake3 1.3.3, Cargo.lock:149-159).

    let hash = blake3::hash(data).into();     // dir_packer.rs:286 (also :320, :353)

`hash(data)` returns the 32-byte BlobHash computed on the GPU; `hash_many` hashes a batch of
independent messages in one launch sequence (the batched form the GPU wants: one call per file
is a synchronous round trip).
"""
import numpy as np


OUT_LEN = 32


def _as_bytes_view(data):
    if isinstance(data, np.ndarray):
        if data.dtype != np.uint8:
            raise TypeError("blake3: expected a uint8 array, got %s" % data.dtype)
        return data.ravel()
    return np.frombuffer(memoryview(data).cast("B"), dtype=np.uint8)


def _immutable(data):
    """True for memory nobody can rewrite through Python: bytes, and read-only buffers (a
    memoryview of bytes, an mmap opened with ACCESS_READ).  Only such memory may be answered from
    the digests a FastCDC drop-in kept (a rewritten bytearray or numpy buffer must be
    hashed again, never answered from an earlier chunking)."""
    if isinstance(data, bytes):
        return True
    if isinstance(data, np.ndarray):
        return False  # writeable=False can be a view of memory writable through its base
    try:
        return memoryview(data).readonly
    except TypeError:
        return False


def hash(data, ctx=None):  # noqa: A001 - mirrors blake3::hash
    """blake3::hash(data) -> 32 bytes (the crate's Hash converted with .into()).  A message of at
    most 64 KiB goes to the library's hash service, a persistent kernel that serves the calls of
    every thread without a launch per call.  Without `ctx` the call goes through the drop-in pool
    (backuwup_amd/pool.py: this thread's home device of every GPU of the node, the Rust crate's
    policy); with one, through that context (bw_blake3_hash_dropin / bw_blake3_hash)."""
    buf = _as_bytes_view(data)
    if ctx is None:
        from .pool import default_pool
        p = default_pool()
        return p.hash_dropin(data) if _immutable(data) else p.with_context(lambda c: c.blake3(buf))
    return ctx.blake3_dropin(buf) if _immutable(data) else ctx.blake3(buf)


def hash_many(data, offsets, lengths, ctx=None):
    """Digests (n x 32 uint8) of data[offsets[i] : offsets[i] + lengths[i]] for every i, in one
    batch.  Ranges may overlap; each must lie inside `data` (ValueError otherwise)."""
    buf = _as_bytes_view(data)
    offs = np.asarray(offsets, dtype=np.uint64).ravel()
    lens = np.asarray(lengths, dtype=np.uint64).ravel()
    if offs.shape != lens.shape:
        raise ValueError("blake3.hash_many: %d offsets but %d lengths" % (offs.size, lens.size))
    if offs.size and int((offs + lens).max()) > buf.size:
        raise ValueError("blake3.hash_many: a message runs past the end of the data")
    if ctx is None:
        from .pool import default_pool
        return default_pool().with_context(lambda c: c.blake3_many(buf, offs, lens))
    return ctx.blake3_many(buf, offs, lens)
