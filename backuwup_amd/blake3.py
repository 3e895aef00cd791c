"""Drop-in for `blake3::hash` as backuwup uses it (crate blake3 1.3.3, Cargo.lock:149-159).

    let hash = blake3::hash(data).into();     // dir_packer.rs:286 (also :320, :353)

`hash(data)` returns the 32-byte BlobHash computed on the GPU; `hash_many` hashes a batch of
independent messages in one launch sequence (the batched form the GPU wants).
"""
from .context import default_context

OUT_LEN = 32


def hash(data, ctx=None):  # noqa: A001 - mirrors blake3::hash
    return (ctx or default_context()).blake3(data)


def hash_many(data, offsets, lengths, ctx=None):
    """digests (n x 32 uint8) of data[offsets[i] : offsets[i] + lengths[i]]."""
    return (ctx or default_context()).blake3_many(data, offsets, lengths)
