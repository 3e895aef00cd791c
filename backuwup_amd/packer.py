"""Drop-in for the dedup front end of backuwup's packer.

Mirrors, on the GPU:
  * dir_packer::process_file / add_file_blob (client/src/backup/filesystem/dir_packer.rs:231-311):
    files larger than BLOB_DESIRED_TARGET_SIZE are cut by FastCDC(256 KiB, 1 MiB, 3 MiB), smaller
    (and empty) files are one blob; every blob gets blake3::hash as its BlobHash;
  * Manager::add_blob's dedup gate (packfile/pack.rs:31-39): BlobTooLarge for > 3 MiB blobs,
    `Ok(None)` for duplicates;
  * BlobIndex (packfile/blob_index.rs:44-148): seeded from the sorted prior index, then
    is_blob_duplicate + blobs_queued insert in canonical order;
  * split_serialize_tree + add_tree_to_blobs (dir_packer.rs:314-390): file and directory trees
    as bincode blobs, split at 10,000 children, through the same gate.
"""
import numpy as np

from .context import (BLOB_DESIRED_TARGET_SIZE, BLOB_MAX_UNCOMPRESSED_SIZE, BLOB_MINIMUM_TARGET_SIZE,
                      BLOB_DTYPE, Context, default_context, make_params, make_tree)

__all__ = ["BlobIndex", "Manager", "BlobTooLarge", "process_files", "process_file", "add_trees_to_blobs", "BLOB_DTYPE",
           "BLOB_MINIMUM_TARGET_SIZE", "BLOB_DESIRED_TARGET_SIZE", "BLOB_MAX_UNCOMPRESSED_SIZE"]


class BlobTooLarge(ValueError):
    """PackfileError::BlobTooLarge (filesystem/mod.rs:80-105, raised at pack.rs:32-34)."""


class BlobIndex:
    """The seen-chunk index, resident in HBM (one per Context)."""

    def __init__(self, sorted_items=None, ctx=None, capacity_hint=0):
        self.ctx = ctx or default_context()
        self.ctx.index_reset(capacity_hint)
        if sorted_items is not None and len(sorted_items):
            self.load(sorted_items)

    def load(self, sorted_digests):
        """BlobIndex::load (blob_index.rs:167-200): prior backups' digests, sorted."""
        self.ctx.index_seed(sorted_digests)

    def is_blob_duplicate(self, blob_hash):
        """is_blob_duplicate (blob_index.rs:130) followed, for a new blob, by its insert
        (blob_index.rs:109) -- the canonical-order form of the add_blob gate."""
        return bool(self.check_insert_many(np.frombuffer(bytes(blob_hash), dtype=np.uint8))[0])

    def check_insert_many(self, digests):
        return self.ctx.index_check_insert(digests)

    def __len__(self):
        return self.ctx.index_size()


class Manager:
    """The dedup gate of packfile::Manager (pack.rs:31-55); compression/encryption/packfile
    writing downstream of the gate are out of scope and unchanged."""

    def __init__(self, index=None, ctx=None):
        self.index = index or BlobIndex(ctx=ctx)

    def add_blob(self, blob_hash, data_len):
        if data_len > BLOB_MAX_UNCOMPRESSED_SIZE:
            raise BlobTooLarge("blob of %d bytes" % data_len)
        if self.index.is_blob_duplicate(blob_hash):
            return None
        return data_len


def process_files(data, file_off, file_len, min_size=BLOB_MINIMUM_TARGET_SIZE, avg_size=BLOB_DESIRED_TARGET_SIZE,
                  max_size=BLOB_MAX_UNCOMPRESSED_SIZE, small_file_threshold=None, dedup=True, ctx=None,
                  flags=0):
    """A batch of files laid out back to back in `data` -> structured array (BLOB_DTYPE) of blobs
    in canonical order with digests and dedup verdicts against ctx's index."""
    from ._lib import BW_F_NO_DEDUP
    ctx = ctx or default_context()
    p = make_params(min_size, avg_size, max_size, small_file_threshold, flags | (0 if dedup else BW_F_NO_DEDUP))
    return ctx.process_files(data, file_off, file_len, p)


def process_file(data, ctx=None, **kw):
    """One file -> list of BlobHash (the file tree's children, dir_packer.rs:261-271)."""
    data = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    blobs = process_files(data, [0], [data.size], ctx=ctx, **kw)
    return [bytes(b) for b in blobs["digest"]]


def add_trees_to_blobs(trees, ctx=None, dedup=True):
    """add_tree_to_blobs for many trees: `trees` = [(kind, name, size, mtime, ctime, children
    bytes)] with kind 0 = File, 1 = Dir and None for an absent metadata field.  Returns (the hash
    each tree gives its parent, per-piece records with dedup verdicts in canonical order)."""
    ctx = ctx or default_context()
    return ctx.tree_blobs([make_tree(*t) for t in trees], dedup=dedup)
