"""backuwup_amd -- MI355X (gfx950) dedup front end for backuwup.

FastCDC-v2020 chunking -> BLAKE3 chunk IDs -> seen-chunk index, as hand-written HIP kernels
behind the C ABI in include/backuwup_gpu.h (libbackuwup_amd.so, built in-tree).  The Python
modules mirror the reference's call sites:

  backuwup_amd.fastcdc.FastCDC   <- fastcdc::v2020::FastCDC   (dir_packer.rs:254-266)
  backuwup_amd.blake3.hash       <- blake3::hash              (dir_packer.rs:286)
  backuwup_amd.packer.BlobIndex  <- packfile::blob_index::BlobIndex (blob_index.rs:44-148)
  backuwup_amd.packer.process_files <- dir_packer::process_file + add_file_blob
  Context.submit_host / submit_device / wait <- the same, pipelined (batches in flight, host-streamed)
  Index + Context.attach_index    <- one BlobIndex shared by every task of a backup session
  Context.tree_blobs / tree_serialize <- split_serialize_tree + add_tree_to_blobs (dir_packer.rs:314-390)
  Context.seal / seal_device      <- derive_backup_key + Aes256Gcm (pack.rs:66-80, key_manager.rs:80-86)
  Context.pack_plan / pack_build  <- Manager::write_packfiles + serialize_packfile (pack.rs:115-227)
  Context.index_files_build / index_load_files <- BlobIndex::push/flush/load (blob_index.rs:151-240)
  backuwup_amd.sharded            <- the index partitioned by digest prefix across ranks (RCCL)
  backuwup_amd.stream_split       <- one long file split across ranks (halo windows, settlement)
"""
from . import _lib
from .context import (BLOB_DTYPE, TREE_BLOB_DTYPE, Context, Index, default_context, host_register, host_unregister,
                      make_params, make_tree, tree_serialize)

__all__ = ["Context", "Index", "default_context", "make_params", "make_tree", "tree_serialize", "BLOB_DTYPE",
           "TREE_BLOB_DTYPE", "host_register", "host_unregister", "load_library"]


def load_library():
    return _lib.load()
