"""ctypes binding of libbackuwup_amd.so (the C ABI in include/backuwup_gpu.h).

There is no fallback: if the HIP library is missing or cannot be loaded this raises, and
every compute call runs on the GPU through the library.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("BW_LIB") or os.path.join(HERE, "libbackuwup_amd.so")

BW_OK, BW_EINVAL, BW_ENOSPC, BW_EHIP, BW_ENOMEM, BW_ECOLLISION, BW_ESTATE = 0, -1, -2, -3, -4, -5, -6
BW_ECRYPTO, BW_EFORMAT, BW_ECOMM, BW_EAGAIN = -7, -8, -9, -10
BW_COMM_ID_BYTES = 128
BW_COMM_DEFAULT_TIMEOUT_MS = 120000
BW_ZSTD_LANES = 6  # include/backuwup_gpu.h: asynchronous zstd batches in flight per context
BW_F_NO_HASH, BW_F_NO_DEDUP, BW_F_SERIAL_RESOLVE = 1, 2, 4
BW_OPT_DEPTH, BW_OPT_SCAN_SMALL_BYTES, BW_OPT_CAND_CAP, BW_OPT_STAGE_CHUNK, BW_OPT_B3_LOADS = 1, 2, 3, 4, 5
BW_OPT_SCAN_WAVES, BW_OPT_LATENCY_STREAM, BW_OPT_ZSTD_SLOTS, BW_OPT_ZSTD_BATCH_BYTES = 6, 7, 8, 9
BW_OPT_ORDER_HASH, BW_OPT_SPLIT = 10, 11
BW_OPT_PROFILE_MASK, BW_OPT_SCAN_FIRST, BW_OPT_B3_UPPER, BW_OPT_B3_GROUP = 12, 13, 14, 15
BW_B3_LOADS_DEFAULT = 2  # the library's BW_OPT_B3_LOADS default (bw_capi.hip)

u8p = ctypes.POINTER(ctypes.c_uint8)
u64p = ctypes.POINTER(ctypes.c_uint64)
vp = ctypes.c_void_p


class BwChunk(ctypes.Structure):
    _fields_ = [("hash", ctypes.c_uint64), ("offset", ctypes.c_uint64), ("length", ctypes.c_uint64)]


class BwBlob(ctypes.Structure):
    _fields_ = [("file", ctypes.c_uint64), ("offset", ctypes.c_uint64), ("length", ctypes.c_uint64),
                ("gear_hash", ctypes.c_uint64), ("digest", ctypes.c_uint8 * 32),
                ("is_dup", ctypes.c_uint8), ("pad", ctypes.c_uint8 * 7)]


class BwParams(ctypes.Structure):
    _fields_ = [("min_size", ctypes.c_uint32), ("avg_size", ctypes.c_uint32),
                ("max_size", ctypes.c_uint32), ("flags", ctypes.c_uint32),
                ("small_file_threshold", ctypes.c_uint64)]


class BwTree(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_uint32), ("flags", ctypes.c_uint32), ("size", ctypes.c_uint64),
                ("mtime", ctypes.c_uint64), ("ctime", ctypes.c_uint64), ("name", vp),
                ("name_len", ctypes.c_uint64), ("children", vp), ("n_children", ctypes.c_uint64)]


class BwTreeBlob(ctypes.Structure):
    _fields_ = [("tree", ctypes.c_uint64), ("piece", ctypes.c_uint64), ("length", ctypes.c_uint64),
                ("hash", ctypes.c_uint8 * 32), ("is_dup", ctypes.c_uint8), ("pad", ctypes.c_uint8 * 7)]


class BwStreamShard(ctypes.Structure):
    _fields_ = [("ticket", ctypes.c_uint64), ("first_blob", ctypes.c_uint64), ("n_blobs", ctypes.c_uint64),
                ("chain_start", ctypes.c_uint64), ("rounds", ctypes.c_uint32), ("pad", ctypes.c_uint32)]


class BwPackfile(ctypes.Structure):
    _fields_ = [("first_blob", ctypes.c_uint64), ("n_blobs", ctypes.c_uint64), ("offset", ctypes.c_uint64),
                ("size", ctypes.c_uint64), ("header_len", ctypes.c_uint64)]


class BwIndexFile(ctypes.Structure):
    _fields_ = [("file_num", ctypes.c_uint32), ("pad", ctypes.c_uint32), ("offset", ctypes.c_uint64),
                ("size", ctypes.c_uint64), ("n_entries", ctypes.c_uint64)]


BW_PACKFILE_TARGET_SIZE, BW_PACKFILE_MAX_SIZE, BW_PACKFILE_MAX_BLOBS = 3 * 1024 * 1024, 16 * 1024 * 1024, 100_000
BW_BLOB_NONCE_SIZE, BW_INDEX_MAX_FILE_ENTRIES, BW_INDEX_ENTRY_BYTES = 12, 50_000, 44
BW_BLOB_FILE_CHUNK, BW_BLOB_TREE = 0, 1
BW_PACK_ZSTD_STORE = 1

BW_TREE_FILE, BW_TREE_DIR = 0, 1
BW_TREE_HAS_SIZE, BW_TREE_HAS_MTIME, BW_TREE_HAS_CTIME = 1, 2, 4
BW_TREE_BLOB_MAX_CHILDREN = 10000

# (name, restype, argtypes) for every symbol of include/backuwup_gpu.h
SIGNATURES = [
    ("bw_params_default", None, [ctypes.POINTER(BwParams)]),
    ("bw_strerror", ctypes.c_char_p, [ctypes.c_int]),
    ("bw_create", ctypes.c_int, [ctypes.c_int, ctypes.POINTER(vp)]),
    ("bw_destroy", None, [vp]),
    ("bw_last_error", ctypes.c_char_p, [vp]),
    ("bw_set_stream", ctypes.c_int, [vp, vp]),
    ("bw_get_stream", vp, [vp]),
    ("bw_fastcdc_chunks", ctypes.c_int, [vp, vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                         ctypes.c_uint32, ctypes.POINTER(BwChunk), ctypes.c_uint64, u64p]),
    ("bw_blake3_hash", ctypes.c_int, [vp, vp, ctypes.c_uint64, u8p]),
    ("bw_blake3_hash_many", ctypes.c_int, [vp, vp, ctypes.c_uint64, u64p, u64p, ctypes.c_uint64, u8p]),
    ("bw_index_reset", ctypes.c_int, [vp, ctypes.c_uint64]),
    ("bw_index_seed", ctypes.c_int, [vp, vp, ctypes.c_uint64]),
    ("bw_index_check_insert", ctypes.c_int, [vp, vp, ctypes.c_uint64, u8p]),
    ("bw_index_size", ctypes.c_int, [vp, u64p]),
    ("bw_index_check", ctypes.c_int, [vp]),
    ("bw_index_create", ctypes.c_int, [ctypes.c_int, ctypes.POINTER(vp)]),
    ("bw_index_destroy", None, [vp]),
    ("bw_attach_index", ctypes.c_int, [vp, vp]),
    ("bw_set_option", ctypes.c_int, [vp, ctypes.c_int, ctypes.c_uint64]),
    ("bw_submit_device", ctypes.c_int, [vp, vp, ctypes.c_uint64, u64p, u64p, ctypes.c_uint64,
                                        ctypes.POINTER(BwParams), u64p]),
    ("bw_submit_host", ctypes.c_int, [vp, vp, ctypes.c_uint64, u64p, u64p, ctypes.c_uint64,
                                      ctypes.POINTER(BwParams), u64p]),
    ("bw_wait", ctypes.c_int, [vp, ctypes.c_uint64, ctypes.POINTER(BwBlob), ctypes.c_uint64, u64p]),
    ("bw_host_register", ctypes.c_int, [vp, ctypes.c_uint64]),
    ("bw_host_unregister", ctypes.c_int, [vp]),
    ("bw_process_files", ctypes.c_int, [vp, vp, ctypes.c_uint64, u64p, u64p, ctypes.c_uint64,
                                        ctypes.POINTER(BwParams), ctypes.POINTER(BwBlob), ctypes.c_uint64,
                                        u64p]),
    ("bw_process_files_device", ctypes.c_int, [vp, vp, ctypes.c_uint64, u64p, u64p, ctypes.c_uint64,
                                               ctypes.POINTER(BwParams)]),
    ("bw_results", ctypes.c_int, [vp, ctypes.POINTER(BwBlob), ctypes.c_uint64, u64p]),
    ("bw_batch_device_views", ctypes.c_int, [vp, u64p, ctypes.POINTER(vp), ctypes.POINTER(vp)]),
    ("bw_partition_by_owner", ctypes.c_int, [vp, vp, ctypes.c_uint64, ctypes.c_uint32, vp, vp, u64p]),
    ("bw_index_check_insert_device", ctypes.c_int, [vp, vp, ctypes.c_uint64, vp]),
    ("bw_scatter_verdicts", ctypes.c_int, [vp, vp, vp, ctypes.c_uint64, vp]),
    ("bw_batch_views", ctypes.c_int, [vp, ctypes.c_uint64, ctypes.POINTER(vp), ctypes.POINTER(vp),
                                      ctypes.POINTER(vp), u64p]),
    ("bw_partition_buckets", ctypes.c_int, [vp, vp, vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, vp, vp,
                                            vp]),
    ("bw_index_check_insert_buckets", ctypes.c_int, [vp, vp, vp, ctypes.c_uint32, ctypes.c_uint64, vp]),
    ("bw_scatter_buckets", ctypes.c_int, [vp, vp, vp, vp, ctypes.c_uint32, ctypes.c_uint64, vp]),
    ("bw_comm_unique_id", ctypes.c_int, [u8p]),
    ("bw_comm_init", ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, u8p, ctypes.POINTER(vp)]),
    ("bw_comm_init_timeout", ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, u8p, ctypes.c_uint32,
                                            ctypes.POINTER(vp)]),
    ("bw_comm_set_timeout", ctypes.c_int, [vp, ctypes.c_uint32]),
    ("bw_comm_status", ctypes.c_int, [vp]),
    ("bw_comm_init_host", ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, vp, ctypes.POINTER(vp)]),
    ("bw_comm_init_all", ctypes.c_int, [ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_uint32, ctypes.POINTER(vp)]),
    ("bw_comm_init_local", ctypes.c_int, [ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.POINTER(vp)]),
    ("bw_comm_destroy", None, [vp]),
    ("bw_comm_last_error", ctypes.c_char_p, [vp]),
    ("bw_comm_set_capacity", ctypes.c_int, [vp, ctypes.c_uint64]),
    ("bw_exchange_dedup", ctypes.c_int, [vp, vp, ctypes.c_uint64]),
    ("bw_comm_progress", ctypes.c_int, [vp]),
    ("bw_stream_window", ctypes.c_int, [ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_uint32, u64p, u64p]),
    ("bw_chunk_stream_shard", ctypes.c_int, [vp, vp, vp, ctypes.c_uint64, ctypes.POINTER(BwParams),
                                             ctypes.POINTER(BwStreamShard)]),
    ("bw_tree_serialize", ctypes.c_int, [ctypes.POINTER(BwTree), vp, vp, ctypes.c_uint64, u64p]),
    ("bw_tree_blobs", ctypes.c_int, [vp, ctypes.POINTER(BwTree), ctypes.c_uint64, ctypes.c_uint32, vp,
                                     ctypes.POINTER(BwTreeBlob), ctypes.c_uint64, u64p]),
    ("bw_seal_device", ctypes.c_int, [vp, vp, vp, u64p, u64p, ctypes.c_uint64, vp, ctypes.c_uint32, vp, vp,
                                      u64p]),
    ("bw_open_device", ctypes.c_int, [vp, vp, vp, u64p, u64p, ctypes.c_uint64, vp, ctypes.c_uint32, vp, vp,
                                      u64p, u8p]),
    ("bw_seal", ctypes.c_int, [vp, vp, vp, u64p, u64p, ctypes.c_uint64, vp, ctypes.c_uint32, vp, vp, u64p]),
    ("bw_open", ctypes.c_int, [vp, vp, vp, u64p, u64p, ctypes.c_uint64, vp, ctypes.c_uint32, vp, vp, u64p, u8p]),
    ("bw_zstd_store_size", ctypes.c_uint64, [ctypes.c_uint64]),
    ("bw_zstd_compress_device", ctypes.c_int, [vp, vp, u64p, u64p, ctypes.c_uint64, vp, u64p, u64p]),
    ("bw_zstd_compress", ctypes.c_int, [vp, vp, u64p, u64p, ctypes.c_uint64, vp, u64p, u64p]),
    ("bw_zstd_submit_device", ctypes.c_int, [vp, vp, u64p, u64p, ctypes.c_uint64, vp, u64p, u64p]),
    ("bw_zstd_wait", ctypes.c_int, [vp, ctypes.c_uint64, u64p]),
    ("bw_pack_plan", ctypes.c_int, [u64p, ctypes.c_uint64, ctypes.c_uint32, ctypes.POINTER(BwPackfile),
                                    ctypes.c_uint64, u64p, u64p]),
    ("bw_pack_plan_session", ctypes.c_int, [vp, vp, u64p, ctypes.c_uint64, ctypes.c_uint32,
                                            ctypes.POINTER(BwPackfile), ctypes.c_uint64, u64p, u64p, u64p]),
    ("bw_pack_build_device", ctypes.c_int, [vp, vp, vp, u64p, u64p, ctypes.c_uint64, vp, vp, vp, ctypes.c_uint32,
                                            ctypes.POINTER(BwPackfile), ctypes.c_uint64, vp, vp]),
    ("bw_pack_build", ctypes.c_int, [vp, vp, vp, u64p, u64p, ctypes.c_uint64, vp, vp, vp, ctypes.c_uint32,
                                     ctypes.POINTER(BwPackfile), ctypes.c_uint64, vp, vp]),
    ("bw_pack_compress_device", ctypes.c_int, [vp, vp, u64p, u64p, ctypes.c_uint64, u64p]),
    ("bw_pack_build_compressed", ctypes.c_int, [vp, vp, vp, vp, vp, ctypes.POINTER(BwPackfile), ctypes.c_uint64,
                                                vp, vp]),
    ("bw_pack_compress", ctypes.c_int, [vp, vp, u64p, u64p, ctypes.c_uint64, u64p]),
    ("bw_pack_build_compressed_host", ctypes.c_int, [vp, vp, vp, vp, vp, ctypes.POINTER(BwPackfile),
                                                     ctypes.c_uint64, vp, vp]),
    ("bw_index_files_build", ctypes.c_int, [vp, vp, vp, ctypes.c_uint64, ctypes.c_uint32, vp, ctypes.c_uint64,
                                            ctypes.POINTER(BwIndexFile), ctypes.c_uint64, u64p, u64p]),
    ("bw_index_load_files", ctypes.c_int, [vp, vp, vp, ctypes.POINTER(BwIndexFile), ctypes.c_uint64, vp,
                                           ctypes.c_uint64, u64p, u64p]),
    ("bw_profile_enable", ctypes.c_int, [vp, ctypes.c_int]),
    ("bw_fastcdc_chunks_hashed", ctypes.c_int, [vp, vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                                ctypes.c_uint32, vp, ctypes.c_uint64, u64p, u64p]),
    ("bw_fastcdc_release", None, [ctypes.c_uint64]),
    ("bw_blake3_kept_hits", ctypes.c_uint64, []),
    ("bw_blake3_hash_dropin", ctypes.c_int, [vp, vp, ctypes.c_uint64, u8p]),
    ("bw_blake3_hash_dropin_device", ctypes.c_int, [ctypes.c_int, vp, ctypes.c_uint64, u8p]),
    ("bw_blake3_coalesce_stats", ctypes.c_int, [ctypes.c_int, u64p, u64p]),
    ("bw_blake3_service_faults", ctypes.c_int, [ctypes.c_int, u64p, u64p, u64p]),
    ("bw_device_count", ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    ("bw_profile_read", ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_double), u64p]),
    ("bw_profile_intervals", ctypes.c_int, [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.c_uint64, u64p]),
    ("bw_calibrate_b3", ctypes.c_int, [vp, ctypes.c_double, ctypes.POINTER(ctypes.c_double)]),
]

STAGES = ["scan", "compact", "resolve", "assemble", "b3_leaf", "b3_tree", "dedup", "pack"]
# the kernel each stage's events bracket (names as rocprofv3 reports them)
STAGE_KERNELS = {"scan": "k_scan", "b3_leaf": "k_b3_lines", "b3_tree": "k_b3_upper"}

_lib = None


def load():
    """Load the HIP library; raises OSError/RuntimeError when it is absent (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError("libbackuwup_amd.so not built (run __graft_entry__.build() or "
                           "python backuwup_amd/build.py); there is no CPU fallback")
    # torch ships its own libamdhip64; load it first so the process holds one HIP runtime (our
    # library binds to the already-loaded soname).  Loaded the other way round, both runtimes end
    # up mapped and bw_create fails with a HIP error on the GPU.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(LIB_PATH)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


class BwError(RuntimeError):
    def __init__(self, rc, msg=""):
        self.rc = rc
        text = load().bw_strerror(rc).decode()
        super().__init__("backuwup_amd error %d (%s)%s" % (rc, text, (": " + msg) if msg else ""))


def check(rc, ctx=None):
    if rc != BW_OK:
        msg = ""
        if ctx is not None:
            m = load().bw_last_error(ctx)
            msg = m.decode() if m else ""
        raise BwError(rc, msg)
