"""GPU context (one bw_ctx: a HIP stream, device workspaces and the in-HBM dedup index)."""
import ctypes

import numpy as np

from . import _lib
from ._lib import BwBlob, BwParams, check

BLOB_DTYPE = np.dtype([("file", "<u8"), ("offset", "<u8"), ("length", "<u8"), ("gear_hash", "<u8"),
                       ("digest", "u1", (32,)), ("is_dup", "u1"), ("pad", "u1", (7,))])
assert BLOB_DTYPE.itemsize == ctypes.sizeof(BwBlob) == 72

# backuwup's chunker constants (client/src/defaults.rs:61-68)
BLOB_MINIMUM_TARGET_SIZE = 256 * 1024
BLOB_DESIRED_TARGET_SIZE = 1024 * 1024
BLOB_MAX_UNCOMPRESSED_SIZE = 3 * 1024 * 1024


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a.size else ctypes.c_void_p(None)


def _as_u8(data):
    if isinstance(data, np.ndarray):
        return np.ascontiguousarray(data).view(np.uint8).reshape(-1)
    return np.frombuffer(bytes(data), dtype=np.uint8)


def make_params(min_size=BLOB_MINIMUM_TARGET_SIZE, avg_size=BLOB_DESIRED_TARGET_SIZE,
                max_size=BLOB_MAX_UNCOMPRESSED_SIZE, small_file_threshold=None, flags=0):
    p = BwParams()
    p.min_size, p.avg_size, p.max_size, p.flags = min_size, avg_size, max_size, flags
    p.small_file_threshold = avg_size if small_file_threshold is None else small_file_threshold
    return p


# the C struct bw_tree as a numpy record, for building many trees without Python objects
TREE_DTYPE = np.dtype([("kind", "<u4"), ("flags", "<u4"), ("size", "<u8"), ("mtime", "<u8"), ("ctime", "<u8"),
                       ("name", "<u8"), ("name_len", "<u8"), ("children", "<u8"), ("n_children", "<u8")])
assert TREE_DTYPE.itemsize == ctypes.sizeof(_lib.BwTree) == 64
TREE_BLOB_DTYPE = np.dtype([("tree", "<u8"), ("piece", "<u8"), ("length", "<u8"), ("hash", "u1", (32,)),
                            ("is_dup", "u1"), ("pad", "u1", (7,))])
assert TREE_BLOB_DTYPE.itemsize == ctypes.sizeof(_lib.BwTreeBlob) == 64
PACKFILE_DTYPE = np.dtype([("first_blob", "<u8"), ("n_blobs", "<u8"), ("offset", "<u8"), ("size", "<u8"),
                           ("header_len", "<u8")])
assert PACKFILE_DTYPE.itemsize == ctypes.sizeof(_lib.BwPackfile) == 40


def make_tree(kind, name, size=None, mtime=None, ctime=None, children=b""):
    """A Tree (client/src/backup/filesystem/mod.rs:63-77) as the C struct plus the buffers it
    points at: kind 0 = File, 1 = Dir; name str/bytes; children = concatenated 32-byte hashes."""
    nm = name.encode("utf-8", "surrogateescape") if isinstance(name, str) else bytes(name)
    ch = np.ascontiguousarray(np.frombuffer(bytes(children), dtype=np.uint8) if not isinstance(children, np.ndarray)
                              else children.reshape(-1).view(np.uint8))
    assert ch.size % 32 == 0
    nb = np.frombuffer(nm, dtype=np.uint8).copy() if nm else np.zeros(0, dtype=np.uint8)
    t = _lib.BwTree()
    t.kind = kind
    t.flags = (_lib.BW_TREE_HAS_SIZE if size is not None else 0) | \
        (_lib.BW_TREE_HAS_MTIME if mtime is not None else 0) | (_lib.BW_TREE_HAS_CTIME if ctime is not None else 0)
    t.size, t.mtime, t.ctime = size or 0, mtime or 0, ctime or 0
    t.name = nb.ctypes.data if nb.size else None
    t.name_len = nb.size
    t.children = ch.ctypes.data if ch.size else None
    t.n_children = ch.size // 32
    return t, (nb, ch)


def tree_serialize(tree, next_sibling=None):
    """bincode bytes of one Tree (host-only entry point of the library)."""
    t, keep = tree
    L = _lib.load()
    n = ctypes.c_uint64()
    sib = None if next_sibling is None else (ctypes.c_uint8 * 32).from_buffer_copy(bytes(next_sibling))
    rc = L.bw_tree_serialize(ctypes.byref(t), sib, None, 0, ctypes.byref(n))
    if rc != _lib.BW_ENOSPC:
        check(rc)
    out = (ctypes.c_uint8 * max(n.value, 1))()
    check(L.bw_tree_serialize(ctypes.byref(t), sib, out, n.value, ctypes.byref(n)))
    return bytes(out[:n.value])


class Index:
    """One seen-chunk index (bw_index) that several contexts gate against: one backup session
    with several batches in flight on several streams (BlobIndex behind the packer mutex,
    blob_index.rs:44-57, packfile/mod.rs:77)."""

    def __init__(self, device=0):
        self._L = _lib.load()
        h = ctypes.c_void_p()
        check(self._L.bw_index_create(device, ctypes.byref(h)))
        self.h = h
        self.device = device

    def close(self):
        if getattr(self, "h", None):
            self._L.bw_index_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def host_register(ptr, length):
    """Page-lock [ptr, ptr + length) so submit_host DMAs it directly."""
    check(_lib.load().bw_host_register(ctypes.c_void_p(ptr), length))


def host_unregister(ptr):
    check(_lib.load().bw_host_unregister(ctypes.c_void_p(ptr)))


class Context:
    """Owns one bw_ctx on `device`.  Not thread-safe (like the reference's packer mutex)."""

    def __init__(self, device=0):
        self._L = _lib.load()
        h = ctypes.c_void_p()
        check(self._L.bw_create(device, ctypes.byref(h)))
        self.h = h
        self.device = device
        self._zs_n = {}  # zstd ticket -> blob count

    def close(self):
        if getattr(self, "h", None):
            self._L.bw_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -------------------------------------------------------------- streams
    def set_stream(self, hip_stream_handle):
        check(self._L.bw_set_stream(self.h, ctypes.c_void_p(hip_stream_handle)), self.h)

    def stream(self):
        return self._L.bw_get_stream(self.h)

    # -------------------------------------------------------------- chunk / hash
    def fastcdc_chunks(self, data, min_size, avg_size, max_size):
        buf = _as_u8(data)
        cap = buf.size // max(min(2 * (min_size // 2), max_size), 1) + 2
        out = (_lib.BwChunk * cap)()
        n = ctypes.c_uint64()
        check(self._L.bw_fastcdc_chunks(self.h, _ptr(buf), buf.size, min_size, avg_size, max_size, out, cap,
                                        ctypes.byref(n)), self.h)
        return [(out[i].hash, out[i].offset, out[i].length) for i in range(n.value)]

    def fastcdc_chunks_hashed(self, buf, min_size, avg_size, max_size):
        """bw_fastcdc_chunks_hashed over a contiguous uint8 numpy array (kept alive by the caller until
        release): ([(hash, offset, length)], handle).  blake3_at(buf, offset, length) of one of these
        chunks then returns the kept digest; fastcdc_release(handle) drops them."""
        assert isinstance(buf, np.ndarray) and buf.dtype == np.uint8 and buf.flags.c_contiguous
        cap = buf.size // max(min(2 * (min_size // 2), max_size), 1) + 2
        out = (_lib.BwChunk * cap)()
        n, h = ctypes.c_uint64(), ctypes.c_uint64()
        check(self._L.bw_fastcdc_chunks_hashed(self.h, _ptr(buf), buf.size, min_size, avg_size, max_size, out, cap,
                                               ctypes.byref(n), ctypes.byref(h)), self.h)
        return [(out[i].hash, out[i].offset, out[i].length) for i in range(n.value)], h.value

    def fastcdc_release(self, handle):
        self._L.bw_fastcdc_release(handle)

    def blake3_at(self, buf, offset, length, kept=False):
        """blake3::hash(&buf[offset..offset+length]) on the caller's own memory (no copy), as the
        reference hashes each chunk slice of its mmap (dir_packer.rs:262-265, :286).  kept=True goes
        through the drop-in entry (bw_blake3_hash_dropin), which answers a chunk of a live
        fastcdc_chunks_hashed handle from its kept digest: only for memory that cannot change."""
        assert isinstance(buf, np.ndarray) and buf.dtype == np.uint8 and offset + length <= buf.size
        out = (ctypes.c_uint8 * 32)()
        fn = self._L.bw_blake3_hash_dropin if kept else self._L.bw_blake3_hash
        check(fn(self.h, ctypes.c_void_p(buf.ctypes.data + offset), length, out), self.h)
        return bytes(out)

    def blake3_dropin(self, data):
        """bw_blake3_hash_dropin over read-only memory (see blake3_at)."""
        buf = _as_u8(data)
        out = (ctypes.c_uint8 * 32)()
        check(self._L.bw_blake3_hash_dropin(self.h, _ptr(buf), buf.size, out), self.h)
        return bytes(out)

    def blake3_many(self, data, offsets, lengths):
        buf = _as_u8(data)
        off = np.ascontiguousarray(offsets, dtype=np.uint64)
        ln = np.ascontiguousarray(lengths, dtype=np.uint64)
        out = np.zeros((len(off), 32), dtype=np.uint8)
        if len(off) == 0:
            return out
        check(self._L.bw_blake3_hash_many(self.h, _ptr(buf), buf.size, off.ctypes.data_as(_lib.u64p),
                                          ln.ctypes.data_as(_lib.u64p), len(off),
                                          out.ctypes.data_as(_lib.u8p)), self.h)
        return out

    def blake3(self, data):
        buf = _as_u8(data)
        out = (ctypes.c_uint8 * 32)()
        check(self._L.bw_blake3_hash(self.h, _ptr(buf), buf.size, out), self.h)
        return bytes(out)

    # -------------------------------------------------------------- sealing (§8f row 3)
    @staticmethod
    def _seal_tables(src_off, src_len, infos, nonces, dst_off):
        so = np.ascontiguousarray(src_off, dtype=np.uint64)
        sl = np.ascontiguousarray(src_len, dtype=np.uint64)
        n = len(so)
        info = np.ascontiguousarray(np.asarray(infos, dtype=np.uint8).reshape(n, -1)) if n else \
            np.zeros((0, 0), np.uint8)
        non = np.ascontiguousarray(np.asarray(nonces, dtype=np.uint8).reshape(n, 12)) if n else \
            np.zeros((0, 12), np.uint8)
        do = np.ascontiguousarray(dst_off, dtype=np.uint64)
        assert len(sl) == n and len(do) == n
        return so, sl, info, non, do, n

    def seal(self, prk, src, src_off, src_len, infos, nonces, dst_off, dst_size, open_=False):
        """Host buffers: derive_backup_key(info_i) + Aes256Gcm encrypt (open_=False) or decrypt
        (open_=True).  infos: n x info_len bytes (blob hashes), nonces: n x 12.  Returns the output
        buffer (and the ok flags when opening)."""
        buf = _as_u8(src)
        so, sl, info, non, do, n = self._seal_tables(src_off, src_len, infos, nonces, dst_off)
        out = np.zeros(max(int(dst_size), 1), dtype=np.uint8)
        k = (ctypes.c_uint8 * 32).from_buffer_copy(bytes(prk))
        args = [self.h, k, _ptr(buf), so.ctypes.data_as(_lib.u64p), sl.ctypes.data_as(_lib.u64p), n, _ptr(info),
                info.shape[1] if n else 0, _ptr(non), _ptr(out), do.ctypes.data_as(_lib.u64p)]
        if open_:
            ok = np.zeros(n, dtype=np.uint8)
            check(self._L.bw_open(*args, ok.ctypes.data_as(_lib.u8p)), self.h)
            return out[:int(dst_size)], ok
        check(self._L.bw_seal(*args), self.h)
        return out[:int(dst_size)]

    def seal_device(self, prk, d_src, src_off, src_len, infos, nonces, d_dst, dst_off, open_=False):
        """Device pointers (ints); tables on the host.  Sealing is asynchronous on the context
        stream; opening synchronizes and returns the ok flags."""
        so, sl, info, non, do, n = self._seal_tables(src_off, src_len, infos, nonces, dst_off)
        k = (ctypes.c_uint8 * 32).from_buffer_copy(bytes(prk))
        args = [self.h, k, ctypes.c_void_p(d_src), so.ctypes.data_as(_lib.u64p), sl.ctypes.data_as(_lib.u64p), n,
                _ptr(info), info.shape[1] if n else 0, _ptr(non), ctypes.c_void_p(d_dst),
                do.ctypes.data_as(_lib.u64p)]
        if open_:
            ok = np.zeros(n, dtype=np.uint8)
            check(self._L.bw_open_device(*args, ok.ctypes.data_as(_lib.u8p)), self.h)
            return ok
        check(self._L.bw_seal_device(*args), self.h)
        return None

    # -------------------------------------------------------------- zstd level 3 (§8f row 2)
    def zstd_compress(self, blobs):
        """Per-blob zstd level 3 as Manager::compress_encrypt_blob runs it (pack.rs:58-64): a
        list of bytes-like blobs (each <= 3 MiB) -> the list of their magicless frames."""
        lens = np.array([len(b) for b in blobs], dtype=np.uint64)
        so = np.zeros(len(blobs), dtype=np.uint64)
        if len(blobs) > 1:
            so[1:] = np.cumsum(lens[:-1])
        src = np.frombuffer(b"".join(bytes(b) for b in blobs) or b"\0", dtype=np.uint8)
        cap = np.array([self._L.bw_zstd_store_size(int(x)) for x in lens], dtype=np.uint64)
        do = np.zeros(len(blobs), dtype=np.uint64)
        if len(blobs) > 1:
            do[1:] = np.cumsum(cap[:-1])
        out = np.zeros(max(int(cap.sum()), 1), dtype=np.uint8)
        fl = np.zeros(len(blobs), dtype=np.uint64)
        check(self._L.bw_zstd_compress(self.h, _ptr(src), so.ctypes.data_as(_lib.u64p), lens.ctypes.data_as(_lib.u64p),
                                       len(blobs), _ptr(out), do.ctypes.data_as(_lib.u64p),
                                       fl.ctypes.data_as(_lib.u64p)), self.h)
        return [out[int(do[i]):int(do[i] + fl[i])].tobytes() for i in range(len(blobs))]

    def zstd_compress_device(self, d_src, src_off, src_len, d_dst, dst_off):
        """Device pointers (ints); frames at dst_off (each with room for bw_zstd_store_size);
        returns the frame lengths (synchronous)."""
        so = np.ascontiguousarray(src_off, dtype=np.uint64)
        sl = np.ascontiguousarray(src_len, dtype=np.uint64)
        do = np.ascontiguousarray(dst_off, dtype=np.uint64)
        fl = np.zeros(so.size, dtype=np.uint64)
        check(self._L.bw_zstd_compress_device(self.h, ctypes.c_void_p(d_src), so.ctypes.data_as(_lib.u64p),
                                              sl.ctypes.data_as(_lib.u64p), so.size, ctypes.c_void_p(d_dst),
                                              do.ctypes.data_as(_lib.u64p), fl.ctypes.data_as(_lib.u64p)), self.h)
        return fl

    def zstd_submit_device(self, d_src, src_off, src_len, d_dst, dst_off):
        """bw_zstd_submit_device: the batch starts on a free lane of the context and the call
        returns its ticket at once (BW_ESTATE: every lane holds a batch); zstd_wait(ticket) blocks
        for it and returns the frame lengths.  The device buffers stay untouched until then."""
        so = np.ascontiguousarray(src_off, dtype=np.uint64)
        sl = np.ascontiguousarray(src_len, dtype=np.uint64)
        do = np.ascontiguousarray(dst_off, dtype=np.uint64)
        t = ctypes.c_uint64()
        check(self._L.bw_zstd_submit_device(self.h, ctypes.c_void_p(d_src), so.ctypes.data_as(_lib.u64p),
                                            sl.ctypes.data_as(_lib.u64p), so.size, ctypes.c_void_p(d_dst),
                                            do.ctypes.data_as(_lib.u64p), ctypes.byref(t)), self.h)
        self._zs_n[t.value] = so.size
        return t.value

    def zstd_wait(self, ticket):
        n = self._zs_n.pop(ticket, 0)
        fl = np.zeros(max(n, 1), dtype=np.uint64)
        check(self._L.bw_zstd_wait(self.h, ticket, fl.ctypes.data_as(_lib.u64p)), self.h)
        return fl[:n]

    # -------------------------------------------------------------- index
    def index_reset(self, capacity_hint=0):
        check(self._L.bw_index_reset(self.h, capacity_hint), self.h)

    def index_seed(self, sorted_digests):
        d = np.ascontiguousarray(np.asarray(sorted_digests, dtype=np.uint8).reshape(-1, 32))
        check(self._L.bw_index_seed(self.h, _ptr(d), d.shape[0]), self.h)

    def index_check_insert(self, digests):
        d = np.ascontiguousarray(np.asarray(digests, dtype=np.uint8).reshape(-1, 32))
        out = np.zeros(d.shape[0], dtype=np.uint8)
        if d.shape[0]:
            check(self._L.bw_index_check_insert(self.h, _ptr(d), d.shape[0], out.ctypes.data_as(_lib.u8p)), self.h)
        return out

    def index_check(self):
        """Raises BwError(BW_ENOSPC) if an exchange bucket overflowed since the last reset."""
        check(self._L.bw_index_check(self.h), self.h)

    def index_size(self):
        n = ctypes.c_uint64()
        check(self._L.bw_index_size(self.h, ctypes.byref(n)), self.h)
        return n.value

    # -------------------------------------------------------------- batches
    def process_files(self, data, file_off, file_len, params=None):
        buf = _as_u8(data)
        fo = np.ascontiguousarray(file_off, dtype=np.uint64)
        fl = np.ascontiguousarray(file_len, dtype=np.uint64)
        p = params or make_params()
        mc = max(min(2 * (p.min_size // 2), p.max_size), 1)
        cap = int(sum(int(x) // mc + 2 for x in fl)) + 1
        out = np.zeros(cap, dtype=BLOB_DTYPE)
        n = ctypes.c_uint64()
        check(self._L.bw_process_files(self.h, _ptr(buf), buf.size, fo.ctypes.data_as(_lib.u64p),
                                       fl.ctypes.data_as(_lib.u64p), len(fo), ctypes.byref(p),
                                       out.ctypes.data_as(ctypes.POINTER(BwBlob)), cap, ctypes.byref(n)), self.h)
        return out[:n.value]

    def submit_device(self, d_ptr, data_len, file_off, file_len, params=None):
        """Enqueue a batch whose bytes are already in HBM (d_ptr = device address) -> its ticket."""
        fo = np.ascontiguousarray(file_off, dtype=np.uint64)
        fl = np.ascontiguousarray(file_len, dtype=np.uint64)
        p = params or make_params()
        t = ctypes.c_uint64()
        check(self._L.bw_submit_device(self.h, ctypes.c_void_p(d_ptr), data_len, fo.ctypes.data_as(_lib.u64p),
                                       fl.ctypes.data_as(_lib.u64p), len(fo), ctypes.byref(p), ctypes.byref(t)),
              self.h)
        return t.value

    def submit_host(self, data, file_off, file_len, params=None, data_len=None):
        """Enqueue a batch whose bytes are in host memory -> its ticket.  `data` is a numpy array
        (pageable: staged through pinned chunks before the call returns) or the address of pinned
        memory (an int, e.g. a pinned torch tensor's data_ptr(), with data_len), which must stay
        unchanged until wait(ticket)."""
        fo = np.ascontiguousarray(file_off, dtype=np.uint64)
        fl = np.ascontiguousarray(file_len, dtype=np.uint64)
        if isinstance(data, int):
            ptr, n = ctypes.c_void_p(data), int(data_len)
        else:
            buf = _as_u8(data)
            ptr, n = _ptr(buf), buf.size
        p = params or make_params()
        t = ctypes.c_uint64()
        check(self._L.bw_submit_host(self.h, ptr, n, fo.ctypes.data_as(_lib.u64p), fl.ctypes.data_as(_lib.u64p),
                                     len(fo), ctypes.byref(p), ctypes.byref(t)), self.h)
        return t.value

    def _fetch(self, fn, cap, out=None):
        n = ctypes.c_uint64()
        if out is not None:
            assert out.dtype == BLOB_DTYPE and out.flags.c_contiguous
            cap = out.size
        elif cap is None:
            rc = fn(None, 0, ctypes.byref(n))
            if rc not in (_lib.BW_OK, _lib.BW_ENOSPC):
                check(rc, self.h)
            cap = n.value
        if out is None:
            out = np.zeros(max(cap, 1), dtype=BLOB_DTYPE)
        check(fn(out.ctypes.data_as(ctypes.POINTER(BwBlob)), cap, ctypes.byref(n)), self.h)
        return out[:n.value]

    def wait(self, ticket, cap=None, out=None):
        """Results of batch `ticket` (blocks until it is done); `out` = a reusable BLOB_DTYPE array."""
        return self._fetch(lambda o, c, n: self._L.bw_wait(self.h, ticket, o, c, n), cap, out)

    def results(self, cap=None):
        """Results of the most recently submitted batch."""
        return self._fetch(lambda o, c, n: self._L.bw_results(self.h, o, c, n), cap)

    def set_option(self, option, value):
        check(self._L.bw_set_option(self.h, option, int(value)), self.h)

    def attach_index(self, index):
        """Gate this context's batches through a shared Index (None: the private one)."""
        check(self._L.bw_attach_index(self.h, index.h if index is not None else None), self.h)
        self._index = index

    def device_views(self):
        n = ctypes.c_uint64()
        d, dup = ctypes.c_void_p(), ctypes.c_void_p()
        check(self._L.bw_batch_device_views(self.h, ctypes.byref(n), ctypes.byref(d), ctypes.byref(dup)), self.h)
        return n.value, d.value, dup.value

    # -------------------------------------------------------------- tree blobs
    def tree_blobs(self, trees, dedup=True):
        """split_serialize_tree + add_tree_to_blobs for a list of make_tree() results ->
        (tree hashes n x 32, every piece as TREE_BLOB_DTYPE records in canonical order)."""
        arr = (_lib.BwTree * max(len(trees), 1))(*[t for t, _ in trees])
        cap = sum(max(1, -(-int(t.n_children) // _lib.BW_TREE_BLOB_MAX_CHILDREN)) for t, _ in trees)
        hashes = np.zeros((max(len(trees), 1), 32), dtype=np.uint8)
        out = np.zeros(max(cap, 1), dtype=TREE_BLOB_DTYPE)
        n = ctypes.c_uint64()
        flags = 0 if dedup else _lib.BW_F_NO_DEDUP
        check(self._L.bw_tree_blobs(self.h, arr, len(trees), flags, ctypes.c_void_p(hashes.ctypes.data),
                                    out.ctypes.data_as(ctypes.POINTER(_lib.BwTreeBlob)), cap, ctypes.byref(n)),
              self.h)
        return hashes[:len(trees)], out[:n.value]

    def tree_blobs_array(self, trees, dedup=True):
        """tree_blobs over a TREE_DTYPE array whose pointers the caller keeps alive."""
        n_ch = trees["n_children"].astype(np.int64)
        cap = int(np.maximum(1, -(-n_ch // _lib.BW_TREE_BLOB_MAX_CHILDREN)).sum())
        hashes = np.zeros((max(len(trees), 1), 32), dtype=np.uint8)
        out = np.zeros(max(cap, 1), dtype=TREE_BLOB_DTYPE)
        n = ctypes.c_uint64()
        flags = 0 if dedup else _lib.BW_F_NO_DEDUP
        check(self._L.bw_tree_blobs(self.h, trees.ctypes.data_as(ctypes.POINTER(_lib.BwTree)), len(trees), flags,
                                    ctypes.c_void_p(hashes.ctypes.data),
                                    out.ctypes.data_as(ctypes.POINTER(_lib.BwTreeBlob)), cap, ctypes.byref(n)),
              self.h)
        return hashes[:len(trees)], out[:n.value]

    # -------------------------------------------------------------- packfiles / index files (§8f row 4)
    def pack_plan(self, payload_len, flags=_lib.BW_PACK_ZSTD_STORE):
        """write_packfiles' grouping (pack.rs:123-148): PACKFILE_DTYPE records and total bytes."""
        pl = np.ascontiguousarray(payload_len, dtype=np.uint64)
        n, total = ctypes.c_uint64(), ctypes.c_uint64()
        rc = self._L.bw_pack_plan(pl.ctypes.data_as(_lib.u64p), pl.size, flags, None, 0, ctypes.byref(n),
                                  ctypes.byref(total))
        if rc not in (_lib.BW_OK, _lib.BW_ENOSPC):
            check(rc)
        out = np.zeros(max(n.value, 1), dtype=PACKFILE_DTYPE)
        check(self._L.bw_pack_plan(pl.ctypes.data_as(_lib.u64p), pl.size, flags,
                                   out.ctypes.data_as(ctypes.POINTER(_lib.BwPackfile)), n.value, ctypes.byref(n),
                                   ctypes.byref(total)))
        return out[:n.value], total.value

    @staticmethod
    def pack_plan_session(digests, is_dup, payload_len, flags=_lib.BW_PACK_ZSTD_STORE):
        """The reference's write cadence over a session's blobs in canonical order (all of them,
        duplicates included): PACKFILE_DTYPE records over the is_dup == 0 blobs, total bytes."""
        d = np.ascontiguousarray(np.asarray(digests, dtype=np.uint8).reshape(-1, 32))
        dup = np.ascontiguousarray(is_dup, dtype=np.uint8)
        pl = np.ascontiguousarray(payload_len, dtype=np.uint64)
        assert d.shape[0] == dup.size == pl.size
        n, total, nu = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        args = [_ptr(d), _ptr(dup), pl.ctypes.data_as(_lib.u64p), pl.size, flags]
        L = _lib.load()
        rc = L.bw_pack_plan_session(*args, None, 0, ctypes.byref(n), ctypes.byref(total), ctypes.byref(nu))
        if rc not in (_lib.BW_OK, _lib.BW_ENOSPC):
            check(rc)
        out = np.zeros(max(n.value, 1), dtype=PACKFILE_DTYPE)
        check(L.bw_pack_plan_session(*args, out.ctypes.data_as(ctypes.POINTER(_lib.BwPackfile)), n.value,
                                           ctypes.byref(n), ctypes.byref(total), ctypes.byref(nu)))
        return out[:n.value], total.value

    def _pack_args(self, prk, src_off, src_len, hashes, kinds, nonces, plan, packfile_ids):
        so = np.ascontiguousarray(src_off, dtype=np.uint64)
        sl = np.ascontiguousarray(src_len, dtype=np.uint64)
        h = np.ascontiguousarray(np.asarray(hashes, dtype=np.uint8).reshape(-1, 32))
        kd = np.ascontiguousarray(kinds, dtype=np.uint8)
        no = np.ascontiguousarray(np.asarray(nonces, dtype=np.uint8).reshape(-1, 12))
        pl = np.ascontiguousarray(plan, dtype=PACKFILE_DTYPE)
        ids = np.ascontiguousarray(np.asarray(packfile_ids, dtype=np.uint8).reshape(-1, 12))
        assert so.size == sl.size == h.shape[0] == kd.size == no.shape[0] and ids.shape[0] >= pl.size
        k = (ctypes.c_uint8 * 32).from_buffer_copy(bytes(prk))
        keep = (so, sl, h, kd, no, pl, ids, k)
        return keep, [k, None, so.ctypes.data_as(_lib.u64p), sl.ctypes.data_as(_lib.u64p), so.size, _ptr(h), _ptr(kd),
                      _ptr(no)], [pl.ctypes.data_as(ctypes.POINTER(_lib.BwPackfile)), pl.size, _ptr(ids)]

    def pack_build(self, prk, src, src_off, src_len, hashes, kinds, nonces, plan, total, packfile_ids,
                   flags=_lib.BW_PACK_ZSTD_STORE):
        """Host buffers: the planned packfiles back to back (numpy u8, `total` bytes)."""
        buf = _as_u8(src)
        keep, a, b = self._pack_args(prk, src_off, src_len, hashes, kinds, nonces, plan, packfile_ids)
        a[1] = _ptr(buf)
        out = np.zeros(max(int(total), 1), dtype=np.uint8)
        check(self._L.bw_pack_build(self.h, *a, flags, *b, _ptr(out)), self.h)
        return out[:int(total)]

    def pack_build_device(self, prk, d_src, src_off, src_len, hashes, kinds, nonces, plan, packfile_ids, d_out,
                          flags=_lib.BW_PACK_ZSTD_STORE):
        """Device pointers (ints) for the payloads and the output; asynchronous on the context stream."""
        keep, a, b = self._pack_args(prk, src_off, src_len, hashes, kinds, nonces, plan, packfile_ids)
        a[1] = ctypes.c_void_p(d_src)
        check(self._L.bw_pack_build_device(self.h, *a, flags, *b, ctypes.c_void_p(d_out)), self.h)
        self._pack_keep = keep

    def pack_compress_device(self, d_src, src_off, src_len):
        """Level-3 frames of the queue's blobs (device pointer d_src) staged in the context for
        pack_build_compressed; returns the frame lengths (synchronous)."""
        so = np.ascontiguousarray(src_off, dtype=np.uint64)
        sl = np.ascontiguousarray(src_len, dtype=np.uint64)
        assert so.size == sl.size
        fl = np.zeros(so.size, dtype=np.uint64)
        check(self._L.bw_pack_compress_device(self.h, ctypes.c_void_p(d_src), so.ctypes.data_as(_lib.u64p),
                                              sl.ctypes.data_as(_lib.u64p), so.size, fl.ctypes.data_as(_lib.u64p)),
              self.h)
        return fl

    def pack_build_compressed(self, prk, hashes, kinds, nonces, plan, packfile_ids, d_out):
        """Seal and lay out the staged frames into the planned packfiles at d_out (asynchronous)."""
        h = np.ascontiguousarray(np.asarray(hashes, dtype=np.uint8).reshape(-1, 32))
        kd = np.ascontiguousarray(kinds, dtype=np.uint8)
        no = np.ascontiguousarray(np.asarray(nonces, dtype=np.uint8).reshape(-1, 12))
        pl = np.ascontiguousarray(plan, dtype=PACKFILE_DTYPE)
        ids = np.ascontiguousarray(np.asarray(packfile_ids, dtype=np.uint8).reshape(-1, 12))
        assert h.shape[0] == kd.size == no.shape[0] and ids.shape[0] >= pl.size
        k = (ctypes.c_uint8 * 32).from_buffer_copy(bytes(prk))
        check(self._L.bw_pack_build_compressed(self.h, k, _ptr(h), _ptr(kd), _ptr(no),
                                               pl.ctypes.data_as(ctypes.POINTER(_lib.BwPackfile)), pl.size,
                                               _ptr(ids), ctypes.c_void_p(d_out)), self.h)
        self._pack_keep = (h, kd, no, pl, ids, k)

    def pack_compress(self, blobs):
        """Host form of pack_compress_device over a list of bytes-like blobs; frame lengths."""
        lens = np.array([len(b) for b in blobs], dtype=np.uint64)
        so = np.zeros(len(blobs), dtype=np.uint64)
        if len(blobs) > 1:
            so[1:] = np.cumsum(lens[:-1])
        src = np.frombuffer(b"".join(bytes(b) for b in blobs) or b"\0", dtype=np.uint8)
        fl = np.zeros(len(blobs), dtype=np.uint64)
        check(self._L.bw_pack_compress(self.h, _ptr(src), so.ctypes.data_as(_lib.u64p), lens.ctypes.data_as(_lib.u64p),
                                       len(blobs), fl.ctypes.data_as(_lib.u64p)), self.h)
        return fl

    def pack_build_compressed_host(self, prk, hashes, kinds, nonces, plan, total, packfile_ids):
        """Host form of pack_build_compressed: the planned packfiles back to back (numpy u8)."""
        h = np.ascontiguousarray(np.asarray(hashes, dtype=np.uint8).reshape(-1, 32))
        kd = np.ascontiguousarray(kinds, dtype=np.uint8)
        no = np.ascontiguousarray(np.asarray(nonces, dtype=np.uint8).reshape(-1, 12))
        pl = np.ascontiguousarray(plan, dtype=PACKFILE_DTYPE)
        ids = np.ascontiguousarray(np.asarray(packfile_ids, dtype=np.uint8).reshape(-1, 12))
        k = (ctypes.c_uint8 * 32).from_buffer_copy(bytes(prk))
        out = np.zeros(max(int(total), 1), dtype=np.uint8)
        check(self._L.bw_pack_build_compressed_host(self.h, k, _ptr(h), _ptr(kd), _ptr(no),
                                                    pl.ctypes.data_as(ctypes.POINTER(_lib.BwPackfile)), pl.size,
                                                    _ptr(ids), _ptr(out)), self.h)
        return out[:int(total)]

    def index_files_build(self, prk, entries, last_file_num=0):
        """BlobIndex::push + flush over n (hash, packfile id) entries (n x 44 bytes):
        [(file_num, bytes)] as the reference writes them to index/{file_num:0>10}."""
        e = np.ascontiguousarray(np.asarray(entries, dtype=np.uint8).reshape(-1, 44))
        k = (ctypes.c_uint8 * 32).from_buffer_copy(bytes(prk))
        nf, total = ctypes.c_uint64(), ctypes.c_uint64()
        rc = self._L.bw_index_files_build(self.h, k, _ptr(e), e.shape[0], last_file_num, None, 0, None, 0,
                                          ctypes.byref(nf), ctypes.byref(total))
        if rc != _lib.BW_ENOSPC:
            check(rc, self.h)
        out = np.zeros(max(total.value, 1), dtype=np.uint8)
        tab = (_lib.BwIndexFile * nf.value)()
        check(self._L.bw_index_files_build(self.h, k, _ptr(e), e.shape[0], last_file_num, _ptr(out), out.size, tab,
                                           nf.value, ctypes.byref(nf), ctypes.byref(total)), self.h)
        return [(t.file_num, out[t.offset:t.offset + t.size].tobytes()) for t in tab]

    def index_load_files(self, prk, files, want_entries=True):
        """BlobIndex::load fused with the device seed: files = [(file_num, bytes)].  Returns the
        (n x 44) records in file order (or their count)."""
        blobs = [bytes(b) for _, b in files]
        data = np.frombuffer(b"".join(blobs) or b"\0", dtype=np.uint8)
        tab = (_lib.BwIndexFile * max(len(files), 1))()
        off = 0
        for i, (num, b) in enumerate(zip([f for f, _ in files], blobs)):
            tab[i].file_num, tab[i].offset, tab[i].size = num, off, len(b)
            off += len(b)
        k = (ctypes.c_uint8 * 32).from_buffer_copy(bytes(prk))
        n, bad = ctypes.c_uint64(), ctypes.c_uint64()
        cap = sum(max(len(b) - 17, 0) // 44 + 1 for b in blobs)
        out = np.zeros((max(cap, 1), 44), dtype=np.uint8) if want_entries else None
        check(self._L.bw_index_load_files(self.h, k, _ptr(data), tab, len(files), _ptr(out) if want_entries else None,
                                          cap if want_entries else 0, ctypes.byref(n), ctypes.byref(bad)), self.h)
        return out[:n.value] if want_entries else n.value

    # -------------------------------------------------------------- stage timing
    def profile_enable(self, on=True):
        check(self._L.bw_profile_enable(self.h, 1 if on else 0), self.h)

    def profile_read(self):
        """{stage: summed ms}, n_batches -- HIP events on the context stream."""
        ms = (ctypes.c_double * len(_lib.STAGES))()
        n = ctypes.c_uint64()
        check(self._L.bw_profile_read(self.h, ms, ctypes.byref(n)), self.h)
        return {s: ms[i] for i, s in enumerate(_lib.STAGES)}, n.value

    def profile_intervals(self, stage):
        """[(start_ms, end_ms)] of one stage over the profiled batches, on the device's timeline
        (shared by every context of the device)."""
        k = _lib.STAGES.index(stage)
        n = ctypes.c_uint64()
        rc = self._L.bw_profile_intervals(self.h, k, None, 0, ctypes.byref(n))
        if rc not in (0, _lib.BW_ENOSPC):
            check(rc, self.h)
        buf = (ctypes.c_double * max(2 * n.value, 1))()
        check(self._L.bw_profile_intervals(self.h, k, buf, n.value, ctypes.byref(n)), self.h)
        return [(buf[2 * i], buf[2 * i + 1]) for i in range(n.value)]

    def calibrate_b3(self, ms=100.0):
        """The BLAKE3 leaf pass's compression from registers on every CU for about `ms` ms:
        {gbs, ghz, bytes_per_clk_cu, launch_ms} -- the pass's integer-issue ceiling on this chip."""
        out = (ctypes.c_double * 4)()
        check(self._L.bw_calibrate_b3(self.h, float(ms), out), self.h)
        return {"gbs": out[0], "ghz": out[1], "bytes_per_clk_cu": out[2], "launch_ms": out[3]}

    # -------------------------------------------------------------- multi-GPU helpers (device pointers)
    def partition_by_owner(self, d_digests, n, n_owners, d_out, d_perm):
        counts = np.zeros(n_owners, dtype=np.uint64)
        check(self._L.bw_partition_by_owner(self.h, ctypes.c_void_p(d_digests), n, n_owners,
                                            ctypes.c_void_p(d_out), ctypes.c_void_p(d_perm),
                                            counts.ctypes.data_as(_lib.u64p)), self.h)
        return counts

    def index_check_insert_device(self, d_digests, n, d_is_dup):
        check(self._L.bw_index_check_insert_device(self.h, ctypes.c_void_p(d_digests), n,
                                                   ctypes.c_void_p(d_is_dup)), self.h)

    def batch_views(self, ticket=0):
        """(d_n_blobs, d_digests, d_is_dup, max_blobs) of a batch, no synchronization."""
        n, d, dup, mx = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_uint64()
        check(self._L.bw_batch_views(self.h, ticket, ctypes.byref(n), ctypes.byref(d), ctypes.byref(dup),
                                     ctypes.byref(mx)), self.h)
        return n.value, d.value, dup.value, mx.value

    def exchange_dedup(self, comm, ticket=0):
        """Batch `ticket` (submitted with BW_F_NO_DEDUP) through the digest-prefix exchange of
        `comm` (a backuwup_amd.comm.Comm): its verdicts land in the batch's results."""
        rc = self._L.bw_exchange_dedup(self.h, comm.h, int(ticket))
        if rc == _lib.BW_ECOMM:
            raise _lib.BwError(rc, comm.last_error() or self._L.bw_last_error(self.h).decode())
        check(rc, self.h)

    def chunk_stream_shard(self, comm, d_window, file_len, params=None):
        """bw_chunk_stream_shard: this rank's part of one file split across the ranks of `comm`
        (d_window = device address of file byte lo of stream_window()).  -> dict(ticket, first_blob,
        n_blobs, chain_start, rounds); bw_wait(ticket) holds the chain, blobs [first_blob, first_blob
        + n_blobs) are the ones this rank emits (and the exchange sends)."""
        out = _lib.BwStreamShard()
        rc = self._L.bw_chunk_stream_shard(self.h, comm.h, ctypes.c_void_p(d_window), int(file_len),
                                           ctypes.byref(params) if params is not None else None, ctypes.byref(out))
        if rc == _lib.BW_ECOMM:
            raise _lib.BwError(rc, comm.last_error() or self._L.bw_last_error(self.h).decode())
        check(rc, self.h)
        return {k: int(getattr(out, k)) for k in ("ticket", "first_blob", "n_blobs", "chain_start", "rounds")}

    def partition_buckets(self, d_digests, d_n, max_n, cap, n_owners, d_buckets, d_perm, d_counts):
        check(self._L.bw_partition_buckets(self.h, ctypes.c_void_p(d_digests), ctypes.c_void_p(d_n), max_n, cap,
                                           n_owners, ctypes.c_void_p(d_buckets), ctypes.c_void_p(d_perm),
                                           ctypes.c_void_p(d_counts)), self.h)

    def index_check_insert_buckets(self, d_buckets, d_counts, n_src, cap, d_verdicts):
        check(self._L.bw_index_check_insert_buckets(self.h, ctypes.c_void_p(d_buckets), ctypes.c_void_p(d_counts),
                                                    n_src, cap, ctypes.c_void_p(d_verdicts)), self.h)

    def scatter_buckets(self, d_verdicts, d_perm, d_counts, n_owners, cap, d_is_dup):
        check(self._L.bw_scatter_buckets(self.h, ctypes.c_void_p(d_verdicts), ctypes.c_void_p(d_perm),
                                         ctypes.c_void_p(d_counts), n_owners, cap, ctypes.c_void_p(d_is_dup)), self.h)

    def scatter_verdicts(self, d_verdict, d_perm, n, d_is_dup):
        check(self._L.bw_scatter_verdicts(self.h, ctypes.c_void_p(d_verdict), ctypes.c_void_p(d_perm), n,
                                          ctypes.c_void_p(d_is_dup)), self.h)


_default = None


def default_context():
    global _default
    if _default is None:
        _default = Context(0)
    return _default
