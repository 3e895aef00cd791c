"""The multi-GPU digest exchange through the C ABI (bw_comm_* and bw_exchange_dedup).

One process per GPU.  Every rank submits its batches with BW_F_NO_DEDUP and then calls
Context.exchange_dedup(comm, ticket) once per batch, in the same batch order on every rank: the
library partitions the batch's digests by owner = digest[0] >> (8 - log2 N), exchanges counts,
buckets and verdicts with all-to-alls, and gates the owner's shard of the index in between
(the one BlobIndex behind the packer mutex of the reference, blob_index.rs:130-148, pack.rs:37,
split by digest prefix).  The transport is RCCL (Comm.rccl) or the caller's host all-to-all
(Comm.host: e.g. gloo, for several ranks on one GPU, which RCCL refuses).
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import check

HOST_A2A = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64)


def unique_id():
    """128 bytes from ncclGetUniqueId (rank 0 draws it; every rank passes it to Comm.rccl)."""
    L = _lib.load()
    buf = (ctypes.c_uint8 * _lib.BW_COMM_ID_BYTES)()
    check(L.bw_comm_unique_id(buf))
    return bytes(buf)


class Comm:
    """A bw_comm handle.  Use Comm.rccl(...) or Comm.host(...)."""

    def __init__(self, handle, keep=None):
        self._L = _lib.load()
        self.h = handle
        self._keep = keep  # the ctypes callback of a host transport must outlive the handle

    @classmethod
    def rccl(cls, device, rank, world, uid, timeout_ms=None):
        """timeout_ms: the deadline of every wait on the peers (default BW_COMM_DEFAULT_TIMEOUT_MS);
        a missed deadline aborts the communicator and returns BW_ECOMM."""
        L = _lib.load()
        assert len(uid) == _lib.BW_COMM_ID_BYTES
        h = ctypes.c_void_p()
        ub = (ctypes.c_uint8 * _lib.BW_COMM_ID_BYTES).from_buffer_copy(uid)
        if timeout_ms is None:
            check(L.bw_comm_init(device, rank, world, ub, ctypes.byref(h)))
        else:
            check(L.bw_comm_init_timeout(device, rank, world, ub, int(timeout_ms), ctypes.byref(h)))
        return cls(h)

    @classmethod
    def host(cls, device, rank, world, all_to_all):
        """all_to_all(send, recv, bytes_per_rank): numpy uint8 arrays of world * bytes_per_rank
        (pinned host memory owned by the library); deliver send[r * b:(r + 1) * b] to rank r's
        recv[rank * b:(rank + 1) * b]."""
        L = _lib.load()

        def fn(_user, send, recv, nbytes):
            try:
                total = int(nbytes) * world
                s = np.ctypeslib.as_array((ctypes.c_uint8 * total).from_address(send))
                r = np.ctypeslib.as_array((ctypes.c_uint8 * total).from_address(recv))
                all_to_all(s, r, int(nbytes))
                return 0
            except Exception:  # never unwind into the library
                import traceback
                traceback.print_exc()
                return 1

        cb = HOST_A2A(fn)
        h = ctypes.c_void_p()
        check(L.bw_comm_init_host(device, rank, world, cb, None, ctypes.byref(h)))
        return cls(h, keep=cb)

    @classmethod
    def local(cls, devices):
        """The ranks of ONE process over an in-process host transport (bw_comm_init_local): a
        list of len(devices) communicators, rank r on devices[r] (a device may repeat).  Drive
        each rank from its own thread."""
        L = _lib.load()
        n = len(devices)
        devs = (ctypes.c_int * n)(*devices)
        hs = (ctypes.c_void_p * n)()
        check(L.bw_comm_init_local(devs, n, hs))
        return [cls(ctypes.c_void_p(h)) for h in hs]

    @classmethod
    def all(cls, devices, timeout_ms=_lib.BW_COMM_DEFAULT_TIMEOUT_MS):
        """The ranks of ONE process over RCCL (bw_comm_init_all): one distinct device per rank."""
        L = _lib.load()
        n = len(devices)
        devs = (ctypes.c_int * n)(*devices)
        hs = (ctypes.c_void_p * n)()
        check(L.bw_comm_init_all(devs, n, int(timeout_ms), hs))
        return [cls(ctypes.c_void_p(h)) for h in hs]

    def set_capacity(self, cap):
        """Obsolete (round 5): exchanges size every transfer from their own counts; ignored."""
        check(self._L.bw_comm_set_capacity(self.h, int(cap)))

    def progress(self):
        """Finish the queued exchanges whose counts have arrived (never waits)."""
        check(self._L.bw_comm_progress(self.h))

    def set_timeout(self, timeout_ms):
        check(self._L.bw_comm_set_timeout(self.h, int(timeout_ms)))

    def status(self):
        """0, or BW_ECOMM once the communicator was aborted (a peer failed or stalled)."""
        return self._L.bw_comm_status(self.h)

    def last_error(self):
        m = self._L.bw_comm_last_error(self.h)
        return m.decode() if m else ""

    def close(self):
        if self.h:
            self._L.bw_comm_destroy(self.h)
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


def gloo_all_to_all(group=None):
    """A host all-to-all over torch.distributed (gloo): the transport of Comm.host in the
    multi-process tests, where several ranks share one GPU."""
    import torch
    import torch.distributed as dist

    def a2a(send, recv, nbytes):
        out = torch.from_numpy(recv)
        dist.all_to_all_single(out, torch.from_numpy(send), group=group)

    return a2a
