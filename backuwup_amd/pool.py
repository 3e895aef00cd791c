"""The drop-ins' context pool over every GPU of the node (the Python mirror of the Rust crate's
`Pool`, rust/backuwup-gpu/src/lib.rs; INTEGRATION.md "Every GPU of the node").

The reference calls `FastCDC::new` and `blake3::hash` with no context, one tokio task per file on
one worker thread per core (client/src/main.rs:43, dir_packer.rs:166, :254-262, :286).  So the
drop-ins share a pool of contexts spread over the node's devices:

  * devices: BACKUWUP_GPU_DEVICES ("all", the default, or a list like "0,1,2,3"; a device may be
    listed twice), else the single BACKUWUP_GPU_DEVICE of earlier versions;
  * BACKUWUP_GPU_CONTEXTS contexts per listed device (default 16); context j is on devices[j % n];
  * thread k (in order of first use) has home slot k: `FastCDC` takes the first free context from its
    home slot on, and `blake3.hash` of a small message goes to its home device's hash service
    (bw_blake3_hash_dropin_device, no context held while it waits); BW_EAGAIN from the service (a
    message over 64 KiB, or a call the service could not take in time) is hashed through a pool
    context instead.

Files are independent (CDC restarts per file, dir_packer.rs:254) and the dedup gate stays the
caller's (pack.rs:37), so spreading calls over devices changes no result.
"""
import ctypes
import itertools
import os
import threading

from . import _lib
from .context import Context, _ptr


def devices_from_env():
    listed = os.environ.get("BACKUWUP_GPU_DEVICES")
    if listed is not None and listed.strip() not in ("", "all"):
        return [int(d) for d in listed.split(",")]
    if listed is None and os.environ.get("BACKUWUP_GPU_DEVICE") is not None:
        return [int(os.environ["BACKUWUP_GPU_DEVICE"])]
    n = ctypes.c_int()
    _lib.check(_lib.load().bw_device_count(ctypes.byref(n)))
    if n.value <= 0:
        raise RuntimeError("backuwup_amd: no GPU for the drop-in pool")
    return list(range(n.value))


class Pool:
    def __init__(self, devices=None, per_device=None):
        self.devices = list(devices) if devices is not None else devices_from_env()
        if not self.devices:
            raise ValueError("Pool: no devices")
        per = per_device or int(os.environ.get("BACKUWUP_GPU_CONTEXTS", "16"))
        self._L = _lib.load()
        self.contexts = [Context(self.devices[j % len(self.devices)]) for j in range(max(1, per) * len(self.devices))]
        self._locks = [threading.Lock() for _ in self.contexts]
        self._next = itertools.count()
        self._tls = threading.local()

    def home_slot(self):
        s = getattr(self._tls, "slot", None)
        if s is None:
            s = self._tls.slot = next(self._next)
        return s

    def home_device(self):
        return self.devices[self.home_slot() % len(self.devices)]

    def with_context(self, fn):
        """fn(context) on the first free context from this thread's home slot on (blocking on the
        home slot's own when every context is busy)."""
        n = len(self.contexts)
        start = self.home_slot() % n
        for k in range(n):
            j = (start + k) % n
            if self._locks[j].acquire(blocking=False):
                try:
                    return fn(self.contexts[j])
                finally:
                    self._locks[j].release()
        with self._locks[start]:
            return fn(self.contexts[start])

    def hash_dropin(self, data):
        """blake3::hash of read-only memory (the Rust drop-in's `hash(&[u8])`): kept chunk digests,
        then the home device's hash service, BW_EAGAIN -> a pool context's launch path."""
        from .blake3 import _as_bytes_view  # (a zero-copy view: the kept digests are found by address)
        buf = _as_bytes_view(data)
        out = (ctypes.c_uint8 * 32)()
        rc = self._L.bw_blake3_hash_dropin_device(self.home_device(), _ptr(buf), buf.size, out)
        if rc == _lib.BW_OK:
            return bytes(out)
        if rc != _lib.BW_EAGAIN:
            _lib.check(rc)
        return bytes(self.with_context(lambda c: c.blake3_many(buf, [0], [buf.size]))[0])

    def close(self):
        for c in self.contexts:
            c.close()


_pool = None
_pool_mu = threading.Lock()


def default_pool():
    global _pool
    with _pool_mu:
        if _pool is None:
            _pool = Pool()
        return _pool


__all__ = ["Pool", "default_pool", "devices_from_env"]
