"""Drop-in for `fastcdc::v2020` as backuwup uses it (crate fastcdc 3.0.3, Cargo.lock:557-560).

    let chunker = FastCDC::new(&mmap, min, avg, max);      // dir_packer.rs:254-259
    for chunk in chunker { &mmap[chunk.offset..chunk.offset + chunk.length] }   // :261-266

Here `FastCDC(source, min_size, avg_size, max_size)` chunks AND hashes the whole source on the GPU
in one submit when it is constructed (bw_fastcdc_chunks_hashed) and iterates `Chunk(hash, offset,
length)` like the crate's iterator.  While the object lives, `blake3.hash(view[offset:offset +
length])` of one of its chunks (a zero-copy view of the same memory, as the reference slices its
mmap) is answered from the kept digests instead of a second trip to the GPU.  Size parameters
outside the crate's asserted ranges raise ValueError (the crate panics), and so does avg > max
(the crate's cut() then reads past max: a chunk longer than max, or an index panic).
"""
from collections import namedtuple

from . import _lib
from ._lib import BW_EINVAL, BwError
from .blake3 import _as_bytes_view, _immutable

MINIMUM_MIN = 64
MINIMUM_MAX = 1_048_576
AVERAGE_MIN = 256
AVERAGE_MAX = 4_194_304
MAXIMUM_MIN = 1024
MAXIMUM_MAX = 16_777_216

Chunk = namedtuple("Chunk", ["hash", "offset", "length"])


class ChunkParameterError(ValueError):
    pass


class FastCDC:
    def __init__(self, source, min_size, avg_size, max_size, ctx=None):
        if not (MINIMUM_MIN <= min_size <= MINIMUM_MAX and AVERAGE_MIN <= avg_size <= AVERAGE_MAX
                and MAXIMUM_MIN <= max_size <= MAXIMUM_MAX):
            raise ChunkParameterError("fastcdc size parameters out of range: %d/%d/%d"
                                      % (min_size, avg_size, max_size))
        if avg_size > max_size:  # the crate's cut() reads past max and panics on most sources
            raise ChunkParameterError("fastcdc avg_size %d > max_size %d" % (avg_size, max_size))
        if ctx is None:  # the drop-in pool over the node's GPUs (backuwup_amd/pool.py)
            from .pool import default_pool
            run = default_pool().with_context
        else:
            def run(fn):
                return fn(ctx)
        self._kept, self._L = 0, _lib.load()
        try:
            buf = _as_bytes_view(source)
            if buf.size and buf.flags.c_contiguous and _immutable(source):
                cuts, self._kept = run(lambda c: c.fastcdc_chunks_hashed(buf, min_size, avg_size, max_size))
                self._buf = buf  # the kept digests name this memory: keep it alive with them
            else:
                cuts = run(lambda c: c.fastcdc_chunks(source, min_size, avg_size, max_size))
            self._chunks = [Chunk(*c) for c in cuts]
        except BwError as e:
            if e.rc == BW_EINVAL:
                raise ChunkParameterError(str(e)) from e
            raise
        self.min_size, self.avg_size, self.max_size = min_size, avg_size, max_size

    def __del__(self):  # the crate's FastCDC borrows the source; its digests go with the object
        kept, self._kept = getattr(self, "_kept", 0), 0
        if kept:
            self._L.bw_fastcdc_release(kept)

    def __iter__(self):
        return iter(self._chunks)

    def __len__(self):
        return len(self._chunks)
