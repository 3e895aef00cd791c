"""One long file split across ranks (SURVEY.md §8e "single long stream"): exact FastCDC
boundaries with one small exchange per round.

The reference chunks a file serially from its start (a new FastCDC per file,
dir_packer.rs:254-266).  Split over N GPUs, rank r owns the file bytes [S_r, S_{r+1}) and holds
the window [S_r - max, S_{r+1} + max) in HBM (the halos overlap its neighbours by one maximum
chunk).  Rank r chunks its window from a speculative start; CDC resynchronises, so its cut
chain soon equals the true one.  The exchange settles where each rank's true chain enters:

  round:  every rank publishes P_r = its last cut <= S_{r+1} (an allgather of one u64); rank r
          takes entry = P_{r-1}; if entry is a cut of its current chain, the chain from entry
          on is the true one (a cut depends only on its start position and the bytes after it);
          otherwise it rechunks its window from entry.  A second allgather tells whether any
          rank rechunked; if none did, every entry is true.  At most N + 1 rounds, normally 1.

Why the windows suffice: true chunks are <= max, so the true last cut <= S_{r+1} lies in
[S_{r+1} - max, S_{r+1}], inside rank r+1's back halo; and a chunk that starts before S_{r+1}
is decided by bytes up to start + max <= S_{r+1} + max, inside rank r's forward halo, so the
cuts rank r keeps are never affected by its window ending early.

Rank r emits the chunks starting in [entry_r, P_r) (the last rank: to the end of the file),
so the chunk straddling S_{r+1} is hashed by rank r+1, which holds it whole in its back halo.
Emitted chunks in rank order are the file's chunks in offset order, i.e. canonical order for
the digest-prefix exchange (sharded.py).

The product path is the C ABI's bw_chunk_stream_shard (backuwup_amd/csrc/bw_stream.hip, round 5),
which runs these rounds in C over the communicator's control channel (RCCL or the caller's host
transport) and hands the final chain to bw_exchange_dedup.  This module keeps the same settlement
as pure logic over a `chunk_fn(start, end) -> cut positions` callback for the world-size-2/4 gloo
tests (the tests' CPU chunker stands in for the device) and for driving several ranks' windows
from one process (`device_chunk_fn`).
"""
import numpy as np


def split_bounds(file_len, world):
    """S_0 .. S_N: the owned ranges (equal split)."""
    return [file_len * k // world for k in range(world + 1)]


def window(file_len, rank, world, max_size):
    """[lo, hi): rank's part of the file in HBM (bw_stream_window computes the same)."""
    s = split_bounds(file_len, world)
    return max(0, s[rank] - max_size), min(file_len, s[rank + 1] + max_size)


class SplitResolver:
    """Rank `rank`'s side of the boundary settlement for one file of `file_len` bytes.

    chunk_fn(start, end) chunks file[start:end) as a file of its own and returns the chunk end
    positions (absolute, ascending; the last is `end`) plus any payload to keep (e.g. the
    batch's blob records): (cuts, payload)."""

    def __init__(self, chunk_fn, file_len, rank, world, max_size):
        self.chunk_fn, self.F, self.rank, self.world = chunk_fn, file_len, rank, world
        self.S = split_bounds(file_len, world)
        self.lo, self.hi = window(file_len, rank, world, max_size)
        self.rounds = 0
        self._chunk(0 if rank == 0 else self.lo)

    def _chunk(self, start):
        self.start = start
        cuts, self.payload = self.chunk_fn(start, self.hi)
        self.cuts = np.asarray(cuts, dtype=np.int64)
        self.rechunks = getattr(self, "rechunks", -1) + 1

    def publish(self):
        """P_rank: the last cut <= S_{rank+1} on the current chain (the chain start counts)."""
        if self.rank == self.world - 1:
            return self.F
        k = int(np.searchsorted(self.cuts, self.S[self.rank + 1], side="right"))
        return int(self.cuts[k - 1]) if k else self.start

    def update(self, published):
        """Take entry = P_{rank-1}; rechunk from it unless it is on the chain.  -> changed?"""
        self.rounds += 1
        self.entry = 0 if self.rank == 0 else int(published[self.rank - 1])
        if not (self.lo <= self.entry <= self.S[self.rank]):
            raise AssertionError("entry %d outside rank %d's back halo [%d, %d]" %
                                 (self.entry, self.rank, self.lo, self.S[self.rank]))
        if self.entry == self.start:
            return False
        k = int(np.searchsorted(self.cuts, self.entry))
        if k < len(self.cuts) and int(self.cuts[k]) == self.entry:
            return False
        self._chunk(self.entry)
        return True

    def emitted(self):
        """(first, count, chunk starts, chunk lengths): the chunks this rank owns, as a range of
        the current chain (chunk i of the chain spans [cut_{i-1}, cut_i), cut_{-1} = start)."""
        ends = self.cuts
        starts = np.concatenate([[self.start], ends[:-1]]) if len(ends) else np.zeros(0, np.int64)
        stop = self.F if self.rank == self.world - 1 else self.last
        sel = np.nonzero((starts >= self.entry) & (starts < stop))[0]
        first = int(sel[0]) if len(sel) else 0
        return first, len(sel), starts[sel], ends[sel] - starts[sel]


def settle(resolvers_or_one, allgather=None):
    """Run the rounds.  Distributed: settle(resolver, allgather) where allgather(x) returns the
    list of every rank's x.  Single process driving all ranks: settle([r0, r1, ...])."""
    if allgather is None:
        rs = resolvers_or_one
        while True:
            pub = [r.publish() for r in rs]
            changed = [r.update(pub) for r in rs]
            if not any(changed):
                for r in rs:
                    r.last = pub[r.rank]
                return rs
    r = resolvers_or_one
    while True:
        pub = allgather(r.publish())
        changed = allgather(bool(r.update(pub)))
        if not any(changed):
            r.last = pub[r.rank]
            return r


def device_chunk_fn(ctx, d_window_ptr, window_lo, params):
    """chunk_fn over this rank's window resident in HBM (file byte x at d_window_ptr + x -
    window_lo; d_window_ptr 16-byte aligned): one bw_process_files_device call per chain, CDC
    forced (the window is part of a file above the small-file threshold), digests computed, no
    index.  Returns the chain's cuts and its blob records."""
    from . import _lib
    from .context import make_params
    p = make_params(min_size=params.min_size, avg_size=params.avg_size, max_size=params.max_size,
                    small_file_threshold=0, flags=params.flags | _lib.BW_F_NO_DEDUP)

    def fn(start, end):
        rel = start - window_lo
        base = rel & ~15
        ctx.submit_device(d_window_ptr + base, end - window_lo - base, [rel - base], [end - start], p)
        res = ctx.results()
        cuts = start + res["offset"].astype(np.int64) + res["length"].astype(np.int64)
        return cuts, res

    return fn
