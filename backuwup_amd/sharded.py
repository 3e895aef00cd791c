"""Multi-GPU dedup: the seen-chunk index partitioned by digest prefix across ranks.

One process per GPU.  Files are sharded rank-major (rank r holds canonical files
[F_r, F_{r+1})), so (rank, local blob index) order IS the canonical order.  Each step:

  1. every rank chunks + hashes its own files (no collective on the data path);
  2. its digests are stably partitioned by owner = digest[0] >> (8 - log2 N) into N buckets of a
     fixed capacity `cap` (one bound agreed per session), with the per-owner counts on the device;
  3. one all-to-all of the counts and one of the buckets (RCCL over xGMI on MI355X; equal splits,
     so nothing has to come back to the host first);
  4. each owner gates the received buckets against its shard of the index in source-rank-major
     order -- the canonical order, so first occurrence = first position;
  5. one all-to-all returns the verdict bytes, scattered back to local blob order.

Nothing in the sequence waits on the host: it is enqueued on the batch's stream behind the
batch's kernels, and the next batch (another stream) computes meanwhile.  The bucket capacity
trades bytes for the host round trip: N x cap x 32 B per rank per batch (C2: 65,538 slots -> 2 MiB
per owner), which xGMI moves in tens of microseconds.

This replaces the reference's single in-process BlobIndex (blob_index.rs:44-148), whose
`blobs_queued` HashSet and sorted `items` become the union of the N shards.

The collective sequence is written once against a small ops interface so the same code runs
on the GPU (DeviceShardOps, backed by libbackuwup_amd.so) and in the world-size-2/4 gloo tests.
"""
import torch
import torch.distributed as dist


def owner_of(first_byte, world):
    bits = world.bit_length() - 1
    return first_byte >> (8 - bits) if bits else 0


class DeviceShardOps:
    """GPU implementation of the three local steps (all device-resident, no synchronization).
    A batch is the tuple Context.batch_views(ticket) returns: (d_n, d_digests, d_is_dup, max_n)."""

    def __init__(self, ctx, device):
        # the collectives run on torch's current stream; the library must use the same stream so
        # its kernels and the all-to-alls are ordered
        self.ctx, self.device = ctx, device
        handle = torch.cuda.current_stream(device).cuda_stream
        if not handle:  # the null stream does not order against the library's non-blocking streams
            raise ValueError("run the exchange under a torch.cuda.Stream (not the default stream)")
        ctx.set_stream(handle)

    def partition(self, batch, cap, world):
        d_n, d_dig, _, max_n = batch
        buckets = torch.empty(world * cap * 32, dtype=torch.uint8, device=self.device)
        perm = torch.empty(world * cap, dtype=torch.int64, device=self.device)
        counts = torch.empty(world, dtype=torch.int64, device=self.device)
        self.ctx.partition_buckets(d_dig, d_n, max_n, cap, world, buckets.data_ptr(), perm.data_ptr(),
                                   counts.data_ptr())
        return buckets, perm, counts

    def decide(self, recv, recv_counts, world, cap):
        verdict = torch.empty(world * cap, dtype=torch.uint8, device=self.device)
        self.ctx.index_check_insert_buckets(recv.data_ptr(), recv_counts.data_ptr(), world, cap, verdict.data_ptr())
        return verdict

    def scatter(self, back, perm, counts, world, cap, batch):
        self.ctx.scatter_buckets(back.data_ptr(), perm.data_ptr(), counts.data_ptr(), world, cap, batch[2])


def exchange_dedup(ops, batch, world, cap, group=None, all_to_all=None):
    """Steps 2-5 above for one batch; verdicts land in the batch's is_dup.  Returns the per-owner
    counts tensor (device) for diagnostics.  all_to_all(out, inp, group) defaults to
    dist.all_to_all_single (RCCL for device tensors)."""
    a2a = all_to_all or (lambda out, inp, group: dist.all_to_all_single(out, inp, group=group))
    buckets, perm, counts = ops.partition(batch, cap, world)
    recv_counts = torch.empty_like(counts)
    a2a(recv_counts, counts, group)
    recv = torch.empty_like(buckets)
    a2a(recv, buckets, group)
    verdict = ops.decide(recv, recv_counts, world, cap)
    back = torch.empty_like(verdict)
    a2a(back, verdict, group)
    ops.scatter(back, perm, counts, world, cap, batch)
    return counts


def session_capacity(max_blobs, device, group=None):
    """The bucket capacity of a session: the largest per-batch blob bound over the ranks (one
    all-reduce when the session starts, never per batch)."""
    t = torch.tensor([int(max_blobs)], dtype=torch.int64, device=device)
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return int(t.item())


def staged_all_to_all(out, inp, group=None):
    """all_to_all_single for a backend without device collectives (gloo): the tensors go through
    host memory.  Used to run the device exchange with several ranks on one GPU (tests)."""
    o = torch.empty(out.shape, dtype=out.dtype)
    dist.all_to_all_single(o, inp.cpu(), group=group)
    out.copy_(o)
