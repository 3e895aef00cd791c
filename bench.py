#!/usr/bin/env python3
"""Benchmark: GB/s chunked + hashed + deduped (BASELINE.json metric).

Default workload C2 = a single 16 GiB random stream per GPU, device-resident (BASELINE.json
configs[1]).  One step = one pass of the hot path over the batch: FastCDC-v2020 (256 KiB / 1 MiB /
3 MiB) -> BLAKE3 of every chunk -> seen-chunk index.  The whole run is one backup session: one
index for every batch, so after the first step every timed blob is a re-submitted duplicate (the
gate does the same work for a duplicate as for a new digest: append, claim, full-digest compare).
Inputs are generated on the GPU (counter-based splitmix64, seed 42 + rank) before timing, so the
timed region starts with the bytes resident in HBM.

N GPUs (weak scaling): every rank owns its own stream; the index is partitioned by digest prefix
and each step exchanges digests with RCCL all-to-alls (and verdicts back).

Other configurations, for DESIGN.md / profiles -- the driver's line is C2:
  --workload c1   1 GiB directory tree, 30% whole-file copies (the reference's CPU config)
  --workload c3   VM images: 4 GiB base + 15 byte-shifted variants = 64 GiB (--gib scales the base)
  --workload c4   1M small files of 4-64 KiB, 30% copies (copies alias their source's bytes)
  --host-stream   the batch starts in pinned host memory: H2D copy of batch k+1 overlaps the
                  processing of batch k (PCIe-inclusive rate; never the headline value)

Prints one JSON line (rank 0).  Extra diagnostics go to stderr.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GB/s chunked+hashed+deduped (whole node, 1/2/4/8 GPU), bit-exact vs CPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s HBM3E (spec)
PCIE_PEAK_GBS = 63.0   # MI355X_MICROARCH.md: PCIe Gen5 x16, 63 GB/s (spec)
# The BLAKE3 leaf pass's own ceiling is integer VALU issue.  It is measured in the
# run: bw_calibrate_b3 runs the pass's compression from registers at its occupancy, giving bytes
# per shader clock per CU, which the line scales to the GFX clock the chip held over the timed steps.
CALIBRATE_MS = 150.0
# stage marks kept in the timed region (BW_OPT_PROFILE_MASK): the two around the BLAKE3 leaf pass,
# the dominant kernel; each mark costs the stream ~5 us, so the full stage split is taken after,
# on the same batch with nothing beside it
PROFILE_MASK_TIMED = (1 << 4) | (1 << 5)  # b3_leaf start, b3_tree start
HOLD_S, HOLD_SKIP_S, PASS_S = 3.0, 0.5, 1.5  # untimed power holds after the timed steps (seconds)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_workload(name, gib, rank, dev, n_files):
    """-> (device uint8 tensor, file_off, file_len, description).  Bytes are generated in HBM."""
    import numpy as np
    import torch
    from backuwup_amd import synth
    if name == "c2":
        n = int(gib * (1 << 30))
        data = synth.splitmix_torch(42 + rank, n, dev)
        return data, [0], [n], ("C2: single %.0f GiB splitmix64 stream per GPU (seed 42+rank), device-resident; "
                                "FastCDC v2020 256K/1M/3M -> BLAKE3 -> index" % gib)
    if name == "c1":
        d, o, l = synth.tree_corpus(int(gib * (1 << 30)), seed=0x6261636B + rank)
        return torch.from_numpy(d).to(dev), o, l, ("C1: %.0f GiB directory tree per GPU, %d files (log-uniform "
                                                    "4 KiB-64 MiB, 30%% whole-file copies)" % (gib, len(l)))
    if name == "c3":
        base = int(gib * (1 << 30))
        data, o, l = synth.vm_image_variants_torch(base, 16, dev, seed=1 + rank)
        return data, o, l, ("C3: VM images per GPU, %.1f GiB base + 15 variants (32 byte indels + 16 x 4 KiB "
                            "overwrites each) = %.1f GiB" % (gib, data.numel() / 2**30))
    if name == "c5":
        # 4 families of C3-style images (base seed 1 + family), 16 files of
        # `gib` GiB each; every family is split over 2 ranks (8 files each), so at 8 GPUs the job
        # holds 256 GiB and ranks r, r^1 share a base image (cross-rank duplicates go through the
        # digest exchange).  The rank's files are staged to pinned host memory by the caller.
        fam, half = (rank // 2, rank % 2)
        base = int(gib * (1 << 30))
        full, o, l = synth.vm_image_variants_torch(base, 16, dev, seed=1 + fam)
        lo, hi = int(o[8 * half]), int(o[8 * half + 7] + l[8 * half + 7])
        data = full[lo:hi].clone()
        del full
        torch.cuda.empty_cache()
        o = (o[8 * half:8 * half + 8] - np.uint64(lo)).astype(np.uint64)
        l = l[8 * half:8 * half + 8]
        return data, o, l, ("C5: VM-image family %d (base seed %d, %.1f GiB base), files %d-%d of its 16 on this "
                            "rank = %.1f GiB, staged in pinned host memory" %
                            (fam, 1 + fam, gib, 8 * half, 8 * half + 7, data.numel() / 2**30))
    if name == "c4":
        u, o, l = synth.small_files_table(n_files, seed=3 + rank)
        data = synth.splitmix_torch(3 + rank, u, dev)
        return data, o, l, ("C4: %d small files per GPU (4-64 KiB uniform, 30%% copies aliasing their source), "
                            "%.1f GB of file bytes" % (n_files, float(np.sum(l)) / 1e9))
    raise SystemExit("unknown workload " + name)


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv):
    """`--gpus N` without a torchrun environment: start N ranks (one process per GPU) as children
    through torch.distributed.run, before this process touches any GPU, and exit with their
    status.  Rank 0 prints the JSON line (its stdout is this process's stdout)."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + argv
    log("bench: launching %d ranks: %s" % (n, " ".join(cmd)))
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); without a torchrun environment bench.py starts them itself")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher check without a GPU: the ranks rendezvous over gloo, verify the world size and "
                         "time a CPU stand-in step (no hot path, value null)")
    ap.add_argument("--dry-run-fail-rank", type=int, default=None, help=argparse.SUPPRESS)  # failure-path test
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default: about 3 s of work for the workload)")
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="c2", choices=["c1", "c2", "c3", "c4", "c5"])
    ap.add_argument("--gib", type=float, default=None,
                    help="C2: stream size per GPU; C1: corpus size; C3/C5: base image size (GiB)")
    ap.add_argument("--files", type=int, default=1000000, help="C4: files per GPU")
    ap.add_argument("--cpu-sample-gib", type=float, default=None,
                    help="CPU baseline sample (default: 8 GiB of C2 on one core, ~10 s; up to 16 GiB of files "
                         "on 16 cores for the other workloads)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-trees", action="store_true",
                    help="C4: the CPU baseline also hashes each file's Tree blob (dir_packer.rs:274 -> :320), the "
                         "reference's second blake3::hash per small file (tools/dropin_c4.cpp's GPU side)")
    ap.add_argument("--cpu-all-cores", action="store_true",
                    help="also time the CPU baseline on os.cpu_count() threads (a whole node that is yours; the "
                         "default measures this GPU's 16-core share and one core, and estimates the node)")
    ap.add_argument("--no-power", action="store_true", help="do not sample socket power during the timed steps")
    ap.add_argument("--no-holds", action="store_true",
                    help="skip the untimed power holds after the timed steps (sustained pipeline, each pass alone)")
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--streams", type=int, default=None,
                    help="batches in flight: consecutive steps alternate between this many contexts/streams "
                         "(default 3 for C1's 1 GiB batches, whose fixed per-batch latency a third batch hides "
                         "(1.42 -> 1.60 TB/s), 2 otherwise: a third gains nothing on large batches)")
    ap.add_argument("--host-stream", action="store_true",
                    help="batches start in pinned host memory (H2D copies overlapped with processing)")
    ap.add_argument("--trees", action="store_true",
                    help="also time the file-tree blobs of the last batch (bw_tree_blobs, §8f row 1)")
    ap.add_argument("--seal", action="store_true",
                    help="also time sealing the last batch's unique blobs (HKDF + AES-256-GCM, §8f row 3)")
    ap.add_argument("--pack", action="store_true",
                    help="also time packing the last batch's unique blobs into packfiles: zstd store frames, "
                         "per-blob + header AES-256-GCM, packfile layout (§8f rows 2-4)")
    ap.add_argument("--pack-l3", action="store_true",
                    help="also time the full chain on the last batch's unique blobs: level-3 zstd on the GPU, "
                         "the packfile grouping over the frame sizes, sealing + layout (§8f rows 2-4)")
    ap.add_argument("--b3-loads", type=int, default=None, choices=[0, 1, 2],
                    help="[BW_DIAG build only: BW_LIB=backuwup_amd/libbackuwup_amd_debug.so] BLAKE3 leaf loads (BW_OPT_B3_LOADS): 0 = one block ahead, 1 = block pairs, "
                         "2 = aligned lines (k_b3_lines)")
    ap.add_argument("--scan-waves", type=int, default=None, choices=[8, 16], help="[BW_DIAG build only: BW_LIB=backuwup_amd/libbackuwup_amd_debug.so] BW_OPT_SCAN_WAVES")
    ap.add_argument("--latency-stream", type=int, default=None, choices=[0, 1], help="[BW_DIAG build only: BW_LIB=backuwup_amd/libbackuwup_amd_debug.so] BW_OPT_LATENCY_STREAM")
    ap.add_argument("--order-hash", type=int, default=None, choices=[0, 1], help="[BW_DIAG build only: BW_LIB=backuwup_amd/libbackuwup_amd_debug.so] BW_OPT_ORDER_HASH")
    ap.add_argument("--split", type=int, default=None, choices=[1, 2],
                    help="[BW_DIAG build only: BW_LIB=backuwup_amd/libbackuwup_amd_debug.so] BW_OPT_SPLIT: 2 = multi-file batches of 64 MiB-4 GiB as a head and a tail part on two streams")
    ap.add_argument("--b3-upper", type=int, default=None, choices=[0, 1],
                    help="[BW_DIAG build only: BW_LIB=backuwup_amd/libbackuwup_amd_debug.so] BW_OPT_B3_UPPER: 0 = upper levels in their own launch (default), 1 = inside the leaf pass")
    ap.add_argument("--b3-group", type=int, default=None, choices=[1, 2, 4],
                    help="BW_OPT_B3_GROUP: BLAKE3 leaves per lane of the leaf pass")
    ap.add_argument("--scan-first", type=int, default=None, choices=[0, 1, 2], help="BW_OPT_SCAN_FIRST")
    ap.add_argument("--all-stage-marks", action="store_true",
                    help="mark every stage in the timed region (each mark costs the stream ~5 us)")
    ap.add_argument("--no-calibrate", action="store_true", help="skip the in-run VALU-issue calibration")
    ap.add_argument("--exchange", action="store_true",
                    help="run the multi-GPU digest exchange (RCCL) even at world size 1 (rehearses the N > 1 path)")
    ap.add_argument("--transport", default="rccl", choices=["rccl", "host"],
                    help="the exchange's transport: RCCL over xGMI (the product), or 'host' = the caller's host "
                         "all-to-all over a gloo process group, with ranks allowed to share a GPU (rank r on "
                         "device r mod the visible count): rehearses the N > 1 bench path on a one-GPU box")
    ap.add_argument("--split-files", action="store_true",
                    help="C3: every rank holds the same corpus and each file is split across the ranks "
                         "(bw_chunk_stream_shard, SURVEY.md §8e single long stream) then exchanged; strong "
                         "scaling: value = the corpus's bytes (once) per second")
    args = ap.parse_args()
    if args.gpus is not None and args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world_env = int(os.environ.get("WORLD_SIZE", 1))
    if args.gpus is not None and args.gpus != world_env:
        raise SystemExit("--gpus %d but WORLD_SIZE=%d: refusing to report a %d-GPU line" %
                         (args.gpus, world_env, world_env))
    if args.dry_run:
        return dry_run(args)
    if args.split_files:
        return split_files_bench(args)
    if args.steps is None:
        args.steps = {"c1": 3000, "c2": 320, "c3": 80, "c4": 200, "c5": 5}[args.workload]
    if args.gib is None:
        args.gib = {"c1": 1.0, "c2": 16.0, "c3": 4.0, "c4": 0.0, "c5": 4.0}[args.workload]
    if args.cpu_sample_gib is None:
        args.cpu_sample_gib = 8.0 if args.workload == "c2" else 16.0
    if args.workload == "c5":
        args.host_stream = True  # C5 is quoted end to end from pinned host memory

    import numpy as np
    import torch
    import torch.distributed as dist

    import ctypes

    from backuwup_amd import BLOB_DTYPE, Context, Index, _lib, make_params
    from backuwup_amd._lib import (BW_B3_LOADS_DEFAULT, BW_F_NO_DEDUP, BW_F_NO_HASH, BW_OPT_B3_LOADS, BW_OPT_DEPTH, BW_OPT_LATENCY_STREAM, BW_OPT_ORDER_HASH,
                                   BW_OPT_B3_GROUP, BW_OPT_B3_UPPER, BW_OPT_PROFILE_MASK, BW_OPT_SCAN_FIRST, BW_OPT_SCAN_WAVES, BW_OPT_SPLIT, STAGES)

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    host_tp = args.transport == "host"
    if host_tp:  # (rehearsal: ranks may share a GPU)
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    multi = world > 1 or args.exchange  # the sharded-index path (digest all-to-all over RCCL)
    if multi:
        if not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29511")
            import datetime  # a rank that never joins (or dies) ends the run instead of hanging it
            if host_tp:
                dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(minutes=5))
            else:
                dist.init_process_group("nccl", device_id=dev, rank=rank, world_size=world,
                                        timeout=datetime.timedelta(minutes=5))
        if dist.get_world_size() != world:
            raise SystemExit("process group has %d ranks, WORLD_SIZE says %d" % (dist.get_world_size(), world))

    t0 = time.time()
    data, file_off, file_len, desc = make_workload(args.workload, args.gib, rank, dev, args.files)
    torch.cuda.synchronize()
    n = int(data.numel())
    processed = int(np.sum(np.asarray(file_len, dtype=np.uint64)))  # file bytes per step (C4 copies alias)
    log("rank %d: %s -- generated in %.1f s" % (rank, desc, time.time() - t0))

    # One backup session: every batch is gated by ONE index (bw_index) shared by the contexts.
    # Device-resident: consecutive batches alternate between two (C1: three) contexts on their streams (one
    # batch's HBM-bound scan beside the other's VALU-bound BLAKE3), the index event chain keeps
    # their dedup in submission order, and batch k's results are read after batch k+1 is queued.
    # Host-streamed: one context; its copy stream brings batch k+1 from pinned host memory while
    # batch k computes (bw_submit_host).  N > 1: the local pass skips the index; each batch's
    # digests go through the RCCL exchange to their owner's index while the next batch computes.
    if args.streams is None:
        args.streams = 3 if args.workload == "c1" else 2
    nctx = 1 if args.host_stream and not multi else (2 if multi else max(1, args.streams))
    index = Index(local)
    ctxs, streams = [], []
    for k in range(nctx):
        c = Context(local)
        st = torch.cuda.Stream(dev)
        c.set_stream(st.cuda_stream)
        c.attach_index(index)
        if args.b3_loads is not None:
            c.set_option(BW_OPT_B3_LOADS, args.b3_loads)
        if args.scan_waves is not None:
            c.set_option(BW_OPT_SCAN_WAVES, args.scan_waves)
        if args.latency_stream is not None:
            c.set_option(BW_OPT_LATENCY_STREAM, args.latency_stream)
        if args.order_hash is not None:
            c.set_option(BW_OPT_ORDER_HASH, args.order_hash)
        if args.split is not None:
            c.set_option(BW_OPT_SPLIT, args.split)
        if args.scan_first is not None:
            c.set_option(BW_OPT_SCAN_FIRST, args.scan_first)
        if args.b3_upper is not None:
            c.set_option(BW_OPT_B3_UPPER, args.b3_upper)
        if args.b3_group is not None:
            c.set_option(BW_OPT_B3_GROUP, args.b3_group)
        if args.host_stream and nctx > 1:
            c.set_option(BW_OPT_DEPTH, 1)  # contexts alternate: one HBM input buffer each is enough
        ctxs.append(c)
        streams.append(st)
    ctx = ctxs[0]
    flags = BW_F_NO_DEDUP if multi else 0
    params = make_params(flags=flags)
    max_blobs = sum(int(x) // (256 << 10) + 2 if int(x) > (1 << 20) else 1 for x in file_len)
    total_batches = args.warmup + args.steps + 4 + (3 if nctx > 1 else 0)
    # the host's bound of the log grows by max_blobs per batch until a result read tightens it
    # (N > 1: by the digests the exchange delivered, about max_blobs); a bound past the table's capacity is
    # tightened by a synchronizing read before it grows, so the session pre-sizes the index
    index_hint = total_batches * max_blobs + 1024
    owner_bits = world.bit_length() - 1
    assert world == 1 << owner_bits, "world size must be a power of two (digest-prefix owners)"

    host = None
    if args.host_stream:
        # the batch lives in pinned host memory; the library copies it in on its copy stream
        host = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        host.copy_(data)
        torch.cuda.synchronize()

    step_no = [0]
    data_ptr = data.data_ptr()
    host_ptr = host.data_ptr() if host is not None else None
    file_off = np.ascontiguousarray(file_off, dtype=np.uint64)
    file_len = np.ascontiguousarray(file_len, dtype=np.uint64)
    host_ms = [0.0]  # host time inside the library's submit calls (metadata build + upload)
    inflight = []  # (context, ticket) of batches whose results are not read yet
    out_buf = np.zeros(max_blobs + 1, dtype=BLOB_DTYPE)

    comm = None
    if multi:
        # the digest exchange through the C ABI (bw_comm_init + bw_exchange_dedup): RCCL over
        # xGMI, every transfer sized from the exchange's own counts, no host wait for the peers;
        # rank 0 draws the RCCL id and the process group hands it to the others
        from backuwup_amd.comm import Comm, gloo_all_to_all, unique_id
        if host_tp:
            comm = Comm.host(local, rank, world, gloo_all_to_all())
        else:
            uid = [unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            comm = Comm.rccl(local, rank, world, uid[0])

    def drain():
        while inflight:
            c, t = inflight.pop(0)
            wait(c, t)

    # The timed loop calls the C ABI with ctypes arguments built once (the Context methods convert
    # and wrap per call, ~10-20 us of Python per batch that a Rust caller does not have; with one
    # batch in flight that time sits between two batches on the GPU)
    L = _lib.load()
    c_data, c_fo, c_fl = ctypes.c_void_p(data_ptr), file_off.ctypes.data_as(_lib.u64p), file_len.ctypes.data_as(_lib.u64p)
    c_nf, c_params = len(file_off), ctypes.byref(params)
    t_out, n_out = ctypes.c_uint64(), ctypes.c_uint64()
    c_t, c_n = ctypes.byref(t_out), ctypes.byref(n_out)
    c_out, c_cap = out_buf.ctypes.data_as(ctypes.POINTER(_lib.BwBlob)), out_buf.size

    def submit(c):
        if host is not None:
            return c.submit_host(host_ptr, file_off, file_len, params, data_len=n)
        rc = L.bw_submit_device(c.h, c_data, n, c_fo, c_fl, c_nf, c_params, c_t)
        if rc:
            _lib.check(rc, c.h)
        return t_out.value

    first_res = [None]  # the session's first batch (fresh index): the whole-result parity check's input

    def wait(c, t):
        rc = L.bw_wait(c.h, t, c_out, c_cap, c_n)
        if rc:
            _lib.check(rc, c.h)
        if first_res[0] is None:
            first_res[0] = out_buf[:n_out.value].copy()

    def step():
        k = step_no[0] % len(ctxs)
        step_no[0] += 1
        c = ctxs[k]
        # (the context runs on the stream set_stream gave it: no torch stream switch per step)
        th = time.perf_counter()
        t = submit(c)
        host_ms[0] += (time.perf_counter() - th) * 1e3
        if multi:
            # owner = digest[0] >> (8 - log2 N): the counts go out now, the digests and verdicts once
            # they arrived (the next exchange or the wait notices); the host never waits for a peer here
            c.exchange_dedup(comm, t)
        inflight.append((c, t))
        if len(inflight) >= len(ctxs):  # one batch per context in flight: read the oldest while the rest run
            c0, t0 = inflight.pop(0)
            wait(c0, t0)

    ctx.index_reset(index_hint)
    for _ in range(args.warmup):
        step()
    if first_res[0] is None and not args.no_check:
        step()  # (--warmup 0: one untimed batch for the parity check)
    drain()
    torch.cuda.synchronize()

    check = None
    if not args.no_check:
        check = parity_spot_check(args, ctx, data, file_off, file_len, rank, first_res[0])
        log("rank %d: parity spot check %s" % (rank, check))
        if not check["bit_exact"]:
            raise SystemExit("parity check failed")

    full_mask = (2 << len(STAGES)) - 1  # every stage and the batch end
    for c in ctxs:
        c.set_option(BW_OPT_PROFILE_MASK, full_mask if args.all_stage_marks else PROFILE_MASK_TIMED)
        c.profile_enable(True)
    if multi:
        dist.barrier()
    torch.cuda.synchronize()
    host_ms[0] = 0.0
    sampler = PowerSampler(local) if (rank == 0 and not args.no_power) else None
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    drain()
    torch.cuda.synchronize()
    if multi:
        dist.barrier()
    el = time.perf_counter() - t0
    power, power_missing = sampler.stop() if sampler else (None, None)
    if multi:
        t = torch.tensor([el], dtype=torch.float64, device="cpu" if host_tp else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    ctx.index_check()  # no sticky index error anywhere in the session
    stage_ms, nbatch = ctx.profile_read()
    per = {s: stage_ms[s] / max(nbatch, 1) for s in STAGES}
    # the leaf pass's active time per step: the union of its launches' intervals over every context
    # (two contexts' leaf passes overlap each other in time, so the mean launch duration can exceed
    # the step time; the union cannot)
    leaf_iv = sorted(iv for c in ctxs for iv in c.profile_intervals("b3_leaf"))
    leaf_union, cur = 0.0, None
    for a, z in leaf_iv:
        if cur is None or a > cur[1]:
            if cur is not None:
                leaf_union += cur[1] - cur[0]
            cur = [a, z]
        else:
            cur[1] = max(cur[1], z)
    if cur is not None:
        leaf_union += cur[1] - cur[0]
    leaf_active_ms = leaf_union / args.steps if leaf_iv else None
    iso = None
    if not multi and host is None:
        # the same batch with nothing beside it (one context, synchronized, every stage marked):
        # each kernel's own duration, reported next to the live one, which shares the GPU with
        # the other batches in flight (and has only the roofline's kernels marked)
        ctx.set_option(BW_OPT_PROFILE_MASK, full_mask)
        ctx.profile_enable(True)
        for _ in range(3):
            with torch.cuda.stream(streams[0]):
                ctx.submit_device(data.data_ptr(), n, file_off, file_len, params)
            torch.cuda.synchronize()
        iso_ms, iso_n = ctx.profile_read()
        iso = {s: iso_ms[s] / max(iso_n, 1) for s in STAGES}
    res = ctx.results()
    log("rank %d: %d blobs/step, stage ms/step: %s, host submit ms/step %.3f" %
        (rank, len(res), {k: round(v, 3) for k, v in per.items()}, host_ms[0] / args.steps))

    # Power evidence, after the timed steps and outside them: socket power lags, so
    # a short timed window mostly samples the ramp.  `sustained` keeps the same pipeline running for
    # HOLD_S and drops the first HOLD_SKIP_S of samples; `passes` holds each pass alone for PASS_S:
    # the scan (the batch chunked with BW_F_NO_HASH) and the BLAKE3 pass (the batch's own chunks
    # submitted as whole-file blobs: unit table + k_b3_lines + k_b3_upper, no scan).
    holds = None
    if not multi and host is None and not args.no_power and not args.no_holds and rank == 0:
        for c in ctxs:
            c.profile_enable(False)

        def hold(seconds, one):
            sampler = PowerSampler(local)
            t0, nb = time.perf_counter(), 0
            while time.perf_counter() - t0 < seconds:
                one()
                nb += 1
            drain()
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            pw, missing = sampler.stop(skip_s=HOLD_SKIP_S)
            return nb, el, pw, missing

        nb, el_h, pw, missing = hold(HOLD_S, step)
        holds = {"sustained": dict(pw or {"missing": missing}, seconds=round(el_h, 3), batches=nb,
                                   gbs=round(processed * nb / el_h / 1e9, 1), skipped_s=HOLD_SKIP_S,
                                   what="the timed pipeline (same contexts, same batch) kept running untimed")}
        pn = make_params(flags=BW_F_NO_HASH | BW_F_NO_DEDUP)
        cut_off = (file_off[res["file"].astype(np.int64)] + res["offset"]).astype(np.uint64)
        cut_len = np.ascontiguousarray(res["length"], dtype=np.uint64)
        ph = make_params(flags=BW_F_NO_DEDUP)
        ph.small_file_threshold = int(cut_len.max()) if len(cut_len) else 0  # every chunk one whole blob
        passes = {}
        for name, pp, fo, fl, what in (
                ("scan", pn, file_off, file_len, "the batch with BW_F_NO_HASH: k_scan + boundary resolution"),
                ("blake3", ph, cut_off, cut_len, "the batch's chunks as whole-file blobs: k_b3_lines + k_b3_upper")):
            def one(pp=pp, fo=fo, fl=fl):
                k = step_no[0] % len(ctxs)
                step_no[0] += 1
                c = ctxs[k]
                rc = L.bw_submit_device(c.h, c_data, n, fo.ctypes.data_as(_lib.u64p), fl.ctypes.data_as(_lib.u64p),
                                        len(fo), ctypes.byref(pp), c_t)
                if rc:
                    _lib.check(rc, c.h)
                inflight.append((c, t_out.value))
                if len(inflight) >= len(ctxs):
                    c0, t0_ = inflight.pop(0)
                    wait(c0, t0_)
            nb, el_h, pw, missing = hold(PASS_S, one)
            passes[name] = dict(pw or {"missing": missing}, seconds=round(el_h, 3), batches=nb,
                                gbs=round(processed * nb / el_h / 1e9, 1), what=what)
            if pw:
                passes[name]["pj_per_byte"] = round(pw["socket_w_median"] / (processed * nb / el_h) * 1e12, 1)
        holds["passes"] = passes
        log("rank 0: power holds %s" % json.dumps(holds))

    total_bytes = processed * world * args.steps
    value = total_bytes / el / 1e9
    ms_per_step = el / args.steps * 1e3

    # roofline for the dominant kernel (largest stage time); algorithmic traffic = every input
    # byte read once per launch, so bytes per launch = the batch's file bytes
    # the dominant kernel is the BLAKE3 leaf pass (the longer pass on a batch alone, `isolated`
    # below, in every configuration); the timed region marks only it
    dom = max(["scan", "b3_leaf"], key=lambda s: per[s]) if args.all_stage_marks else "b3_leaf"
    algo = processed if dom == "b3_leaf" else n
    # achieved = the launch's bytes / the kernel's active time per step (the union above); the
    # mean launch duration (live, overlapping) stays beside it
    active_ms = leaf_active_ms if (dom == "b3_leaf" and leaf_active_ms) else per[dom]
    achieved = algo / (active_ms * 1e-3) / 1e9
    loads = args.b3_loads if args.b3_loads is not None else BW_B3_LOADS_DEFAULT
    leaf_kernel = "k_b3_lines" if loads == 2 else "k_b3_groups"
    kernel = {"scan": "k_scan", "b3_leaf": leaf_kernel}[dom]
    traffic, traffic_src, path_bytes = pmc_traffic(args, kernel)
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
                "kernel": kernel,
                "algorithmic_bytes_per_launch": algo,
                "kernel_active_ms_per_step": round(active_ms, 4),
                "kernel_active_basis": ("union of the %s launches' intervals over the %d contexts, per timed step "
                                        "(library events on the launches' own streams)" % (kernel, len(ctxs))
                                        if active_ms is leaf_active_ms else "mean launch duration"),
                "launch_ms_mean": round(per[dom], 4),
                # the whole pipeline against HBM: this GPU's input bytes per second / 8 TB/s
                "pipeline_frac": round(value / world / HBM_PEAK_GBS, 4),
                # every kernel of a batch (PMC FETCH + WRITE), per input byte: 1.0 would be one pass
                "path_bytes_per_input_byte": path_bytes,
                # the bound the contract prices against is HBM; the limit this kernel meets is integer
                # VALU issue (valu_issue.frac below) and the pipeline's is the socket power cap (power)
                "limiter": "integer VALU issue (BLAKE3 compressions; see valu_issue), at the socket power cap",
                "marked_stage_ms_per_step": ({k: round(v, 3) for k, v in per.items()} if args.all_stage_marks else
                                             {dom: round(per[dom], 3)}),
                "marked_stage_note": ("every stage marked (--all-stage-marks)" if args.all_stage_marks else
                                      "only the leaf pass is marked in the timed region (each mark costs ~5 us); "
                                      "the full stage split is isolated.stage_ms_per_step")}
    valu = None
    if kernel == leaf_kernel and not args.no_calibrate:
        # the limit this kernel actually meets: integer VALU issue, measured now on this chip
        cal = ctx.calibrate_b3(CALIBRATE_MS)
        mhz = power["gfx_mhz_mean"] if power is not None else None
        ceiling = cal["gbs"] * (mhz / 1e3) / cal["ghz"] if mhz and cal["ghz"] > 0 else cal["gbs"]
        valu = {"ceiling": round(ceiling, 1), "unit": "GB/s", "frac": round(achieved / ceiling, 4),
                "basis": ("bw_calibrate_b3: the leaf pass's compression from registers at its occupancy, "
                          "%.3f B per shader clock per CU, scaled to the %s" %
                          (cal["bytes_per_clk_cu"], "%d MHz GFX clock of the timed steps" % mhz if mhz
                           else "calibration's own clock (no power samples)")),
                "calibration": {k: round(v, 4) for k, v in cal.items()}}
        roofline["valu_issue"] = valu
    if host is not None:
        roofline.update({"host_stream_pcie_frac": round(value / PCIE_PEAK_GBS, 4)})
    if power is not None:
        # the limit the whole pipeline meets: the socket power cap; energy per byte
        # of this GPU's share of the work = its power / its throughput
        power["pj_per_byte"] = round(power["socket_w_median"] / (value / world * 1e9) * 1e12, 1)
        power["window"] = "the timed steps (%.2f s; amdsmi's socket power lags a short window)" % el
        roofline["power"] = power
    elif sampler is not None:
        roofline["power"] = None
        roofline["power_missing"] = power_missing
    if holds is not None:
        sus = holds["sustained"]
        if "socket_w_median" in sus:
            sus["pj_per_byte"] = round(sus["socket_w_median"] / (sus["gbs"] * 1e9) * 1e12, 1)
        roofline.setdefault("power", None)
        if roofline["power"] is None:
            roofline["power"] = {}
        roofline["power"]["sustained"] = sus
    if iso is not None:
        # live durations above include the overlap with the other batch in flight
        a_iso = algo / (iso["b3_leaf" if kernel == leaf_kernel else "scan"] * 1e-3) / 1e9
        if len(ctxs) > 1:
            roofline["live_shares_gpu_with"] = "the other batches in flight (%d contexts)" % len(ctxs)
        roofline["isolated"] = {"achieved": round(a_iso, 1), "frac": round(a_iso / HBM_PEAK_GBS, 4),
                                "valu_issue_frac": (round(a_iso / valu["ceiling"], 4) if valu else None),
                                "stage_ms_per_step": {k: round(v, 3) for k, v in iso.items()}}
        if holds is not None:
            roofline["isolated"]["passes"] = holds["passes"]

    trees = time_file_trees(ctx, res, file_len, args.steps) if args.trees else None
    seal = time_seal(ctx, data, res, file_off, args.steps) if args.seal else None
    pack = time_pack(ctx, data, res, file_off, args.steps) if args.pack else None
    pack_l3 = time_pack_l3(ctx, data, res, file_off, min(args.steps, 10)) if args.pack_l3 else None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, data, file_off, file_len)

    if rank == 0:
        line = {"metric": METRIC, "value": round(value, 3), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
                "config": {"workload": desc + (" -- streamed from pinned host memory" if host is not None else "") +
                           (" -- REHEARSAL: host transport, %d ranks on %d GPU(s)" % (world, torch.cuda.device_count())
                            if host_tp and multi else ""),
                           "bytes_per_gpu": processed, "blobs_per_gpu": int(len(res)),
                           "files_per_gpu": len(file_len),
                           "parallelism": "dp%d (files sharded, index by digest prefix)" % world,
                           "batches_in_flight": len(ctxs) if len(ctxs) > 1 else (2 if host is not None else 1),
                           "index": "one shared index for every batch (a single backup session)"},
                "roofline": roofline, "cpu_baseline": cpu, "parity": check}
        if trees:
            line["file_trees"] = trees
        if seal:
            line["seal"] = seal
        if pack:
            line["pack"] = pack
        if pack_l3:
            line["pack_l3"] = pack_l3
        print(json.dumps(line), flush=True)
    for c in ctxs:
        c.close()
    index.close()
    if comm is not None:
        comm.close()
    if multi:
        dist.destroy_process_group()


def split_files_bench(args):
    """--split-files: one corpus for the whole job, every file chunked by all the ranks together
    (bw_chunk_stream_shard: each rank chunks and hashes its window of the file, the ranks settle the
    boundaries, bw_exchange_dedup sends the chunks each rank emits to their owners).  One step = the
    whole corpus once.  Strong scaling."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from backuwup_amd import Context, Index, make_params
    from backuwup_amd._lib import BW_OPT_DEPTH
    from backuwup_amd.comm import Comm, unique_id
    from backuwup_amd.stream_split import window
    if args.workload not in ("c3", "c2"):
        raise SystemExit("--split-files applies to c2 (one stream) and c3 (VM images)")
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if args.steps is None:
        args.steps = 20 if args.workload == "c3" else 100
    if args.gib is None:
        args.gib = 4.0 if args.workload == "c3" else 16.0
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        import datetime
        dist.init_process_group("nccl", device_id=dev, rank=rank, world_size=world,
                                timeout=datetime.timedelta(minutes=5))
    t0 = time.time()
    data, file_off, file_len, desc = make_workload(args.workload, args.gib, 0, dev, args.files)  # same corpus on every rank
    torch.cuda.synchronize()
    log("rank %d: %s -- generated in %.1f s" % (rank, desc, time.time() - t0))
    file_off = np.asarray(file_off, dtype=np.uint64)
    file_len = np.asarray(file_len, dtype=np.uint64)
    params = make_params()
    uid = [unique_id() if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    comm = Comm.rccl(local, rank, world, uid[0])
    ctx = Context(local)
    ctx.set_stream(torch.cuda.Stream(dev).cuda_stream)
    ctx.set_option(BW_OPT_DEPTH, 8)
    index = Index(local)
    ctx.attach_index(index)
    total = int(np.sum(file_len))
    ctx.index_reset(int((args.warmup + args.steps + 1) * (total // (256 << 10) + 2 * len(file_len)) // world + 4096))
    wins = [window(int(file_len[f]), rank, world, params.max_size) for f in range(len(file_len))]
    base = data.data_ptr()
    rounds = []

    def step(keep=False):
        held, out = [], []
        for f in range(len(file_len)):
            lo, hi = wins[f]
            sh = ctx.chunk_stream_shard(comm, base + int(file_off[f]) + lo, int(file_len[f]), params)
            rounds.append(sh["rounds"])
            if sh["ticket"]:
                ctx.exchange_dedup(comm, sh["ticket"])
                held.append((f, sh))
        for f, sh in held[-8:]:  # the ring keeps the last 8; earlier exchanges finished as slots were reused
            r = ctx.wait(sh["ticket"])
            if keep:
                out.append((f, sh, r[sh["first_blob"]:sh["first_blob"] + sh["n_blobs"]].copy()))
        return out

    for _ in range(args.warmup):
        step()
    check = None
    if not args.no_check:
        got = step(keep=True)
        f0 = [(f, sh, r) for f, sh, r in got if f == got[0][0]] if got else []
        mine = [(int(sh["chain_start"] + b["offset"]), int(b["length"]), bytes(b["digest"])) for f, sh, r in f0
                for b in r]
        allm = [None] * world
        dist.all_gather_object(allm, (got[0][0] if got else -1, mine))
        if rank == 0:
            from oracle import oracle
            f = allm[0][0]
            chunks = sorted(c for fm, m in allm if fm == f for c in m)
            pre = min(int(file_len[f]), 96 << 20)  # the oracle over a prefix: its cuts before pre - max are the file's
            host = data[int(file_off[f]):int(file_off[f]) + pre].cpu().numpy()
            want = oracle.process_files(host, [0], [pre], small_threshold=0)
            lim = pre - params.max_size if pre < int(file_len[f]) else pre
            w = [(int(o), int(l), bytes(d)) for o, l, d in zip(want["offset"], want["length"], want["digest"])
                 if int(o) + int(l) <= lim]
            g = [c for c in chunks if c[0] + c[1] <= lim]
            check = {"bit_exact": w == g, "file": int(f), "chunks_compared": len(w),
                     "sample": "the emitted chunks of every rank in the first %d MiB of file %d against the oracle's "
                               "serial chunking (boundaries and digests)" % (lim >> 20, f)}
            log("rank 0: split parity %s" % check)
            if not check["bit_exact"]:
                raise SystemExit("parity check failed")
    rounds.clear()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())
    ctx.index_check()
    value = total * args.steps / el / 1e9
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": round(value, 3), "unit": "GB/s", "n_gpus": world,
                          "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3),
                          "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u8",
                          "data": "synthetic",
                          "config": {"workload": desc + " -- the same corpus on every rank, every file split across "
                                                        "the %d ranks (bw_chunk_stream_shard)" % world,
                                     "corpus_bytes": total, "files": len(file_len),
                                     "parallelism": "each file split over %d ranks, index by digest prefix" % world,
                                     "settlement_rounds_max": max(rounds) if rounds else 0,
                                     "settlement_rounds_mean": round(float(np.mean(rounds)), 3) if rounds else 0},
                          "roofline": None, "roofline_note": "the headline C2 line carries the roofline; this mode "
                                                             "adds the per-file settlement (host round trips)",
                          "cpu_baseline": None, "parity": check}), flush=True)
    ctx.close()
    index.close()
    comm.close()
    dist.destroy_process_group()


def dry_run(args):
    """--dry-run: the launcher, the rendezvous and the timing protocol without a GPU.  The ranks
    join over gloo, check the world size, and time a CPU stand-in step (a byte sum over 1 MiB)
    between barriers, max over ranks.  The line carries n_gpus and value null: nothing of the hot
    path runs."""
    import numpy as np
    import torch
    import torch.distributed as dist
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        if dist.get_world_size() != world:
            raise SystemExit("process group has %d ranks, WORLD_SIZE says %d" % (dist.get_world_size(), world))
    steps = args.steps or 3
    buf = np.random.default_rng(rank).integers(0, 256, 1 << 20, dtype=np.uint8)
    for _ in range(args.warmup):
        int(buf.sum())
    if args.dry_run_fail_rank == rank:  # a rank that dies mid-run: the launcher must exit non-zero
        log("bench: dry run: rank %d fails on purpose" % rank)
        os._exit(3)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        int(buf.sum())
    if world > 1:
        dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "GB/s", "n_gpus": world, "steps": steps,
                          "warmup": args.warmup, "ms_per_step": round(float(el.item()) / steps * 1e3, 4),
                          "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
                          "data": "synthetic", "dry_run": True,
                          "config": {"workload": "dry run: CPU stand-in step, no hot path",
                                     "parallelism": "dp%d" % world}}), flush=True)
    if world > 1:
        dist.destroy_process_group()


class PowerSampler:
    """Socket power and GFX clock of this process's GPU, read in-process through the amdsmi library
    (libamd_smi, read-only queries, no program launched) on a background thread while the timed
    steps run: the path holds the chip at its power cap, so energy per byte =
    power / throughput is the figure that bounds it.  The GPU is found by its PCI bus id (amdsmi
    lists every GPU of the host).  Fewer than MIN_SAMPLES samples in the timed window, or no
    amdsmi, gives power = null in the line (with the reason)."""
    MIN_SAMPLES = 5
    PERIOD_S = 0.02

    def __init__(self, dev):
        import threading
        self.samples, self.note = [], None
        self.t0 = time.perf_counter()
        self._stop = threading.Event()
        self.h = None
        try:
            import amdsmi
            import torch
            self.smi = amdsmi
            amdsmi.amdsmi_init()
            props = torch.cuda.get_device_properties(dev)
            want = (getattr(props, "pci_domain_id", 0), getattr(props, "pci_bus_id", None),
                    getattr(props, "pci_device_id", None))
            handles = amdsmi.amdsmi_get_processor_handles()
            for h in handles:
                bdf = amdsmi.amdsmi_get_gpu_device_bdf(h)  # "DDDD:BB:DD.F"
                dom, bus, df = bdf.split(":")
                if want[1] is not None and (int(dom, 16), int(bus, 16), int(df.split(".")[0], 16)) == want:
                    self.h, self.bdf = h, bdf
            if self.h is None and len(handles) == 1:
                self.h, self.bdf = handles[0], amdsmi.amdsmi_get_gpu_device_bdf(handles[0])
            if self.h is None:
                self.note = "no amdsmi GPU matches this device's PCI id %s" % (want,)
        except Exception as e:  # amdsmi absent or refusing: the line says so
            self.note = "amdsmi unavailable: %s" % e
        self.t = threading.Thread(target=self._run, daemon=True)
        if self.h is not None:
            self.t.start()

    def _read(self):
        p = self.smi.amdsmi_get_power_info(self.h)
        w = p.get("current_socket_power")
        if not isinstance(w, (int, float)) or w <= 0:
            w = p.get("average_socket_power")
        try:
            clk = self.smi.amdsmi_get_clock_info(self.h, self.smi.AmdSmiClkType.GFX).get("clk")
        except Exception:
            clk = None
        return (w if isinstance(w, (int, float)) and w > 0 else None,
                clk if isinstance(clk, (int, float)) and clk > 0 else None)

    def _run(self):
        while not self._stop.is_set():
            try:
                w, clk = self._read()
            except Exception as e:
                self.note = "amdsmi query failed: %s" % e
                return
            if w is not None and not self._stop.is_set():
                self.samples.append((time.perf_counter() - self.t0, w, clk))
            self._stop.wait(self.PERIOD_S)

    def stop(self, skip_s=0.0):
        """(summary, None) or (None, reason).  skip_s drops the samples of the first seconds (the
        socket power reading lags: a window that starts at an idle GPU first samples the ramp)."""
        self._stop.set()
        if self.h is not None:
            self.t.join(timeout=10)
        try:
            self.smi.amdsmi_shut_down()
        except Exception:
            pass
        kept = [(w, c) for t, w, c in self.samples if t >= skip_s]
        if len(kept) < self.MIN_SAMPLES:
            return None, {"samples": len(kept), "note": self.note or
                          "fewer than %d samples in the timed window" % self.MIN_SAMPLES}
        ps = sorted(p for p, _ in kept)
        cs = [c for _, c in kept if c]
        return {"samples": len(ps), "period_s": self.PERIOD_S, "socket_w_median": ps[len(ps) // 2],
                "socket_w_max": ps[-1], "gfx_mhz_mean": round(sum(cs) / len(cs)) if cs else None,
                "source": "amdsmi (in-process): current_socket_power, GFX clock", "gpu_bdf": self.bdf}, None


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_share():
    """(CPUs this process may run on, cgroup CPU quota in CPUs or None)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return aff, quota


def cpu_baseline(args, data, file_off, file_len, reps=5):
    """The reference's CPU path restated (oracle/bw_oracle.c FastCDC + index, with the crate's
    16-way SIMD BLAKE3 strategy, bw_oracle_simd.c), timed on this box's host cores: the median of
    `reps` runs on the cores this GPU's share of the node offers (16) and on one core.  Threading
    follows the reference: one task per file, serial within a file (dir_packer.rs:148-166); a
    single stream (C2) is cut into one file per thread for the multi-core figures, which moves
    the cuts of those files' heads but not the work per byte.  The whole node (os.cpu_count()
    threads, the reference's tokio pool on every core) is measured with --cpu-all-cores; by
    default it is estimated from the 16-core share, labelled as such, because a one-GPU box lends
    this process 16 cores and the rest belong to other jobs.  About 10-20 s of CPU time."""
    import numpy as np
    from oracle import oracle
    simd = oracle.set_blake3_simd(True)
    nproc = os.cpu_count() or 1
    threads = min(16, nproc)
    fo = np.asarray(file_off, dtype=np.uint64)
    fl = np.asarray(file_len, dtype=np.uint64)

    def timed(host, offs, lens, t):
        runs = []
        for _ in range(reps):
            t1 = time.perf_counter()
            r = oracle.process_files(host, offs, lens, threads=t)
            runs.append(time.perf_counter() - t1)
        m = float(np.sum(np.asarray(lens, dtype=np.uint64)))
        return m, sorted(runs)[len(runs) // 2], len(r)

    try:
        if args.workload == "c2":
            one = int(1 << 30)
            allc = int(min(args.cpu_sample_gib, 8.0) * (1 << 30))
            host = data[:max(one, allc)].cpu().numpy()
            m1, t1, b1 = timed(host, [0], [one], 1)
            per = allc // threads
            offs = np.arange(threads, dtype=np.uint64) * np.uint64(per)
            mA, tA, bA = timed(host, offs, np.full(threads, per, dtype=np.uint64), threads)
            sample = ("C2 stream: one core = its first 1 GiB as one file (%d blobs); 16 cores = its first %.0f GiB "
                      "cut into %d files of %.2f GiB, one per task (%d blobs)" % (b1, allc / 2**30, threads,
                                                                                 per / 2**30, bA))
            if args.cpu_all_cores:
                perN = allc // nproc
                offsN = np.arange(nproc, dtype=np.uint64) * np.uint64(perN)
                mN, tN, _ = timed(host, offsN, np.full(nproc, perN, dtype=np.uint64), nproc)
        else:
            cum = np.cumsum(fl)
            kA = max(1, int(np.searchsorted(cum, int(min(args.cpu_sample_gib, 8.0) * (1 << 30)))))
            k1 = max(1, int(np.searchsorted(cum, 1 << 30)))
            end = int(np.max(fo[:kA] + fl[:kA]))
            host = data[:end].cpu().numpy()
            m1, t1, b1 = timed(host, fo[:k1], fl[:k1], 1)
            mA, tA, bA = timed(host, fo[:kA], fl[:kA], threads)
            sample = ("first %d files (%.2f GB, %d blobs) on 16 cores, one file per task; first %d files "
                      "(%.2f GB) on one core" % (kA, mA / 1e9, bA, k1, m1 / 1e9))
            if getattr(args, "cpu_trees", False):
                # each file's Tree { File, "file_NNNNNNN.bin", Some(size), Some(mtime), Some(ctime),
                # [hash], None } in bincode (96 bytes, tools/dropin_c4.cpp's layout), hashed as one
                # blob per file on the same threads: the reference's second blake3::hash per file
                def trees(k):
                    t = np.zeros((k, 96), dtype=np.uint8)
                    t[:, 4] = 16  # name length (u64 LE)
                    names = np.frombuffer(b"".join(b"file_%07d.bin" % i for i in range(k)), np.uint8).reshape(k, 16)
                    t[:, 12:28] = names
                    for j, v in enumerate((fl[:k], 1700000000 + np.arange(k), 1700000000 + np.arange(k) // 2)):
                        t[:, 28 + 9 * j] = 1
                        t[:, 29 + 9 * j:37 + 9 * j] = np.asarray(v, np.uint64)[:, None].view(np.uint8)
                    t[:, 55] = 1  # one child; its 32 digest bytes follow at 63, next_sibling None at 95
                    return t.reshape(-1)
                for k, one_core in ((kA, False), (k1, True)):
                    tb = trees(k)
                    offs = np.arange(k, dtype=np.uint64) * np.uint64(96)
                    mt, tt, _ = timed(tb, offs, np.full(k, 96, np.uint64), 1 if one_core else threads)
                    if one_core:
                        t1 += tt
                    else:
                        tA += tt
                sample += "; plus each file's 96-byte Tree blob hashed (the per-file tree hash, dir_packer.rs:320)"
            if args.cpu_all_cores:
                mN, tN, _ = timed(host, fo[:kA], fl[:kA], nproc)
    finally:
        oracle.set_blake3_simd(False)
    share, one = mA / tA / 1e9, m1 / t1 / 1e9
    aff, quota = cpu_share()
    if args.cpu_all_cores:
        whole = {"value": round(mN / tN / 1e9, 3), "threads": nproc, "kind": "measured", "seconds": round(tN, 3)}
    else:
        # the share's per-core rate over every core of the node (parallel efficiency of 16 threads
        # kept; SMT siblings counted as cores, so this flatters the CPU)
        whole = {"value": round(share / threads * nproc, 3), "threads": nproc, "kind": "estimate",
                 "basis": "16-core share x nproc / 16 (not run: the box lends this process 16 cores; "
                          "bench.py --cpu-all-cores measures it on a node of your own)"}
    return {"value": round(share, 3), "unit": "GB/s", "cores": threads, "kind": "port",
            "scope": "this GPU's share of the node: 16 of nproc host cores (8 GPUs per node share them)",
            "sample": sample, "stat": "median of %d runs" % reps, "seconds": round(tA, 3),
            "one_core": {"value": round(one, 3), "seconds": round(t1, 3)},
            "whole_node": whole,
            "blake3": "16-way AVX-512 (the crate's hash_many strategy)" if simd else "scalar (no AVX-512 here)",
            "cpu_model": cpu_model(), "nproc": nproc, "affinity_cpus": aff, "cgroup_cpu_quota": quota}


def time_file_trees(ctx, res, file_len, reps):
    """The File tree of every file of the last batch (dir_packer.rs:237-274: name, size, mtime,
    children = the file's chunk hashes) through bw_tree_blobs -- bincode, BLAKE3 on the GPU and
    the dedup gate -- timed over `reps` fresh indexes; spot-checked against the oracle."""
    import numpy as np
    from backuwup_amd.context import TREE_DTYPE
    from oracle import oracle
    nf = len(file_len)
    fidx = res["file"].astype(np.int64)
    first = np.searchsorted(fidx, np.arange(nf))
    count = np.bincount(fidx, minlength=nf)
    names = np.frombuffer(b"".join(b"f%07d" % i for i in range(nf)), dtype=np.uint8)
    t = np.zeros(nf, dtype=TREE_DTYPE)
    t["kind"] = 0
    t["flags"] = 1 | 2  # size, mtime
    t["size"] = np.asarray(file_len, dtype=np.uint64)
    t["mtime"] = 1700000000 + np.arange(nf, dtype=np.uint64)
    t["name"] = names.ctypes.data + 8 * np.arange(nf, dtype=np.uint64)
    t["name_len"] = 8
    digests = np.ascontiguousarray(res["digest"])  # a file's chunk hashes, 32 B apart
    t["children"] = digests.ctypes.data + 32 * first.astype(np.uint64)
    t["n_children"] = count
    best = None
    for _ in range(max(1, reps)):
        ctx.index_reset(2 * nf + 1024)
        t0 = time.perf_counter()
        hashes, pieces = ctx.tree_blobs_array(t)
        el = time.perf_counter() - t0
        best = el if best is None else min(best, el)
    ok = True
    for i in np.random.default_rng(0).integers(0, nf, 16):
        ch = b"".join(bytes(d) for d in res["digest"][first[i]:first[i] + count[i]])
        want = oracle.split_serialize_tree(0, b"f%07d" % i, int(file_len[i]), 1700000000 + int(i), None, ch)
        ok = ok and bytes(hashes[i]) == want[0][1]
    return {"trees": nf, "pieces": int(len(pieces)), "ms": round(best * 1e3, 2),
            "trees_per_s": round(nf / best, 1), "bytes_serialized": int(pieces["length"].sum()),
            "bit_exact_sample": bool(ok)}


def unique_queue(res):
    """The blobs the packer would queue for the batch as the first of a session: the first
    occurrence of every digest, in canonical order.  (The bench's session index has seen the
    batch's data in earlier steps, so its own verdicts mark everything a duplicate.)"""
    import numpy as np
    d = np.ascontiguousarray(res["digest"]).view(np.dtype((np.void, 32))).ravel()
    _, first = np.unique(d, return_index=True)
    return res[np.sort(first)]


def time_seal(ctx, data, res, file_off, reps):
    """Seal every unique blob of the last batch in HBM (derive_backup_key(hash) + AES-256-GCM,
    pack.rs:70-80), as the packer would after compression; the blob bytes stand in for the zstd
    payload (synthetic data is incompressible, so level-3 zstd stores it raw).  Timed over `reps`
    calls with events on the context stream; spot-checked against the oracle."""
    import numpy as np
    import torch
    from oracle import oracle
    u = unique_queue(res)
    fo = np.asarray(file_off, dtype=np.uint64)
    src_off = fo[u["file"].astype(np.int64)] + u["offset"]
    lens = u["length"].astype(np.uint64)
    dst_off = np.concatenate([[0], np.cumsum(lens + 16)[:-1]]).astype(np.uint64)
    total = int(np.sum(lens + 16))
    dst = torch.empty(total, dtype=torch.uint8, device=data.device)
    nonces = np.random.default_rng(1).integers(0, 256, (len(u), 12), dtype=np.uint8)
    prk = bytes(range(32))
    ctx.seal_device(prk, data.data_ptr(), src_off, lens, u["digest"], nonces, dst.data_ptr(), dst_off)  # warm-up
    torch.cuda.synchronize()
    # the context runs on its own stream (torch's default stream is the null handle), so the
    # calls are bracketed by device-wide synchronizes and timed on the host clock
    t0 = time.perf_counter()
    for _ in range(max(1, reps)):
        ctx.seal_device(prk, data.data_ptr(), src_off, lens, u["digest"], nonces, dst.data_ptr(), dst_off)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / max(1, reps)
    ok = True
    for i in np.random.default_rng(2).integers(0, len(u), 4):
        pt = data[int(src_off[i]):int(src_off[i] + lens[i])].cpu().numpy()
        got = dst[int(dst_off[i]):int(dst_off[i] + lens[i]) + 16].cpu().numpy().tobytes()
        ok = ok and got == oracle.seal_blob(prk, bytes(u["digest"][i]), bytes(nonces[i]), pt)
    payload = int(np.sum(lens))
    return {"blobs": int(len(u)), "payload_bytes": payload, "ms": round(ms, 3),
            "GBps": round(payload / (ms * 1e-3) / 1e9, 1),
            "hbm_algorithmic_bytes": payload + total, "bit_exact_sample": bool(ok)}


def time_pack(ctx, data, res, file_off, reps):
    """write_packfiles over every unique blob of the last batch, from HBM to HBM (pack.rs:58-80,
    115-227): zstd store frames (synthetic data is incompressible, so these are the bytes level-3
    zstd emits), derive_backup_key + AES-256-GCM per blob and per header, the packfile layout.
    Timed over `reps` calls; one packfile is checked byte for byte against the format oracle and
    one blob read back through the oracle's get_blob + zstd store parse."""
    import numpy as np
    import torch
    from oracle import pack_oracle as po
    u = unique_queue(res)
    fo = np.asarray(file_off, dtype=np.uint64)
    src_off = fo[u["file"].astype(np.int64)] + u["offset"]
    lens = u["length"].astype(np.uint64)
    rng = np.random.default_rng(4)
    nonces = rng.integers(0, 256, (len(u), 12), dtype=np.uint8)
    kinds = np.zeros(len(u), dtype=np.uint8)
    plan, total = ctx.pack_plan(lens)
    ids = rng.integers(0, 256, (len(plan), 12), dtype=np.uint8)
    out = torch.empty(total, dtype=torch.uint8, device=data.device)
    prk = bytes(range(32))
    args = (prk, data.data_ptr(), src_off, lens, u["digest"], kinds, nonces, plan, ids, out.data_ptr())
    ctx.pack_build_device(*args)  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(max(1, reps)):
        ctx.pack_build_device(*args)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / max(1, reps)
    k = int(rng.integers(0, len(plan)))
    p = plan[k]
    blobs = []
    for i in range(int(p["first_blob"]), int(p["first_blob"] + p["n_blobs"])):
        pt = data[int(src_off[i]):int(src_off[i] + lens[i])].cpu().numpy().tobytes()
        blobs.append((bytes(u["digest"][i]), 0, bytes(nonces[i]),
                      po.seal_blob_payload(prk, u["digest"][i], nonces[i], po.zstd_store(pt))))
    got = out[int(p["offset"]):int(p["offset"] + p["size"])].cpu().numpy().tobytes()
    ok = got == po.serialize_packfile(prk, bytes(ids[k]), blobs)
    payload = int(np.sum(lens))
    return {"blobs": int(len(u)), "packfiles": int(len(plan)), "payload_bytes": payload,
            "packfile_bytes": int(total), "ms": round(ms, 3), "GBps": round(payload / (ms * 1e-3) / 1e9, 1),
            "bit_exact_packfile_sample": bool(ok)}


def time_pack_l3(ctx, data, res, file_off, reps):
    """The whole downstream chain of add_blob over every unique blob of the last batch, from HBM
    to HBM (pack.rs:58-80, 115-227): level-3 zstd on the GPU (bw_pack_compress_device, the real
    compressor's decisions, not store frames), write_packfiles' grouping over the frame sizes on
    the host, sealing + packfile layout (bw_pack_build_compressed).  One packfile is checked byte
    for byte against the oracle chain (zstd restatement -> seal -> serialize)."""
    import numpy as np
    import torch
    from oracle import oracle as orc
    from oracle import pack_oracle as po
    u = unique_queue(res)
    fo = np.asarray(file_off, dtype=np.uint64)
    src_off = fo[u["file"].astype(np.int64)] + u["offset"]
    lens = u["length"].astype(np.uint64)
    rng = np.random.default_rng(5)
    nonces = rng.integers(0, 256, (len(u), 12), dtype=np.uint8)
    kinds = np.zeros(len(u), dtype=np.uint8)
    prk = bytes(range(32))
    out = None

    def once():
        nonlocal out
        fl = ctx.pack_compress_device(data.data_ptr(), src_off, lens)
        plan, total = ctx.pack_plan(fl, flags=0)
        ids = np.random.default_rng(6).integers(0, 256, (len(plan), 12), dtype=np.uint8)
        if out is None or out.numel() < total:
            out = torch.empty(total, dtype=torch.uint8, device=data.device)
        ctx.pack_build_compressed(prk, u["digest"], kinds, nonces, plan, ids, out.data_ptr())
        return fl, plan, total, ids

    once()  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(max(1, reps)):
        fl, plan, total, ids = once()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / max(1, reps)
    k = int(rng.integers(0, len(plan)))
    p = plan[k]
    blobs = []
    for i in range(int(p["first_blob"]), int(p["first_blob"] + p["n_blobs"])):
        pt = data[int(src_off[i]):int(src_off[i] + lens[i])].cpu().numpy().tobytes()
        blobs.append((bytes(u["digest"][i]), 0, bytes(nonces[i]),
                      po.seal_blob_payload(prk, u["digest"][i], nonces[i], orc.zstd3_compress(pt))))
    got = out[int(p["offset"]):int(p["offset"] + p["size"])].cpu().numpy().tobytes()
    ok = got == po.serialize_packfile(prk, bytes(ids[k]), blobs)
    payload = int(np.sum(lens))
    return {"blobs": int(len(u)), "packfiles": int(len(plan)), "payload_bytes": payload,
            "frame_bytes": int(np.sum(fl)), "packfile_bytes": int(total), "ms": round(ms, 3),
            "GBps": round(payload / (ms * 1e-3) / 1e9, 1), "bit_exact_packfile_sample": bool(ok)}


def pmc_traffic(args, kernel):
    """(HBM bytes per launch of `kernel`, provenance) from the committed PMC summary of the same
    workload (tools/pmc_traffic.py: FETCH_SIZE x2 + WRITE_SIZE, gfx950 corrections).  The bytes
    are reported only when the summary was measured on these kernel sources (its source digest
    equals this tree's); otherwise None and the provenance says why."""
    from backuwup_amd.build import source_digest
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if args.workload != "c2" or args.host_stream or not os.path.exists(path):
        return None, None, None
    try:
        pmc = json.load(open(path))
    except (OSError, ValueError):
        return None, {"file": "profiles/pmc_traffic.json", "status": "unreadable"}, None
    prov = {"file": "profiles/pmc_traffic.json", "commit": pmc.get("commit"),
            "source_digest": pmc.get("source_digest")}
    if pmc.get("source_digest") != source_digest():
        prov["status"] = "stale: measured on other kernel sources"
        return None, prov, None
    if pmc.get("gib") != args.gib or kernel not in pmc.get("kernels", {}):
        prov["status"] = "no entry for this workload/kernel"
        return None, prov, None
    prov["status"] = "measured on this tree's kernels"
    # every kernel of the measured batch launches once per batch: their sum is the batch's traffic
    path_bytes = sum(v["hbm_bytes_per_launch"] for k, v in pmc["kernels"].items()
                     if k not in ("k_table_clear", "k_b3_calib"))  # session setup / calibration, not the batch
    return pmc["kernels"][kernel]["hbm_bytes_per_launch"], prov, round(path_bytes / (args.gib * (1 << 30)), 3)


def whole_result_fixture(args, rank):
    """The committed oracle fixture of this rank's whole first batch, if one exists for exactly this
    workload (tests/golden/c{1..5}_full.json: bench.py's rank-0 corpora at their default sizes; rank 0's
    verdicts at N > 1 are the same: files are sharded rank-major, so rank 0's come first)."""
    name = args.workload
    path = os.path.join(ROOT, "tests", "golden", "%s_full.json" % name)
    if rank != 0 or not os.path.exists(path):
        return None, path
    fx = json.load(open(path))
    same = {"c1": args.gib * (1 << 30) == fx.get("total_bytes"),
            "c2": args.gib * (1 << 30) == fx.get("bytes"),
            "c3": args.gib * (1 << 30) == fx.get("base_bytes"),
            "c4": args.files == fx.get("files"),
            "c5": args.gib * (1 << 30) == fx.get("base_bytes")}.get(name, False)
    return (fx if same else None), path


def parity_spot_check(args, ctx, data, file_off, file_len, rank, first=None):
    """Bit-exactness of the session's first batch (fresh index).  WHOLE result: where the oracle's
    fixture of this exact corpus is committed (C2 16 GiB, C3 4 GiB x 16, C4 1 M files; rank 0), the
    sha256 over every blob's (file, offset, length, gear_hash, digest, is_dup) must equal it (C1 and C5
    too).  Plus a
    live oracle run here: the first ~64 MiB of blobs (C2) or a sample of files (other workloads)."""
    from backuwup_amd import synth
    out = {}
    res = first if first is not None else ctx.results()
    fx, path = whole_result_fixture(args, rank)
    if fx is not None and first is not None:
        have = synth.result_digest(res)
        keys = ("blobs", "dup_blobs", "bytes", "dup_bytes", "sha256_digests", "sha256_records")
        ok = all(have[k] == fx[k] for k in keys)
        out["whole_result_detail"] = {
            "bit_exact": ok, "fixture": os.path.relpath(path, ROOT), "blobs": have["blobs"],
            "dup_blobs": have["dup_blobs"], "sha256_records": have["sha256_records"],
            "scope": "every blob of the first batch against the oracle's fixture of the same corpus"}
    spot = spot_check(args.workload, res, data, file_off, file_len, rank)
    out.update(spot)
    whole = out.get("whole_result_detail")
    # true only when the whole first batch was compared and equal; false when no fixture applies
    out["whole_result"] = bool(whole and whole["bit_exact"])
    out["bit_exact"] = bool(spot["bit_exact"] and (whole is None or whole["bit_exact"]))
    return out


def spot_check(workload, res, data, file_off, file_len, rank):
    """The oracle run live on the first ~64 MiB of blobs (C2) or on a sample of files."""
    import numpy as np
    from oracle import oracle
    if workload == "c2":
        n = int(file_len[0])
        ends = np.cumsum(res["length"].astype(np.int64))
        assert int(ends[-1]) == n and int(res["offset"][0]) == 0
        k = int(np.searchsorted(ends, 64 << 20)) + 1
        upto = int(ends[k - 1])
        host = data[:upto + (4 << 20)].cpu().numpy()
        want = oracle.fastcdc(host, 262144, 1048576, 3145728)
        ok = all(want[i][1] == int(res["offset"][i]) and want[i][2] == int(res["length"][i]) and
                 want[i][0] == int(res["gear_hash"][i]) for i in range(k - 1))
        ok = ok and all(oracle.blake3(host[int(res["offset"][i]):int(res["offset"][i] + res["length"][i])]) ==
                        bytes(res["digest"][i]) for i in range(k - 1))
        return {"chunks_checked": k - 1, "bytes_checked": int(ends[k - 2]), "bit_exact": bool(ok)}
    # sample files: each file's blobs re-derived by the oracle (chunking + digests; dedup verdicts
    # need the whole batch and are covered by tests/test_gpu_configs.py)
    rng = np.random.default_rng(rank)
    nf = len(file_len)
    pick = sorted(set(rng.integers(0, nf, min(nf, 64)).tolist()))
    fo = np.asarray(file_off, dtype=np.uint64)
    fl = np.asarray(file_len, dtype=np.uint64)
    ok, nb, nbytes = True, 0, 0
    for f in pick:
        got = res[res["file"] == f]
        if int(fl[f]) > (256 << 20):
            # a large file: its blobs up to 64 MiB, from the file start (CDC restarts per file)
            ends = np.cumsum(got["length"].astype(np.int64))
            k = int(np.searchsorted(ends, 64 << 20)) + 1
            host = data[int(fo[f]):int(fo[f]) + int(ends[k - 1]) + (4 << 20)].cpu().numpy()
            want = oracle.fastcdc(host, 262144, 1048576, 3145728)[:k - 1]
            got = got[:k - 1]
            ok = ok and [(int(g["gear_hash"]), int(g["offset"]), int(g["length"])) for g in got] == want and \
                all(oracle.blake3(host[int(g["offset"]):int(g["offset"] + g["length"])]) == bytes(g["digest"])
                    for g in got)
            nbytes += int(ends[k - 2])
        else:
            host = data[int(fo[f]):int(fo[f] + fl[f])].cpu().numpy()
            want = oracle.process_files(host, [0], [int(fl[f])])
            ok = ok and len(got) == len(want) and np.array_equal(got["length"], want["length"]) and \
                np.array_equal(got["digest"], want["digest"]) and np.array_equal(got["gear_hash"], want["gear_hash"])
            nbytes += int(fl[f])
        nb += len(got)
    return {"files_checked": len(pick), "blobs_checked": nb, "bytes_checked": nbytes, "bit_exact": bool(ok)}


if __name__ == "__main__":
    main()
