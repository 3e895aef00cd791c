#!/usr/bin/env python3
"""Benchmark: GB/s chunked + hashed + deduped (BASELINE.json metric) on configuration C2.

C2 = a single 16 GiB random stream, device-resident (BASELINE.json configs[1]).  One step = one
pass of the hot path over the stream: FastCDC-v2020 (256 KiB / 1 MiB / 3 MiB) -> BLAKE3 of every
chunk -> seen-chunk index (fresh index per step: one backup session).  Inputs are generated on
the GPU (counter-based splitmix64, seed 42 + rank) before timing, so the timed region starts
with the bytes resident in HBM.

N GPUs (weak scaling): every rank owns its own 16 GiB stream; the index is partitioned by digest
prefix and each step exchanges digests with one RCCL all-to-all (and verdicts back).

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


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--gib", type=float, default=16.0, help="stream size per GPU (GiB)")
    ap.add_argument("--cpu-sample-gib", type=float, default=4.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--streams", type=int, default=1,
                    help="batches in flight: consecutive steps alternate between this many contexts/streams")
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    from backuwup_amd import Context, make_params
    from backuwup_amd._lib import BW_F_NO_DEDUP, STAGES
    from backuwup_amd.synth import splitmix_torch

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    n = int(args.gib * (1 << 30))
    t0 = time.time()
    data = splitmix_torch(42 + rank, n, dev)
    torch.cuda.synchronize()
    log("rank %d: generated %.1f GiB in %.1f s" % (rank, n / 2**30, time.time() - t0))

    ctxs, streams = [], []
    for k in range(max(1, args.streams)):
        c = Context(local)
        st = torch.cuda.current_stream(dev) if k == 0 else torch.cuda.Stream(dev)
        c.set_stream(st.cuda_stream)
        ctxs.append(c)
        streams.append(st)
    ctx = ctxs[0]
    stream = streams[0]
    flags = BW_F_NO_DEDUP if world > 1 else 0
    params = make_params(flags=flags)
    index_hint = 2 * (n // (256 << 10)) + 1024
    owner_bits = world.bit_length() - 1
    assert world == 1 << owner_bits, "world size must be a power of two (digest-prefix owners)"

    from backuwup_amd.sharded import DeviceShardOps, exchange_dedup
    step_no = [0]

    def step():
        k = step_no[0] % len(ctxs)
        step_no[0] += 1
        c = ctxs[k]
        with torch.cuda.stream(streams[k]):
            c.index_reset(index_hint)
            c.submit_device(data.data_ptr(), n, [0], [n], params)
            if world > 1:
                # digest all-to-all by owner = digest[0] >> (8 - log2 N); verdicts come back
                nb, d_dig, d_dup = c.device_views()
                exchange_dedup(DeviceShardOps(c, dev), d_dig, nb, d_dup, world, dev)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    check = None
    if not args.no_check:
        # bit-exactness spot check against the CPU oracle on the first 64 MiB of chunks
        from oracle import oracle
        res = ctx.results()
        ends = np.cumsum(res["length"].astype(np.int64))
        assert int(ends[-1]) == n and int(res["offset"][0]) == 0
        k = int(np.searchsorted(ends, 64 << 20)) + 1
        upto = int(ends[k - 1])
        host = data[:upto + (4 << 20)].cpu().numpy()
        want = oracle.fastcdc(host[:upto + (4 << 20)], 262144, 1048576, 3145728)
        ok = all(want[i][1] == int(res["offset"][i]) and want[i][2] == int(res["length"][i]) and
                 want[i][0] == int(res["gear_hash"][i]) for i in range(k - 1))
        ok = ok and all(oracle.blake3(host[int(res["offset"][i]):int(res["offset"][i] + res["length"][i])]) ==
                        bytes(res["digest"][i]) for i in range(k - 1))
        check = {"chunks_checked": k - 1, "bytes_checked": int(ends[k - 2]), "bit_exact": bool(ok)}
        log("rank %d: parity spot check %s" % (rank, check))
        if not ok:
            raise SystemExit("parity check failed")

    for c in ctxs:
        c.profile_enable(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    stage_ms, nbatch = ctx.profile_read()
    per = {s: stage_ms[s] / max(nbatch, 1) for s in STAGES}
    res = ctx.results()
    log("rank %d: %d blobs/step, stage ms/step: %s" % (rank, len(res), {k: round(v, 3) for k, v in per.items()}))

    total_bytes = n * world * args.steps
    value = total_bytes / el / 1e9
    ms_per_step = el / args.steps * 1e3

    # roofline for the dominant kernel (largest stage time); algorithmic traffic = every input byte
    # read once per launch, so bytes per launch = n
    dom = max(["scan", "b3_leaf"], key=lambda s: per[s])
    achieved = n / (per[dom] * 1e-3) / 1e9
    kernel = {"scan": "k_scan", "b3_leaf": "k_b3_groups"}[dom]
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc_path):
        try:
            pmc = json.load(open(pmc_path))
            if pmc.get("gib") == args.gib and kernel in pmc.get("kernels", {}):
                traffic = pmc["kernels"][kernel]["hbm_bytes_per_launch"]
        except Exception:
            traffic = None
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": kernel,
                "algorithmic_bytes_per_launch": n,
                "stage_ms_per_step": {k: round(v, 3) for k, v in per.items()}}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import oracle
        m = int(args.cpu_sample_gib * (1 << 30))
        host = data[:m].cpu().numpy()
        t1 = time.perf_counter()
        r = oracle.process_files(host, [0], [m], threads=1)
        ct = time.perf_counter() - t1
        cpu = {"value": round(m / ct / 1e9, 4), "unit": "GB/s", "cores": 1, "kind": "port",
               "sample": "first %.0f GiB of the C2 stream as one file (%d blobs), oracle/bw_oracle.c "
                         "FastCDC+BLAKE3+index, serial within a file like the reference" % (args.cpu_sample_gib, len(r)),
               "seconds": round(ct, 2)}

    if rank == 0:
        line = {"metric": METRIC, "value": round(value, 3), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
                "config": {"workload": "C2: single %.0f GiB splitmix64 stream per GPU (seed 42+rank), "
                                       "device-resident; FastCDC v2020 256K/1M/3M -> BLAKE3 -> index" % args.gib,
                           "bytes_per_gpu": n, "blobs_per_gpu": int(len(res)),
                           "parallelism": "dp%d (files sharded, index by digest prefix)" % world,
                           "batches_in_flight": len(ctxs)},
                "roofline": roofline, "cpu_baseline": cpu, "parity": check}
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
