#!/usr/bin/env python3
"""what limits the overlap of the gear scan and the BLAKE3 leaf pass on C2.

Runs bench.py's C2 pipeline -- one 16 GiB splitmix64 stream, consecutive batches alternating between
two contexts on two streams, one shared index -- on the clock-stamp library
(libbackuwup_amd_clock.so: `python backuwup_amd/build.py --clock`), whose k_scan stamps every 128 KiB
tile (one in 16) and whose k_b3_lines stamps every wave (of one workgroup in 4) with the 100 MHz
real-time counter (s_memrealtime) and the shader clock counter (s_memtime); stamping every unit put
one global atomic per 128 KiB tile into the scan and slowed its tiles 2.5x.  Socket power and the GFX clock are sampled through amdsmi
(bench.PowerSampler) over the whole timed run (>= 3 s); the stamps cover a window of steps inside it.

From the stamps, on the chip's own clock:
  * the timeline split into both passes running / the scan alone / the leaf pass alone / neither
    (unions of the stamped intervals of each kind);
  * the shader clock inside each class: sum of shader cycles / sum of real time over the work units
    that lie (>= 90 %) inside it;
  * each pass's rate (bytes of its stamped units per second of the class) alone and beside the other:
    if the two rates beside each other, as fractions of the rates alone, add up to ~1, running them
    together buys nothing (the chip delivers the same work either way); the clock says whether it is
    the clock that gives way.
Prints one JSON object (stdout) and writes it to --out.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("BW_LIB", os.path.join(ROOT, "backuwup_amd", "libbackuwup_amd_clock.so"))

REC = None  # numpy dtype, set in main


def union(iv):
    """iv: (n, 2) sorted by start -> the merged, disjoint intervals (m, 2)."""
    import numpy as np
    if not len(iv):
        return np.zeros((0, 2))
    s, e = iv[:, 0], np.maximum.accumulate(iv[:, 1])
    new = np.ones(len(s), dtype=bool)
    new[1:] = s[1:] > e[:-1]  # a gap before this interval: a new merged one starts
    first = np.nonzero(new)[0]
    last = np.append(first[1:] - 1, len(s) - 1)
    return np.stack([s[first], e[last]], 1)


def intersect(A, B):
    import numpy as np
    out, i, j = [], 0, 0
    while i < len(A) and j < len(B):
        s, e = max(A[i][0], B[j][0]), min(A[i][1], B[j][1])
        if s < e:
            out.append((s, e))
        if A[i][1] < B[j][1]:
            i += 1
        else:
            j += 1
    return np.array(out, dtype=np.float64).reshape(-1, 2)


def covered(iv, U):
    """per interval of iv, the length of its intersection with the union U (sorted, disjoint)."""
    import numpy as np
    if not len(U):
        return np.zeros(len(iv))
    lens = U[:, 1] - U[:, 0]
    cum = np.concatenate([[0.0], np.cumsum(lens)])

    def F(x):  # length of U up to x
        j = np.searchsorted(U[:, 0], x, side="right") - 1
        jj = np.maximum(j, 0)
        part = np.clip(x - U[jj, 0], 0.0, lens[jj])
        return np.where(j >= 0, cum[jj] + part, 0.0)

    return F(iv[:, 1]) - F(iv[:, 0])


def main():
    import numpy as np
    import torch
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=400, help="timed steps (~9 ms each: >= 3 s of power samples)")
    ap.add_argument("--window", type=int, default=24, help="steps in the middle of the run that are stamped")
    ap.add_argument("--gib", type=float, default=16.0)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "clock_windows.json"))
    args = ap.parse_args()
    from backuwup_amd import Context, Index, _lib, make_params, synth
    from bench import PowerSampler
    L = _lib.load()
    L.bw_clock_log.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_int]
    L.bw_clock_log.restype = ctypes.c_int
    L.bw_clock_log_read.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]
    L.bw_clock_log_read.restype = ctypes.c_int
    rec = np.dtype([("kind", "<u4"), ("pad", "<u4"), ("t0", "<u8"), ("t1", "<u8"), ("c0", "<u8"), ("c1", "<u8")])
    dev = torch.device("cuda", 0)
    n = int(args.gib * (1 << 30))
    data = synth.splitmix_torch(42, n, dev)
    torch.cuda.synchronize()
    # a scan record stands for 16 tiles of 128 KiB (one tile in 16 is stamped: C2 >= 4 GiB), a leaf
    # record for 4 waves of 64 4-leaf groups (the waves of one block in 4)
    tile, wave_bytes = 16 * (128 << 10), 4 * 64 * 4096
    cap = args.window * (n // tile + n // wave_bytes + 4096) * 2 + (1 << 20)
    _lib.check(L.bw_clock_log(0, cap, 0))
    index = Index(0)
    ctxs = []
    for _ in range(2):
        c = Context(0)
        c.set_stream(torch.cuda.Stream(dev).cuda_stream)
        c.attach_index(index)
        ctxs.append(c)
    params = make_params()
    max_blobs = n // (256 << 10) + 2
    ctxs[0].index_reset((args.steps + 8) * max_blobs + 1024)
    inflight, k = [], [0]

    def step():
        c = ctxs[k[0] % 2]
        k[0] += 1
        t = c.submit_device(data.data_ptr(), n, [0], [n], params)
        inflight.append((c, t))
        if len(inflight) >= 2:
            c0, t0 = inflight.pop(0)
            c0.wait(t0)

    for _ in range(4):
        step()
    torch.cuda.synchronize()
    lo = (args.steps - args.window) // 2
    sampler = PowerSampler(0)
    t_start = time.perf_counter()
    t_w0 = t_w1 = None
    for s in range(args.steps):
        if s == lo:
            _lib.check(L.bw_clock_log(0, cap, 1))  # synchronizes: a short gap in the pipeline
            t_w0 = time.perf_counter()
        if s == lo + args.window:
            t_w1 = time.perf_counter()
            _lib.check(L.bw_clock_log(0, cap, 0))
        step()
    while inflight:
        c0, t0 = inflight.pop(0)
        c0.wait(t0)
    torch.cuda.synchronize()
    el = time.perf_counter() - t_start
    power, missing = sampler.stop()
    nrec = ctypes.c_uint64()
    buf = np.zeros(cap, dtype=rec)
    _lib.check(L.bw_clock_log_read(buf.ctypes.data, cap, ctypes.byref(nrec)))
    r = buf[:min(nrec.value, cap)]
    # the 100 MHz counter in microseconds
    t0 = r["t0"].astype(np.float64) / 100.0
    t1 = r["t1"].astype(np.float64) / 100.0
    cyc = (r["c1"] - r["c0"]).astype(np.float64)
    base = t0.min()
    t0 -= base
    t1 -= base
    dur = t1 - t0
    out = {"steps": args.steps, "ms_per_step": round(el / args.steps * 1e3, 3),
           "gbs": round(n * args.steps / el / 1e9, 1), "stamped_steps": args.window,
           "records": int(len(r)), "dropped": int(max(0, nrec.value - cap)),
           "power": power, "power_missing": missing}
    kinds = {}
    for kind, name in ((0, "scan"), (1, "leaf")):
        m = r["kind"] == kind
        iv = np.stack([t0[m], t1[m]], 1)
        iv = iv[np.argsort(iv[:, 0])]
        kinds[name] = (m, union(iv))
    Us, Ul = kinds["scan"][1], kinds["leaf"][1]
    both = intersect(Us, Ul)
    span = max(t1.max(), 1e-9)
    tot = lambda U: float((U[:, 1] - U[:, 0]).sum()) if len(U) else 0.0
    t_scan, t_leaf, t_both = tot(Us), tot(Ul), tot(both)
    out["timeline_us"] = {"span": round(span, 1), "both": round(t_both, 1), "scan_only": round(t_scan - t_both, 1),
                          "leaf_only": round(t_leaf - t_both, 1), "neither": round(span - t_scan - t_leaf + t_both, 1)}
    out["timeline_frac"] = {k: round(v / span, 4) for k, v in out["timeline_us"].items() if k != "span"}
    classes = {}
    for name, (m, U) in kinds.items():
        iv = np.stack([t0[m], t1[m]], 1)
        fb = covered(iv, both) / np.maximum(dur[m], 1e-9)
        unit = tile if name == "scan" else wave_bytes
        for cls, sel in (("beside_other", fb >= 0.9), ("alone", fb <= 0.1)):
            d, c = dur[m][sel], cyc[m][sel]
            ghz = float(c.sum() / d.sum() / 1e3) if d.sum() > 0 else None
            # the pass's rate in this class: its units there, over the class's time
            cls_time = t_both if cls == "beside_other" else (tot(U) - t_both)
            rate = float(sel.sum() * unit / (cls_time * 1e-6) / 1e9) if cls_time > 0 else None
            classes["%s_%s" % (name, cls)] = {"units": int(sel.sum()), "shader_ghz": round(ghz, 3) if ghz else None,
                                              "unit_us_mean": round(float(d.mean()), 2) if len(d) else None,
                                              "rate_gbs": round(rate, 1) if rate else None}
    out["classes"] = classes
    sa, sb = classes["scan_alone"]["rate_gbs"], classes["scan_beside_other"]["rate_gbs"]
    la, lb = classes["leaf_alone"]["rate_gbs"], classes["leaf_beside_other"]["rate_gbs"]
    if sa and sb and la and lb:
        out["overlap_sum_of_fractions"] = round(sb / sa + lb / la, 3)
    print(json.dumps(out), flush=True)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    for c in ctxs:
        c.close()
    index.close()


if __name__ == "__main__":
    main()
