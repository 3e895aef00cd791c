"""Split a rocprofv3 kernel trace of `bench.py` into its phases for one kernel: warm-up launches,
the timed launches (two batches in flight, sharing the GPU) and the isolated launches that
follow (one context, synchronized).  Usage:
    trace_split.py run_kernel_trace.csv k_b3_lines W K [bytes_per_launch]
For the timed launches it also gives the union of their intervals per step (the kernel's active
time per step: two contexts' launches overlap each other, so the mean duration can exceed the step
time), and with bytes_per_launch the achieved GB/s on that union and its fraction of the 8 TB/s
HBM peak -- the figures the bench line's roofline.achieved / frac come from (bench.py reads the
same union from the library's events)."""
import csv
import json
import sys

HBM_PEAK_GBS = 8000.0


def union_ms(iv):
    tot, cur = 0, None
    for a, z in sorted(iv):
        if cur is None or a > cur[1]:
            if cur is not None:
                tot += cur[1] - cur[0]
            cur = [a, z]
        else:
            cur[1] = max(cur[1], z)
    if cur is not None:
        tot += cur[1] - cur[0]
    return tot / 1e6


def main():
    path, kernel, warm, steps = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    nbytes = float(sys.argv[5]) if len(sys.argv) > 5 else None
    rows = [r for r in csv.DictReader(open(path)) if kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    dur = [(z - a) / 1e6 for a, z in iv]
    out = {"kernel": kernel, "launches": len(dur)}
    phases = {"warmup": dur[:warm], "timed": dur[warm:warm + steps], "after_timed": dur[warm + steps:]}
    for k, v in phases.items():
        if v:
            out[k] = {"n": len(v), "mean_ms": round(sum(v) / len(v), 4), "min_ms": round(min(v), 4)}
    timed = iv[warm:warm + steps]
    if timed:
        act = union_ms(timed) / len(timed)
        out["timed"]["active_ms_per_step"] = round(act, 4)
        out["timed"]["window_ms_per_step"] = round((max(z for _, z in timed) - min(a for a, _ in timed)) / 1e6 / len(timed), 4)
        if nbytes:
            out["timed"]["achieved_gbs"] = round(nbytes / (act * 1e-3) / 1e9, 1)
            out["timed"]["frac"] = round(nbytes / (act * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    if nbytes and phases["after_timed"]:
        m = sum(phases["after_timed"]) / len(phases["after_timed"])
        out["after_timed"]["achieved_gbs"] = round(nbytes / (m * 1e-3) / 1e9, 1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
