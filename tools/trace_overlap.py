"""Occupancy of the GPU timeline by the hot path's kernels in a rocprofv3 kernel trace of
`bench.py` (C2, two batches in flight): over the timed launches of k_scan, the fraction of the
wall time during which a scan runs, a BLAKE3 leaf pass runs, both run at once (the overlap the
two-stream design relies on), and no kernel of the path runs at all (bubbles).

Usage: trace_overlap.py run_kernel_trace.csv WARMUP STEPS [out.json]
The timed window is [start of the first timed k_scan, end of the last timed k_b3_groups]."""
import csv
import json
import sys


def intervals(rows, name):
    return sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if name in r["Kernel_Name"])


def union(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def clip(iv, lo, hi):
    return [(max(s, lo), min(e, hi)) for s, e in iv if e > lo and s < hi]


def length(iv):
    return sum(e - s for s, e in iv)


def intersect(a, b):
    out, i, j = [], 0, 0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if s < e:
            out.append((s, e))
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return out


def main():
    path, warm, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    rows = list(csv.DictReader(open(path)))
    rows = [r for r in rows if "bw::" in r["Kernel_Name"]]
    leaf = "k_b3_lines" if any("k_b3_lines" in r["Kernel_Name"] for r in rows) else "k_b3_groups"
    scans, b3 = intervals(rows, "k_scan"), intervals(rows, leaf)
    lo, hi = scans[warm][0], b3[warm + steps - 1][1]
    span = hi - lo
    us = union(clip(scans, lo, hi))
    ub = union(clip(b3, lo, hi))
    anyk = union(clip([(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows], lo, hi))
    both = intersect(us, ub)
    res = {
        "window_ms": round(span / 1e6, 3), "steps": steps, "ms_per_step": round(span / 1e6 / steps, 4),
        "scan_active_frac": round(length(us) / span, 4), "b3_leaf_active_frac": round(length(ub) / span, 4),
        "scan_and_b3_concurrent_frac": round(length(both) / span, 4),
        "no_hot_path_kernel_frac": round(1 - length(anyk) / span, 4),
        "scan_mean_ms": round(sum(e - s for s, e in scans[warm:warm + steps]) / steps / 1e6, 4),
        "b3_leaf_mean_ms": round(sum(e - s for s, e in b3[warm:warm + steps]) / steps / 1e6, 4),
    }
    print(json.dumps(res, indent=1))
    if len(sys.argv) > 4:
        json.dump(res, open(sys.argv[4], "w"), indent=1)


if __name__ == "__main__":
    main()
