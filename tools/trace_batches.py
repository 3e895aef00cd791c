"""Per-batch timeline of a single-stream run (e.g. `bench.py --workload c1 --streams 1`) from a
rocprofv3 kernel trace: batches start at each k_scan launch.  For the timed batches it reports the
mean batch period (scan start to next scan start), the busy time (union of the batch's kernels),
the idle gap inside the batch and between batches, and the mean duration and count of every kernel
per batch, so the fixed costs a single batch in flight cannot hide are visible by name.

Usage: trace_batches.py run_kernel_trace.csv [skip_batches] [out.json] [scans_per_batch]
(scans_per_batch = 2 for batches split into a head and a tail part, BW_OPT_SPLIT)"""
import collections
import csv
import json
import sys


def main():
    path = sys.argv[1]
    skip = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ks = [(r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0].split("::")[-1],
           int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if "bw::" in r["Kernel_Name"]]
    per_batch = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    starts = [s for n, s, e in ks if n == "k_scan"][::per_batch]
    if len(starts) < skip + 3:
        raise SystemExit("too few batches in the trace")
    starts = starts[skip:-1]
    per = collections.defaultdict(list)
    periods, busy, inner_gap = [], [], []
    for a, b in zip(starts, starts[1:]):
        batch = [(n, s, e) for n, s, e in ks if a <= s < b]
        periods.append(b - a)
        iv, u = sorted((s, e) for _, s, e in batch), []
        for s, e in iv:
            if u and s <= u[-1][1]:
                u[-1][1] = max(u[-1][1], e)
            else:
                u.append([s, e])
        busy.append(sum(e - s for s, e in u))
        inner_gap.append((u[-1][1] - u[0][0]) - busy[-1])
        c = collections.defaultdict(lambda: [0, 0])
        for n, s, e in batch:
            c[n][0] += 1
            c[n][1] += e - s
        for n, (cnt, t) in c.items():
            per[n].append((cnt, t))
    nb = len(periods)
    mean = lambda v: sum(v) / len(v) / 1e3  # ns -> us
    out = {"batches": nb, "period_us": round(mean(periods), 2), "busy_us": round(mean(busy), 2),
           "idle_inside_batch_us": round(mean(inner_gap), 2),
           "idle_between_batches_us": round(mean(periods) - mean(busy) - mean(inner_gap), 2),
           "kernels": {n: {"launches_per_batch": round(sum(c for c, _ in v) / nb, 2),
                           "us_per_batch": round(sum(t for _, t in v) / nb / 1e3, 2)}
                       for n, v in sorted(per.items(), key=lambda kv: -sum(t for _, t in kv[1]))}}
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 3:
        json.dump(out, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
