"""Split a rocprofv3 kernel trace of `bench.py` into its phases for one kernel: warm-up launches,
the timed launches (two batches in flight, sharing the GPU) and the isolated launches that
follow (one context, synchronized).  Usage: trace_split.py run_kernel_trace.csv k_b3_groups W K"""
import csv
import json
import sys


def main():
    path, kernel, warm, steps = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    rows = [r for r in csv.DictReader(open(path)) if kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    out = {"kernel": kernel, "launches": len(dur)}
    phases = {"warmup": dur[:warm], "timed": dur[warm:warm + steps], "after_timed": dur[warm + steps:]}
    for k, v in phases.items():
        if v:
            out[k] = {"n": len(v), "mean_ms": round(sum(v) / len(v), 4), "min_ms": round(min(v), 4)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
