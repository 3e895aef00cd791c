"""Summarise a tools/gpu_abv.sh run: bench value and isolated stage times per library variant
(mean over rounds), and FETCH_SIZE per launch of k_scan / k_b3_groups relative to the input."""
import collections
import csv
import glob
import json
import os
import re
import sys

out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
rows = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(out, "*bench_*_[0-9].log"))):
    m = re.match(r"(.*)bench_(.+)_(\d+)\.log", os.path.basename(f))
    tag, var = m.group(1), m.group(2)
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            iso = d["roofline"].get("isolated", {}).get("stage_ms_per_step") or d["roofline"]["stage_ms_per_step"]
            rows[(tag, var)].append((d["value"], d["ms_per_step"], iso, d["config"]["bytes_per_gpu"]))
for (tag, var), rs in rows.items():
    v = sum(r[0] for r in rs) / len(rs)
    st = {k: round(sum(r[2][k] for r in rs) / len(rs), 3) for k in rs[0][2]}
    print("%-6s %-10s %8.1f GB/s  (%s)  isolated %s" % (tag or "c2", var, v, " ".join("%.0f" % r[0] for r in rs), st))
for f in sorted(glob.glob(os.path.join(out, "*pmc_*/**/*counter_collection.csv"), recursive=True)):
    var = f[len(out) + 1:].split("/")[0]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == "FETCH_SIZE":
            acc[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    nbytes = rows[("", "base")][0][3] if ("", "base") in rows else 16 << 30
    for k, vv in acc.items():
        if "k_scan" in k or "k_b3_groups" in k:
            print("%-16s %-40s n=%d fetch x%.3f" % (var, k.replace("void ", ""), len(vv), sum(vv) / len(vv) * 2048 / nbytes))
