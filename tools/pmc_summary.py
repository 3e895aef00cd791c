#!/usr/bin/env python3
"""Summarise rocprofv3 counter CSVs (gpurun_out/pmc*/run_counter_collection.csv) per bw:: kernel."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(root + "/pmc*/*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        if k.startswith("bw::"):
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(agg):
    d = {c: sum(v) / len(v) for c, v in agg[k].items()}
    line = ", ".join("%s=%.4g" % (c, v) for c, v in sorted(d.items()))
    extra = ""
    if "SQ_WAVE_CYCLES" in d and d["SQ_WAVE_CYCLES"]:
        extra = " | wait_any %.0f%% wait_inst %.0f%%" % (100 * d.get("SQ_WAIT_ANY", 0) / d["SQ_WAVE_CYCLES"],
                                                       100 * d.get("SQ_WAIT_INST_ANY", 0) / d["SQ_WAVE_CYCLES"])
    print(k, ":", line, extra)
