#!/usr/bin/env python3
"""Turn rocprofv3 FETCH_SIZE / WRITE_SIZE passes into per-launch HBM bytes for the bw:: kernels.

Usage: pmc_traffic.py <fetch_dir> <write_dir> <gib> <out.json>
The summary is stamped with the digest of the library sources it was measured on
(backuwup_amd.build.source_digest) and $BW_COMMIT when set; bench.py reports the traffic only
when the digest matches its own tree.

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE is reported in KiB and on gfx950 counts
exactly half of the bytes of a wide coalesced streaming read, so it is doubled; WRITE_SIZE (KiB)
reads exactly for 16-B-per-lane stores.  Values are averaged over the profiled launches.
"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def per_kernel(d, counter):
    acc = collections.defaultdict(list)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            if k.startswith("bw::"):
                acc[(k, r.get("Dispatch_Id", r.get("Correlation_Id", "")))].append(float(r["Counter_Value"]))
    out = collections.defaultdict(list)
    for (k, _), v in acc.items():
        out[k].append(sum(v))  # a counter may be reported per XCD / instance: sum within a dispatch
    return {k: sum(v) / len(v) for k, v in out.items()}


def main():
    fdir, wdir, gib, path = sys.argv[1], sys.argv[2], float(sys.argv[3]), sys.argv[4]
    fetch = per_kernel(fdir, "FETCH_SIZE")
    write = per_kernel(wdir, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        name = k.split("::")[-1].split("<")[0]
        rd = fetch.get(k)
        wr = write.get(k)
        e = {"fetch_size_kib_raw": rd, "write_size_kib_raw": wr,
             "hbm_read_bytes_per_launch": None if rd is None else int(rd * 1024 * 2),
             "hbm_write_bytes_per_launch": None if wr is None else int(wr * 1024)}
        e["hbm_bytes_per_launch"] = (e["hbm_read_bytes_per_launch"] or 0) + (e["hbm_write_bytes_per_launch"] or 0)
        kernels[name] = e
    from backuwup_amd.build import source_digest
    json.dump({"gib": gib, "note": "FETCH_SIZE x2 (gfx950 half-count) + WRITE_SIZE, KiB->bytes, mean per launch",
               "source_digest": source_digest(), "commit": os.environ.get("BW_COMMIT"),
               "kernels": kernels}, open(path, "w"), indent=1)
    for k, e in kernels.items():
        print(k, e)


if __name__ == "__main__":
    main()
