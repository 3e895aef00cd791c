"""Per-wave SQ counter summary of the zstd kernels from tools/gpu_zstd_pmc.sh's two passes."""
import collections
import csv
import sys

for f in sys.argv[1:]:
    agg = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if "zs_" not in r["Kernel_Name"]:
            continue
        agg[(int(r["Dispatch_Id"]), r["Kernel_Name"].split("(")[0], r["Counter_Name"])] += float(r["Counter_Value"])
    seen = sorted(set(k[:2] for k in agg))
    for d, name in seen:
        c = {k[2]: v for k, v in agg.items() if k[:2] == (d, name)}
        w = c.get("SQ_WAVES", 1) or 1
        print(d, name, "waves %d" % w, " ".join("%s/wave=%.4g" % (k[3:] if k.startswith("SQ_") else k, v / w)
                                                  for k, v in sorted(c.items()) if k != "SQ_WAVES"))
