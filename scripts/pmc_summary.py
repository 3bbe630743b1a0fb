"""Summarise a rocprofv3 --pmc counter_collection.csv per kernel (sum over dispatches)."""
import csv
import glob
import sys

for f in sys.argv[1:]:
    for path in glob.glob(f):
        agg = {}
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"].split("(")[0]
            if name.startswith("__amd") or "at::native" in name:
                continue
            d = agg.setdefault(name, {"VGPR": r.get("VGPR_Count"), "Scratch": r.get("Scratch_Size")})
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        for k, d in agg.items():
            print(path.split("/")[-3] if "/" in path else path, k)
            for c, v in sorted(d.items()):
                print("   %-22s %s" % (c, ("%.4g" % v) if isinstance(v, float) else v))
