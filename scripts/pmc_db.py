"""Summarise rocprofv3 --pmc results (sqlite .db or counter_collection.csv) per kernel:
sums over dispatches, plus derived ratios when the counters are present.

    python scripts/pmc_db.py gpurun_out/pmc_x/run_results.db [more ...]
"""
import csv
import sqlite3
import sys


def rows(path):
    if path.endswith(".db"):
        db = sqlite3.connect(path)
        for k, c, v, d in db.execute("select kernel_name, counter_name, value, dispatch_id from counters_collection"):
            yield k, c, float(v), d
    else:
        for r in csv.DictReader(open(path)):
            yield r["Kernel_Name"], r["Counter_Name"], float(r["Counter_Value"]), r.get("Dispatch_Id")


def short(k):
    k = k.split("(")[0]
    return k.replace("void ", "")


for path in sys.argv[1:]:
    agg, disp = {}, {}
    for k, c, v, d in rows(path):
        if k.startswith("__amd") or "at::native" in k or "rocprim" in k:
            continue
        k = short(k)
        agg.setdefault(k, {})
        agg[k][c] = agg[k].get(c, 0.0) + v
        disp.setdefault(k, set()).add(d)
    print("==", path)
    for k, d in agg.items():
        n = len(disp[k])
        print(" %s  (%d dispatches; per dispatch)" % (k, n))
        for c, v in sorted(d.items()):
            print("   %-24s %.4g" % (c, v / n))
        g = d.get
        if g("SQ_WAVE_CYCLES"):
            wc = g("SQ_WAVE_CYCLES")
            for c in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU"):
                if g(c) is not None:
                    print("   %-24s %.1f %%" % (c + "/WAVE_CYC", 100 * g(c) / wc))
        if g("SQ_THREAD_CYCLES_VALU") and g("SQ_ACTIVE_INST_VALU"):
            print("   %-24s %.1f %%" % ("lane util (VALU)", 100 * g("SQ_THREAD_CYCLES_VALU") / (64 * g("SQ_ACTIVE_INST_VALU"))))
