"""Turn rocprofv3 FETCH_SIZE / WRITE_SIZE passes into per-launch HBM traffic.

    python scripts/pmc_traffic.py KEY KERNEL FETCH_CSV WRITE_CSV [--note TEXT]

KEY is "<scene>/<mode>" (e.g. standard/pt), KERNEL a substring of the dominant
kernel's name, *_CSV the counter_collection.csv of a `rocprofv3 --pmc FETCH_SIZE
--kernel-trace` and a separate `--pmc WRITE_SIZE` pass (TCC slots do not fit both,
MI355X_MICROARCH.md §rocprofv3 PMC slots).  Both counters are in KB, summed over
the XCDs.  Per MI355X_MICROARCH.md §HBM, gfx950's FETCH_SIZE reports half the bytes
of a wide coalesced read (128-B requests tallied at 64 B), so it is doubled;
WRITE_SIZE is taken as is.  Infinity-Cache hits are counted by these counters, so
the figure is memory-side fabric traffic, an upper bound on HBM bytes.

The result is merged into profiles/traffic.json, which bench.py reports as
roofline.traffic.
"""
import argparse
import csv
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_launch(path, kernel, counter, frames=None):
    tot, disp = 0.0, set()
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
            tot += float(r["Counter_Value"])
            disp.add(r.get("Dispatch_Id") or r.get("Correlation_Id") or len(disp))
    if not disp:
        raise SystemExit("no %s rows for kernel %r in %s" % (counter, kernel, path))
    return tot / (frames or len(disp)), len(disp)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("key")
    ap.add_argument("kernel")
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("--note", default="")
    ap.add_argument("--frames", type=float, default=None,
                    help="sum every matching dispatch and divide by this many frames (BDPT: the "
                         "wavefront sequence of one frame is the 'launch')")
    a = ap.parse_args()
    f_kb, nf = per_launch(a.fetch_csv, a.kernel, "FETCH_SIZE", a.frames)
    w_kb, nw = per_launch(a.write_csv, a.kernel, "WRITE_SIZE", a.frames)
    entry = {"kernel": a.kernel, "fetch_size_kb": round(f_kb, 1), "write_size_kb": round(w_kb, 1),
             "bytes_per_launch": round((2.0 * f_kb + w_kb) * 1024.0),
             "correction": "bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 (gfx950 FETCH_SIZE halving)",
             "dispatches": [nf, nw], "note": a.note}
    out = os.path.join(ROOT, "profiles", "traffic.json")
    db = json.load(open(out)) if os.path.exists(out) else {}
    db[a.key] = entry
    json.dump(db, open(out, "w"), indent=1, sort_keys=True)
    print(a.key, entry)


if __name__ == "__main__":
    main()
