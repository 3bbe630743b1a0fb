"""Summarise a rocprofv3 kernel trace: per kernel name count / total / mean, the span,
and (BDPT) the busy time of the gen and connect streams.
    python scripts/diag/trace_timeline.py path/to/kernel_trace.csv"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", ""))
            for r in rows)
t0, t1 = ev[0][0], max(e[1] for e in ev)
agg = collections.defaultdict(lambda: [0, 0])
for s, e, n in ev:
    agg[n][0] += 1
    agg[n][1] += e - s
print("span %.3f ms" % ((t1 - t0) / 1e6))
for n, (c, d) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print("%-40s n=%5d total %9.3f ms mean %8.1f us" % (n[:40], c, d / 1e6, d / c / 1e3))
# union of busy intervals of all kernels
busy, cur_s, cur_e = 0, None, None
for s, e, _ in ev:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
print("any-kernel busy %.3f ms of span (%.1f %%)" % (busy / 1e6, 100.0 * busy / (t1 - t0)))
gens = [(s, e) for s, e, n in ev if "gen_kernel" in n]
conns = [(s, e) for s, e, n in ev if "conn_kernel" in n]
if gens:
    g = [e - s for s, e in gens]
    c = [e - s for s, e in conns]
    print("gen   per launch: mean %.1f us min %.1f max %.1f" % (sum(g) / len(g) / 1e3, min(g) / 1e3, max(g) / 1e3))
    print("conn  per launch: mean %.1f us min %.1f max %.1f" % (sum(c) / len(c) / 1e3, min(c) / 1e3, max(c) / 1e3))
    # time when neither gen nor conn runs
    iv = sorted(gens + conns)
    b2, cs, ce = 0, None, None
    for s, e in iv:
        if ce is None or s > ce:
            if ce is not None:
                b2 += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    b2 += ce - cs
    print("gen|conn busy %.3f ms (%.1f %% of span)" % (b2 / 1e6, 100.0 * b2 / (t1 - t0)))
    # sweep: time by the set of kernel kinds running (gen count, conn count)
    pts = []
    for s, e, n in ev:
        kind = "g" if "gen_kernel" in n else "c" if "conn_kernel" in n else "o"
        pts.append((s, 1, kind))
        pts.append((e, -1, kind))
    pts.sort()
    cnt = {"g": 0, "c": 0, "o": 0}
    acc = collections.defaultdict(int)
    last = pts[0][0]
    for t, d, kind in pts:
        if t > last:
            acc[(min(cnt["g"], 2), min(cnt["c"], 1), min(cnt["o"], 1))] += t - last
        cnt[kind] += d
        last = t
    for key, v in sorted(acc.items(), key=lambda x: -x[1]):
        print("gens=%d conn=%d other=%d : %8.3f ms (%.1f %%)" % (key + (v / 1e6, 100.0 * v / (t1 - t0))))
