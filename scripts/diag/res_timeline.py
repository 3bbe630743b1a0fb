"""Per-wavefront wait / connect timeline of the LAST render of a resident-chains run
(rocprofv3 kernel trace).   python scripts/diag/res_timeline.py path/to/kernel_trace.csv"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
g = [e for e in ev if "gen_res" in e[2]]
print("gen launches (ms):", ["%.2f" % ((x[1] - x[0]) / 1e6) for x in g])
base = g[-1][0]
w = [e for e in ev if "wait_kernel" in e[2] and e[0] >= base]
c = [e for e in ev if "conn_kernel" in e[2] and e[0] >= base]
idle = 0
for i in range(len(c)):
    idle += (w[i][1] - w[i][0]) / 1e6
    print("f=%2d wait %7.2f-%7.2f (%5.2f) conn %7.2f-%7.2f (%5.2f)" % (
        i, (w[i][0] - base) / 1e6, (w[i][1] - base) / 1e6, (w[i][1] - w[i][0]) / 1e6,
        (c[i][0] - base) / 1e6, (c[i][1] - base) / 1e6, (c[i][1] - c[i][0]) / 1e6))
print("connect stream waiting on gen: %.2f ms" % idle)
