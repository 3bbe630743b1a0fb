"""Per-wavefront gen / connect start-end of the LAST render in a rocprofv3 kernel trace.
    python scripts/diag/wf_timeline.py path/to/kernel_trace.csv RENDERS"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
g = [e for e in ev if "gen_kernel" in e[2]]
c = [e for e in ev if "conn_kernel" in e[2]]
nf = len(g) // reps
g, c = g[-nf:], c[-nf:]
base = g[0][0]
for i in range(nf):
    print("f=%2d gen %7.2f-%7.2f (%5.2f)  conn %7.2f-%7.2f (%5.2f)" % (
        i, (g[i][0] - base) / 1e6, (g[i][1] - base) / 1e6, (g[i][1] - g[i][0]) / 1e6,
        (c[i][0] - base) / 1e6, (c[i][1] - base) / 1e6, (c[i][1] - c[i][0]) / 1e6))
