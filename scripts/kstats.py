"""Print a rocprofv3 kernel_stats.csv compactly: name (templates/args stripped), calls, avg/total ms, %."""
import csv
import re
import sys

for path in sys.argv[1:]:
    print("==", path)
    for r in csv.DictReader(open(path)):
        n = r["Name"]
        n = re.sub(r"\(.*", "", n)
        n = n.replace("void ", "")
        if "rocprim" in n:
            n = "rocprim::" + ("scan" if "scan_impl" in n else n.split("::")[-1])[:40]
        print("  %-42s %6s  avg %9.3f ms  total %9.2f ms  %5.1f%%" % (n[:42], r["Calls"], float(r["AverageNs"]) / 1e6,
              float(r["TotalDurationNs"]) / 1e6, float(r["Percentage"])))
