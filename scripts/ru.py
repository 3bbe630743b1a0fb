"""One line per tpt kernel: VGPRs, scratch, occupancy (make resource-usage, filtered)."""
import re
import subprocess
import sys

out = subprocess.run(["make", "-s", "-C", "toypathtracer-games101-assignment7_amd", "resource-usage"] + sys.argv[1:],
                     capture_output=True, text=True).stdout
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1) if "tpt_" in m.group(1) else None
        if cur:
            rows[cur] = {}
        continue
    if cur:
        m = re.search(r"(VGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]|TotalSGPRs): (\d+)", line)
        if m:
            rows[cur][m.group(1).split()[0]] = int(m.group(2))
for k, v in rows.items():
    print("%-60s vgpr %3s sgpr %3s scratch %4s occ %s lds %s" % (k[:60], v.get("VGPRs"), v.get("TotalSGPRs"),
          v.get("ScratchSize"), v.get("Occupancy"), v.get("LDS")))
