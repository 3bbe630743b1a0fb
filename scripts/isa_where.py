"""Source lines of the scratch (spill) instructions of one kernel.
    python scripts/isa_where.py FILE.s KERNEL-SUBSTRING"""
import collections
import re
import sys

files, cur, loc = {}, None, None
res = collections.Counter()
for l in open(sys.argv[1]):
    m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', l)
    if m:
        files[m.group(1)] = (m.group(3) or m.group(2)).split("/")[-1]
    m = re.match(r"^(_Z\w+):", l)
    if m:
        cur = m.group(1)
    m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", l)
    if m:
        loc = "%s:%s" % (files.get(m.group(1), m.group(1)), m.group(2))
    if cur and sys.argv[2] in cur and ("scratch_store" in l or "scratch_load" in l):
        t = l.split()
        res[(loc, t[0], t[1] if "store" in t[0] else t[1].rstrip(","))] += 1
for k, v in sorted(res.items()):
    print(" ".join(map(str, k)), v)
