"""Source-line trail before each scratch store of one kernel (which values spill).
    python scripts/isa_trail.py FILE.s KERNEL-SUBSTRING [N]"""
import re
import sys

lines = open(sys.argv[1]).read().split("\n")
n = int(sys.argv[3]) if len(sys.argv) > 3 else 6
files = {}
for l in lines:
    m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', l)
    if m:
        files[m.group(1)] = (m.group(3) or m.group(2)).split("/")[-1]
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\w*%s\w*:" % sys.argv[2], l))
hist = []
for l in lines[start:]:
    if l.startswith(".Lfunc_end"):
        break
    m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", l)
    if m:
        loc = "%s:%s" % (files.get(m.group(1)), m.group(2))
        if not hist or hist[-1] != loc:
            hist.append(loc)
    if "scratch_store" in l or "scratch_load" in l:
        print(l.strip()[:58], "<-", " ".join(hist[-n:]))
