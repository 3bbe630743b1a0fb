"""Scratch (spill) instructions per kernel in a device assembly file.

    hipcc ... --cuda-device-only -S -o /tmp/x.s csrc/tpt_capi.hip
    python scripts/isa_spills.py /tmp/x.s [name-substring ...]
"""
import re
import sys


def split(path):
    cur, out = None, {}
    for line in open(path):
        m = re.match(r"^(_Z\w+):", line)
        if m:
            cur = m.group(1)
            out[cur] = []
        elif cur is not None:
            out[cur].append(line)
    return out


def main():
    funcs = split(sys.argv[1])
    pats = sys.argv[2:] or ["kernel"]
    for name, lines in funcs.items():
        if "rocprim" in name or not any(p in name for p in pats):
            continue
        st = sum("scratch_store" in l or ("buffer_store" in l and "offen" not in l and "s[0:3]" in l) for l in lines)
        ld = sum("scratch_load" in l for l in lines)
        n = sum(1 for l in lines if l.startswith("\t") and not l.startswith("\t."))
        print("%-70s insts %6d scratch st %4d ld %4d" % (name[:70], n, st, ld))


if __name__ == "__main__":
    main()
