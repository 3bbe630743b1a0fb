"""Static VALU opcode breakdown of kernels, in the PMC's classes (VERDICT r5 Next #4).

    python scripts/isa_hist.py FILE.s KERNEL-SUBSTRING [...]   (FILE.s: scripts/isa.sh, line tables on)

For each kernel: VALU instructions by the rocprofv3 SQ_INSTS_VALU_* class they count in
(ADD/MUL/FMA F32/F64, TRANS F32/F64, INT32, INT64, CVT) and the rest -- the "other"
share of the VALU model -- split into moves, compares, selects, bit ops, lane ops,
min/max/med3 and the remainder; then where the moves come from (source line of each
v_mov) and the instructions attributed to the empty-asm launderings (`asm volatile(""
: "+v"(x))` lines).  Static counts: every instruction once, however often it runs."""
import collections
import re
import sys

CLS = [
    ("TRANS_F64", r"v_(rcp|rsq|sqrt)_f64|v_(sin|cos|exp|log)_f64"),
    ("TRANS_F32", r"v_(rcp|rsq|sqrt|sin|cos|exp|log|rcp_iflag)_f32|v_(exp|log)_legacy"),
    ("FMA_F64", r"v_(fma|fmac)_f64|v_div_fmas_f64|v_div_scale_f64"),
    ("MUL_F64", r"v_mul_f64|v_ldexp_f64"),
    ("ADD_F64", r"v_add_f64"),
    ("FMA_F32", r"v_(fma|fmac|mac|mad|madak|madmk|fmaak|fmamk)_f32|v_div_fmas_f32|v_div_scale_f32|v_pk_fma_f32"),
    ("MUL_F32", r"v_mul_f32|v_pk_mul_f32|v_ldexp_f32"),
    ("ADD_F32", r"v_(add|sub|subrev)_f32|v_pk_add_f32"),
    ("CVT", r"v_cvt_"),
    ("INT64", r"v_(lshlrev|lshrrev|ashrrev|lshl|lshr|ashr)_(b|i|u)64|v_(add|sub)_(co_)?u64|v_mad_u64|v_mad_i64|v_lshl_add_u64"),
    ("INT32", r"v_(add|sub|subrev)(_co|_nc)?(_ci)?_[ui]32|v_mul_(lo|hi)_[ui]32|v_mul_u32_u24|v_mad_u32_u24|v_mad_[ui]32|v_add3_u32|v_lshl_add_u32|v_add_lshl_u32|v_mul_i32_i24|v_sad"),
]
OTHER = [
    ("mov", r"v_mov_|v_accvgpr|v_swap"),
    ("cmp", r"v_cmp|v_cmpx"),
    ("cndmask", r"v_cndmask"),
    ("bitops", r"v_(and|or|xor|not|xnor|bfe|bfi|bfm|alignbit|alignbyte|perm|lshlrev_b32|lshrrev_b32|ashrrev_i32|lshl_or|and_or|or3|xor3|bcnt|ffbh|ffbl|ffbh|bitop3|lshl_b32|lshr_b32)"),
    ("lane", r"v_readlane|v_readfirstlane|v_writelane|v_mbcnt|_dpp|v_permlane"),
    ("minmax", r"v_(max|min|med3|max3|min3)_"),
    ("fp-misc", r"v_(div_fixup|frexp|fract|floor|ceil|trunc|rndne|class)"),
]


def classify(op):
    for name, rx in CLS:
        if re.match(rx, op):
            return name, None
    for name, rx in OTHER:
        if re.match(rx, op):
            return "OTHER", name
    return "OTHER", "rest:" + op


def main():
    path, subs = sys.argv[1], sys.argv[2:]
    files, loc, cur = {}, None, None
    srclines = {}
    per = collections.defaultdict(lambda: {"cls": collections.Counter(), "oth": collections.Counter(),
                                           "mov_loc": collections.Counter(), "loc": collections.Counter(), "n": 0})
    for l in open(path):
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', l)
        if m:
            files[m.group(1)] = (m.group(2), m.group(3))
            continue
        m = re.match(r"^(_Z\w+):", l)
        if m:
            cur = m.group(1) if any(s in m.group(1) for s in subs) else None
            continue
        if l.startswith(".Lfunc_end"):
            cur = None
        m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", l)
        if m:
            f = files.get(m.group(1), ("?", None))
            loc = (f, int(m.group(2)))
            continue
        if cur is None:
            continue
        t = l.strip()
        if not t.startswith("v_"):
            continue
        op = t.split()[0]
        c, o = classify(op)
        k = per[cur]
        k["n"] += 1
        k["cls"][c] += 1
        if o:
            k["oth"][o] += 1
        if o == "mov":
            k["mov_loc"][loc] += 1
        k["loc"][loc] += 1
    for kname, k in per.items():
        n = k["n"]
        print("== %s: %d VALU instructions (static)" % (kname[:90], n))
        for c, v in k["cls"].most_common():
            print("   %-10s %6d  %5.1f %%" % (c, v, 100.0 * v / n))
        print("   OTHER by kind:")
        for o, v in k["oth"].most_common(14):
            print("     %-22s %6d  %5.1f %% of all" % (o, v, 100.0 * v / n))
        print("   v_mov by source line (top 12):")
        for key, v in k["mov_loc"].most_common(12):
            f, ln = key if key else (None, 0)
            name = (f[1] or f[0]).split("/")[-1] if f else "?"
            print("     %-28s %5d" % ("%s:%s" % (name, ln), v))
        # instructions on the launderings' own lines
        asm_lines = collections.Counter()
        for key, v in k["loc"].items():
            if not key or not key[0] or key[0] == "?":
                continue
            f, ln = key
            full = (f[0] + "/" + f[1]) if f[1] and not f[1].startswith("/") else (f[1] or f[0])
            try:
                src = srclines.setdefault(full, open(full).read().split("\n"))
            except OSError:
                continue
            if 0 < ln <= len(src) and 'asm volatile(""' in src[ln - 1]:
                asm_lines["%s:%d" % (full.split("/")[-1], ln)] += v
        print("   VALU on empty-asm laundering lines: %d" % sum(asm_lines.values()))
        for a, v in asm_lines.most_common(10):
            print("     %-28s %5d" % (a, v))


if __name__ == "__main__":
    main()
