"""VALU-issue roofline inputs from one profile_round.sh run -> profiles/valu_model.json.

    python scripts/valu_model.py PROF_DIR KEY WORKLOAD KERNEL [--frames F] [--waves W] [--scale S]

PROF_DIR  gpurun_out/prof_TAG (scripts/profile_round.sh)
KEY       "<scene>/<mode>" entry in valu_model.json (e.g. standard/pt)
WORKLOAD  the pass prefix in PROF_DIR (pt, bdpt, c5, pti)
KERNEL    substring of the kernel names to sum (tpt_pt_kernel, tpt_bdpt_)
--frames  frames in the profiled run (PT: --warmup 1 --steps 1 = 2; BDPT: 1); the
          per-launch figures are totals / frames
--scale   multiply per-frame counts (a BDPT profile at 32 spp scaled to the 256-spp
          frame bench.py times: 8)
--waves   valu_cost.log column (default 8 waves per SIMD: the issue-saturated rate)

Issue cycles = sum over classes of (wave-instruction count x cycles per wave-
instruction), the costs measured by scripts/valu_cost.hip on the same box (costs()):
  ADD/MUL/FMA_F32 -> v_add/v_mul/v_fma_f32     ADD/MUL/FMA_F64 -> v_add/v_mul/v_fma_f64
  TRANS_F32 -> mean(v_rcp_f32, v_sqrt_f32)     TRANS_F64 -> mean(v_rcp_f64, v_sqrt_f64)
  INT32 -> v_add_u32   INT64 -> v_lshlrev_b64   CVT -> (v_cvt_f32_f64 + v_cvt_f64_f32) / 2
  the rest of SQ_INSTS_VALU (moves, selects, compares, bit ops) -> mean(v_mov_b32,
  v_and_b32, (v_cmp + v_cndmask) / 2)
Clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel wall time (MI355X_MICROARCH.md, DVFS give-back).
"""
import argparse
import csv
import glob
import json
import os
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLASSES = ["ADD_F32", "MUL_F32", "FMA_F32", "TRANS_F32", "ADD_F64", "MUL_F64", "FMA_F64", "TRANS_F64", "INT32",
           "INT64", "CVT"]


def costs(log, waves):
    """Cycles per wave-instruction of each class on one SIMD: valu_cost's event-time
    figure at `waves` waves per SIMD (default 8: issue-saturated).  It includes the
    benchmark's loop overhead (3 SALU per 32 VALU), so it errs high by ~0.2 cycle."""
    c = {}
    for line in open(log):
        line = line.strip()
        if line.startswith("{"):
            r = json.loads(line)
            if r["waves_per_simd"] == waves:
                c[r["inst"]] = r["cycles_per_wave_inst_event"] / (2.0 if "+" in r["inst"] else 1.0)
    m = statistics.mean
    return {"ADD_F32": c["v_add_f32"], "MUL_F32": c["v_mul_f32"], "FMA_F32": c["v_fma_f32"],
            "TRANS_F32": m([c["v_rcp_f32"], c["v_sqrt_f32"]]), "ADD_F64": c["v_add_f64"], "MUL_F64": c["v_mul_f64"],
            "FMA_F64": c["v_fma_f64"], "TRANS_F64": m([c["v_rcp_f64"], c["v_sqrt_f64"]]), "INT32": c["v_add_u32"],
            "INT64": c["v_lshlrev_b64"], "CVT": c["v_cvt_f64_f32+v_cvt_f32_f64"],
            "OTHER": m([c["v_mov_b32"], c["v_and_b32"], c["v_cmp_lt_f32+v_cndmask_b32"]])}


def counters(pass_dir, kernel):
    tot, per_kernel = {}, {}
    for path in glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if kernel not in r["Kernel_Name"]:
                continue
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            v = float(r["Counter_Value"])
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + v
            pk = per_kernel.setdefault(name, {})
            pk[r["Counter_Name"]] = pk.get(r["Counter_Name"], 0.0) + v
    return tot, per_kernel


def kernel_ns(pass_dir, kernel):
    """Summed duration (ns) of the matching dispatches in the pass's kernel trace."""
    tot, per = 0, {}
    for path in glob.glob(os.path.join(pass_dir, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if kernel in r["Kernel_Name"]:
                d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                tot += d
                name = r["Kernel_Name"].split("(")[0].replace("void ", "")
                per[name] = per.get(name, 0) + d
    return tot, per


def lane_util(pass_dir, kernel):
    """VALU lane utilisation from a `lane` pass (SQ_THREAD_CYCLES_VALU / (64 x
    SQ_ACTIVE_INST_VALU), counter_defs.yaml's VALUUtilization): overall and per kernel."""
    tot, per = counters(pass_dir, kernel)
    f = lambda c: c["SQ_THREAD_CYCLES_VALU"] / (64.0 * c["SQ_ACTIVE_INST_VALU"])  # noqa: E731
    ok = lambda c: c.get("SQ_THREAD_CYCLES_VALU") and c.get("SQ_ACTIVE_INST_VALU")  # noqa: E731
    return (round(f(tot), 4) if ok(tot) else None), {k: round(f(c), 4) for k, c in per.items() if ok(c)}


def add_lane(entry, pass_dir, kernel, source):
    """Lane fields of a valu_model.json entry: lane_util (issue-cycle weighted over the
    entry's kernels when it has several) and per-kernel lane_util."""
    overall, per = lane_util(pass_dir, kernel)
    if overall is None:
        return entry
    pk = entry.get("per_kernel", {})
    w = sum(v.get("issue_cycles_per_launch", 0) * per[k] for k, v in pk.items() if k in per)
    tw = sum(v.get("issue_cycles_per_launch", 0) for k, v in pk.items() if k in per)
    for k, v in pk.items():
        if k in per:
            v["lane_util"] = per[k]
    entry["lane_util"] = round(w / tw, 4) if tw else overall
    entry["lane_util_thread_cycles"] = overall
    entry["lane_source"] = source
    return entry


def issue_cycles(cnt, cost):
    classes = {k: cnt.get("SQ_INSTS_VALU_" + k, 0.0) for k in CLASSES}
    other = max(0.0, cnt.get("SQ_INSTS_VALU", 0.0) - sum(classes.values()))
    cyc = sum(classes[k] * cost[k] for k in CLASSES) + other * cost["OTHER"]
    return cyc, classes, other


def patch_lane(argv):
    """--patch-lane PROF_DIR KEY WORKLOAD KERNEL SOURCE: add the lane fields of a `lane`
    pass to an existing entry (a build whose kernels are byte-identical to the entry's)."""
    prof_dir, key, workload, kernel, source = argv
    out = os.path.join(ROOT, "profiles", "valu_model.json")
    db = json.load(open(out))
    add_lane(db[key], os.path.join(prof_dir, "%s_lane" % workload), kernel, source)
    json.dump(db, open(out, "w"), indent=1, sort_keys=True)
    print(key, db[key]["lane_util"], {k: v.get("lane_util") for k, v in db[key].get("per_kernel", {}).items()})


def main():
    import sys
    if len(sys.argv) > 1 and sys.argv[1] == "--patch-lane":
        return patch_lane(sys.argv[2:])
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("key")
    ap.add_argument("workload")
    ap.add_argument("kernel")
    ap.add_argument("--frames", type=float, default=1.0)
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--waves", type=int, default=8, help="valu_cost column (8: issue-saturated)")
    ap.add_argument("--samples", type=int, required=True,
                    help="pixel-samples of the launch the figures are scaled to (784*784*spp)")
    ap.add_argument("--note", default="")
    ap.add_argument("--source", default=None, help="committed summary the figures come from (profiles/...)")
    a = ap.parse_args()
    cost = costs(os.path.join(a.prof_dir, "valu_cost.log"), a.waves)
    p = lambda s: os.path.join(a.prof_dir, "%s_%s" % (a.workload, s))  # noqa: E731
    c1, k1 = counters(p("valu1"), a.kernel)
    c2, k2 = counters(p("valu2"), a.kernel)
    cnt = dict(c1)
    cnt.update(c2)
    ns2, _ = kernel_ns(p("valu2"), a.kernel)
    clock_mhz = cnt["GRBM_GUI_ACTIVE"] / 8.0 / (ns2 * 1e-9) / 1e6 if ns2 else None
    ns_kt, per_kt = kernel_ns(p("kt"), a.kernel)
    f = a.scale / a.frames
    cyc, classes, other = issue_cycles(cnt, cost)
    per = {}
    for name in sorted(set(k1) | set(k2)):
        kc = dict(k1.get(name, {}))
        kc.update(k2.get(name, {}))
        kcyc, _, _ = issue_cycles(kc, cost)
        per[name] = {"issue_cycles_per_launch": round(kcyc * f), "valu_insts_per_launch": round(kc.get("SQ_INSTS_VALU", 0) * f),
                     "kernel_ms_per_launch_kt": round(per_kt.get(name, 0) * 1e-6 * f, 3)}
    busy = cnt.get("SQ_BUSY_CYCLES")
    entry = {"kernel": a.kernel, "issue_cycles_per_launch": round(cyc * f), "samples_per_launch": a.samples,
             "valu_insts_per_launch": round(cnt.get("SQ_INSTS_VALU", 0) * f),
             "class_insts_per_launch": {k: round(v * f) for k, v in classes.items()},
             "other_insts_per_launch": round(other * f),
             "cycles_per_wave_inst": {k: round(v, 3) for k, v in cost.items()},
             "cost_waves_per_simd": a.waves,
             "clock_mhz": round(clock_mhz, 1) if clock_mhz else None,
             "sq_busy_cycles_per_se": round(busy / 32.0 / a.frames) if busy else None,
             "kernel_ms_per_launch_kt": round(ns_kt * 1e-6 * f, 3),
             "valu_frac_in_profile": round(cyc / (1024 * clock_mhz * 1e6 * ns2 * 1e-9), 4) if ns2 and clock_mhz else None,
             "active_inst_valu_quad": cnt.get("SQ_ACTIVE_INST_VALU"), "wave_cycles_quad": cnt.get("SQ_WAVE_CYCLES"),
             "wait_inst_any_quad": cnt.get("SQ_WAIT_INST_ANY"),
             "per_kernel": per, "source": a.source or os.path.relpath(a.prof_dir, ROOT), "note": a.note}
    if os.path.isdir(p("lane")):
        add_lane(entry, p("lane"), a.kernel, a.source or os.path.relpath(a.prof_dir, ROOT))
    out = os.path.join(ROOT, "profiles", "valu_model.json")
    db = json.load(open(out)) if os.path.exists(out) else {}
    db[a.key] = entry
    json.dump(db, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps({a.key: entry}, indent=1))


if __name__ == "__main__":
    main()
