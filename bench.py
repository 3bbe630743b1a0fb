"""bench.py -- Msamples/s (pixels x spp / s) of the integration loop on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--mode pt|bdpt|c5|pti] [--scene S] [--spp SPP]

With no --mode the ONE JSON line carries every BASELINE config, each a full 784x784
frame per step with the flattened scene already resident in HBM:
  * the headline, BASELINE.json configs[1]: Standard Cornell Box, PT, 1024 spp;
  * "bdpt": configs[2], Standard Cornell Box, BDPT, 256 spp;
  * "c4_ball" / "c4_smooth": configs[3], refractive ball / smooth dielectric, PT, 4096 spp;
  * "c5":   configs[4], Cornell + bunny, BDPT, 4096 spp (one frame: ~18 s on one GPU);
  * configs[0] (PT 16 spp, -j 1, CPU only) is the headline cpu_baseline's "j1" leg;
  * "shard_model" (N = 1 only): the 1/2/4/8-way pixel split of configs 2, 3 and 5 timed
    shard by shard on this one GPU (sharding.shard_model): the frame each rank of an
    N-GPU run would render, its kernel time, and T_full / (N * T_slowest_shard).
--mode runs one workload alone (profiling runs use it).

`python bench.py --gpus N` (N > 1) without a launcher starts the N ranks itself: it
counts the visible GPUs (exit 2 if fewer than N) and runs torch.distributed.run as a
child process.  With N > 1 (one process per GPU) each rank
renders its pixel shard (i = rank; i += N, the reference's own interleave,
Renderer.cpp:38) into HBM and the [rgb; splat] buffer is summed onto rank 0 with one
RCCL reduce over xGMI.  The frame is fixed as N grows: strong scaling.
The timed region is render + reduce, bracketed by barrier + synchronize, max over ranks.

roofline: the dominant kernel's VALU issue rate.  Nothing on this path is a dense
contraction and the scene is LDS/L2-resident, so the bound is vector-instruction
issue.  profiles/valu_model.json (scripts/valu_model.py) holds the
kernel's SIMD issue-cycles per launch = sum over instruction classes of
rocprofv3 SQ_INSTS_VALU_* counts x the cycles per wave-instruction measured on
MI355X by scripts/valu_cost.hip; `achieved` divides that by the kernel's average
duration measured live here (HIP events inside libtpt on the stream the kernel runs
on); `peak` = 1,024 SIMDs x the clock the profiled run held (GRBM_GUI_ACTIVE).
scene_fetch_model (was roofline_hbm_model until round 5): SURVEY §8(d)'s algorithmic
scene-fetch bytes / kernel time, with reuse_factor = that rate / 8 TB/s -- the reads are
served from LDS / L2, so it is no roofline (a "frac" above 1 read as a violated bound).
roofline_hbm_measured: the measured memory-side bytes (rocprofv3 FETCH_SIZE /
WRITE_SIZE of the profiled build) / the live kernel time / 8 TB/s.  An N-rank
line adds `ranks` (device PCI ids, kernel and reduce ms per rank); every line ends with a
compact per-config `summary`.

cpu_baseline: the REAL reference renderer (oracle/_ref/libref.so, Renderer::Render
with std::async threads, one per CPU this process may run on) on a bounded sample,
rank 0 at N = 1 only, plus the -j 1 leg of configs[0]; falls back to the CPU
restatement (oracle/liboracle.so, kind "port") if the reference build is absent.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "toypathtracer-games101-assignment7_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, os.path.join(ROOT, "tests"))

# SURVEY.md §8(d) / BASELINE.md: algorithmic bytes per sample (reference traversal counts)
B_ALG = {("standard", "pt"): 2073, ("standard", "bdpt"): 18481, ("refractive_ball", "pt"): 2109,
         ("refractive_ball", "bdpt"): 19377, ("bunny", "pt"): 2123, ("bunny", "bdpt"): 21229,
         # scripts/b_alg.py (oracle traversal counts, full frame at 1 spp; reproduces the six above)
         ("smooth_dielectric", "pt"): 2076, ("smooth_dielectric", "bdpt"): 26715,
         ("silver", "pt"): 2075, ("silver", "bdpt"): 25386}
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s
N_SIMD = 1024          # 256 CUs x 4 SIMDs
MAX_CLOCK_MHZ = 2400.0

# (scene, mode, spp) of each workload; BASELINE.json configs[1], [2], [3] (two scenes), [4]
WORKLOADS = {"pt": ("standard", "pt", 1024), "bdpt": ("standard", "bdpt", 256),
             "c4_ball": ("refractive_ball", "pt", 4096), "c4_smooth": ("smooth_dielectric", "pt", 4096),
             "c5": ("bunny", "bdpt", 4096), "pti": ("standard", "pti", 1024)}
CONFIG_NAME = {"pt": "configs[1]: Standard Cornell Box 784x784, PT, 1024 spp",
               "bdpt": "configs[2]: Standard Cornell Box 784x784, BDPT, 256 spp",
               "c4_ball": "configs[3]: Refractive Ball Cornell 784x784, PT, 4096 spp",
               "c4_smooth": "configs[3]: Smooth Dielectric Cornell 784x784, PT, 4096 spp",
               "c5": "configs[4]: Cornell + bunny OBJ 784x784, BDPT, 4096 spp, pixel-sharded + RCCL reduce",
               "pti": "PathTrace with the indirect bounce (not a BASELINE config), Standard 784x784, 1024 spp"}
# (steps, warmup) of the workloads after the first one in a default run
SUB_STEPS = {"bdpt": (2, 1), "c4_ball": (2, 1), "c4_smooth": (2, 1), "c5": (1, 0)}
# shard model: (workload, spp) -- c5 at a reduced spp (its per-iteration launch chain is
# the same at every spp, so the split's efficiency is too; stated in the line)
SHARD_MODEL = (("pt", 1024), ("bdpt", 256), ("c5", 256))
SHARD_NS = (2, 4, 8)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5, help="timed frames of the headline PT workload")
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--mode", choices=tuple(WORKLOADS), default=None,
                    help="run one workload alone (default: PT headline + every other config in one line)")
    ap.add_argument("--scene", default=None, help="override the workload's scene")
    ap.add_argument("--spp", type=int, default=None, help="override the workload's spp")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline legs")
    ap.add_argument("--no-c5", action="store_true", help="default line without the c5 sub-object")
    ap.add_argument("--no-shard-model", action="store_true", help="default line without the shard_model sub-object")
    ap.add_argument("--shard-only", action="store_true", help="print the shard_model object alone (A/B runs)")
    ap.add_argument("--shard-keys", default=None, help="--shard-only: comma list of the shard-model legs (pt,bdpt,c5)")
    ap.add_argument("--sample-seed", action="store_true",
                    help="--mode pt|pti only: per-sample seeding (TPT_FLAG_SAMPLE_SEED), a non-replay throughput mode")
    ap.add_argument("--cpu-threads", type=int, default=None)
    ap.add_argument("--rehearse", action="store_true",
                    help="CPU rehearsal of the N-rank plumbing (gloo, no GPU, no renderer): each rank "
                         "writes a known pattern into its pixel shard, rank 0 checks the reduced frame; "
                         "the line carries value null (tests/test_multiproc.py)")
    return ap.parse_args()


def _load_json(name):
    path = os.path.join(ROOT, "profiles", name)
    return json.load(open(path)) if os.path.exists(path) else {}


def cpu_info():
    """Host CPU as this process sees it: model, nproc, the CPUs it may run on and the
    cgroup CPU quota (the GPU box shares its host between jobs)."""
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    affinity = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    return {"model": model, "nproc": os.cpu_count(), "affinity": affinity, "cgroup_cpus": quota}


def _quiet(fn):
    """Run fn() with fd 1 redirected: the reference prints progress from C++."""
    import ctypes
    sys.stdout.flush()
    saved = os.dup(1)
    devnull = os.open(os.devnull, os.O_WRONLY)
    os.dup2(devnull, 1)
    try:
        return fn()
    finally:
        ctypes.CDLL(None).fflush(None)
        os.dup2(saved, 1)
        os.close(saved)
        os.close(devnull)


def cpu_render(scene, mode, spp, threads):
    """Wall seconds of one full-frame render on the CPU; (seconds, kind)."""
    from oracle_bind import Oracle, Reference, ref_available
    m = {"pt": 0, "bdpt": 1, "pti": 2}[mode]
    # Renderer::Render has no switch for the indirect bounce: for "pti" the baseline is
    # the restatement (bit-exact to the reference built without PathTracer.cpp:109)
    if ref_available() and mode != "pti":
        R = Reference(scene)

        def run():
            t0 = time.perf_counter()
            R.render(m, spp, threads=threads)
            return time.perf_counter() - t0
        return _quiet(run), "reference"
    _, ms = Oracle(scene).render(m, spp, threads=threads)
    return ms / 1e3, "port"


def cpu_baseline(key, scene, mode, threads, info):
    """Bounded CPU sample of the workload on this host: full frames at a reduced spp
    (throughput does not depend on spp: the per-pixel stream is serial either way)."""
    spp = {"pt": 64, "pti": 16, "bdpt": 2}[mode] if key != "c5" else 1
    if key.startswith("c4"):
        spp = 32  # the glass / smooth scenes: ~1 s at 16 threads, lengthened below
    dt, kind = cpu_render(scene, mode, spp, threads)
    if dt < 2.0 and mode == "pt":  # many-core host: lengthen the sample to a few seconds
        spp *= max(2, int(round(4.0 / max(dt, 1e-3))))
        dt, kind = cpu_render(scene, mode, spp, threads)
    n = 784 * 784 * spp
    cores = threads if info["cgroup_cpus"] is None else min(threads, info["cgroup_cpus"])
    out = {"value": round(n / dt / 1e6, 4), "unit": "Msamples/s", "cores": cores, "threads": threads,
           "kind": kind,
           "sample": "full 784x784 %s frame of '%s' at %d spp, Renderer::Render with %d std::async threads, "
                     "wall %.2f s" % (mode.upper(), scene, spp, threads, dt),
           "host": info}
    if key == "pt":
        # BASELINE.json configs[0]: Standard PT 16 spp with -j 1, the whole config
        dt1, kind1 = cpu_render(scene, mode, 16, 1)
        out["j1"] = {"value": round(784 * 784 * 16 / dt1 / 1e6, 4), "unit": "Msamples/s", "cores": 1,
                     "kind": kind1, "sample": "configs[0] itself: full 784x784 PT frame of 'standard' at 16 spp, "
                                              "Renderer::Render with 1 thread (-j 1), wall %.2f s" % dt1}
    return out


ISA_CYCLES = {"ADD_F32": 2.0, "MUL_F32": 2.0, "FMA_F32": 2.0, "ADD_F64": 4.0, "MUL_F64": 4.0, "FMA_F64": 4.0,
              "INT32": 2.0, "INT64": 4.0, "CVT": 2.0, "TRANS_F32": 8.0, "TRANS_F64": 16.0}


def valu_roofline(key, kernel_ms, samples):
    """VALU-issue roofline of the workload's dominant kernel (see module docstring).
    `samples`: pixel-samples this rank's launch traced; the profiled issue cycles are
    per-sample constants of the workload, scaled to it."""
    model = _load_json("valu_model.json").get(key)
    if not model:
        return {"bound": "valu", "achieved": None, "peak": None, "unit": "G SIMD-cycles/s", "frac": None,
                "traffic": None, "note": "profiles/valu_model.json has no entry for %s" % key}
    shard_frac = samples / float(model["samples_per_launch"])
    cyc = model["issue_cycles_per_launch"] * shard_frac  # this rank's share of the profiled frame
    ms = kernel_ms
    achieved = cyc / (ms / 1e3) / 1e9
    clk = model.get("clock_mhz") or MAX_CLOCK_MHZ
    peak = N_SIMD * clk / 1e3
    t = _load_json("traffic.json").get(key)
    out = {"bound": "valu", "achieved": round(achieved, 1), "peak": round(peak, 1), "unit": "G SIMD-cycles/s",
            "frac": round(achieved / peak, 4), "frac_at_2400mhz": round(achieved / (N_SIMD * MAX_CLOCK_MHZ / 1e3), 4),
            "traffic": float(t["bytes_per_launch"]) * shard_frac if t else None,
            "kernel": model["kernel"], "kernel_ms": round(ms, 3),
            "issue_cycles_per_launch": round(cyc), "clock_mhz": clk,
            "source": model.get("source"),
            "note": "VALU issue cycles per launch (PMC class counts x measured cycles per wave-instruction, "
                    "profiles/valu_model.json) / live kernel time / (1,024 SIMDs x the profiled clock); "
                    "traffic = measured memory-side bytes per launch (profiles/traffic.json)"}
    # the same class counts priced at the ISA's nominal issue rates instead of the measured
    # table (full-rate 32-bit ops 2 cycles per wave64 instruction, 64-bit 4,
    # quarter-rate transcendentals 8 / 16)
    cls = model.get("class_insts_per_launch")
    if cls:
        isa = sum(n * ISA_CYCLES.get(c, 2.0) for c, n in cls.items()) + 2.0 * model.get("other_insts_per_launch", 0)
        out["issue_cycles_per_launch_isa"] = round(isa * shard_frac)
        out["frac_at_isa_rate"] = round(isa * shard_frac / (ms / 1e3) / 1e9 / peak, 4)
    # lane utilisation (round 6): the share of a VALU wave-instruction's 64 lanes that
    # work (SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU)); the issue fraction
    # counts wave-instructions whatever their lanes, so frac x lane_util is the fraction
    # of the SIMDs' lane-cycles spent on useful lanes (issue-cycle weighted over BDPT's
    # kernels)
    lu = model.get("lane_util")
    if lu:
        out["lane_util"] = lu
        out["frac_lane_weighted"] = round(achieved / peak * lu, 4)
        out["lane_source"] = model.get("lane_source")
    if len(model.get("per_kernel", {})) > 1:  # BDPT: a sequence of kernels on two streams
        out["per_kernel_profiled"] = model["per_kernel"]
    return out


def scene_fetch_model(scene, mode, kernel_ms, samples, traffic_key):
    """SURVEY §8(d)'s algorithmic scene-fetch bytes (B_ALG) over the kernel time: a MODEL
    of the reference traversal's reads, not a bound.  The scene is LDS/L2-resident, so the
    rate exceeds the HBM peak; reuse_factor = rate / 8 TB/s says by how much the on-chip
    memories multiply HBM here.  The HBM roofline is roofline_hbm_measured."""
    b_alg = B_ALG.get((scene, "pt" if mode == "pti" else mode))
    if not b_alg:
        return None
    achieved = samples * b_alg / (kernel_ms / 1e3) / 1e9
    t = _load_json("traffic.json").get(traffic_key)
    return {"achieved": round(achieved, 1), "unit": "GB/s", "reuse_factor": round(achieved / HBM_PEAK_GBS, 4),
            "hbm_peak": HBM_PEAK_GBS, "measured_traffic": float(t["bytes_per_launch"]) if t else None,
            "bytes_per_sample_alg": b_alg, "samples_per_launch": samples,
            "note": "MODEL (SURVEY 8d): algorithmic scene-fetch bytes / kernel time, served from LDS / L2; "
                    "reuse_factor = that rate / the HBM peak (not a roofline fraction); measured_traffic = "
                    "memory-side bytes per launch (roofline_hbm_measured prices them)"}


def _free_port():
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _apply_visible(devs, spec):
    """The devices a *_VISIBLE_DEVICES value selects from `devs` (a list of (ordinal-free)
    device records with a "uuid"): comma-separated ordinals into `devs` or GPU-<uuid>
    tokens; duplicates count once, and -- as the HIP/ROCr parsers do -- the list ends at
    the first token that names no device (out of range, unknown uuid, garbage)."""
    out = []
    for tok in spec.split(","):
        tok = tok.strip()
        if not tok:
            break
        d = None
        if tok.isdigit():
            i = int(tok)
            d = devs[i] if i < len(devs) else None
        elif tok.upper().startswith("GPU-"):
            d = next((x for x in devs if x.get("uuid") and x["uuid"].lower() == tok[4:].lower()), None)
        if d is None:
            break
        if d not in out:
            out.append(d)
    return out


def visible_gpus(root=None):
    """GPUs this process may open, counted WITHOUT the HIP runtime (the launcher must
    not initialise the GPU before it starts the ranks): the kfd topology nodes that
    have SIMDs and a DRM render node this user can open (/dev/dri/renderD<minor>, what
    ROCr opens), then narrowed by ROCR_VISIBLE_DEVICES and HIP_VISIBLE_DEVICES (or
    CUDA_VISIBLE_DEVICES when HIP's is unset), each an ordered list of ordinals into the
    devices left by the previous level or GPU-<uuid> tokens (ordinals out of
    range and duplicates no longer count; _apply_visible).  Returns (count, source), or
    (None, reason) when there is no such view; then amdsmi is tried (its devices' render
    nodes must be openable too), and nothing else: torch.cuda.device_count() may fall
    back to hipGetDeviceCount.  `root` (tests: TPT_BENCH_SYSFS_ROOT) prefixes /sys and /dev."""
    root = root if root is not None else os.environ.get("TPT_BENCH_SYSFS_ROOT", "/")
    base = os.path.join(root, "sys/class/kfd/kfd/topology/nodes")
    try:
        nodes = sorted((d for d in os.listdir(base) if d.isdigit()), key=int)
    except OSError:
        nodes = None

    def openable(minor):
        return os.access(os.path.join(root, "dev/dri/renderD%s" % minor), os.R_OK | os.W_OK)

    devs = []
    if nodes is not None:
        for nd in nodes:
            props = {}
            try:
                with open(os.path.join(base, nd, "properties")) as f:
                    for line in f:
                        k, _, v = line.strip().partition(" ")
                        props[k] = v.strip()
            except OSError:
                continue
            if int(props.get("simd_count", "0") or 0) <= 0 or "drm_render_minor" not in props:
                continue  # a CPU node
            if openable(props["drm_render_minor"]):
                uid = props.get("unique_id")
                devs.append({"node": int(nd), "uuid": ("%016x" % int(uid)) if uid and uid.isdigit() and int(uid) else None})
        source = "kfd topology"
    elif root == "/" and not os.environ.get("TPT_BENCH_NO_AMDSMI"):
        try:
            import amdsmi
            amdsmi.amdsmi_init()
            try:
                for h in amdsmi.amdsmi_get_processor_handles():
                    e = amdsmi.amdsmi_get_gpu_enumeration_info(h)
                    if openable(e["drm_render"]):
                        u = (e.get("hip_uuid") or "")
                        devs.append({"node": e.get("hsa_id"), "uuid": u[4:] if u.upper().startswith("GPU-") else u or None})
            finally:
                amdsmi.amdsmi_shut_down()
            source = "amdsmi"
        except Exception as e:  # noqa: BLE001 -- any failure means "cannot count"
            return None, "no kfd topology under %s and amdsmi failed (%s)" % (base, type(e).__name__)
    else:
        return None, "no kfd topology under %s" % base
    v = os.environ.get("ROCR_VISIBLE_DEVICES")
    if v is not None:
        devs = _apply_visible(devs, v)
    v = os.environ.get("HIP_VISIBLE_DEVICES")
    if v is None:
        v = os.environ.get("CUDA_VISIBLE_DEVICES")
    if v is not None:
        devs = _apply_visible(devs, v)
    return len(devs), source


def check_distinct(line, world):
    """An N-rank line must come from N different GPUs (distinct PCI ids of the ranks'
    devices); returns the reason it does not, or None."""
    if world <= 1 or "distinct_devices" not in line:
        return None
    if line["distinct_devices"] != world:
        return "the %d ranks ran on %d distinct GPUs (PCI ids %s)" % (
            world, line["distinct_devices"], sorted({str(r.get("pci_bus_id")) for r in line.get("ranks", [])}))
    return None


def spawn_ranks(a):
    """`bench.py --gpus N` (N > 1) run without a launcher: start N ranks through
    torch.distributed.run as a CHILD process (never an exec: this process may not
    replace itself once anything has touched the GPU) and return its exit code; rank
    0 prints the line.  Nothing here initialises the GPU: the visible devices are
    counted from the kfd topology (visible_gpus), never through HIP; when they cannot be
    counted that way the run is refused (exit 2)."""
    import subprocess
    if not a.rehearse:
        n, source = visible_gpus()
        if n is None:
            print("bench.py: --gpus %d: cannot count GPUs without the HIP runtime (%s); start the ranks "
                  "with torch.distributed.run instead" % (a.gpus, source), file=sys.stderr, flush=True)
            return 2
        if n < a.gpus:
            print("bench.py: --gpus %d needs %d visible GPUs, this box has %d (%s)" % (a.gpus, a.gpus, n, source),
                  file=sys.stderr, flush=True)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(a.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL (see README)
    env.setdefault("OMP_NUM_THREADS", "1")
    sys.stdout.flush()
    return subprocess.call(cmd, env=env)


def hbm_measured(traffic_key, kernel_ms, samples):
    """Measured memory-side traffic of the workload (profiles/traffic.json: rocprofv3
    FETCH_SIZE / WRITE_SIZE passes, (2 x FETCH + WRITE) per MI355X_MICROARCH.md's gfx950
    correction) per launch, scaled to this rank's samples, over the live kernel time:
    the fraction of the 8 TB/s HBM peak the kernels really move."""
    t = _load_json("traffic.json").get(traffic_key)
    model = _load_json("valu_model.json").get(traffic_key)
    if not t or not model:
        return None
    b = float(t["bytes_per_launch"]) * samples / float(model["samples_per_launch"])
    gbs = b / (kernel_ms / 1e3) / 1e9
    return {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(gbs / HBM_PEAK_GBS, 4), "bytes_per_launch": round(b),
            "fetch_size_kb": t["fetch_size_kb"], "write_size_kb": t["write_size_kb"],
            "source": t.get("note"),
            "note": "MEASURED memory-side bytes (2 x FETCH_SIZE + WRITE_SIZE, rocprofv3 PMC) / live kernel time"}


class Rehearsal:
    """--rehearse: the N-rank plumbing of Runner (rendezvous, shard split, the one
    reduce onto rank 0, max-over-ranks timing, per-rank records) on the CPU over gloo,
    with no renderer: rank r writes pixel index + 1 into its shard's pixels
    (i = r mod N, Renderer.cpp:38) and rank 0 checks that the reduced frame holds every
    pixel's value exactly once."""
    W = H = 64

    def __init__(self, args):
        import torch
        import torch.distributed as dist
        import sharding
        self.torch, self.dist, self.sharding, self.args = torch, dist, sharding, args
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        if self.world > 1:
            dist.init_process_group("gloo")
        else:
            self.dist = None

    def run(self):
        torch = self.torch
        npix = self.W * self.H
        begin, stride = self.sharding.shard(self.rank, self.world)
        want = torch.arange(1, npix + 1, dtype=torch.float32).repeat_interleave(3)
        fb = torch.zeros(2, npix * 3)
        ok = True
        red_ms = []
        t0 = time.perf_counter()
        for _ in range(self.args.warmup + self.args.steps):
            fb.zero_()
            idx = torch.arange(begin, npix, stride)
            fb[0].view(npix, 3)[idx] = (idx + 1).to(torch.float32)[:, None]
            t1 = time.perf_counter()
            self.sharding.reduce_frame(self.dist, fb, dst=0)
            red_ms.append((time.perf_counter() - t1) * 1e3)
            if self.rank == 0:
                ok = ok and bool(torch.equal(fb[0], want)) and not fb[1].any()
        dt = time.perf_counter() - t0
        rec = {"rank": self.rank, "device": "cpu", "pci_bus_id": None, "kernel_ms": 0.0,
               "reduce_ms": round(sum(red_ms) / len(red_ms), 3), "pixels": len(range(begin, npix, stride))}
        ranks = [None] * self.world
        if self.dist is not None:
            self.dist.all_gather_object(ranks, rec)
            t = torch.tensor([dt], dtype=torch.float64)
            self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
            dt = float(t.item())
        else:
            ranks = [rec]
        if self.rank == 0:
            print(json.dumps({"metric": "rehearsal (no renderer): N-rank shard + reduce plumbing", "value": None,
                              "unit": "Msamples/s", "n_gpus": self.world, "steps": self.args.steps,
                              "warmup": self.args.warmup, "rehearsal": True, "reduce_check": ok,
                              "wall_s_max_over_ranks": round(dt, 4), "ranks": ranks}), flush=True)
        if self.dist is not None:
            self.dist.destroy_process_group()
        return 0 if ok else 1


class Runner:
    def __init__(self, args):
        import torch
        self.torch = torch
        self.args = args
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        if args.gpus != self.world:
            sys.exit("bench.py: --gpus %d but WORLD_SIZE %d" % (args.gpus, self.world))
        self.local = local
        self.dist = None
        if self.world > 1:
            import torch.distributed as dist
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            self.dist = dist
        else:
            torch.cuda.set_device(0)
        import pytpt
        import sharding
        self.pytpt, self.sharding = pytpt, sharding
        self.ctx = pytpt.Context(torch.cuda.current_device())
        self.scene = None
        self.fb = None
        dev = torch.cuda.current_device()
        p = torch.cuda.get_device_properties(dev)
        self.device_rec = {"rank": self.rank, "local_rank": local, "device": dev, "name": p.name,
                           "pci_bus_id": "%04x:%02x:%02x" % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id),
                           "uuid": str(p.uuid)}

    def barrier(self):
        self.torch.cuda.synchronize()
        if self.dist is not None:
            self.dist.barrier()
        self.torch.cuda.synchronize()

    def run(self, key, steps, warmup):
        torch, pytpt = self.torch, self.pytpt
        scene, mode, spp = WORKLOADS[key]
        if self.args.mode is not None:
            scene = self.args.scene or scene
            spp = self.args.spp or spp
        if self.scene != scene:
            self.ctx.upload(pytpt.Preset(scene))
            self.scene = scene
        W, H = self.ctx.width, self.ctx.height
        if self.fb is None or self.fb.shape[1] != H * W * 3:
            self.fb = torch.zeros(2, H * W * 3, dtype=torch.float32, device="cuda")  # rgb + splat, one reduce
        fb = self.fb
        m = {"pt": pytpt.MODE_PT, "bdpt": pytpt.MODE_BDPT, "pti": pytpt.MODE_PT_INDIRECT}[mode]
        begin, stride = self.sharding.shard(self.rank, self.world)  # Renderer.cpp:38 interleave
        stream = torch.cuda.current_stream()
        flags = pytpt.FLAG_SAMPLE_SEED if (self.args.sample_seed and self.args.mode in ("pt", "pti")) else 0

        # PT modes write no splats (PathTrace has no light-tracing strategy), so only the
        # rgb half of the buffer is summed; BDPT sums rgb and splat in one reduce.
        red = fb if mode == "bdpt" else fb[:1]

        events = []

        def step(timed=False):
            # libtpt renders on its own stream: everything torch's stream has queued on
            # fb (the zero fill, the previous step's reduce) must finish before it
            # rewrites the buffers.
            stream.synchronize()
            st = self.ctx.render_device(spp, m, fb[0].data_ptr(), fb[1].data_ptr(), begin, stride, flags)
            if timed and self.dist is not None:  # the reduce alone, on the stream it runs on
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                self.sharding.reduce_frame(self.dist, red, dst=0)  # onto rank 0 (RCCL over xGMI)
                e1.record(stream)
                events.append((e0, e1))
            else:
                self.sharding.reduce_frame(self.dist, red, dst=0)
            return st

        for _ in range(warmup):
            step()
        self.barrier()
        kms = []
        t0 = time.perf_counter()
        for _ in range(steps):
            st = step(timed=True)
            kms.append(st.kernel_ms)
        self.barrier()
        dt = time.perf_counter() - t0
        ranks = None
        if self.dist is not None:
            t = torch.tensor([dt], dtype=torch.float64, device="cuda")
            self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
            rec = dict(self.device_rec, kernel_ms=round(sum(kms) / len(kms), 3),
                       reduce_ms=round(sum(a.elapsed_time(b) for a, b in events) / len(events), 4),
                       reduce_bytes=red.numel() * 4, wall_s=round(dt, 4), samples=st.samples)
            ranks = [None] * self.world
            self.dist.all_gather_object(ranks, rec)
            dt = float(t.item())
        samples = W * H * spp * steps  # all ranks together cover the frame each step
        kernel_ms = sum(kms) / len(kms)
        shard_samples = st.samples
        # the VALU model is profiled on the replay kernels; a seeded run has no entry
        tkey = "%s/%s%s" % (scene, mode, "/seeded" if flags else "")
        line = {"metric": "Msamples/s (pixels x spp / s), %s %s %dx%d%s" % (
                    scene, mode.upper(), W, H, ", per-sample seeding (not the reference's replay)" if flags else ""),
                "value": round(samples / dt / 1e6, 2), "unit": "Msamples/s", "n_gpus": self.world, "steps": steps,
                "warmup": warmup, "ms_per_step": round(dt / steps * 1e3, 3),
                "config": {"workload": CONFIG_NAME[key] if self.args.mode is None or
                           (scene, spp) == WORKLOADS[key][::2] else "%s %s %d spp" % (scene, mode.upper(), spp),
                           "scene": scene, "mode": mode, "spp": spp, "width": W, "height": H,
                           "parallelism": "pixel-shard x%d + RCCL reduce" % self.world if self.world > 1
                           else "1 GPU"},
                "roofline": valu_roofline(tkey, kernel_ms, shard_samples),
                "scene_fetch_model": scene_fetch_model(scene, mode, kernel_ms, shard_samples, tkey),
                "roofline_hbm_measured": hbm_measured(tkey, kernel_ms, shard_samples),
                "kernel_ms_per_step": round(kernel_ms, 3), "samples_per_rank_step": shard_samples,
                "nonfinite_pixels": st.nonfinite + st.nonfinite_splat}
        if ranks is not None:
            line["ranks"] = ranks
            line["distinct_devices"] = len({r["pci_bus_id"] for r in ranks})
            # kernel time of the slowest rank: the roofline of the N-GPU step
            line["kernel_ms_max_over_ranks"] = max(r["kernel_ms"] for r in ranks)
        return line

    def shard_model(self, c5_line=None):
        """The N-way pixel split of configs 2, 3 and 5 modelled on this one GPU: every
        stride-N shard is rendered alone (tpt_render_device, as rank r of an N-GPU run
        renders it) and timed with the library's HIP events (sharding.shard_model)."""
        pytpt = self.pytpt
        out = {"note": "one-GPU model of the N-GPU split, not a scaling run: each stride-N shard "
                       "(pixels i = r mod N, Renderer.cpp:38) rendered alone on this GPU; eff = T_full / "
                       "(N x slowest shard), kernel time (HIP events); the reduce (one 7.4 / 14.7 MB RCCL "
                       "reduce) is not modelled", "ns": list(SHARD_NS)}
        keys = self.args.shard_keys.split(",") if getattr(self.args, "shard_keys", None) else None
        for key, spp in SHARD_MODEL:
            if keys is not None and key not in keys:
                continue
            scene, mode, _ = WORKLOADS[key]
            if self.scene != scene:
                self.ctx.upload(pytpt.Preset(scene))
                self.scene = scene
            m = {"pt": pytpt.MODE_PT, "bdpt": pytpt.MODE_BDPT}[mode]
            fb = self.fb

            def render(begin, stride):
                st = self.ctx.render_device(spp, m, fb[0].data_ptr(), fb[1].data_ptr(), begin, stride, 0)
                return st.kernel_ms, st.total_ms

            render(0, 1)  # warm-up
            res = self.sharding.shard_model(render, SHARD_NS)
            res["workload"] = "%s %s %d spp%s" % (scene, mode.upper(), spp,
                                                  "" if spp == WORKLOADS[key][2] else
                                                  " (configs[4] at a reduced spp: same per-iteration chain)")
            out[key] = res
        if c5_line is not None:
            # configs[4] at its own 4096 spp, split 8 ways (the run BASELINE defines it on):
            # every 1/8 shard against the c5 line's whole frame (same process, same scene)
            scene, mode, spp = WORKLOADS["c5"]
            if self.scene != scene:
                self.ctx.upload(pytpt.Preset(scene))
                self.scene = scene
            fb = self.fb

            def render8(begin, stride):
                st = self.ctx.render_device(spp, pytpt.MODE_BDPT, fb[0].data_ptr(), fb[1].data_ptr(), begin, stride, 0)
                return st.kernel_ms, st.total_ms

            res = self.sharding.shard_model(render8, (8,), full=(c5_line["kernel_ms_per_step"], c5_line["ms_per_step"]))
            res["workload"] = "bunny BDPT 4096 spp (configs[4] itself); whole frame = the c5 line's"
            out["c5_4096"] = res
        return out
    
    def close(self):
        self.ctx.close()
        if self.dist is not None:
            self.dist.destroy_process_group()


def summary(lines):
    """Compact per-config figures, last in the line so a tail of the output shows them."""
    out = {}
    for k, l in lines.items():
        rf, hm = l.get("roofline") or {}, l.get("roofline_hbm_measured") or {}
        out[k] = {"value": l["value"], "ms": l["ms_per_step"], "kernel_ms": l["kernel_ms_per_step"],
                  "valu_frac": rf.get("frac"), "valu_frac_at_isa_rate": rf.get("frac_at_isa_rate"),
                  "lane_util": rf.get("lane_util"), "valu_frac_lane_weighted": rf.get("frac_lane_weighted"),
                  "hbm_frac_measured": hm.get("frac"),
                  "cpu": (l.get("cpu_baseline") or {}).get("value")}
    return out


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(a))
    if a.rehearse:
        sys.exit(Rehearsal(a).run())
    r = Runner(a)
    if a.shard_only:
        r.fb = r.torch.zeros(2, 784 * 784 * 3, dtype=r.torch.float32, device="cuda")
        print(json.dumps({"shard_model": r.shard_model()}), flush=True)
        r.close()
        return
    info = cpu_info()
    want_cpu = not a.no_cpu and r.world == 1 and r.rank == 0
    # every CPU this process may use: the affinity mask, capped by the cgroup's CPU
    # quota (the GPU box gives each job a 16-CPU share of a 256-CPU host; more threads
    # than that only time-slice)
    threads = a.cpu_threads or (min(info["affinity"], max(1, int(info["cgroup_cpus"])))
                                if info["cgroup_cpus"] else info["affinity"])
    keys = [a.mode] if a.mode else ["pt", "bdpt", "c4_ball", "c4_smooth"] + ([] if a.no_c5 else ["c5"])
    lines = {}
    for k in keys:
        steps, warmup = (a.steps, a.warmup) if k == keys[0] else SUB_STEPS[k]
        lines[k] = r.run(k, steps, warmup)
    shard_model = r.shard_model(lines.get("c5")) if (a.mode is None and r.world == 1 and not a.no_shard_model) else None
    if r.rank == 0:
        if want_cpu:
            for k in keys:
                scene, mode = lines[k]["config"]["scene"], lines[k]["config"]["mode"]
                lines[k]["cpu_baseline"] = cpu_baseline(k, scene, mode, threads, info)
        head = lines[keys[0]]
        out = {"metric": head["metric"], "value": head["value"], "unit": "Msamples/s", "n_gpus": r.world,
               "steps": head["steps"], "warmup": head["warmup"], "ms_per_step": head["ms_per_step"],
               "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32+f64",
               "data": "synthetic (deterministic Cornell scenes, %s)" % (
                   "per-sample seeding: sample j of pixel i seeds tpt_sample_seed(i, j)" if a.sample_seed
                   else "reference seeds pixel+1"),
               "config": head["config"], "roofline": head["roofline"],
               "scene_fetch_model": head["scene_fetch_model"],
               "roofline_hbm_measured": head["roofline_hbm_measured"], "cpu_baseline": head.get("cpu_baseline"),
               "kernel_ms_per_step": head["kernel_ms_per_step"], "nonfinite_pixels": head["nonfinite_pixels"]}
        for f in ("ranks", "distinct_devices", "kernel_ms_max_over_ranks"):
            if f in head:
                out[f] = head[f]
        for k in keys[1:]:
            out[k] = lines[k]
        if shard_model is not None:
            out["shard_model"] = shard_model
        out["summary"] = summary(lines)
        if shard_model is not None:  # the one-GPU model's efficiencies (kernel time), N = 2 / 4 / 8
            out["summary"]["shard_eff"] = {k: [v["n%d" % n]["eff_kernel"] for n in SHARD_NS if "n%d" % n in v]
                                           for k, v in shard_model.items() if isinstance(v, dict)}
        bad = check_distinct(out, r.world)
        if bad:
            out["distinct_devices_error"] = bad
        print(json.dumps(out), flush=True)
        if bad:
            print("bench.py: " + bad, file=sys.stderr, flush=True)
            r.close()
            sys.exit(3)
    r.close()


if __name__ == "__main__":
    main()
