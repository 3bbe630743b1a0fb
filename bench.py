"""bench.py -- Msamples/s (pixels x spp / s) of the integration loop on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--mode pt|bdpt] [--scene S] [--spp SPP]

A step is one full render of the 784x784 frame (BASELINE.json configs[1]:
Standard Cornell Box, PT, 1024 spp on 1 MI355X).  With N > 1 (launched by
torch.distributed.run) each rank renders its pixel shard (i = rank; i += N, the
reference's own interleave, Renderer.cpp:38) into HBM and the framebuffers are
summed onto rank 0 with one RCCL reduce over xGMI; per-GPU work is
fixed by the frame, so scaling is strong.  Inputs (the flattened scene) are
resident in HBM before timing; the timed region is render + reduce.

Roofline: the hot kernel's ALGORITHMIC scene-fetch bytes (BVH nodes
popped x 32 B + triangle tests x 48 B, counted on the reference traversal; 2,073 B
per Standard PT sample) / its average device time (HIP events inside libtpt on the
stream the kernel runs on) against 8 TB/s.  The scene is L2-resident, so this is a
modelled yardstick; `traffic` is the memory-side bytes per launch measured by
rocprofv3 FETCH_SIZE/WRITE_SIZE passes (profiles/traffic.json, scripts/pmc_traffic.py).

cpu_baseline: the REAL reference renderer (oracle/_ref/libref.so, Renderer::Render
with std::async threads) on a bounded sample, rank 0 only; falls back to the CPU
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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--mode", choices=("pt", "bdpt", "pti"), default="pt",
                    help="pti: PathTrace with the indirect bounce on (TPT_MODE_PT_INDIRECT, not a BASELINE config)")
    ap.add_argument("--scene", default="standard")
    ap.add_argument("--spp", type=int, default=None, help="default 1024 (PT) / 256 (BDPT), BASELINE configs 1-2")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-threads", type=int, default=None)
    ap.add_argument("--traffic-bytes", type=float, default=None,
                    help="HBM bytes per launch (default: profiles/traffic.json, made by scripts/pmc_traffic.py)")
    return ap.parse_args()


def pmc_traffic(scene, mode):
    """Per-launch memory-side bytes of the dominant kernel, measured by rocprofv3
    FETCH_SIZE / WRITE_SIZE passes of this build (profiles/traffic.json)."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(path):
        return None
    e = json.load(open(path)).get("%s/%s" % (scene, mode))
    return float(e["bytes_per_launch"]) if e else None


def cpu_baseline(mode, scene, threads):
    """Bounded CPU sample on this host (about 10-30 s of CPU work)."""
    import numpy as np
    from oracle_bind import Oracle, Reference, ref_available
    spp = {"pt": 64, "pti": 16}.get(mode, 2)
    m = {"pt": 0, "bdpt": 1, "pti": 2}[mode]
    # Renderer::Render has no switch for the indirect bounce: for "pti" the baseline is
    # the restatement (bit-exact to the reference built without PathTracer.cpp:109)
    if ref_available() and mode != "pti":
        # the reference prints its progress lines from C++ (fd 1): keep them off the
        # bench's one-JSON-line stdout
        sys.stdout.flush()
        saved = os.dup(1)
        devnull = os.open(os.devnull, os.O_WRONLY)
        os.dup2(devnull, 1)
        try:
            R = Reference(scene)
            t0 = time.perf_counter()
            R.render(m, spp, threads=threads)
            dt = time.perf_counter() - t0
        finally:
            import ctypes
            ctypes.CDLL(None).fflush(None)  # C stdio buffers still hold reference output
            os.dup2(saved, 1)
            os.close(saved)
            os.close(devnull)
        kind = "reference"
    else:
        o = Oracle(scene)
        _, ms = o.render(m, spp, threads=threads)
        dt = ms / 1e3
        kind = "port"
    n = 784 * 784 * spp
    return {"value": round(n / dt / 1e6, 4), "unit": "Msamples/s", "cores": threads, "kind": kind,
            "sample": "full 784x784 %s frame of '%s' at %d spp, Renderer::Render with %d std::async threads, "
                      "wall %.2f s" % (mode.upper(), scene, spp, threads, dt)}


def main():
    a = parse()
    import numpy as np
    import torch

    mode = a.mode
    spp = a.spp or (256 if mode == "bdpt" else 1024)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus > 1 and world == 1:
        sys.exit("--gpus > 1 must be launched with torch.distributed.run (one process per GPU)")
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)

    import pytpt
    import sharding
    dev = torch.cuda.current_device()
    ctx = pytpt.Context(dev)
    preset = pytpt.Preset(a.scene)
    ctx.upload(preset)
    W, H = ctx.width, ctx.height
    fb = torch.zeros(2, H * W * 3, dtype=torch.float32, device="cuda")  # rgb + splat, one reduce buffer
    m = {"pt": pytpt.MODE_PT, "bdpt": pytpt.MODE_BDPT, "pti": pytpt.MODE_PT_INDIRECT}[mode]
    shard_begin, shard_stride = sharding.shard(rank, world)  # Renderer.cpp:38 interleave

    def step():
        st = ctx.render_device(spp, m, fb[0].data_ptr(), fb[1].data_ptr(), shard_begin, shard_stride)
        sharding.reduce_frame(dist, fb, dst=0)  # framebuffer + splat sum onto rank 0 (RCCL over xGMI)
        return st

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    kms = []
    t0 = time.perf_counter()
    for _ in range(a.steps):
        st = step()
        kms.append(st.kernel_ms)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    samples = W * H * spp * a.steps  # all ranks together cover the frame each step
    value = samples / dt / 1e6
    if rank == 0:
        kernel_ms = float(np.mean(kms))
        shard_samples = st.samples
        b_alg = B_ALG.get((a.scene, mode))
        achieved = (shard_samples * b_alg / (kernel_ms / 1e3) / 1e9) if b_alg else None
        roofline = {"bound": "hbm", "achieved": round(achieved, 1) if achieved else None, "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                    "traffic": a.traffic_bytes if a.traffic_bytes is not None else pmc_traffic(a.scene, mode),
                    "kernel": {"pt": "tpt_pt_kernel", "pti": "tpt_pti_kernel"}.get(mode, "bdpt wavefront sequence (gen+scan+scatter+conn+fold) x spp"), "kernel_ms": round(kernel_ms, 3),
                    "bytes_per_sample_alg": b_alg, "samples_per_launch": shard_samples,
                    "note": "algorithmic scene-fetch bytes (SURVEY 8d); scene is L2-resident, real bound is VALU"}
        cpu = None
        if not a.no_cpu and world == 1:
            threads = a.cpu_threads or min(16, os.cpu_count() or 1)
            cpu = cpu_baseline(mode, a.scene, threads)
        line = {"metric": "Msamples/s (pixels x spp / s), %s %s 784x784" % (a.scene, mode.upper()),
                "value": round(value, 2), "unit": "Msamples/s", "n_gpus": world, "steps": a.steps,
                "warmup": a.warmup, "ms_per_step": round(dt / a.steps * 1e3, 3), "higher_is_better": True,
                "scaling": "strong", "vs_baseline": None, "dtype": "f32+f64",
                "data": "synthetic (deterministic Cornell scene, reference seeds pixel+1)",
                "config": {"workload": "%s Cornell Box 784x784, %s, %d spp" % (a.scene, mode.upper(), spp),
                           "scene": a.scene, "mode": mode, "spp": spp, "width": W, "height": H,
                           "parallelism": "pixel-shard x%d + RCCL reduce" % world if world > 1 else "1 GPU"},
                "roofline": roofline, "cpu_baseline": cpu}
        print(json.dumps(line), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
