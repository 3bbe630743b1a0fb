"""Full-frame fixtures at the BASELINE configs' spp, from the REAL reference
(oracle/_ref/libref.so, built by oracle/build_ref.sh from /root/reference).  Data only:
no reference source is copied.  SURVEY.md §4 item 3; VERDICT r2 "Next" #2.

    python tests/golden/make_frames.py [c1 c2 c4_ball c4_smooth c3 c5r ...]

One file per config, tests/golden/frame_<cfg>.npz (silver16: the reference main.cpp's
own HEAD scene, silver boxes, PT 16 spp -- the in-reference binding's check):

  * PT configs (c1 = configs[0] PT 16 spp, c2 = configs[1] PT 1024 spp, c4_ball /
    c4_smooth = configs[3] PT 4096 spp): the framebuffer of the real
    Renderer::Render (Renderer.cpp:68-127, 8 std::async workers; PT frames do not
    depend on the worker count) summarised as
      - rgb_sha256   sha256 of the W*H*3 float32 frame (NaN bit patterns canonicalised
                     to 0x7fc00000), the whole-frame bit-exact pin;
      - rgb_rowxor / rgb_colxor   per row / per column and channel XOR of the float
                     bit patterns (locates any differing pixel);
      - rgb_blocks   8x8 block means (f64 mean stored as f32), rgb_crops 64x64
                     full-resolution crops at crop_origins;
      - nonfinite    the flat pixel indices whose radiance is not finite.
  * BDPT configs (c3 = configs[2] Standard BDPT 256 spp, c5r = configs[4]'s bunny scene
    at a REDUCED 256 spp, stated in `spp`): the same summary of the per-pixel
    radiance (the t > 1 strategies, Renderer.cpp:49), from the reference's own
    FillBufferThread loop replayed per pixel (ref_trace_pixels: ResetRandom(i+1), the
    spp loop over BDPT(), BDPT.cpp:282-315) in 8 worker processes; splat_blocks /
    splat_crops of the t = 1 light-tracing splats (DrawToImage,
    SceneRenderingHelper.cpp:24-55, scaled 1/spp as Renderer.cpp:59); and
    render_blocks / render_crops of the real Renderer::Render frame (radiance plus the
    merged per-thread splat buffers, Renderer.cpp:98-114).  The generator checks that
    the two routes agree (radiance + splats vs Render, splats summed in another order).
"""
import multiprocessing as mp
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import frames  # noqa: E402  (tests/frames.py: the summary the tests check against)

W = H = 784
WORKERS = int(os.environ.get("FRAME_WORKERS", "8"))
# cfg -> (preset, mode, spp); mode 0 PathTrace, 1 BDPT
CONFIGS = {"silver16": ("silver", 0, 16), "c1": ("standard", 0, 16), "c2": ("standard", 0, 1024), "c4_ball": ("refractive_ball", 0, 4096),
           "c4_smooth": ("smooth_dielectric", 0, 4096), "c3": ("standard", 1, 256), "c5r": ("bunny", 1, 256),
           "c5": ("bunny", 1, 4096)}
# BDPT configs made through the per-pixel route alone: configs[4] at its own 4096 spp takes
# ~3 h of the container's 8 cores per route, and c5r already checks at 256 spp that the
# per-pixel route and Renderer::Render agree on this scene
TRACE_ONLY = {"c5"}
# chunked, resumable per-pixel route for long configs: chunk c holds pixels i = c (mod CHUNKS)
CHUNKS = {"c5": 32}
CACHE = os.path.join(os.path.dirname(os.path.dirname(HERE)), ".frame_cache")
# 64x64 crops: the image centre, the light's corner of the ceiling, a floor/left-wall corner
CROP_ORIGINS = np.array([[360, 360], [40, 300], [700, 60]], np.int32)  # (row, col)


def frame_summary(img, prefix):
    return frames.frame_summary(np.ascontiguousarray(img, np.float32).reshape(H, W, 3), prefix, CROP_ORIGINS)


def frame_blocks(img, prefix):
    return frames.frame_blocks(np.ascontiguousarray(img, np.float32).reshape(H, W, 3), prefix, CROP_ORIGINS)


def _trace_worker(args):
    preset, mode, spp, pix = args
    from oracle_bind import Reference
    R = Reference(preset)
    rgb, splat, _ = R.trace_pixels(mode, spp, pix, want_splat=True)
    return rgb, splat


def trace_frame(preset, mode, spp, chunks=1, tag=None):
    """The whole frame through ref_trace_pixels, pixels dealt i = w (mod WORKERS).
    With chunks > 1 the frame is traced as `chunks` interleaved pixel sets, each saved
    under .frame_cache/ when done so an interrupted run resumes; the splat buffers are
    summed in chunk order, then worker order."""
    allpix = np.arange(W * H, dtype=np.int64)
    rgb = np.zeros((W * H, 3), np.float32)
    splat = np.zeros((H, W, 3), np.float32)
    ctx = mp.get_context("spawn")
    with ctx.Pool(WORKERS) as pool:
        for c in range(chunks):
            pix = allpix[c::chunks]
            path = os.path.join(CACHE, "%s_%d_of_%d.npz" % (tag, c, chunks)) if chunks > 1 else None
            if path and os.path.exists(path):
                z = np.load(path)
                rgb[pix], s = z["rgb"], z["splat"]
            else:
                t0 = time.time()
                res = pool.map(_trace_worker, [(preset, mode, spp, pix[w::WORKERS]) for w in range(WORKERS)])
                r = np.zeros((len(pix), 3), np.float32)
                s = np.zeros((H, W, 3), np.float32)
                for w, (rw, sw) in enumerate(res):
                    r[w::WORKERS] = rw
                    s += sw
                rgb[pix] = r
                if path:
                    os.makedirs(CACHE, exist_ok=True)
                    np.savez(path, rgb=r, splat=s)
                    print("%s chunk %d/%d in %.0f s" % (tag, c + 1, chunks, time.time() - t0), flush=True)
            splat += s
    return rgb.reshape(H, W, 3), splat


def make(cfg):
    from oracle_bind import Reference
    preset, mode, spp = CONFIGS[cfg]
    t0 = time.time()
    out = {"preset": np.array(preset), "mode": np.int32(mode), "spp": np.int32(spp), "width": np.int32(W),
           "height": np.int32(H), "crop_origins": CROP_ORIGINS}
    if mode == 0:
        img = Reference(preset).render(0, spp, threads=WORKERS)
        out.update(frame_summary(img, "rgb"))
    else:
        rgb, splat = trace_frame(preset, mode, spp, CHUNKS.get(cfg, 1), cfg)
        out.update(frame_summary(rgb, "rgb"))
        out.update(frame_blocks(splat, "splat"))
        out["splat_sum"] = splat.astype(np.float64).sum((0, 1))
        if cfg in TRACE_ONLY:
            out["trace_only"] = np.int32(1)
            np.savez_compressed(os.path.join(HERE, "frame_%s.npz" % cfg), **out)
            print("%s (%s mode %d spp %d, per-pixel route only) done in %.0f s" % (cfg, preset, mode, spp,
                                                                                 time.time() - t0), flush=True)
            return
        render = Reference(preset).render(1, spp, threads=WORKERS)
        out.update(frame_blocks(render, "render"))
        # the two routes: Render = radiance + per-thread splat buffers merged in thread order
        both = (rgb.astype(np.float64) + splat)
        fin = np.isfinite(both).all(2) & np.isfinite(render).all(2)
        d = np.abs(both[fin] - render[fin]).max()
        rel = np.linalg.norm(both[fin] - render[fin]) / np.linalg.norm(render[fin])
        print("%s: Render vs radiance + splats: max|d| %.3g relL2 %.3g" % (cfg, d, rel), flush=True)
        assert rel < 1e-5, rel
        out["render_vs_trace_relL2"] = np.float64(rel)
    np.savez_compressed(os.path.join(HERE, "frame_%s.npz" % cfg), **out)
    print("%s (%s mode %d spp %d) done in %.0f s" % (cfg, preset, mode, spp, time.time() - t0), flush=True)


def main():
    from oracle_bind import ref_available
    if not ref_available():
        sys.exit("oracle/_ref/libref.so missing: run oracle/build_ref.sh first")
    for cfg in sys.argv[1:] or list(CONFIGS):
        make(cfg)


if __name__ == "__main__":
    main()
