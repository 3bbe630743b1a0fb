"""Generate tests/golden/*.npz from the REAL reference (oracle/_ref/libref.so, built
by oracle/build_ref.sh from /root/reference).  Fixtures are data only (inputs and
expected outputs); no reference source is copied.  Re-run after changing inputs:

    python tests/golden/make_golden.py

Contents (all float32 unless noted):
  rng.npz               XorShift32 / GetRandomFloat streams (global.cpp:5-22)
  kat_material.npz      Material::sample/pdf/evalGivenSample/fresnel + cosine sample
  kat_helpers.npz       Reflect/Refract/AnyPerpendicular/GGX/SolveQuadratic/DotProduct
  intersect_<p>.npz     Scene::Intersect closest hits (x, N, primitive ordinal)
  pixels_<p>.npz        per-pixel replay (Renderer.cpp:38-52): PT spp 1/16, BDPT spp 4
                        (+ BDPT t=1 splats of those pixels as a sparse list)
  image_standard.npz    real Renderer::Render framebuffers: PT 16 spp (8x8 block
                        means + a 64x64 full-res crop), BDPT 2 spp -j1 (same)
  pt_indirect.npz       TPT_MODE_PT_INDIRECT: per-pixel replay through the reference's
                        PathTrace compiled without the `break` at PathTracer.cpp:109
                        (oracle/build_ref.sh), spp 1 and 8, radiance + outBounces sums
  edge_<case>.npz       the reference's edge cases (VERDICT r1 Missing #4):
                        multi_light (three emitters, two of them coplanar and
                        overlapping: PathTracer.cpp:82's loop, closest-hit ties),
                        emissive_sphere (a Sphere as m_emissionObjects[0]: Sphere::Sample,
                        Sphere.cpp:48-55), background (Scene.hpp:23's default colour,
                        BDPT.cpp:182 / BDPT.hpp:124), standard_1280x960 (Scene.hpp:19-20's
                        default frame: integer aspect 1, splat index ix + height*iy,
                        SceneRenderingHelper.cpp:17, :50).  Each: closest hits, PT 1/16 spp
                        and BDPT 4 spp per-pixel replay (+ splats, bounces), PT-indirect
                        4 spp, and a real Renderer::Render frame (PT 4 spp -j8, BDPT 1 spp -j1)
                        as 8x8 block means

    python tests/golden/make_golden.py indirect   # only pt_indirect.npz
    python tests/golden/make_golden.py edge       # only edge_<case>.npz
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from oracle_bind import Reference, ref_available  # noqa: E402

PRESETS = ("silver", "standard", "refractive_ball", "occlusion", "smooth_dielectric", "bunny")
W = H = 784


def f32(x):
    return np.float32(x)


def rough(s):
    r = (f32(1.0) - f32(s)) * (f32(1.0) - f32(s))
    return max(f32(0.002), r)


# {type, ior_d, ior_m(3), ior_m_k(3), kd(3), rough} -- main.cpp:52-81
DEF_M = [0.131, 0.55758, 1.4561]
DEF_K = [4.0624, 2.2039, 1.9541]
MATERIALS = {
    "white": [0, 1.5] + DEF_M + DEF_K + [0.725, 0.71, 0.68, rough(0.1)],
    "white_smooth": [0, 1.5] + DEF_M + DEF_K + [0.725, 0.71, 0.68, rough(0.7)],
    "light": [0, 1.5] + DEF_M + DEF_K + [0.65, 0.65, 0.65, 0.2],
    "silver": [1, 1.5, 0.041, 0.53285, 0.049317, 4.8025, 3.4101, 2.8545, 0.5, 0.5, 0.5, rough(1.0)],
    "copper": [1, 1.5, 0.211, 1.2174, 1.2493, 4.1592, 2.5978, 2.4771, 0.5, 0.5, 0.5, rough(0.7)],
    "glass": [2, 1.5] + DEF_M + DEF_K + [0.5, 0.5, 0.5, rough(0.9)],
    "glass_rough": [2, 1.33] + DEF_M + DEF_K + [0.5, 0.5, 0.5, 0.3],
}


def unit(rng, n):
    v = rng.normal(size=(n, 3))
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    return v.astype(np.float32)


def material_cases(rng, n):
    wo, nn, wi = unit(rng, n), unit(rng, n), unit(rng, n)
    # half the cases: w_o on the normal's side, a quarter: axis-aligned normals
    flip = (np.sum(wo * nn, 1) < 0) & (rng.random(n) < 0.5)
    wo[flip] *= -1
    ax = rng.random(n) < 0.25
    nn[ax] = np.array([0, 1, 0], np.float32)
    seeds = rng.integers(1, 2**31 - 1, size=n).astype(np.uint32)
    cases = np.zeros((n, 10), np.float32)
    cases[:, 0:3], cases[:, 3:6], cases[:, 6:9] = wo, nn, wi
    cases[:, 9] = seeds.view(np.float32)
    return cases


def pixel_set(seed, n, w=W, h=H):
    rng = np.random.default_rng(seed)
    return np.sort(rng.choice(w * h, n, replace=False)).astype(np.int64)


def ray_set(rng, n):
    eye = np.array([278, 278, -800], np.float32)
    o = np.empty((n, 3), np.float32)
    d = np.empty((n, 3), np.float32)
    k = n // 2
    o[:k] = eye
    tgt = rng.uniform([0, 0, 0], [556, 548.8, 559.2], size=(k, 3)).astype(np.float32)
    d[:k] = tgt - eye
    o[k:] = rng.uniform([1, 1, 1], [555, 548, 558], size=(n - k, 3)).astype(np.float32)
    d[k:] = unit(rng, n - k)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return np.concatenate([o, d.astype(np.float32)], 1).astype(np.float32)


# name -> (preset, width, height)
EDGE = {"multi_light": ("multi_light", 784, 784), "emissive_sphere": ("emissive_sphere", 784, 784),
        "background": ("background", 784, 784), "standard_1280x960": ("standard", 1280, 960)}


def light_rays(rng, n):
    """Rays from inside the box toward the ceiling-light plane (y = 548.7) over all
    three light quads, two of which overlap (light.obj / light3.obj): tie order."""
    o = rng.uniform([20, 20, 20], [540, 500, 540], size=(n, 3)).astype(np.float32)
    t = np.stack([rng.uniform(10, 500, n), np.full(n, 548.7), rng.uniform(227, 332, n)], 1).astype(np.float32)
    d = t - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return np.concatenate([o, d.astype(np.float32)], 1).astype(np.float32)


def blocks(img, b=8):
    h, w = img.shape[:2]
    return img.reshape(h // b, b, w // b, b, 3).astype(np.float64).mean((1, 3)).astype(np.float32)


def edge():
    rng = np.random.default_rng(20261016)
    for k, (name, (p, w, h)) in enumerate(EDGE.items()):
        R = Reference(p, w, h)
        out = {"width": np.int32(w), "height": np.int32(h)}
        rays = np.concatenate([ray_set(rng, 1536), light_rays(rng, 512)])
        out["rays"] = rays
        out["hits"] = np.stack([R.intersect(rays, c) for c in (0, 1, 2)])
        pix = pixel_set(300 + k, 2048, w, h)
        out["pix"] = pix
        out["pt1"], _, _ = R.trace_pixels(0, 1, pix)
        out["pt16"], _, _ = R.trace_pixels(0, 16, pix)
        bpix = pix[::8]
        out["bpix"] = bpix
        bd4, splat, bounces = R.trace_pixels(1, 4, bpix, want_splat=True)
        nz = np.nonzero(splat.reshape(-1))[0].astype(np.int64)
        out["bdpt4"], out["bdpt4_bounces"] = bd4, bounces
        out["splat_idx"], out["splat_val"] = nz, splat.reshape(-1)[nz]
        out["pti4"], _, out["pti4_bounces"] = R.trace_pixels(2, 4, pix[::4])
        out["pt4_blocks"] = blocks(R.render(0, 4, threads=8))
        out["bdpt1_blocks"] = blocks(R.render(1, 1, threads=1))
        np.savez_compressed(os.path.join(HERE, "edge_%s.npz" % name), **out)
        print("edge", name, "done", flush=True)


def indirect():
    out = {}
    for p in PRESETS:
        R = Reference(p)
        pix = pixel_set(101 + PRESETS.index(p), 1024)
        out[p + "_pix"] = pix
        out[p + "_spp1"], _, out[p + "_spp1_bounces"] = R.trace_pixels(2, 1, pix)
        out[p + "_spp8"], _, out[p + "_spp8_bounces"] = R.trace_pixels(2, 8, pix)
    np.savez_compressed(os.path.join(HERE, "pt_indirect.npz"), **out)
    print("pt_indirect done", flush=True)


def main():
    if not ref_available():
        sys.exit("oracle/_ref/libref.so missing: run oracle/build_ref.sh first")
    if sys.argv[1:] == ["indirect"]:
        return indirect()
    if sys.argv[1:] == ["edge"]:
        return edge()
    rng = np.random.default_rng(20261015)
    R = Reference("standard")

    seeds = np.array([1, 2, 3, 392 * 784 + 392 + 1, 614656, 0x7fffffff], np.uint32)
    us, fs = zip(*[R.rng(int(s), 4096) for s in seeds])
    np.savez_compressed(os.path.join(HERE, "rng.npz"), seeds=seeds, u32=np.stack(us), f=np.stack(fs))

    names = sorted(MATERIALS)
    mats = np.array([MATERIALS[k] for k in names], np.float32)
    cases = material_cases(rng, 1024)
    outs = np.stack([R.material_kat(m, cases) for m in mats])
    np.savez_compressed(os.path.join(HERE, "kat_material.npz"), names=np.array(names), mats=mats, cases=cases, out=outs)

    hc = np.zeros((2048, 8), np.float32)
    hc[:, 0:3], hc[:, 3:6] = unit(rng, 2048), unit(rng, 2048)
    hc[:512, 0:3] = np.round(hc[:512, 0:3])  # axis-aligned / zero components (AnyPerpendicular branches)
    hc[:, 6] = rng.uniform(-2, 2, 2048)
    hc[:, 7] = rng.uniform(-2, 2, 2048)
    np.savez_compressed(os.path.join(HERE, "kat_helpers.npz"), cases=hc, out=R.helper_kat(hc))

    for p in PRESETS:
        R = Reference(p)
        rays = ray_set(rng, 2048)
        hits = np.stack([R.intersect(rays, c) for c in (0, 1, 2)])
        np.savez_compressed(os.path.join(HERE, "intersect_%s.npz" % p), rays=rays, hits=hits)
        pix = pixel_set(7 + PRESETS.index(p), 2048)
        pt1, _, _ = R.trace_pixels(0, 1, pix)
        pt16, _, _ = R.trace_pixels(0, 16, pix)
        bpix = pix[::8]
        bd4, splat, bounces = R.trace_pixels(1, 4, bpix, want_splat=True)
        nz = np.nonzero(splat.reshape(-1))[0].astype(np.int64)
        np.savez_compressed(os.path.join(HERE, "pixels_%s.npz" % p), pix=pix, pt1=pt1, pt16=pt16, bpix=bpix,
                            bdpt4=bd4, bdpt4_bounces=bounces, splat_idx=nz, splat_val=splat.reshape(-1)[nz])
        print("preset", p, "done", flush=True)

    R = Reference("standard")
    img_pt = R.render(0, 16, threads=8)
    img_bd = R.render(1, 2, threads=1)

    def blocks(img):
        return img.reshape(H // 8, 8, W // 8, 8, 3).astype(np.float64).mean((1, 3)).astype(np.float32)

    np.savez_compressed(os.path.join(HERE, "image_standard.npz"), pt16_blocks=blocks(img_pt),
                        pt16_crop=img_pt[360:424, 360:424], bdpt2_blocks=blocks(img_bd),
                        bdpt2_crop=img_bd[360:424, 360:424], crop_origin=np.array([360, 360]))
    indirect()
    edge()
    print("done")


if __name__ == "__main__":
    main()
