"""Pin the CPU restatement (oracle/tpt_oracle.cpp) against the reference.

1. against the committed golden fixtures (made by tests/golden/make_golden.py from
   the REAL reference build, oracle/_ref) -- bit-exact;
2. live against oracle/_ref/libref.so on fresh inputs, where that library exists.
"""
import numpy as np
import pytest

from conftest import EDGE, PRESETS, bits, blocks, golden
from oracle_bind import Oracle, Reference, ref_available


def eq_bits(a, b):
    return np.array_equal(bits(a), bits(b))


def test_rng_stream():
    g = golden("rng.npz")
    o = Oracle("standard")
    for k, s in enumerate(g["seeds"]):
        u, f = o.rng(int(s), g["u32"].shape[1])
        assert np.array_equal(u, g["u32"][k])
        assert eq_bits(f, g["f"][k])
    # known answer quoted in SURVEY.md §8(c): seed 1 -> 268476417, 1157628417, ...
    assert list(g["u32"][0][:4]) == [268476417, 1157628417, 1158709409, 269814307]


def test_material_kat():
    g = golden("kat_material.npz")
    o = Oracle("standard")
    for k, name in enumerate(g["names"]):
        out = o.material_kat(g["mats"][k], g["cases"])
        assert eq_bits(out, g["out"][k]), name


def test_helper_kat():
    g = golden("kat_helpers.npz")
    assert eq_bits(Oracle("standard").helper_kat(g["cases"]), g["out"])


@pytest.mark.parametrize("preset", PRESETS)
def test_intersect(preset):
    g = golden("intersect_%s.npz" % preset)
    o = Oracle(preset)
    for c in range(3):
        assert eq_bits(o.intersect(g["rays"], c), g["hits"][c])


@pytest.mark.parametrize("preset", PRESETS)
def test_pixels_pt(preset):
    g = golden("pixels_%s.npz" % preset)
    o = Oracle(preset)
    assert eq_bits(o.trace_pixels(0, 1, g["pix"])[0], g["pt1"])
    assert eq_bits(o.trace_pixels(0, 16, g["pix"])[0], g["pt16"])


@pytest.mark.parametrize("preset", PRESETS)
def test_pixels_bdpt(preset):
    g = golden("pixels_%s.npz" % preset)
    o = Oracle(preset)
    rgb, splat, b = o.trace_pixels(1, 4, g["bpix"], want_splat=True)
    assert eq_bits(rgb, g["bdpt4"])
    assert np.array_equal(b, g["bdpt4_bounces"])
    flat = splat.reshape(-1)
    assert np.array_equal(np.nonzero(flat)[0], g["splat_idx"])
    assert eq_bits(flat[g["splat_idx"]], g["splat_val"])


def test_full_image_pt():
    g = golden("image_standard.npz")
    img, _ = Oracle("standard").render(0, 16, threads=8)
    blocks = img.reshape(98, 8, 98, 8, 3).astype(np.float64).mean((1, 3)).astype(np.float32)
    assert eq_bits(blocks, g["pt16_blocks"])
    y, x = g["crop_origin"]
    assert eq_bits(img[y:y + 64, x:x + 64], g["pt16_crop"])


def test_full_frame_pins_c1():
    """The whole configs[0] frame (Standard PT 16 spp, 784x784) of the CPU restatement
    against the real Renderer::Render's, pinned by tests/golden/frame_c1.npz
    (make_frames.py): sha256 of every float, so the full-frame pins the GPU tests use
    are themselves checked here."""
    from frames import check_exact
    g = golden("frame_c1.npz")
    img, _ = Oracle("standard").render(0, 16, threads=8)
    check_exact(img, g, "rgb", "oracle PT16 frame")


def test_full_image_bdpt():
    # Renderer::Render with -j1: splat buffers merged after the radiance (Renderer.cpp:98-114)
    g = golden("image_standard.npz")
    img, _ = Oracle("standard").render(1, 2, threads=1)
    blocks = img.reshape(98, 8, 98, 8, 3).astype(np.float64).mean((1, 3)).astype(np.float32)
    assert eq_bits(blocks, g["bdpt2_blocks"])
    y, x = g["crop_origin"]
    assert eq_bits(img[y:y + 64, x:x + 64], g["bdpt2_crop"])


@pytest.mark.skipif(not ref_available(), reason="oracle/_ref/libref.so not built")
@pytest.mark.parametrize("preset", PRESETS)
def test_live_against_reference(preset):
    rng = np.random.default_rng(hash(preset) % 2**32)
    pix = np.sort(rng.choice(784 * 784, 3000, replace=False))
    R, o = Reference(preset), Oracle(preset)
    assert eq_bits(o.trace_pixels(0, 8, pix)[0], R.trace_pixels(0, 8, pix)[0])
    a = o.trace_pixels(1, 2, pix[:400], want_splat=True)
    b = R.trace_pixels(1, 2, pix[:400], want_splat=True)
    assert eq_bits(a[0], b[0]) and eq_bits(a[1], b[1]) and np.array_equal(a[2], b[2])


@pytest.mark.parametrize("preset", PRESETS)
def test_pixels_pt_indirect(preset):
    """TPT_MODE_PT_INDIRECT (PathTrace without the HEAD `break`, PathTracer.cpp:109):
    radiance and outBounces sums against the sed-built reference's fixtures."""
    g = golden("pt_indirect.npz")
    o = Oracle(preset)
    pix = g[preset + "_pix"]
    for spp in (1, 8):
        rgb, _, b = o.trace_pixels(2, spp, pix)
        assert eq_bits(rgb, g["%s_spp%d" % (preset, spp)])
        assert np.array_equal(b, g["%s_spp%d_bounces" % (preset, spp)])


@pytest.mark.skipif(not ref_available(), reason="oracle/_ref/libref.so not built")
@pytest.mark.parametrize("preset", ["standard", "refractive_ball", "silver"])
def test_live_indirect_against_reference(preset):
    rng = np.random.default_rng(17 + len(preset))
    pix = np.sort(rng.choice(784 * 784, 2000, replace=False))
    R, o = Reference(preset), Oracle(preset)
    a, b = o.trace_pixels(2, 8, pix), R.trace_pixels(2, 8, pix)
    assert eq_bits(a[0], b[0]) and np.array_equal(a[2], b[2])


def test_traversal_counts_b_alg():
    """bench.py's B_ALG (nodes x 32 B + triangle tests x 48 B per sample)
    against the oracle's traversal counters on every 7th pixel of the Standard frame."""
    import bench
    o = Oracle("standard")
    pix = np.arange(0, 784 * 784, 7, dtype=np.int64)
    for mode, name in ((0, "pt"), (1, "bdpt")):
        nodes, tris = o.traversal_counts(mode, 1, pix)
        b = (nodes * 32 + tris * 48) / len(pix)
        assert abs(b / bench.B_ALG[("standard", name)] - 1) < 0.01, (name, b)


@pytest.mark.parametrize("name", sorted(EDGE))
def test_edge_cases(name):
    """The reference's edge cases (golden edge_<name>.npz): several emitters with
    coplanar overlapping quads, a sphere as emitter 0, a non-zero background, the
    default 1280x960 frame.  Closest hits, PT / BDPT / PT-indirect per-pixel replay,
    splats and bounce counts, and a full PT frame -- all bit-exact."""
    g = golden("edge_%s.npz" % name)
    p, w, h = EDGE[name]
    o = Oracle(p, w, h)
    for c in range(3):
        assert eq_bits(o.intersect(g["rays"], c), g["hits"][c]), c
    assert eq_bits(o.trace_pixels(0, 1, g["pix"])[0], g["pt1"])
    assert eq_bits(o.trace_pixels(0, 16, g["pix"])[0], g["pt16"])
    rgb, splat, b = o.trace_pixels(1, 4, g["bpix"], want_splat=True)
    assert eq_bits(rgb, g["bdpt4"]) and np.array_equal(b, g["bdpt4_bounces"])
    flat = splat.reshape(-1)
    assert np.array_equal(np.nonzero(flat)[0], g["splat_idx"])
    assert eq_bits(flat[g["splat_idx"]], g["splat_val"])
    rgb, _, b = o.trace_pixels(2, 4, g["pix"][::4])
    assert eq_bits(rgb, g["pti4"]) and np.array_equal(b, g["pti4_bounces"])
    img, _ = o.render(0, 4, threads=8)
    assert eq_bits(blocks(img), g["pt4_blocks"])


def test_edge_full_frame_bdpt_1280x960():
    """Renderer::Render's BDPT frame at 1280x960 (-j1): radiance plus splats that land
    at the reference's `ix + height*iy` (SceneRenderingHelper.cpp:50)."""
    g = golden("edge_standard_1280x960.npz")
    img, _ = Oracle("standard", 1280, 960).render(1, 1, threads=1)
    assert eq_bits(blocks(img), g["bdpt1_blocks"])


def test_frame_c5_crop_pixels_match_oracle():
    """tests/golden/frame_c5.npz (configs[4], the bunny scene at its own 4096 spp, made by
    the real reference's per-pixel route) against the CPU restatement on 12 pixels of
    its full-resolution crops: the radiance bit for bit.  Bounded sample: ~1 s of
    BDPT at 4096 spp per pixel on one core."""
    import os
    from conftest import GOLDEN
    if not os.path.exists(os.path.join(GOLDEN, "frame_c5.npz")):
        pytest.skip("frame_c5.npz not generated")
    g = golden("frame_c5.npz")
    assert int(g["spp"]) == 4096 and str(g["preset"]) == "bunny"
    rng = np.random.default_rng(7)
    pix, want = [], []
    for ci, (r0, c0) in enumerate(g["crop_origins"]):
        for _ in range(4):
            dy, dx = rng.integers(0, 64, 2)
            pix.append((r0 + dy) * 784 + (c0 + dx))
            want.append(g["rgb_crops"][ci, dy, dx])
    got = Oracle("bunny").trace_pixels(1, 4096, np.array(pix, np.int64))[0]
    assert eq_bits(got, np.array(want, np.float32))
