"""Diagnostics on the GPU box (round 2): emissive_sphere closest-hit mismatches and
non-finite values in the bunny BDPT 4096-spp frame."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "toypathtracer-games101-assignment7_amd")]
import pytpt  # noqa: E402
from conftest import bits, golden  # noqa: E402
from oracle_bind import Oracle  # noqa: E402

np.set_printoptions(precision=9, linewidth=200)
g = golden("edge_emissive_sphere.npz")
c = pytpt.Context(0)
c.upload(pytpt.Preset("emissive_sphere"))
o = Oracle("emissive_sphere")
for cull in range(3):
    got = c.intersect(g["rays"], cull)
    want = g["hits"][cull]
    bad = np.nonzero(np.any(bits(got) != bits(want), axis=1))[0]
    print("cull", cull, "mismatching rays", len(bad), bad[:20])
    for k in bad[:6]:
        print(" ray", g["rays"][k])
        print("  gpu ", got[k])
        print("  ref ", want[k])
        print("  orc ", o.intersect(g["rays"][k:k + 1], cull)[0])
sys.stdout.flush()

c.upload(pytpt.Preset("bunny"))
spp = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
rgb, splat, st = c.render(spp, pytpt.MODE_BDPT)
for name, a in (("rgb", rgb), ("splat", splat)):
    nf = ~np.isfinite(a.reshape(-1, 3)).all(1)
    idx = np.nonzero(nf)[0]
    print(name, "non-finite pixels", len(idx), idx[:20], a.reshape(-1, 3)[idx[:5]])
sys.stdout.flush()
# bisect the pixels whose splats are non-finite: render pixel lists, check the splat
W = 784
if not np.isfinite(splat).all():
    lo = np.arange(W * W, dtype=np.int64)
    while len(lo) > 1:
        half = lo[: len(lo) // 2]
        _, s, _ = c.render_pixels(spp, pytpt.MODE_BDPT, half)
        lo = half if not np.isfinite(s).all() else lo[len(lo) // 2:]
        print("bisect", len(lo), flush=True)
    p = lo
    r, s, _ = c.render_pixels(spp, pytpt.MODE_BDPT, p)
    print("culprit pixel", p, "rgb", r, "splat non-finite at", np.nonzero(~np.isfinite(s.reshape(-1)))[0][:10])
    orr, os_, _ = o.trace_pixels(1, spp, p, want_splat=True)
    print("oracle rgb", orr, "oracle splat non-finite at", np.nonzero(~np.isfinite(os_.reshape(-1)))[0][:10],
          "values", os_.reshape(-1)[~np.isfinite(os_.reshape(-1))][:6])
bad = np.nonzero(~np.isfinite(rgb.reshape(-1, 3)).all(1))[0]
if len(bad):
    p = bad[:4].astype(np.int64)
    print("rgb culprits", p, rgb.reshape(-1, 3)[p])
    print("oracle", o.trace_pixels(1, spp, p)[0])
