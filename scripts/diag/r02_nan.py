"""Round-2 diagnostic: the bunny BDPT pixel whose 4096-spp radiance is NaN on the GPU."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "toypathtracer-games101-assignment7_amd")]
import pytpt  # noqa: E402
from oracle_bind import Oracle  # noqa: E402

np.set_printoptions(precision=9, linewidth=200)
pix = np.array([int(sys.argv[1]) if len(sys.argv) > 1 else 485594], np.int64)
o = Oracle("bunny")


def ctx(**env):
    for k in ("TPT_BDPT_KERNEL", "TPT_FLAT"):
        os.environ.pop(k, None)
    os.environ.update(env)
    c = pytpt.Context(0)
    c.upload(pytpt.Preset("bunny"))
    return c


c = ctx()
lo, hi = 1, 4096
assert not np.isfinite(c.render_pixels(hi, pytpt.MODE_BDPT, pix)[0]).all()
while lo < hi:
    mid = (lo + hi) // 2
    if np.isfinite(c.render_pixels(mid, pytpt.MODE_BDPT, pix)[0]).all():
        lo = mid + 1
    else:
        hi = mid
spp = lo
print("first spp with NaN:", spp, flush=True)
for s in (spp - 1, spp):
    print("spp", s, "wavefront", c.render_pixels(s, pytpt.MODE_BDPT, pix)[0], "oracle", o.trace_pixels(1, s, pix)[0])
for env in ({"TPT_BDPT_KERNEL": "mono"}, {"TPT_FLAT": "0"}, {"TPT_BDPT_KERNEL": "mono", "TPT_FLAT": "0"}):
    c2 = ctx(**env)
    print(env, "spp", spp, c2.render_pixels(spp, pytpt.MODE_BDPT, pix)[0], flush=True)
    c2.close()
