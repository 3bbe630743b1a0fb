"""Render one frame with two library builds (TPT_LIB) and compare them pixel by pixel.
    python scripts/diag/cmp_libs.py LIB_A LIB_B [preset] [mode] [spp]   (LIB "default" = in-tree)"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CHILD = r'''
import sys, numpy as np
sys.path.insert(0, %r)
import pytpt
c = pytpt.Context(0)
c.upload(pytpt.Preset(sys.argv[1]))
rgb, splat, st = c.render(int(sys.argv[3]), pytpt.MODE_BDPT if sys.argv[2] == "bdpt" else pytpt.MODE_PT)
np.save(sys.argv[4], rgb)
c.close()
''' % os.path.join(ROOT, "toypathtracer-games101-assignment7_amd")


def run(lib, preset, mode, spp, out):
    env = dict(os.environ)
    if lib != "default":
        env["TPT_LIB"] = lib
    subprocess.run([sys.executable, "-c", CHILD, preset, mode, str(spp), out], env=env, check=True, timeout=120)
    return np.load(out)


def main():
    a, b = sys.argv[1], sys.argv[2]
    preset = sys.argv[3] if len(sys.argv) > 3 else "bunny"
    mode = sys.argv[4] if len(sys.argv) > 4 else "bdpt"
    spp = int(sys.argv[5]) if len(sys.argv) > 5 else 4
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    fa = run(a, preset, mode, spp, os.path.join(ROOT, "gpurun_out", "cmp_a.npy"))
    fb = run(b, preset, mode, spp, os.path.join(ROOT, "gpurun_out", "cmp_b.npy"))
    ra, rb = fa.reshape(-1, 3).view(np.uint32), fb.reshape(-1, 3).view(np.uint32)
    diff = np.nonzero((ra != rb).any(1))[0]
    print("pixels %d differing %d" % (len(ra), len(diff)))
    if len(diff):
        fa2, fb2 = fa.reshape(-1, 3), fb.reshape(-1, 3)
        print("first", diff[:10].tolist())
        print("a", fa2[diff[:5]].tolist())
        print("b", fb2[diff[:5]].tolist())
        d = np.abs(fa2[diff] - fb2[diff])
        print("sum a %.6g b %.6g  max|d| %.3g" % (np.nansum(fa2), np.nansum(fb2), np.nanmax(d)))


if __name__ == "__main__":
    main()
