"""SURVEY.md §8(d) algorithmic bytes per sample from the oracle's traversal counts.

    python scripts/b_alg.py [scene ...]

B_alg = nodes popped x 32 B + triangle tests x 48 B per sample, counted over every
pixel of the 784x784 frame at 1 spp (the reference traversal, oracle/tpt_oracle.cpp).
The values feed bench.py's B_ALG table.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle_bind import Oracle  # noqa: E402

scenes = sys.argv[1:] or ["standard", "refractive_ball", "bunny", "smooth_dielectric", "silver"]
pix = np.arange(0, 784 * 784, dtype=np.int64)
for sc in scenes:
    o = Oracle(sc)
    for mode, name in ((0, "pt"), (1, "bdpt")):
        nodes, tris = o.traversal_counts(mode, 1, pix)
        n = len(pix)
        print("%-18s %-4s nodes/sample %7.2f tris/sample %6.2f B_alg %6d" % (
            sc, name, nodes / n, tris / n, round((nodes * 32 + tris * 48) / n)), flush=True)
