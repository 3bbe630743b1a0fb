import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "toypathtracer-games101-assignment7_amd")
for p in (os.path.join(ROOT, "tests"), PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")
PRESETS = ("silver", "standard", "refractive_ball", "occlusion", "smooth_dielectric", "bunny")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP path)")


def golden(name):
    import numpy as np
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def bits(a):
    import numpy as np
    return np.ascontiguousarray(a, np.float32).view(np.uint32)
