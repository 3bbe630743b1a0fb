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

# reference edge cases (tests/golden/make_golden.py edge): name -> (preset, width, height)
EDGE = {"multi_light": ("multi_light", 784, 784), "emissive_sphere": ("emissive_sphere", 784, 784),
        "background": ("background", 784, 784), "standard_1280x960": ("standard", 1280, 960)}


def blocks(img, b=8):
    import numpy as np
    h, w = img.shape[:2]
    return img.reshape(h // b, b, w // b, b, 3).astype(np.float64).mean((1, 3)).astype(np.float32)
