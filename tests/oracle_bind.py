"""ctypes bindings of the TEST-ONLY oracles (never the product path):

  oracle/liboracle.so   CPU restatement of the reference hot path (oracle/tpt_oracle.cpp)
  oracle/_ref/libref.so the reference itself, compiled in place by oracle/build_ref.sh
                        (present only where it was built; travels to the GPU box)
"""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "liboracle.so")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libref.so")
MODELS = os.path.join(ROOT, "toypathtracer-games101-assignment7_amd", "models")
P = ctypes.c_void_p


def _p(a):
    return P(a.ctypes.data) if a is not None else None


class Oracle:
    """CPU restatement (oracle/tpt_oracle.cpp)."""

    def __init__(self, preset=None, width=784, height=784, desc=None):
        if not os.path.exists(ORACLE_SO):
            raise RuntimeError("oracle/liboracle.so not built (make -C oracle)")
        L = ctypes.CDLL(ORACLE_SO)
        L.oracle_preset.restype = P
        L.oracle_preset.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int]
        L.oracle_create.restype = P
        L.oracle_create.argtypes = [P]
        L.oracle_destroy.argtypes = [P]
        L.oracle_trace_pixels.argtypes = [P, ctypes.c_int, ctypes.c_int, P, ctypes.c_int64, P, P, P]
        L.oracle_trace_pixels_seeded.argtypes = [P, ctypes.c_int, ctypes.c_int, P, ctypes.c_int64, ctypes.c_int, P, P]
        L.oracle_sample_seed.argtypes = [ctypes.c_int64, ctypes.c_int32]
        L.oracle_sample_seed.restype = ctypes.c_uint32
        L.oracle_render.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int64, P]
        L.oracle_render.restype = ctypes.c_double
        L.oracle_rng.argtypes = [ctypes.c_uint32, ctypes.c_int, P, P]
        L.oracle_traversal_counts.argtypes = [P, ctypes.c_int, ctypes.c_int, P, ctypes.c_int64, P]
        L.oracle_intersect.argtypes = [P, P, ctypes.c_int64, ctypes.c_int, P]
        L.oracle_material_kat.argtypes = [P, P, ctypes.c_int, P]
        L.oracle_helper_kat.argtypes = [P, ctypes.c_int, P]
        L.oracle_camera_scale.argtypes = [ctypes.c_double]
        L.oracle_camera_scale.restype = ctypes.c_float
        self.L = L
        self.h = None
        self.width, self.height = width, height
        if preset is not None:
            self.h = L.oracle_preset(MODELS.encode(), preset.encode(), width, height)
            if not self.h:
                raise ValueError(preset)
        elif desc is not None:
            self.h = L.oracle_create(ctypes.cast(desc, P))

    def trace_pixels(self, mode, spp, pix, want_splat=False):
        pix = np.ascontiguousarray(pix, np.int64)
        out = np.zeros((len(pix), 3), np.float32)
        splat = np.zeros(self.width * self.height * 3, np.float32) if want_splat else None
        b = np.zeros(len(pix), np.int64)
        self.L.oracle_trace_pixels(P(self.h), mode, spp, _p(pix), len(pix), _p(out), _p(splat), _p(b))
        return out, (splat.reshape(self.height, self.width, 3) if want_splat else None), b

    def trace_pixels_seeded(self, mode, spp, pix, lanes=1):
        """TPT_FLAG_SAMPLE_SEED restated (oracle_trace_pixels_seeded): PT with lanes=1,
        PT-indirect with the library's TPT_PT_LANES."""
        pix = np.ascontiguousarray(pix, np.int64)
        out = np.zeros((len(pix), 3), np.float32)
        b = np.zeros(len(pix), np.int64)
        self.L.oracle_trace_pixels_seeded(P(self.h), mode, spp, _p(pix), len(pix), lanes, _p(out), _p(b))
        return out, b

    def sample_seed(self, i, j):
        return int(self.L.oracle_sample_seed(ctypes.c_int64(i), ctypes.c_int32(j)))

    def traversal_counts(self, mode, spp, pix):
        """(nodes popped, triangle tests) summed over `pix` x `spp` (SURVEY §8(d) B_alg)."""
        pix = np.ascontiguousarray(pix, np.int64)
        out = np.zeros(2, np.uint64)
        self.L.oracle_traversal_counts(P(self.h), mode, spp, _p(pix), len(pix), _p(out))
        return int(out[0]), int(out[1])

    def render(self, mode, spp, threads=1, pixel_limit=0):
        out = np.zeros(self.width * self.height * 3, np.float32)
        ms = self.L.oracle_render(P(self.h), mode, spp, threads, pixel_limit, _p(out))
        return out.reshape(self.height, self.width, 3), ms

    def intersect(self, rays, cull):
        rays = np.ascontiguousarray(rays, np.float32)
        out = np.zeros((len(rays), 8), np.float32)
        self.L.oracle_intersect(P(self.h), _p(rays), len(rays), cull, _p(out))
        return out

    def rng(self, seed, n):
        u = np.zeros(n, np.uint32)
        f = np.zeros(n, np.float32)
        self.L.oracle_rng(seed, n, _p(u), _p(f))
        return u, f

    def material_kat(self, mat, cases):
        mat = np.ascontiguousarray(mat, np.float32)
        cases = np.ascontiguousarray(cases, np.float32)
        out = np.zeros((len(cases), 17), np.float32)
        self.L.oracle_material_kat(_p(mat), _p(cases), len(cases), _p(out))
        return out

    def helper_kat(self, cases):
        cases = np.ascontiguousarray(cases, np.float32)
        out = np.zeros((len(cases), 16), np.float32)
        self.L.oracle_helper_kat(_p(cases), len(cases), _p(out))
        return out

    def __del__(self):
        if getattr(self, "h", None):
            self.L.oracle_destroy(P(self.h))
            self.h = None


def ref_available():
    return os.path.exists(REF_SO)


class Reference:
    """The reference renderer itself (oracle/_ref/libref.so).  One scene at a time
    (the reference keeps global state: Renderer.cpp:29-30)."""

    _L = None

    def __init__(self, preset, width=784, height=784):
        if Reference._L is None:
            L = ctypes.CDLL(REF_SO)
            L.ref_setup.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int]
            L.ref_render.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, P]
            L.ref_trace_pixels.argtypes = [ctypes.c_int, ctypes.c_int, P, ctypes.c_int, P, P, P]
            L.ref_rng.argtypes = [ctypes.c_uint32, ctypes.c_int, P, P]
            L.ref_intersect.argtypes = [P, ctypes.c_int, ctypes.c_int, P]
            L.ref_material_kat.argtypes = [P, P, ctypes.c_int, P]
            L.ref_helper_kat.argtypes = [P, ctypes.c_int, P]
            L.ref_scale.argtypes = [ctypes.c_float]
            L.ref_scale.restype = ctypes.c_float
            Reference._L = L
        self.L = Reference._L
        self.width, self.height = width, height
        if preset is not None and self.L.ref_setup(MODELS.encode(), preset.encode(), width, height) != 0:
            raise ValueError(preset)

    def trace_pixels(self, mode, spp, pix, want_splat=False):
        pix = np.ascontiguousarray(pix, np.int64)
        out = np.zeros((len(pix), 3), np.float32)
        splat = np.zeros(self.width * self.height * 3, np.float32) if want_splat else None
        b = np.zeros(len(pix), np.int64)
        self.L.ref_trace_pixels(mode, spp, _p(pix), len(pix), _p(out), _p(splat), _p(b))
        return out, (splat.reshape(self.height, self.width, 3) if want_splat else None), b

    def render(self, mode, spp, threads=1):
        out = np.zeros(self.width * self.height * 3, np.float32)
        self.L.ref_render(spp, threads, mode, _p(out))
        return out.reshape(self.height, self.width, 3)

    def intersect(self, rays, cull):
        rays = np.ascontiguousarray(rays, np.float32)
        out = np.zeros((len(rays), 8), np.float32)
        self.L.ref_intersect(_p(rays), len(rays), cull, _p(out))
        return out

    def rng(self, seed, n):
        u = np.zeros(n, np.uint32)
        f = np.zeros(n, np.float32)
        self.L.ref_rng(seed, n, _p(u), _p(f))
        return u, f

    def material_kat(self, mat, cases):
        mat = np.ascontiguousarray(mat, np.float32)
        cases = np.ascontiguousarray(cases, np.float32)
        out = np.zeros((len(cases), 17), np.float32)
        self.L.ref_material_kat(_p(mat), _p(cases), len(cases), _p(out))
        return out

    def helper_kat(self, cases):
        cases = np.ascontiguousarray(cases, np.float32)
        out = np.zeros((len(cases), 16), np.float32)
        self.L.ref_helper_kat(_p(cases), len(cases), _p(out))
        return out
