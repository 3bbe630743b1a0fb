"""pytpt -- ctypes binding of libtpt.so (include/tpt.h, include/tpt_host.h).

This is how Python (tests, bench.py, __graft_entry__) drives the HIP path.  It is
the same binding a maintainer would add to call the library from any FFI (see
INTEGRATION.md).  There is no CPU fallback: if libtpt.so is missing or a call
fails, an exception is raised.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TPT_LIB") or os.path.join(HERE, "libtpt.so")  # TPT_LIB: profiling A/B only
MODELS_DIR = os.path.join(HERE, "models")
ABI_VERSION = 2  # TPT_ABI_VERSION of include/tpt.h

TPT_OK = 0
TPT_E_INVALID = -1
TPT_E_DEVICE = -2
TPT_E_NOSCENE = -3
TPT_E_ALLOC = -4
TPT_E_UNSUPPORTED = -5
MODE_PT, MODE_BDPT = 0, 1
MODE_PT_INDIRECT = 2  # PathTrace without the HEAD `break` (PathTracer.cpp:109); off by default
FLAG_SAMPLE_SEED = 1  # per-sample seeding (tpt.h TPT_FLAG_SAMPLE_SEED): a non-replay throughput mode
CULL_BACK, CULL_FRONT, NO_CULL = 0, 1, 2
PRESETS = ("silver", "standard", "refractive_ball", "occlusion", "smooth_dielectric", "bunny")
EDGE_PRESETS = ("multi_light", "emissive_sphere", "background")


class Material(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int32), ("emission", ctypes.c_float * 3), ("ior_d", ctypes.c_float),
                ("ior_m", ctypes.c_float * 3), ("ior_m_k", ctypes.c_float * 3), ("kd", ctypes.c_float * 3),
                ("rough", ctypes.c_float)]


class Object(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("material", ctypes.c_int32), ("first_triangle", ctypes.c_int32),
                ("num_triangles", ctypes.c_int32), ("center", ctypes.c_float * 3), ("radius", ctypes.c_float)]


class SceneDesc(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32), ("eye", ctypes.c_float * 3),
                ("background", ctypes.c_float * 3), ("fov", ctypes.c_double),
                ("num_materials", ctypes.c_int32), ("materials", ctypes.POINTER(Material)),
                ("num_objects", ctypes.c_int32), ("objects", ctypes.POINTER(Object)),
                ("num_vertices", ctypes.c_int64), ("vertices", ctypes.POINTER(ctypes.c_float))]


class RenderParams(ctypes.Structure):
    _fields_ = [("spp", ctypes.c_int32), ("mode", ctypes.c_int32), ("pixel_begin", ctypes.c_int64),
                ("pixel_stride", ctypes.c_int64), ("flags", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class Stats(ctypes.Structure):
    _fields_ = [("pixels", ctypes.c_int64), ("samples", ctypes.c_int64), ("bounces", ctypes.c_int64),
                ("kernel_ms", ctypes.c_double), ("total_ms", ctypes.c_double),
                ("nonfinite", ctypes.c_int64), ("nonfinite_splat", ctypes.c_int64)]


# Every symbol declared in include/tpt.h and include/tpt_host.h.
EXPORTS = ("tpt_create", "tpt_destroy", "tpt_last_error", "tpt_abi_version", "tpt_hip_versions",
           "tpt_upload_scene", "tpt_render",
           "tpt_render_pixels", "tpt_render_device", "tpt_intersect", "tpt_camera_scale", "tpt_sample_seed",
           "tpt_multi_create", "tpt_multi_destroy", "tpt_multi_last_error", "tpt_multi_upload_scene",
           "tpt_render_multi",
           "tpt_preset_load", "tpt_preset_desc", "tpt_preset_free", "tpt_save_image")

_lib = None


def lib():
    """Load libtpt.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError("libtpt.so not built (run `make -C %s` or __graft_entry__.build())" % HERE)
    # One HIP runtime per process: torch ships its own libamdhip64 and ROCr.  Loaded
    # after libtpt had pulled in /opt/rocm's, torch finds no GPU ("No HIP GPUs are
    # available") and RCCL cannot initialise; loaded first, libtpt binds to torch's
    # runtime (same soname).  So torch, where installed, is loaded before libtpt.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    P = ctypes.c_void_p
    L.tpt_create.argtypes = [ctypes.c_int, ctypes.POINTER(P)]
    L.tpt_destroy.argtypes = [P]
    L.tpt_destroy.restype = None
    L.tpt_last_error.argtypes = [P]
    L.tpt_last_error.restype = ctypes.c_char_p
    L.tpt_upload_scene.argtypes = [P, ctypes.POINTER(SceneDesc)]
    L.tpt_render.argtypes = [P, ctypes.POINTER(RenderParams), P, P, ctypes.POINTER(Stats)]
    L.tpt_render_device.argtypes = [P, ctypes.POINTER(RenderParams), P, P, ctypes.POINTER(Stats)]
    L.tpt_render_pixels.argtypes = [P, ctypes.c_int32, ctypes.c_int32, P, ctypes.c_int64, P, P,
                                    ctypes.POINTER(Stats)]
    L.tpt_intersect.argtypes = [P, P, ctypes.c_int64, ctypes.c_int32, P]
    L.tpt_camera_scale.argtypes = [ctypes.c_double]
    L.tpt_camera_scale.restype = ctypes.c_float
    L.tpt_sample_seed.argtypes = [ctypes.c_int64, ctypes.c_int32]
    L.tpt_sample_seed.restype = ctypes.c_uint32
    L.tpt_preset_load.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int32, ctypes.c_int32,
                                  ctypes.POINTER(P)]
    L.tpt_preset_desc.argtypes = [P]
    L.tpt_preset_desc.restype = ctypes.POINTER(SceneDesc)
    L.tpt_preset_free.argtypes = [P]
    L.tpt_preset_free.restype = None
    L.tpt_save_image.argtypes = [P, ctypes.c_int32, ctypes.c_int32, ctypes.c_char_p]
    L.tpt_multi_create.argtypes = [ctypes.c_int, P, ctypes.POINTER(P)]
    L.tpt_multi_destroy.argtypes = [P]
    L.tpt_multi_destroy.restype = None
    L.tpt_multi_last_error.argtypes = [P]
    L.tpt_multi_last_error.restype = ctypes.c_char_p
    L.tpt_multi_upload_scene.argtypes = [P, ctypes.POINTER(SceneDesc)]
    L.tpt_render_multi.argtypes = [P, ctypes.POINTER(RenderParams), P, P, ctypes.POINTER(Stats)]
    if L.tpt_abi_version() != ABI_VERSION:  # Stats is ABI 2's layout (include/tpt.h)
        raise RuntimeError("%s has ABI %d, pytpt expects %d" % (LIB_PATH, L.tpt_abi_version(), ABI_VERSION))
    L.tpt_hip_versions.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
    L.tpt_hip_versions.restype = None
    _lib = L
    return L


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


class Preset:
    """One of the reference's hard-coded scenes, built by the C++ host mirror."""

    def __init__(self, name, width=784, height=784, models_dir=MODELS_DIR):
        h = ctypes.c_void_p()
        rc = lib().tpt_preset_load(models_dir.encode(), name.encode(), width, height, ctypes.byref(h))
        if rc != TPT_OK:
            raise ValueError("unknown preset or missing models: %s" % name)
        self.handle = h
        self.name = name
        self.width, self.height = width, height

    @property
    def desc(self):
        return lib().tpt_preset_desc(self.handle)

    def __del__(self):
        if getattr(self, "handle", None) and _lib is not None:
            _lib.tpt_preset_free(self.handle)
            self.handle = None


class TptError(RuntimeError):
    pass


def hip_versions():
    """(HIP_VERSION libtpt was compiled against, the loaded runtime's; -1 if unknown).
    Call after a context exists: reading the runtime's version initialises HIP."""
    c, r = ctypes.c_int(0), ctypes.c_int(0)
    lib().tpt_hip_versions(ctypes.byref(c), ctypes.byref(r))
    return c.value, r.value


class Context:
    """A libtpt context on one HIP device."""

    def __init__(self, device=0):
        h = ctypes.c_void_p()
        rc = lib().tpt_create(device, ctypes.byref(h))
        if rc != TPT_OK:
            raise TptError("tpt_create(%d) failed: %d" % (device, rc))
        self.h = h
        self.width = self.height = 0
        self.hip_versions = hip_versions()
        comp, run = self.hip_versions
        if run >= 0 and run // 10000000 != comp // 10000000:
            import warnings
            warnings.warn("libtpt was compiled against HIP %d but runs on HIP runtime %d (another libamdhip64 "
                          "was loaded first)" % (comp, run), RuntimeWarning)

    def _check(self, rc, what):
        if rc != TPT_OK:
            raise TptError("%s failed (%d): %s" % (what, rc, lib().tpt_last_error(self.h).decode()))

    def upload(self, preset_or_desc):
        desc = preset_or_desc.desc if isinstance(preset_or_desc, Preset) else preset_or_desc
        self._check(lib().tpt_upload_scene(self.h, desc), "tpt_upload_scene")
        self.width, self.height = desc.contents.width, desc.contents.height
        self._keep = preset_or_desc

    def render(self, spp, mode=MODE_PT, begin=0, stride=1, flags=0):
        n = self.width * self.height * 3
        rgb = np.zeros(n, np.float32)
        splat = np.zeros(n, np.float32) if mode == MODE_BDPT else None
        p = RenderParams(spp, mode, begin, stride, flags, 0)
        st = Stats()
        self._check(lib().tpt_render(self.h, ctypes.byref(p), _ptr(rgb), _ptr(splat), ctypes.byref(st)),
                    "tpt_render")
        rgb = rgb.reshape(self.height, self.width, 3)
        if splat is not None:
            splat = splat.reshape(self.height, self.width, 3)
        return rgb, splat, st

    def render_device(self, spp, mode, rgb_dev_ptr, splat_dev_ptr, begin=0, stride=1, flags=0):
        p = RenderParams(spp, mode, begin, stride, flags, 0)
        st = Stats()
        self._check(lib().tpt_render_device(self.h, ctypes.byref(p), ctypes.c_void_p(rgb_dev_ptr),
                                            ctypes.c_void_p(splat_dev_ptr) if splat_dev_ptr else None,
                                            ctypes.byref(st)), "tpt_render_device")
        return st

    def render_pixels(self, spp, mode, pixels):
        pixels = np.ascontiguousarray(pixels, dtype=np.int64)
        rgb = np.zeros((len(pixels), 3), np.float32)
        splat = np.zeros(self.width * self.height * 3, np.float32) if mode == MODE_BDPT else None
        st = Stats()
        self._check(lib().tpt_render_pixels(self.h, spp, mode, _ptr(pixels), len(pixels), _ptr(rgb), _ptr(splat),
                                            ctypes.byref(st)), "tpt_render_pixels")
        if splat is not None:
            splat = splat.reshape(self.height, self.width, 3)
        return rgb, splat, st

    def intersect(self, rays, cull=CULL_BACK):
        rays = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 6)
        out = np.zeros((len(rays), 8), np.float32)
        self._check(lib().tpt_intersect(self.h, _ptr(rays), len(rays), cull, _ptr(out)), "tpt_intersect")
        return out

    def close(self):
        if self.h:
            lib().tpt_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Multi:
    """tpt_multi: one frame over several GPUs of this process (pixel shards + one RCCL
    reduce onto the first device; Renderer.cpp:86-114 across devices)."""

    def __init__(self, devices):
        devs = np.ascontiguousarray(devices, np.int32)
        h = ctypes.c_void_p()
        rc = lib().tpt_multi_create(len(devs), _ptr(devs), ctypes.byref(h))
        if rc != TPT_OK:
            raise TptError("tpt_multi_create(%s) failed: %d" % (list(devs), rc))
        self.h = h
        self.width = self.height = 0
        self.hip_versions = hip_versions()
        comp, run = self.hip_versions
        if run >= 0 and run // 10000000 != comp // 10000000:
            import warnings
            warnings.warn("libtpt was compiled against HIP %d but runs on HIP runtime %d (another libamdhip64 "
                          "was loaded first)" % (comp, run), RuntimeWarning)

    def _check(self, rc, what):
        if rc != TPT_OK:
            raise TptError("%s failed (%d): %s" % (what, rc, lib().tpt_multi_last_error(self.h).decode()))

    def upload(self, preset_or_desc):
        desc = preset_or_desc.desc if isinstance(preset_or_desc, Preset) else preset_or_desc
        self._check(lib().tpt_multi_upload_scene(self.h, desc), "tpt_multi_upload_scene")
        self.width, self.height = desc.contents.width, desc.contents.height
        self._keep = preset_or_desc

    def render(self, spp, mode=MODE_PT):
        n = self.width * self.height * 3
        rgb = np.zeros(n, np.float32)
        splat = np.zeros(n, np.float32) if mode == MODE_BDPT else None
        p = RenderParams(spp, mode, 0, 1, 0, 0)
        st = Stats()
        self._check(lib().tpt_render_multi(self.h, ctypes.byref(p), _ptr(rgb), _ptr(splat), ctypes.byref(st)),
                    "tpt_render_multi")
        rgb = rgb.reshape(self.height, self.width, 3)
        if splat is not None:
            splat = splat.reshape(self.height, self.width, 3)
        return rgb, splat, st

    def close(self):
        if self.h:
            lib().tpt_multi_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def save_image(rgb, path):
    rgb = np.ascontiguousarray(rgb, dtype=np.float32)
    h, w = rgb.shape[:2]
    rc = lib().tpt_save_image(_ptr(rgb), w, h, path.encode())
    if rc != TPT_OK:
        raise TptError("tpt_save_image failed")
