"""PT's shadow-cone masks change no bit.

pt_cone_mask (csrc/tpt_device.h) lets PT's two shadow queries skip
every flat leaf whose box cannot meet conv(emitters' box ∪ {the pixel's camera hit}),
grown by a rounding margin.  TPT_FLAT bit 8 (read at upload) turns the masks off; full
PT frames with and without them must be bit-identical -- on the presets with occluders
(occlusion: a blocker under the light), several emitters, a sphere emitter, glass, and on
scenes built here with a small box whose corner lies ON the boundary of that hull (on the
segment from a floor point to a corner of the emitters' box: tangent to the cone of the
pixels around that point), for a mesh emitter and a sphere emitter."""
import ctypes

import numpy as np
import pytest

import pytpt
from conftest import bits

pytestmark = pytest.mark.gpu

SPP = 32


def _frame(desc_or_preset, flat):
    import os
    old = os.environ.get("TPT_FLAT")
    os.environ["TPT_FLAT"] = str(flat)
    c = pytpt.Context(0)
    try:
        c.upload(desc_or_preset)
        rgb, _, st = c.render(SPP, pytpt.MODE_PT)
    finally:
        c.close()
        if old is None:
            del os.environ["TPT_FLAT"]
        else:
            os.environ["TPT_FLAT"] = old
    return rgb, st


class Scene:
    """A preset's scene plus extra mesh objects (kept alive with the desc)."""

    def __init__(self, preset, extra_tris, material):
        d = preset.desc.contents
        nm, no, nv = d.num_materials, d.num_objects, d.num_vertices
        self.mats = (pytpt.Material * nm)(*[d.materials[i] for i in range(nm)])
        verts = np.ctypeslib.as_array(d.vertices, shape=(nv * 3,)).copy()
        objs = [d.objects[i] for i in range(no)]
        first = nv // 3
        extra = np.asarray(extra_tris, np.float32).reshape(-1)
        o = pytpt.Object()
        o.kind, o.material, o.first_triangle, o.num_triangles = 0, material, first, len(extra) // 9
        objs.append(o)
        self.objs = (pytpt.Object * len(objs))(*objs)
        self.verts = np.ascontiguousarray(np.concatenate([verts, extra]), np.float32)
        self.d = pytpt.SceneDesc()
        self.d.width, self.d.height = d.width, d.height
        self.d.eye[:] = list(d.eye)
        self.d.background[:] = list(d.background)
        self.d.fov = d.fov
        self.d.num_materials, self.d.materials = nm, self.mats
        self.d.num_objects, self.d.objects = len(objs), self.objs
        self.d.num_vertices = len(self.verts) // 3
        self.d.vertices = self.verts.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
        self.desc = ctypes.pointer(self.d)
        self.preset = preset


def _box(lo, hi):
    """12 triangles of an axis-aligned box (outward-facing)."""
    x0, y0, z0 = lo
    x1, y1, z1 = hi
    v = [(x0, y0, z0), (x1, y0, z0), (x1, y1, z0), (x0, y1, z0), (x0, y0, z1), (x1, y0, z1), (x1, y1, z1), (x0, y1, z1)]
    quads = [(0, 3, 2, 1), (4, 5, 6, 7), (0, 1, 5, 4), (3, 7, 6, 2), (0, 4, 7, 3), (1, 2, 6, 5)]
    out = []
    for a, b, c, e in quads:
        out += [v[a], v[b], v[c], v[a], v[c], v[e]]
    return out


def _emitter_box(preset, obj):
    d = preset.desc.contents
    o = d.objects[obj]
    if o.kind == 1:  # sphere
        c, r = np.array(o.center[:], np.float64), float(o.radius)
        return c - r, c + r
    v = np.ctypeslib.as_array(d.vertices, shape=(d.num_vertices * 3,)).reshape(-1, 3)
    t = v[3 * o.first_triangle: 3 * (o.first_triangle + o.num_triangles)]
    return t.min(0).astype(np.float64), t.max(0).astype(np.float64)


@pytest.mark.parametrize("preset", ["standard", "occlusion", "multi_light", "emissive_sphere", "refractive_ball"])
def test_cone_masks_change_nothing_on_presets(preset):
    p = pytpt.Preset(preset)
    a, sa = _frame(p, 3)
    b, sb = _frame(p, 3 | 8)
    assert np.array_equal(bits(a), bits(b)), "%s: frames differ with / without the shadow-cone masks" % preset


@pytest.mark.parametrize("preset,emitter", [("standard", 5), ("emissive_sphere", 5)])
def test_cone_masks_change_nothing_with_a_tangent_blocker(preset, emitter):
    p = pytpt.Preset(preset)
    lo, hi = _emitter_box(p, emitter)  # standard: light.obj; emissive_sphere: the glowing ball
    for x in ((278.0, 0.5, 280.0), (150.0, 0.5, 120.0), (420.0, 0.5, 400.0)):
        x = np.array(x)
        for corner in ((lo[0], lo[1], lo[2]), (hi[0], lo[1], hi[2]), (lo[0], lo[1], hi[2])):
            c = np.array(corner)
            q = x + 0.5 * (c - x)  # on the segment x -> corner: the hull's boundary near x
            out = np.sign(q - 0.5 * (lo + hi))  # away from the emitters' centre
            tip = q + 12.0 * out
            box_lo, box_hi = np.minimum(q, tip), np.maximum(q, tip)
            sc = Scene(p, _box(box_lo, box_hi), material=2)
            a, _ = _frame(sc.desc, 3)
            b, _ = _frame(sc.desc, 3 | 8)
            assert np.array_equal(bits(a), bits(b)), "%s, blocker at %s: frames differ" % (preset, q)
