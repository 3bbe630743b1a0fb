// tpt_device.h -- gfx950 device code of the hot path: BVH traversal, primitive
// tests, GGX/Lambert/Fresnel BSDF, light sampling, the PT sample and the BDPT
// sample.  Every function cites the reference code it reproduces; arithmetic
// follows the numerics contract of tpt_devmath.h (kernels are built with
// -ffp-contract=off).
//
// Memory model: the scene (tpt_scene.h) is staged in LDS when it fits (the Cornell
// presets, a few KB) and read through L1/L2 otherwise (the bunny mesh, <1 MB); ray
// queries are stackless (flat all-leaves loops or threaded-tree walks).
#pragma once

#include <hip/hip_runtime.h>

#include "../../include/tpt.h"
#include "tpt_devmath.h"
#include "tpt_scene.h"

namespace tpt {

#define TPT_D __device__ __forceinline__
// tpt_conn2.hip compiles tpt_capi.hip's walk-scene connect kernel alone (TPT_TU_CONN2): its
// device globals get internal linkage there, so the two objects link side by side
#if defined(TPT_TU_CONN2) && TPT_TU_CONN2
#define TPT_TU_STATIC static
#else
#define TPT_TU_STATIC
#endif

constexpr int kBlock = 256;     // threads per workgroup (4 waves)
// ------------------------------------------------------------------ rays --
struct Ray {
    V3 o, d, inv;
};
// Ray.hpp:12-15 computes float(1.0 / (double)d).  A single correctly rounded
// operation on floats carried out in double and rounded to float equals the
// correctly rounded float operation (double rounding is innocuous since
// 53 >= 2*24 + 2), so the exact f32 divide is used.
#ifndef TPT_FAST_RCP
#define TPT_FAST_RCP 1
#endif
TPT_D Ray make_ray(V3 o, V3 d) {
    Ray r;
    r.o = o;
    r.d = d;
#if TPT_FAST_RCP && !defined(TPT_HOST_EMU)
    // rcp_fast_f32 equals the IEEE quotient on its range (tpt_devmath.h); a wave with a
    // component outside it (0, denormal, huge: rare) divides.  (The host emulation of
    // tests/native/wave_emu.h divides: both forms give the same bits, and its waves do not
    // model a ballot reached by only some lanes, as owner_ray's call in walk4_steal is.)
    if (__ballot(!(rcp_fast_ok(d.x) & rcp_fast_ok(d.y) & rcp_fast_ok(d.z))) == 0) {
        r.inv = v3(rcp_fast_f32(d.x), rcp_fast_f32(d.y), rcp_fast_f32(d.z));
        return r;
    }
#endif
    r.inv = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    return r;
}

struct Hit {
    double dist;
    int prim;  // -1: no hit
};

// Bounds3::IntersectP (Bounds3.hpp:92-115): nmin starts at FLT_MIN, std::max /
// std::min ignore a NaN second argument, hit iff nmax > 0 && nmin <= nmax.
TPT_D bool slab_hit(float x0, float y0, float z0, float x1, float y1, float z1, const Ray& r) {
    float nmin = 1.17549435e-38f, nmax = 3.40282347e+38f;
    {
        float t1 = (x0 - r.o.x) * r.inv.x, t2 = (x1 - r.o.x) * r.inv.x;
        if (t1 > t2) { float t = t1; t1 = t2; t2 = t; }
        nmin = smax(nmin, t1); nmax = smin(nmax, t2);
    }
    {
        float t1 = (y0 - r.o.y) * r.inv.y, t2 = (y1 - r.o.y) * r.inv.y;
        if (t1 > t2) { float t = t1; t1 = t2; t2 = t; }
        nmin = smax(nmin, t1); nmax = smin(nmax, t2);
    }
    {
        float t1 = (z0 - r.o.z) * r.inv.z, t2 = (z1 - r.o.z) * r.inv.z;
        if (t1 > t2) { float t = t1; t1 = t2; t2 = t; }
        nmin = smax(nmin, t1); nmax = smin(nmax, t2);
    }
    return (nmax > 0.0f) & (nmin <= nmax);
}
TPT_D bool box_hit(const DNode& n, const Ray& r) {
    return slab_hit(n.bmin[0], n.bmin[1], n.bmin[2], n.bmax[0], n.bmax[1], n.bmax[2], r);
}
// slab_hit for a ray with finite inv (ray_monotone): (b - o) * inv is then never
// NaN, so std::max/std::min equal the hardware max/min and the swap is a min/max
// pair (a +-0 difference cannot change `nmax > 0` or `nmin <= nmax`).  Same
// decision as slab_hit, half the instructions.
TPT_D bool slab_hit_finite(float x0, float y0, float z0, float x1, float y1, float z1, const Ray& r) {
    const float ax = (x0 - r.o.x) * r.inv.x, bx = (x1 - r.o.x) * r.inv.x;
    const float ay = (y0 - r.o.y) * r.inv.y, by = (y1 - r.o.y) * r.inv.y;
    const float az = (z0 - r.o.z) * r.inv.z, bz = (z1 - r.o.z) * r.inv.z;
    const float nmin = fmaxf(fmaxf(1.17549435e-38f, fminf(ax, bx)), fmaxf(fminf(ay, by), fminf(az, bz)));
    const float nmax = fminf(fminf(3.40282347e+38f, fmaxf(ax, bx)), fminf(fmaxf(ay, by), fmaxf(az, bz)));
    return (nmax > 0.0f) & (nmin <= nmax);
}
// kFin: every ray of the (sub)wave has a finite inv (wave_finite), so the NaN-free
// form gives the same decision.
template <bool kFin>
TPT_D bool box_hit_t(const DNode& n, const Ray& r) {
    return kFin ? slab_hit_finite(n.bmin[0], n.bmin[1], n.bmin[2], n.bmax[0], n.bmax[1], n.bmax[2], r)
                : slab_hit(n.bmin[0], n.bmin[1], n.bmin[2], n.bmax[0], n.bmax[1], n.bmax[2], r);
}

// The slab test (Bounds3::IntersectP) is monotone in the box bounds -- fl(b - o) and
// fl(x * inv) are monotone in b and std::max / std::min preserve order -- unless a
// direction component is +-0 or tiny enough that 1/d overflows: with inv = -inf a
// box flat at o.x passes while a box [o.x, o.x + w] does not.  Rays with an infinite
// inv component are walked on the threaded tree instead.
TPT_D bool ray_monotone(const Ray& r) {
    const float inf = 3.40282347e+38f;
    return fabs_(r.inv.x) <= inf && fabs_(r.inv.y) <= inf && fabs_(r.inv.z) <= inf;
}
// True when every active lane's ray has a finite inv: the walk can then use the
// NaN-free slab test (wave-uniform, so the choice costs no divergence).
TPT_D bool wave_finite(const Ray& r) { return __ballot(!ray_monotone(r)) == 0; }

TPT_D V3 tri_normal(const DTri& t) { return v3(t.nx, t.ny, t.nz); }

#ifndef TPT_TRI_BF
#define TPT_TRI_BF 1  // tri_test's form in the per-lane walks and per-leaf loops (see below)
#endif
#ifndef TPT_TRI_BF_C
#define TPT_TRI_BF_C 2  // ... and in the dense rounds of the compacted flat queries
#endif
// Triangle::GetIntersection (Triangle.cpp:77-118): culling on the f64 sign of
// dot(d, n), then f64 Moller-Trumbore with |det| < EPSILON(1e-4f) rejection.
// Every rejection returns the same `false` and every quantity is a pure function of
// the ray and the triangle, so the tests may be evaluated in any order.
template <int kBF>
TPT_D bool tri_test_t(const DTri t, const Ray& r, int cull, double& dist) {  // by value: all 48 B load up front
    V3 n = tri_normal(t);
    if (kBF < 2) {
        if (cull == TPT_CULL_BACK) {
            if (dot3(r.d, n) > 0) return false;
        } else if (cull == TPT_CULL_FRONT) {
            if (dot3(r.d, n) < 0) return false;
        }
    }
    V3 e1 = v3(t.e1[0], t.e1[1], t.e1[2]), e2 = v3(t.e2[0], t.e2[1], t.e2[2]);
    V3 pvec = cross(r.d, e2);
    double det = dot3(e1, pvec);
    if (kBF < 2 && dabs_(det) < (double)1e-4f) return false;
    V3 tvec = r.o - v3(t.v0[0], t.v0[1], t.v0[2]);
    const double ua = dot3(tvec, pvec);
    V3 qvec = cross(tvec, e1);
    const double vb = dot3(r.d, qvec);
    double det_inv = 1. / det;
    double u = ua * det_inv;
    if (kBF == 0) {
        if (u < 0 || u > 1) return false;
        double v = vb * det_inv;
        if (v < 0 || u + v > 1) return false;
        double tt = dot3(e2, qvec) * det_inv;
        if (tt < 0.0f) return false;
        dist = tt;
        return true;
    }
    // kBF >= 1: one predicate, the same comparisons (NaN passes each of them, as above);
    // kBF == 2 folds the culling and |det| tests into it too (no branch at all)
    const double v = vb * det_inv;
    const double tt = dot3(e2, qvec) * det_inv;
    bool rej = (u < 0) | (u > 1) | (v < 0) | (u + v > 1) | (tt < 0.0f);
    if (kBF >= 2) {
        const double dn = dot3(r.d, n);
        rej = rej | (dabs_(det) < (double)1e-4f) | ((cull == TPT_CULL_BACK) & (dn > 0)) |
              ((cull == TPT_CULL_FRONT) & (dn < 0));
    }
    dist = tt;
    return !rej;
}
TPT_D bool tri_test(const DTri t, const Ray& r, int cull, double& dist) { return tri_test_t<TPT_TRI_BF>(t, r, cull, dist); }

// SolveQuadratic (SampleHelperFunctions.cpp:4-18), float parameters.
TPT_D bool solve_quadratic(float a, float b, float c, float& x0, float& x1) {
    double discr = (double)b * b - 4.0 * a * c;
    if (discr < 0) return false;
    if (discr == 0) {
        x0 = x1 = (float)(-0.5 * b / a);
    } else {
        float q = (b > 0) ? (float)(-0.5 * (b + sqrt_d(discr))) : (float)(-0.5 * (b - sqrt_d(discr)));
        x0 = q / a;
        x1 = c / q;
    }
    if (x0 > x1) { float t = x0; x0 = x1; x1 = t; }
    return true;
}
// Sphere::GetIntersection (Sphere.cpp:4-41)
TPT_D bool sphere_test(const DSphere& s, const Ray& r, int cull, double& dist) {
    V3 L = r.o - v3(s.c[0], s.c[1], s.c[2]);
    double a = dot3(r.d, r.d);
    double b = 2.0 * dot3(r.d, L);
    double c = dot3(L, L) - s.r2;
    float t0, t1;
    if (!solve_quadratic((float)a, (float)b, (float)c, t0, t1)) return false;
    float tk;
    if (cull == TPT_CULL_BACK) tk = t0;
    else if (cull == TPT_CULL_FRONT) tk = t1;
    else tk = t0 <= 0 ? t1 : t0;
    if (tk > 0.0f) { dist = tk; return true; }
    return false;
}

// BVHAccel::Intersect (BVH.cpp:103-143) from `root`, both levels spliced
// (tpt_scene.h).  Same pop order (right child first), strict `>` on the f64
// distance, so ties resolve exactly as in the reference.
template <bool kFin>
TPT_D Hit traverse_t(const DScene& s, int root, const Ray& r, int cull) {
    // stackless walk of the threaded tree (tpt_scene.h): one node fetch per step
    Hit best;
    best.prim = -1;
    best.dist = 0.0;
    int cur = root, cont = kWalkEnd;
    while (cur >= 0) {
        const DNode n = s.tnodes[cur];
        int nxt = n.b;
        if (box_hit_t<kFin>(n, r)) {
            if (n.a >= 0) {
                if (n.a & kSpliceBit) {  // entering a mesh: resume at n.b when it is done
                    cont = n.b;
                    nxt = n.a & ~kSpliceBit;
                } else {
                    nxt = n.a;
                }
            } else if (n.a != kEmptyLeaf) {
                const int prim = -1 - n.a;
                double dist;
                bool h;
                if (prim < s.ntri) h = tri_test(s.tris[prim], r, cull, dist);
                else h = sphere_test(s.sph[prim - s.ntri], r, cull, dist);
                if (h && (best.prim < 0 || best.dist > dist)) {
                    best.dist = dist;
                    best.prim = prim;
                }
            }
        }
        cur = nxt == kMeshExit ? cont : nxt;
    }
    return best;
}
// ---- flat queries: every primitive leaf box, no interior nodes ----------------
// For a ray with finite inv the slab test is monotone in the box bounds (see
// ray_monotone) and every interior box is the union of its children's
// (BVH.cpp:58-98), so a leaf's box passing implies every ancestor's box passes: the
// primitives the reference tests are exactly those whose own leaf box passes.
// Testing all leaf boxes in the reference's DFS leaf order (HostScene::leaves)
// therefore visits the same primitives in the same relative order -- the same
// closest hit, ties included (strict `>`), and the same any-hit answer.  The leaf
// index is wave-uniform: no divergence in the loop, the primitive test runs only
// when some lane's box passed.  For scenes with few leaves (the Cornell presets: 32
// triangles) this beats a per-lane walk; rays with an infinite inv component keep
// the walk.
enum { kFlatShadow = 1, kFlatHit = 2, kFlatCompactAll = 4, kFlatNoCone = 8 };  // DScene::flat bits (4: tests force the
// compacted form; 8: tests turn PT's shadow-cone masks off, pt_cone_mask)
// A walk group (groups[g].b < 0) is a mesh too large for the flat list (the bunny):
// a lane whose ray passed the group box -- the mesh root's box, tpt_scene.h -- walks
// the mesh's threaded subtree from the root's right child (a) until kMeshExit, i.e.
// exactly the reference's DFS below that box, at the group's place in the leaf
// order.  Nodes and triangles come through L2 (s.tnodes / s.tris).
TPT_D void walk_group_closest(const DScene& s, int cur, const Ray& r, int cull, Hit& best) {
    while (cur >= 0) {
        const DNode n = s.tnodes[cur];
        int nxt = n.b;
        if (box_hit_t<true>(n, r)) {
            if (n.a >= 0) {
                nxt = n.a;
            } else if (n.a != kEmptyLeaf) {
                const int prim = -1 - n.a;
                double dist;
                if (tri_test(s.tris[prim], r, cull, dist) && (best.prim < 0 || best.dist > dist)) {
                    best.dist = dist;
                    best.prim = prim;
                }
            }
        }
        cur = nxt;
    }
}
TPT_D bool walk_group_shadow(const DScene& s, int cur, const Ray& r, V3 lc, double thr, int cull) {
    while (cur >= 0) {
        const DNode n = s.tnodes[cur];
        int nxt = n.b;
        if (box_hit_t<true>(n, r)) {
            if (n.a >= 0) {
                nxt = n.a;
            } else if (n.a != kEmptyLeaf) {
                double dist;
                if (tri_test(s.tris[-1 - n.a], r, cull, dist)) {
                    const V3 hx = r.o + mul(r.d, (float)dist);
                    if (dot3(hx - lc, hx - lc) < thr) return true;
                }
            }
        }
        cur = nxt;
    }
    return false;
}
// The same walk on the group's 4-wide tree (tpt_scene.h QNode4), for lanes with a
// per-lane LDS stack (s.ws; the BDPT kernels).  A QNode's four entry boxes are tested
// at once from one 128-B record, so a ray descends two binary levels per dependent
// fetch.  Passing entries are visited in entry order -- the first at once, the others
// from the stack -- and a leaf entry is tested when its turn comes, so the triangles
// reached and their order are the binary walk's (the skipped binary boxes enclose the
// entries' boxes; slab monotonicity, finite inv): closest-hit ties resolve the same.
// A QNode4's box rows and entry codes as 16-B vector loads: a by-value copy of the
// struct came out as a dwordx3 + dword pair per row (13 VMEM instructions per node;
// the vector memory pipeline serves a divergent load per lane address, whatever its
// width), this is 7.
TPT_D QNode4 load_qnode(const QNode4* p) {
    const float4* v = reinterpret_cast<const float4*>(p);
    QNode4 n;
    static_assert(kWalkW == 4, "load_qnode reads 4-entry rows");
    const float4 r0 = v[0], r1 = v[1], r2 = v[2], r3 = v[3], r4 = v[4], r5 = v[5], r6 = v[6];
    const float4 rows[6] = {r0, r1, r2, r3, r4, r5};
    for (int a = 0; a < 3; ++a) {
        n.bmin[a][0] = rows[a].x; n.bmin[a][1] = rows[a].y; n.bmin[a][2] = rows[a].z; n.bmin[a][3] = rows[a].w;
        n.bmax[a][0] = rows[3 + a].x; n.bmax[a][1] = rows[3 + a].y; n.bmax[a][2] = rows[3 + a].z; n.bmax[a][3] = rows[3 + a].w;
    }
    n.e[0] = __builtin_bit_cast(int32_t, r6.x); n.e[1] = __builtin_bit_cast(int32_t, r6.y);
    n.e[2] = __builtin_bit_cast(int32_t, r6.z); n.e[3] = __builtin_bit_cast(int32_t, r6.w);
    return n;
}
// A walk group's triangle from `gtris`, which is never re-pointed to LDS, so the
// compiler emits global loads; through `tris` (LDS in small scenes) they were flat
// loads, which also count against lgkmcnt, so the walk's LDS stack reads waited on them.
TPT_D DTri load_gtri(const DTri* p) {
    const float4* v = reinterpret_cast<const float4*>(p);
    const float4 a = v[0], b = v[1], c = v[2];
    DTri t;
    t.v0[0] = a.x; t.v0[1] = a.y; t.v0[2] = a.z; t.nx = a.w;
    t.e1[0] = b.x; t.e1[1] = b.y; t.e1[2] = b.z; t.ny = b.w;
    t.e2[0] = c.x; t.e2[1] = c.y; t.e2[2] = c.z; t.nz = c.w;
    return t;
}
template <bool kShadow>
TPT_D bool walk4(const DScene& s, int q, const Ray& r, int cull, Hit& best, V3 lc, double thr, int* iters = nullptr) {
    uint16_t* st = s.ws + threadIdx.x;  // [slot][lane]
    int sp = 0;
    int cur = q;
    for (;;) {
        if (iters) ++*iters;
        // a leaf: its triangle test (BVHAccel::Intersect's strict `>` fold, or the
        // shadow answer), then the next entry -- in the same step, so a lane does one
        // triangle and one QNode per step and the two kinds of work do not alternate
        if (cur < 0) {
            const int prim = -1 - cur;
            double dist;
            if (tri_test(load_gtri(s.gtris + prim), r, cull, dist)) {
                if (kShadow) {
                    const V3 hx = r.o + mul(r.d, (float)dist);
                    if (dot3(hx - lc, hx - lc) < thr) return true;
                } else if (best.prim < 0 || best.dist > dist) {
                    best.dist = dist;
                    best.prim = prim;
                }
            }
            if (sp == 0) break;
            cur = (int)(int16_t)st[kBlock * --sp];
        }
        if (cur >= 0) {
            const QNode4 n = load_qnode(s.qnodes + cur);
            int held = kQNone;
            for (int j = kWalkW - 1; j >= 0; --j) {
                const bool pass = n.e[j] != kQNone && slab_hit_finite(n.bmin[0][j], n.bmin[1][j], n.bmin[2][j],
                                                                      n.bmax[0][j], n.bmax[1][j], n.bmax[2][j], r);
                if (pass) {
                    if (held != kQNone) st[kBlock * sp++] = (uint16_t)held;
                    held = n.e[j];
                }
            }
            if (held != kQNone) {
                cur = held;
            } else {
                if (sp == 0) break;
                cur = (int)(int16_t)st[kBlock * --sp];
            }
        }
    }
    return false;
}
// A walk group's closest hit / shadow answer: the 4-wide walk where the group has a
// 4-wide tree and the kernel gave its lanes stacks, else the threaded binary walk.
// (`iters`: diagnostics builds count the lane's walk steps.)
#ifndef TPT_WALK4
#define TPT_WALK4 1
#endif
TPT_D void group_closest(const DScene& s, const DNode& gn, const Ray& r, int cull, Hit& best, int* iters = nullptr) {
    if (TPT_WALK4 && gn.b <= -2 && s.ws) walk4<false>(s, -2 - gn.b, r, cull, best, r.o, 0.0, iters);
    else walk_group_closest(s, gn.a, r, cull, best);
}
TPT_D bool group_shadow(const DScene& s, const DNode& gn, const Ray& r, V3 lc, double thr, int cull) {
    Hit unused;
    if (TPT_WALK4 && gn.b <= -2 && s.ws) return walk4<true>(s, -2 - gn.b, r, cull, unused, lc, thr);
    return walk_group_shadow(s, gn.a, r, lc, thr, cull);
}
// Objects are tested first (their box is the union of their leaves' boxes, so a
// failed object box means every leaf box of it fails): a wave skips the leaves of an
// object no lane's ray reaches.
TPT_D Hit traverse_flat(const DScene& s, const Ray& r, int cull) {
    Hit best;
    best.prim = -1;
    best.dist = 0.0;
    for (int gi = 0; gi < s.ngroup; ++gi) {
        const DNode gn = s.groups[gi];
        const bool pass = slab_hit_finite(gn.bmin[0], gn.bmin[1], gn.bmin[2], gn.bmax[0], gn.bmax[1], gn.bmax[2], r);
        if (__ballot(pass) == 0) continue;
        if (s.big && gn.b < 0) {
            if (pass) group_closest(s, gn, r, cull, best);
            continue;
        }
        const int j1 = gn.a + gn.b;
        for (int j = gn.a; j < j1; ++j) {
            const DNode n = s.leaves[j];
            if (slab_hit_finite(n.bmin[0], n.bmin[1], n.bmin[2], n.bmax[0], n.bmax[1], n.bmax[2], r)) {
                const int prim = -1 - n.a;
                double dist;
                bool h;
                if (prim < s.ntri) h = tri_test(s.ftris[n.b], r, cull, dist);
                else h = sphere_test(s.sph[prim - s.ntri], r, cull, dist);
                if (h && (best.prim < 0 || best.dist > dist)) {
                    best.dist = dist;
                    best.prim = prim;
                }
            }
        }
    }
    return best;
}
// Any hit with |hit - lc|^2 < thr over all leaves (see shadow_pts for why any-hit is exact).
// `wm` (wave-uniform): the flat leaves that can hold a counting hit for every active
// lane's query (PT's shadow-cone mask, pt_cone_mask); the others are skipped untested.
TPT_D bool shadow_flat(const DScene& s, const Ray& r, V3 lc, double thr, int cull, uint64_t wm = ~0ull) {
    bool sh = false;
    for (int gi = 0; gi < s.ngroup; ++gi) {
        const DNode gn = s.groups[gi];
        if (!(s.big && gn.b < 0)) {  // a flat group: skip it whole when none of its leaves is a candidate
            const uint64_t gbits = (gn.b >= 64 ? ~0ull : (1ull << gn.b) - 1) << gn.a;
            if ((wm & gbits) == 0) continue;
        }
        const bool pass =
            !sh && slab_hit_finite(gn.bmin[0], gn.bmin[1], gn.bmin[2], gn.bmax[0], gn.bmax[1], gn.bmax[2], r);
        if (__ballot(pass) == 0) continue;
        if (s.big && gn.b < 0) {
            if (pass) sh = group_shadow(s, gn, r, lc, thr, cull);
            continue;
        }
        const int j1 = gn.a + gn.b;
        for (int j = gn.a; j < j1; ++j) {
            if (!((wm >> j) & 1)) continue;
            const DNode n = s.leaves[j];
            if (!sh && slab_hit_finite(n.bmin[0], n.bmin[1], n.bmin[2], n.bmax[0], n.bmax[1], n.bmax[2], r)) {
                const int prim = -1 - n.a;
                double dist = 0.0;
                bool h;
                if (prim < s.ntri) h = tri_test(s.ftris[n.b], r, cull, dist);
                else h = sphere_test(s.sph[prim - s.ntri], r, cull, dist);
                if (h) {
                    const V3 hx = r.o + mul(r.d, (float)dist);
                    if (dot3(hx - lc, hx - lc) < thr) sh = true;
                }
            }
        }
    }
    return sh;
}

// ---- compacted flat queries (the BDPT kernels) --------------------------------
// In the loops above a primitive test runs for the whole wave as soon as ONE lane's
// ray passes the leaf box.  Waves of incoherent rays (BDPT's path extensions and
// connections) pass almost every leaf box somewhere in the wave while each ray passes
// only a few: Standard, uniform surface-to-surface rays pass 4.4 of 32 leaf boxes
// per ray but 31.4 per wave of 64, so most lanes of most primitive tests idle.  The
// compacted form splits the query:
//   1. each lane slab-tests the leaves (wave-uniform loop, as above) into a 64-bit
//      mask of the leaves its ray passes (kFlatMaxLeaves = 64);
//   2. the (ray, leaf) pairs are listed in LDS, lane-major and in leaf order within a
//      lane, and dealt densely to the active lanes: a lane takes pair p, fetches the
//      owner's ray with ds_bpermute and runs the same primitive test on it;
//   3. the owner folds its pairs' results in leaf order: the sequential strict-`>`
//      update of BVHAccel::Intersect (BVH.cpp:103-143) for a closest hit, any hit
//      below the threshold for a shadow query.
// Same (ray, primitive) pairs, the same tests on bit-identical operands and, per ray,
// the same order: the result is the flat loop's, bit for bit.  A wave whose rays are
// coherent (few leaves passed, by many lanes each) keeps the per-leaf loop; the
// choice is made per wave and query.
#ifndef TPT_QC
#define TPT_QC 256
#endif
#ifndef TPT_QC_COST
#define TPT_QC_COST 5  // a dense round costs about 5/4 of one wave-wide primitive test
#endif
constexpr int kQC = TPT_QC;  // pair slots per chunk
struct QScratch {         // per wave, in LDS
    uint16_t pair[kQC];   // owner lane | leaf << 6
    double res[kQC];      // closest hit: the pair's nearest distance and primitive (-1: none)
    int32_t prim[kQC];
    uint32_t flag[64];    // shadow query: the owner's ray is blocked
};
#ifndef TPT_QS_SGPR
#define TPT_QS_SGPR 0  // 1: same-box A/B, Standard BDPT 441.0 -> 444.3 ms, bunny 256 spp 917 -> 923 ms
#endif
TPT_D QScratch* wave_qs(const DScene& s) {  // TPT_QS_SGPR: wave index in an SGPR, no per-lane copy of the base
    return reinterpret_cast<QScratch*>(s.qs) + (TPT_QS_SGPR ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : (threadIdx.x >> 6));
}
// LDS writes of some lanes made visible to reads of other lanes of the same wave
TPT_D void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
TPT_D int mbcnt64(uint64_t m) {
    return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}
// Step 1 over the flat groups [g0, g1): `mask` = leaves this lane's ray passes, `any`
// (wave-uniform) = leaves some lane's ray passes.  A leaf box passing implies its
// group box passes (the group box is the union), so `pass &&` changes nothing.
TPT_D void leaf_masks(const DScene& s, int g0, int g1, const Ray& r, bool on, uint64_t& mask, uint64_t& any) {
    mask = 0;
    any = 0;
    for (int gi = g0; gi < g1; ++gi) {
        const DNode gn = s.groups[gi];
        if (s.big && gn.b < 0) continue;  // walk group: handled by the caller
        const bool pass = on && slab_hit_finite(gn.bmin[0], gn.bmin[1], gn.bmin[2], gn.bmax[0], gn.bmax[1], gn.bmax[2], r);
        if (__ballot(pass) == 0) continue;
        const int j1 = gn.a + gn.b;
        for (int j = gn.a; j < j1; ++j) {
            const DNode n = s.leaves[j];
            const bool p = pass && slab_hit_finite(n.bmin[0], n.bmin[1], n.bmin[2], n.bmax[0], n.bmax[1], n.bmax[2], r);
            if (__ballot(p) != 0) any |= 1ull << j;
            if (p) mask |= 1ull << j;
        }
    }
}
// Step 2's plan: this lane's pairs occupy slots [off, off + cnt) of the wave's list
// (exclusive prefix over the active lanes, from ballots of the count's bits, so
// inactive lanes count for nothing); n pairs in all, dealt over the na active lanes.
struct QPlan {
    int off, cnt, n, na, rank;
};
TPT_D QPlan q_plan(uint64_t mask) {
    QPlan q;
    q.cnt = __popcll(mask);
    q.off = 0;
    q.n = 0;
    for (int b = 0; b < 7; ++b) {
        const uint64_t m = __ballot((q.cnt >> b) & 1);
        q.off += mbcnt64(m) << b;
        q.n += __popcll(m) << b;
    }
    const uint64_t act = __ballot(true);
    q.na = __popcll(act);
    q.rank = mbcnt64(act);
    return q;
}
// Dense rounds beat one wave-wide test per passed leaf by a wide margin or not at all.
TPT_D bool q_compact_pays(const DScene& s, const QPlan& q, uint64_t any) {
    const int rounds = (q.n + q.na - 1) / q.na;
    return (s.flat & kFlatCompactAll) || (rounds + 1) * TPT_QC_COST < __popcll(any) * 4;
}
// The primitive test of flat leaf n (as in traverse_flat / shadow_flat).
template <int kBF = TPT_TRI_BF>
TPT_D bool leaf_test(const DScene& s, const DNode& n, const Ray& r, int cull, double& dist) {
    const int prim = -1 - n.a;
    if (prim < s.ntri) return tri_test_t<kBF>(s.ftris[n.b], r, cull, dist);
    return sphere_test(s.sph[prim - s.ntri], r, cull, dist);
}
// Flat leaf n folded into `best` with BVHAccel::Intersect's strict `>` (BVH.cpp:103-143).
template <int kBF = TPT_TRI_BF>
TPT_D void entry_closest(const DScene& s, const DNode& n, const Ray& r, int cull, Hit& best) {
    double dist;
    if (leaf_test<kBF>(s, n, r, cull, dist) && (best.prim < 0 || best.dist > dist)) {
        best.dist = dist;
        best.prim = -1 - n.a;
    }
}
// Shadow answer of flat leaf n (a hit with |hit - r.o|^2 < thr).
template <int kBF = TPT_TRI_BF>
TPT_D bool entry_blocks(const DScene& s, const DNode& n, const Ray& r, double thr, int cull) {
    double dist = 0.0;
    if (!leaf_test<kBF>(s, n, r, cull, dist)) return false;
    const V3 hx = r.o + mul(r.d, (float)dist);
    return dot3(hx - r.o, hx - r.o) < thr;
}

TPT_D V3 shfl3(V3 a, int l) { return v3(__shfl(a.x, l), __shfl(a.y, l), __shfl(a.z, l)); }
// Step 2a for the chunk of slots [c0, c1): each lane writes its pairs that fall in it
// (mw / sw: its leaves and the slot of the next pair still to be listed).
TPT_D void q_list(QScratch* qs, int c0, int c1, int end, uint64_t& mw, int& sw) {
    const int lane = (int)__lane_id();
    while (sw < end && sw < c1) {
        const int j = __builtin_ctzll(mw);
        mw &= mw - 1;
        qs->pair[sw - c0] = (uint16_t)(lane | j << 6);
        ++sw;
    }
    wave_lds_sync();
}

// Closest hit over the flat groups [g0, g1), folded into `best` (which already holds
// the hits of the leaves before g0, in the reference's order).
TPT_D void flat_closest_c(const DScene& s, int g0, int g1, const Ray& r, int cull, Hit& best) {
    uint64_t mask, any;
    leaf_masks(s, g0, g1, r, true, mask, any);
    if (any == 0) return;
    const QPlan q = q_plan(mask);
    if (!q_compact_pays(s, q, any)) {
        for (uint64_t m = any; m != 0; m &= m - 1) {
            const int j = __builtin_ctzll(m);
            if ((mask >> j) & 1) entry_closest(s, s.leaves[j], r, cull, best);
        }
        return;
    }
    QScratch* qs = wave_qs(s);
    uint64_t mw = mask;
    int sw = q.off, sr = q.off;
    const int end = q.off + q.cnt;
    for (int c0 = 0; c0 < q.n; c0 += kQC) {
        const int c1 = c0 + kQC < q.n ? c0 + kQC : q.n;
        q_list(qs, c0, c1, end, mw, sw);
        for (int p0 = 0; p0 < c1 - c0; p0 += q.na) {
            const int p = p0 + q.rank;
            const bool v = p < c1 - c0;
            const int pr = v ? (int)qs->pair[p] : 0;
            const int l = pr & 63;
            Ray rr;
            rr.o = shfl3(r.o, l);
            rr.d = shfl3(r.d, l);
            rr.inv = rr.d;  // not read by the primitive tests
            const int cl = __shfl(cull, l);
            if (v) {
                Hit h;
                h.prim = -1;
                h.dist = 0.0;
                entry_closest<TPT_TRI_BF_C>(s, s.leaves[pr >> 6], rr, cl, h);
                qs->res[p] = h.dist;
                qs->prim[p] = h.prim;
            }
        }
        wave_lds_sync();
        while (sr < end && sr < c1) {  // step 3, in this ray's leaf order
            const double d = qs->res[sr - c0];
            const int pp = qs->prim[sr - c0];
            if (pp >= 0 && (best.prim < 0 || best.dist > d)) {
                best.dist = d;
                best.prim = pp;
            }
            ++sr;
        }
        wave_lds_sync();  // the next chunk reuses the slots
    }
}
// Closest hit over the groups [g0, g1) in the DFS order, folded into `best`: runs of
// flat groups through the compacted query, split at walk groups, which are walked.
TPT_D void closest_groups_c(const DScene& s, int g0, int g1, const Ray& r, int cull, Hit& best) {
    while (g0 < g1) {
        int ge = g0;
        while (ge < g1 && !(s.big && s.groups[ge].b < 0)) ++ge;
        if (ge > g0) flat_closest_c(s, g0, ge, r, cull, best);
        if (ge < g1) {  // a walk group
            const DNode gn = s.groups[ge];
            if (slab_hit_finite(gn.bmin[0], gn.bmin[1], gn.bmin[2], gn.bmax[0], gn.bmax[1], gn.bmax[2], r))
                group_closest(s, gn, r, cull, best);
            ++ge;
        }
        g0 = ge;
    }
}
TPT_D Hit traverse_flat_c(const DScene& s, const Ray& r, int cull) {
    Hit best;
    best.prim = -1;
    best.dist = 0.0;
    closest_groups_c(s, 0, s.ngroup, r, cull, best);
    return best;
}
// Connect's shadow walks with work stealing (TPT_CONN_STEAL; see walk4_steal in
// tpt_bdpt.h for the closest-hit form): lanes of the query whose ray misses the walk
// group's box, or whose walk has ended, walk subtrees from other lanes' stacks with the
// owner's ray.  Any hit below the owner's threshold marks the owner shadowed; its other
// jobs then end.  The answer is the any-hit answer, so the order of the jobs is free.
#ifndef TPT_CONN_STEAL
#define TPT_CONN_STEAL 1  // round 6, with the compiler changes: bunny BDPT 256 spp 609.3-611.7 -> 600.4-601.6 ms
                          // same-box, three interleaved rounds (round 5, before them: no gain)
#endif
#ifndef TPT_CONN_STEAL_CAP
#define TPT_CONN_STEAL_CAP 0  // steals per query round (0: no cap; round 6, bunny BDPT 256 spp: cap 64 / 256 / 1024 /
                              // none 600.5 / 557-559 / 561 / 559 ms same-box; the walks are finite, so stealing ends)
#endif
TPT_D bool walk4_shadow_steal(const DScene& s, int root, bool need, Ray r, double thr, int cl) {
    QScratch* qs = wave_qs(s);
    const int lane = (int)__lane_id();
    float* rv = reinterpret_cast<float*>(qs->res);  // [slot][lane]: o, d, cull, thr (lo, hi)
    uint16_t* blocked = qs->pair;
    uint16_t* st = s.ws + threadIdx.x;
    wave_lds_sync();
    if (need) {
        rv[0 * 64 + lane] = r.o.x; rv[1 * 64 + lane] = r.o.y; rv[2 * 64 + lane] = r.o.z;
        rv[3 * 64 + lane] = r.d.x; rv[4 * 64 + lane] = r.d.y; rv[5 * 64 + lane] = r.d.z;
        rv[6 * 64 + lane] = __int_as_float(cl);
        rv[7 * 64 + lane] = __int_as_float(__double2loint(thr));
        rv[8 * 64 + lane] = __int_as_float(__double2hiint(thr));
    }
    blocked[lane] = 0;
    wave_lds_sync();
    int sb = 0, sp = 0, cur = root, owner = lane, jobs = 0;
    bool job = need;
    for (;;) {
        bool done = job && blocked[owner] != 0;
        if (job && !done) {
            if (cur < 0) {
                double dist;
                if (tri_test(load_gtri(s.gtris + (-1 - cur)), r, cl, dist)) {
                    const V3 hx = r.o + mul(r.d, (float)dist);
                    if (dot3(hx - r.o, hx - r.o) < thr) {
                        blocked[owner] = 1;
                        done = true;
                    }
                }
                if (!done) {
                    if (sp == sb) done = true;
                    else cur = (int)(int16_t)st[kBlock * --sp];
                }
            }
            if (!done && cur >= 0) {
                const QNode4 n = load_qnode(s.qnodes + cur);
                int held = kQNone;
                for (int j = kWalkW - 1; j >= 0; --j) {
                    const bool pass = n.e[j] != kQNone && slab_hit_finite(n.bmin[0][j], n.bmin[1][j], n.bmin[2][j],
                                                                          n.bmax[0][j], n.bmax[1][j], n.bmax[2][j], r);
                    if (pass) {
                        if (held != kQNone) st[kBlock * sp++] = (uint16_t)held;
                        held = n.e[j];
                    }
                }
                if (held != kQNone) cur = held;
                else if (sp == sb) done = true;
                else cur = (int)(int16_t)st[kBlock * --sp];
            }
        }
        if (done) job = false;
        if (__ballot(job) == 0) break;
        const uint64_t vm = __ballot(job && sp > sb);
        const uint64_t im = __ballot(!job);
        int m = __popcll(im) < __popcll(vm) ? __popcll(im) : __popcll(vm);
#if TPT_CONN_STEAL_CAP > 0
        {
            int cap = TPT_CONN_STEAL_CAP;
#if TPT_STEAL_CAP_OPAQUE
            asm volatile("" : "+s"(cap));
#endif
            if (m > cap - jobs) m = cap - jobs;  // a bounded number of steals per query
        }
#else
        (void)jobs;
#endif
        if (m > 0) {
            if (job && sp > sb) {
                const int k = mbcnt64(vm);
                if (k < m) {
                    qs->flag[k] = (uint32_t)st[kBlock * sb] | (uint32_t)owner << 16;
                    ++sb;
                }
            }
            wave_lds_sync();
            if (!job) {
                const int k = mbcnt64(im);
                if (k < m) {
                    const uint32_t mb = qs->flag[k];
                    cur = (int)(int16_t)(mb & 0xffffu);
                    owner = (int)(mb >> 16);
                    r = make_ray(v3(rv[0 * 64 + owner], rv[1 * 64 + owner], rv[2 * 64 + owner]),
                                 v3(rv[3 * 64 + owner], rv[4 * 64 + owner], rv[5 * 64 + owner]));
                    cl = __float_as_int(rv[6 * 64 + owner]);
                    thr = __hiloint2double(__float_as_int(rv[8 * 64 + owner]), __float_as_int(rv[7 * 64 + owner]));
                    job = true;
                    sb = sp = 0;
                }
            }
            jobs += m;
            wave_lds_sync();
        }
    }
    wave_lds_sync();
    const bool sh = need && blocked[lane] != 0;
    wave_lds_sync();
    return sh;
}

// Shadow query (any hit with |hit - r.o|^2 < thr; r.o is the query's lc, see shadow_ray).
TPT_D bool shadow_flat_c(const DScene& s, const Ray& r, double thr, int cull) {
    uint64_t mask, any;
    leaf_masks(s, 0, s.ngroup, r, true, mask, any);
    bool sh = false;
    if (any != 0) {
        const QPlan q = q_plan(mask);
        if (!q_compact_pays(s, q, any)) {
            for (uint64_t m = any; m != 0; m &= m - 1) {
                const int j = __builtin_ctzll(m);
                if (((mask >> j) & 1) && !sh) sh = entry_blocks(s, s.leaves[j], r, thr, cull);
            }
        } else {
            QScratch* qs = wave_qs(s);
            const int lane = (int)__lane_id();
            qs->flag[lane] = 0u;
            uint64_t mw = mask;
            int sw = q.off;
            const int end = q.off + q.cnt;
            for (int c0 = 0; c0 < q.n; c0 += kQC) {
                const int c1 = c0 + kQC < q.n ? c0 + kQC : q.n;
                q_list(qs, c0, c1, end, mw, sw);
                for (int p0 = 0; p0 < c1 - c0; p0 += q.na) {
                    const int p = p0 + q.rank;
                    const bool v = p < c1 - c0;
                    const int pr = v ? (int)qs->pair[p] : 0;
                    const int l = pr & 63;
                    Ray rr;
                    rr.o = shfl3(r.o, l);
                    rr.d = shfl3(r.d, l);
                    rr.inv = rr.d;
                    const int cl = __shfl(cull, l);
                    const double th = __shfl(thr, l);
                    if (v && entry_blocks<TPT_TRI_BF_C>(s, s.leaves[pr >> 6], rr, th, cl)) qs->flag[l] = 1u;
                }
                wave_lds_sync();  // the flags are final / the next chunk reuses the slots
            }
            sh = qs->flag[lane] != 0u;
        }
    }
#ifndef TPT_DIAG_NO_GROUP_SHADOW
#define TPT_DIAG_NO_GROUP_SHADOW 0  // diagnostics builds only (timing attribution; wrong images)
#endif
    for (int gi = 0; s.big && !TPT_DIAG_NO_GROUP_SHADOW && gi < s.ngroup; ++gi) {  // walk groups (any-hit: order is free)
        const DNode gn = s.groups[gi];
        if (gn.b >= 0) continue;
        const bool pass =
            !sh && slab_hit_finite(gn.bmin[0], gn.bmin[1], gn.bmin[2], gn.bmax[0], gn.bmax[1], gn.bmax[2], r);
        if (TPT_CONN_STEAL && gn.b <= -2 && s.ws) {
            if (walk4_shadow_steal(s, -2 - gn.b, pass, r, thr, cull)) sh = true;
        } else if (pass) {
            sh = group_shadow(s, gn, r, r.o, thr, cull);
        }
    }
    return sh;
}

TPT_D Hit traverse(const DScene& s, int root, const Ray& r, int cull) {
    const bool fin = wave_finite(r);
    if (fin && root == 0 && (s.flat & kFlatHit)) return s.qs ? traverse_flat_c(s, r, cull) : traverse_flat(s, r, cull);
    return fin ? traverse_t<true>(s, root, r, cull) : traverse_t<false>(s, root, r, cull);
}

// Intersection fields of a hit (Triangle.cpp:109-114, Sphere.cpp:30-36)
TPT_D void hit_geometry(const DScene& s, const Ray& r, const Hit& h, V3& x, V3& n) {
    if (h.prim < s.ntri) {
        x = r.o + mul(r.d, (float)h.dist);
        n = tri_normal(s.tris[h.prim]);
    } else {
        const DSphere& sp = s.sph[h.prim - s.ntri];
        x = r.o + mul(r.d, (float)h.dist);
        n = normalized(x - v3(sp.c[0], sp.c[1], sp.c[2]));
    }
}
TPT_D int prim_mat(const DScene& s, int prim) {
    return prim < s.ntri ? s.trix[prim].mat : s.sph[prim - s.ntri].mat;
}

// PTVertex (PTVertex.hpp:6-21).  prim = Object* of the reference (-1 = nullptr).
enum { T_BG = 0, T_MID = 1, T_LIGHT = 2, T_CAM = 3 };
struct PTV {
    V3 x, N;
    int type;
    int prim;
};
TPT_D PTV ptv_bg() {
    PTV v;
    v.x = v3s(0.0f);
    v.N = v3s(0.0f);
    v.type = T_BG;
    v.prim = -1;
    return v;
}
// Scene::Intersect (Scene.cpp:21-35)
TPT_D PTV scene_intersect(const DScene& s, const Ray& r, int cull) {
    Hit h = traverse(s, 0, r, cull);
    PTV v = ptv_bg();
    if (h.prim >= 0) {
        hit_geometry(s, r, h, v.x, v.N);
        v.type = T_MID;
        v.prim = h.prim;
    }
    return v;
}
TPT_D int lane_id() { return __lane_id(); }

// Scene::ShadowCheck(Vector3f, Vector3f, FaceCulling) (Scene.cpp:37-48):
// shadowed iff the CLOSEST hit of the ray lc -> x has |hit - lc|^2 < |x - lc|^2 - 1.
// The hit point is lc + float(t)*d rounded per component and its squared distance
// is summed in double: every step is monotone, so d2(t) is non-decreasing in t and
// "closest hit's d2 < thr"  <=>  "some reachable hit's d2 < thr".  Hence an any-hit
// traversal with early exit is exact.  Box tests are the reference's, so the set
// of reachable primitives is unchanged.
template <bool kFin>
TPT_D bool shadow_walk(const DScene& s, const Ray& r, V3 lc, double thr, int cull) {
    int cur = 0, cont = kWalkEnd;
    while (cur >= 0) {
        const DNode n = s.tnodes[cur];
        int nxt = n.b;
        if (box_hit_t<kFin>(n, r)) {
            if (n.a >= 0) {
                if (n.a & kSpliceBit) {
                    cont = n.b;
                    nxt = n.a & ~kSpliceBit;
                } else {
                    nxt = n.a;
                }
            } else if (n.a != kEmptyLeaf) {
                const int prim = -1 - n.a;
                double dist;
                bool h;
                if (prim < s.ntri) h = tri_test(s.tris[prim], r, cull, dist);
                else h = sphere_test(s.sph[prim - s.ntri], r, cull, dist);
                if (h) {
                    const V3 hx = r.o + mul(r.d, (float)dist);
                    if (dot3(hx - lc, hx - lc) < thr) return true;
                }
            }
        }
        cur = nxt == kMeshExit ? cont : nxt;
    }
    return false;
}
// The shadow query of Scene::ShadowCheck from lc toward x: flat all-leaves query
// when every ray of the wave has a finite inv, else a per-lane threaded walk.
// `cone` (PT only): the wave's shadow-cone mask for queries from an emitter point toward
// the lanes' camera hits (pt_cone_mask); used when every active lane's origin is a hit on
// an emitter (`on_e`), else every leaf is a candidate.
TPT_D bool shadow_ray(const DScene& s, V3 lc, V3 x, int cull, uint64_t cone = ~0ull, bool on_e = false) {
    const double ld2 = dot3(lc - x, lc - x);
    const double thr = ld2 - 1.0f;
    if (!(thr > 0.0)) return false;  // d2 >= 0 can never be < thr (the lane leaves the wave's query)
    const Ray r = make_ray(lc, normalized(x - lc));
    const bool fin = wave_finite(r);
    if (fin && (s.flat & kFlatShadow)) {
        if (s.qs) return shadow_flat_c(s, r, thr, cull);
        if (cone != ~0ull && __ballot(!on_e) != 0) cone = ~0ull;  // e.g. the light branch's query from (0,0,0)
        return shadow_flat(s, r, lc, thr, cull, cone);
    }
    return fin ? shadow_walk<true>(s, r, lc, thr, cull) : shadow_walk<false>(s, r, lc, thr, cull);
}

// PT shadow-cone mask (round 5).  Both of PathTrace's shadow queries run from a point on
// an emitter (the light sample's re-intersection, or the BSDF ray's hit on the light --
// hit points computed within a few ulps of the emitter's triangles or sphere) to
// the pixel's camera hit x, which is the same for all its samples.  A hit that counts
// (|hit - lc|^2 < |x - lc|^2 - 1, Scene.cpp:37-48) lies on that segment, so inside
// H = conv(E u {x}), E the emitters' box; its primitive lies in its leaf box, so a leaf
// whose box cannot meet H (both grown by cone_delta, which covers the rounding of the
// origin, the direction, the hit point and Moller-Trumbore's float edges) holds no
// counting hit and may be skipped: the any-hit answer is unchanged.  H is exactly the
// union over s in [0, 1] of the boxes x + s (E - x), so a leaf box L meets it iff the
// per-axis conditions  x + s (Emin - x) <= Lmax,  x + s (Emax - x) >= Lmin  have a common
// s in [0, 1]: six linear bounds on s per leaf.  Bit j: flat leaf j is a candidate.
TPT_D uint64_t pt_cone_mask(const DScene& s, V3 x) {
    const float dl = s.cone_delta;
    const float xv[3] = {x.x, x.y, x.z};
    float c1[3], c2[3], i1[3], i2[3];
    for (int a = 0; a < 3; ++a) {
        c1[a] = (s.lbox[a] - dl) - xv[a];
        c2[a] = (s.lbox[3 + a] + dl) - xv[a];
        i1[a] = __builtin_amdgcn_rcpf(c1[a]);
        i2[a] = __builtin_amdgcn_rcpf(c2[a]);
    }
    uint64_t m = 0;
    for (int j = 0; j < s.nleaf && j < 64; ++j) {
        const DNode n = s.leaves[j];
        float lo = 0.0f, hi = 1.0f;
        bool ok = true;
        for (int a = 0; a < 3; ++a) {
            const float r1 = (n.bmax[a] + dl) - xv[a];  // c1 s <= r1
            const float r2 = (n.bmin[a] - dl) - xv[a];  // c2 s >= r2
            if (c1[a] > 0.0f) hi = fminf(hi, r1 * i1[a]);
            else if (c1[a] < 0.0f) lo = fmaxf(lo, r1 * i1[a]);
            else ok = ok && r1 >= 0.0f;
            if (c2[a] > 0.0f) lo = fmaxf(lo, r2 * i2[a]);
            else if (c2[a] < 0.0f) hi = fminf(hi, r2 * i2[a]);
            else ok = ok && r2 <= 0.0f;
        }
        // the bounds are quotients rounded a few ulps either way: a relative slack keeps
        // the test conservative (the margins above are far larger)
        if (ok && lo <= hi + 1e-5f * (1.0f + fabs_(hi))) m |= 1ull << j;
    }
    return m;
}

// ------------------------------------------------------------ materials --
struct Mat {
    int type;
    V3 em, ior_m, ior_m_k, kd;
    float ior_d, rough;
};
TPT_D Mat load_mat(const DScene& s, int mi) {
    const DMat& m = s.mats[mi];
    Mat r;
    r.type = m.type;
    r.em = v3(m.em[0], m.em[1], m.em[2]);
    r.ior_m = v3(m.ior_m[0], m.ior_m[1], m.ior_m[2]);
    r.ior_m_k = v3(m.ior_m_k[0], m.ior_m_k[1], m.ior_m_k[2]);
    r.kd = v3(m.kd[0], m.kd[1], m.kd[2]);
    r.ior_d = m.ior_d;
    r.rough = m.rough;
    return r;
}

TPT_D float saturate(float t) { return smin(smax(t, 0.0f), 1.0f); }  // std::clamp(t, 0, 1)
TPT_D double clampd(double v) { return v < -1.0 ? -1.0 : (1.0 < v ? 1.0 : v); }

// AnyPerpendicular (SampleHelperFunctions.cpp:51-67)
TPT_D V3 any_perp(V3 i) {
    if (i.z == 0.0f) {
        if (i.y == 0.0f) return v3(0.0f, 1.0f, 0.0f);
        return normalized(v3(1.0f, -i.x / i.y, 0.0f));
    }
    return normalized(v3(0.0f, 1.0f, -1.0f * i.y / i.z));
}
// Shading frame of a surface point seen from wo: the normal, the tangent frame
// TransformVectorToWorld builds from it (SampleHelperFunctions.hpp:46-54:
// t = AnyPerpendicular(n), b = n x t) and n.wo as the material code rounds it.  All
// are functions of (n, wo) only, so a caller that shades the same point many times
// (PT: every sample of a pixel) computes them once; the values are identical.
struct Shade {
    V3 n, t, b;
    float nv;  // (float)DotProduct(n, wo)
};
TPT_D Shade make_shade(V3 n, V3 wo) {
    Shade f;
    f.n = n;
    f.t = any_perp(n);
    f.b = cross(n, f.t);
    f.nv = (float)dot3(n, wo);
    return f;
}
// TransformVectorToWorld (SampleHelperFunctions.hpp:46-54)
TPT_D V3 to_world(V3 a, const Shade& f) {
    const V3 t = f.t, b = f.b, n = f.n;
    return v3(a.x * t.x + a.y * b.x + a.z * n.x, a.x * t.y + a.y * b.y + a.z * n.y,
              a.x * t.z + a.y * b.z + a.z * n.z);
}
// Reflect (SampleHelperFunctions.cpp:21-25)
TPT_D V3 reflect(V3 I, V3 N) {
    I = -I;
    return I - mul(N, (float)(2 * dot3(I, N)));
}
// Refract (SampleHelperFunctions.cpp:38-49)
TPT_D V3 refract(V3 I, V3 N, float ior) {
    I = -I;
    float cosi = (float)clampd(dot3(I, N));
    float etai = 1, etat = ior;
    V3 n = N;
    if (cosi < 0) cosi = -cosi;
    else { float t = etai; etai = etat; etat = t; n = -N; }
    float eta = etai / etat;
    float k = 1 - eta * eta * (1 - cosi * cosi);
    return k < 0 ? v3s(0.0f) : normalized(mul(I, eta) + mul(n, eta * cosi - sqrt_f(k)));
}
// GetInsideOutsideIOR (SampleHelperFunctions.hpp:57-73); nv = (float)DotProduct(N, wo)
TPT_D void inout_ior(V3 N, V3 wi, float nv, float mior, float& ior_i, float& ior_o) {
    float nl = (float)dot3(N, wi);
    ior_i = nl < 0.0f ? mior : 1.0f;
    ior_o = nv < 0.0f ? mior : 1.0f;
}
TPT_D void inout_ior(V3 N, V3 wi, V3 wo, float mior, float& ior_i, float& ior_o) {
    inout_ior(N, wi, (float)dot3(N, wo), mior, ior_i, ior_o);
}
// GetHalfDir (SampleHelperFunctions.hpp:79-102); nv = (float)DotProduct(N, wo)
TPT_D V3 half_dir(V3 N, V3 wi, V3 wo, float nv, float mior) {
    float nl = (float)dot3(N, wi);
    if (nl == 0.0f || nv == 0.0f) return v3s(0.0f);
    if (nl * nv > 0.0f) {
        V3 h = normalized(wi + wo);
        return nv < 0.0f ? -h : h;
    }
    if (nv < 0.0f) return -normalized(mul(wo, mior) + wi);
    return -normalized(wo + mul(wi, mior));
}
TPT_D V3 half_dir(V3 N, V3 wi, V3 wo, float mior) { return half_dir(N, wi, wo, (float)dot3(N, wo), mior); }
// GetCosineWeightedSample (SampleHelperFunctions.hpp:105-115); cos/sin in double
TPT_D V3 cosine_sample(const Shade& f, float& pdf, uint32_t& rs) {
    const V3 N = f.n;
    float u1 = rng_float(rs);
    float r = sqrt_f(u1);
    float theta = 2 * kPi * rng_float(rs);
    double sd, cd;
    tpt_sincos_d((double)theta, &sd, &cd);
    float x = (float)((double)r * cd), y = (float)((double)r * sd);
    V3 wi = normalized(to_world(v3(x, y, sqrt_f(1.0f - u1)), f));
    pdf = (float)(dot3(wi, N) / (double)kPi);
    return wi;
}
TPT_D V3 cosine_sample(V3 N, float& pdf, uint32_t& rs) { return cosine_sample(make_shade(N, N), pdf, rs); }
// GetCosineWeightedPdf (SampleHelperFunctions.hpp:118-120)
TPT_D float cosine_pdf(V3 N, V3 wi) { return saturate((float)dot3(wi, N)) / kPi; }

// GGX.hpp:8-14
TPT_D float ggx_vis(float vn, float vh, float r) {
    if (vh * vn <= 0.0f) return 0.0f;
    float vh2 = vh * vh;
    float tan2 = (1.0f - vh2) / vh2;
    return 2.0f / (1 + sqrt_f(1.0f + r * r * tan2));
}
// GGX.hpp:17-30
TPT_D float ggx_d(float c, float r) {
    float a2 = r * r;
    float c2 = c * c;
    float c4 = c2 * c2;
    float t2 = (1.0f - c2) / c2;
    float b = a2 + t2;
    b = b * b;
    return a2 / (kPi * c4 * b);
}
// GGX.hpp:33-35 (float(|d|) into GGXTerm, product with |d| in double)
TPT_D float ggx_half_pdf(V3 n, V3 h, float r) {
    double d = dabs_(dot3(n, h));
    return (float)((double)ggx_d((float)d, r) * d);
}
// GGX.hpp:46-59
TPT_D V3 ggx_h(const Shade& f, float r, float d1, float d2) {
    float theta = tpt_atan2f(r * sqrt_f(d1), sqrt_f(1.0f - d1));
    float phi = 2.0f * kPi * d2;
    float st, ct, sp, cp;
    tpt_sincosf(theta, &st, &ct);
    tpt_sincosf(phi, &sp, &cp);
    V3 local = v3(st * cp, st * sp, ct);
    return normalized(to_world(local, f));
}
TPT_D V3 ggx_sample_h(const Shade& f, float r, uint32_t& rs) {
    float d1 = rng_float(rs), d2 = rng_float(rs);
    return ggx_h(f, r, d1, d2);
}

// Material::fresnel (Material.cpp:221-252)
TPT_D V3 fresnel(const Mat& m, V3 I, V3 N) {
    if (m.type == TPT_METAL) {
        float c = (float)dot3(I, N);
        float c2 = c * c;
        V3 two = mul(mul(m.ior_m, 2.0f), c);
        V3 t0 = m.ior_m * m.ior_m + m.ior_m_k * m.ior_m_k;
        V3 t1 = mul(t0, c2);
        V3 Rs = (t0 - two + v3s(c2)) / (t0 + two + v3s(c2));
        V3 Rp = (t1 - two + v3s(1.0f)) / (t1 + two + v3s(1.0f));
        return mul(Rp + Rs, 0.5f);
    }
    I = -I;
    float cosi = (float)clampd(dot3(I, N));
    float etai = 1, etat = m.ior_d;
    if (cosi > 0) { float t = etai; etai = etat; etat = t; }
    float sint = etai / etat * sqrt_f(smax(0.f, 1 - cosi * cosi));
    if (sint >= 1) return v3s(1.0f);
    float cost = sqrt_f(smax(0.f, 1 - sint * sint));
    cosi = fabs_(cosi);
    float Rs = ((etat * cosi) - (etai * cost)) / ((etat * cosi) + (etai * cost));
    float Rp = ((etai * cosi) - (etat * cost)) / ((etai * cosi) + (etat * cost));
    return v3s((Rs * Rs + Rp * Rp) / 2);
}

// Material::evalGivenSample (Material.cpp:11-72)
TPT_D V3 eval_bsdf(const Mat& m, V3 wo, V3 wi, const Shade& sh, bool cosine) {
    const V3 N = sh.n;
    float nl = (float)dot3(N, wi);
    float nv = sh.nv;
    if (nl == 0.0f || nv == 0.0f) return v3s(0.0f);
    V3 h = half_dir(N, wi, wo, nv, m.ior_d);
    float nh = (float)dot3(N, h);
    float lh = (float)dot3(wi, h);
    float vh = (float)dot3(wo, h);
    float D = ggx_d(nh, m.rough);
    float G = ggx_vis(nv, vh, m.rough) * ggx_vis(nl, lh, m.rough);
    V3 f = fresnel(m, wi, h);
    if (nl * nv > 0.0f) {
        V3 spec = v3s(0.0f);
        if (G != 0.0f) {
            spec = divs(mul(mul(f, D), G), (float)(4.0 * (double)fabs_(nv)));
            if (!cosine) spec = divs(spec, fabs_(nl));
        }
        V3 diff = v3s(0.0f);
        if (m.type == TPT_DIELETRIC) {
            diff = divs(m.kd * (v3s(1.0f) - f), kPi);
            if (cosine) diff = mul(diff, saturate(nl));
        }
        return diff + spec;
    }
    if (m.type != TPT_TRANSPARENT) return v3s(0.0f);
    float ior_i, ior_o;
    if (nv < 0.0f) { ior_i = 1.0f; ior_o = m.ior_d; }
    else { ior_i = m.ior_d; ior_o = 1.0f; }
    float pa = fabs_(vh) * fabs_(lh) / (fabs_(nv));
    if (!cosine) pa /= fabs_(nl);
    float pb = ior_o * ior_o * (1.0f - f.x) * G * D;
    if (pa * pb == 0.0f) return v3s(0.0f);
    float pc = ior_i * lh + ior_o * vh;
    pc *= pc;
    return v3s(pa * pb / pc);
}
TPT_D V3 eval_bsdf(const Mat& m, V3 wo, V3 wi, V3 N, bool cosine) {
    return eval_bsdf(m, wo, wi, make_shade(N, wo), cosine);
}

TPT_D float safe_div(float v, float p) { return p == 0.0f ? 0.0f : v / p; }  // SampleHelperFunctions.hpp:24-32
TPT_D V3 safe_div(V3 v, float p) { return p == 0.0f ? v3s(0.0f) : divs(v, p); }

// Material::pdf (Material.cpp:105-147)
TPT_D float mat_pdf(const Mat& m, V3 wo, const Shade& sh, V3 wi) {
    const V3 n = sh.n;
    float nv = sh.nv, nl = (float)dot3(n, wi);
    if (nv == 0.0f || nl == 0.0f) return 0.0f;
    V3 h = half_dir(n, wi, wo, nv, m.ior_d);
    V3 f = fresnel(m, wo, h);
    float pdf_h = ggx_half_pdf(n, h, m.rough);
    float vh = (float)dot3(wo, h);
    float avh = fabs_(vh);
    float lh = (float)dot3(wi, h);
    float ior_i, ior_o;
    inout_ior(n, wi, nv, m.ior_d, ior_i, ior_o);
    if (nv * nl < 0.0f) {
        float den = ior_i * lh + ior_o * vh;
        float jac = safe_div(ior_o * ior_o * avh, den * den);
        if (m.type != TPT_TRANSPARENT) return 0.0f;
        return pdf_h * (1.0f - f.x) * jac;
    }
    if (nv * nl > 0.0f) {
        float jac = safe_div(1.0f, 4.0f * avh);
        float diff = cosine_pdf(n, wi);
        if (m.type == TPT_METAL) return pdf_h * jac;
        if (m.type == TPT_DIELETRIC) return (diff + pdf_h * jac) * 0.5f;
        return pdf_h * f.x * jac;
    }
    return 0.0f;
}
TPT_D float mat_pdf(const Mat& m, V3 wo, V3 n, V3 wi) { return mat_pdf(m, wo, make_shade(n, wo), wi); }

// eval_bsdf(m, wo, wi, N, false) and mat_pdf(m, wo, N, wi) of one direction pair,
// computed together: both start from the same nl, nv, half vector, n.h (ggx_d is
// even in its argument, so GGXTerm(|n.h|) == GGXTerm(n.h)), v.h and l.h; only the
// Fresnel argument differs (evalGivenSample uses fresnel(wi, h), pdf uses
// fresnel(wo, h): Material.cpp:24 vs :112).  Same float ops as the two functions.
// kCos: evalGivenSample with combineCosineTerm = true (PathTrace's light branch);
// nv = (float)DotProduct(N, wo) as the caller has it (the Shade).
template <bool kCos>
TPT_D void bsdf_pdf_t(const Mat& m, V3 wo, V3 wi, V3 N, float nv, V3& f_out, float& pdf_out) {
    f_out = v3s(0.0f);
    pdf_out = 0.0f;
    float nl = (float)dot3(N, wi);
    if (nl == 0.0f || nv == 0.0f) return;
    V3 h = half_dir(N, wi, wo, nv, m.ior_d);
    const double dnh = dot3(N, h);
    float nh = (float)dnh;
    float lh = (float)dot3(wi, h);
    float vh = (float)dot3(wo, h);
    float D = ggx_d(nh, m.rough);
    // ---- Material::pdf (Material.cpp:105-147)
    {
        V3 fp = fresnel(m, wo, h);
        const double d = dabs_(dnh);
        float pdf_h = (float)((double)D * d);  // ggx_half_pdf
        float avh = fabs_(vh);
        float ior_i, ior_o;
        inout_ior(N, wi, nv, m.ior_d, ior_i, ior_o);
        if (nv * nl < 0.0f) {
            float den = ior_i * lh + ior_o * vh;
            float jac = safe_div(ior_o * ior_o * avh, den * den);
            if (m.type == TPT_TRANSPARENT) pdf_out = pdf_h * (1.0f - fp.x) * jac;
        } else if (nv * nl > 0.0f) {
            float jac = safe_div(1.0f, 4.0f * avh);
            float diff = cosine_pdf(N, wi);
            if (m.type == TPT_METAL) pdf_out = pdf_h * jac;
            else if (m.type == TPT_DIELETRIC) pdf_out = (diff + pdf_h * jac) * 0.5f;
            else pdf_out = pdf_h * fp.x * jac;
        }
    }
    // ---- Material::evalGivenSample (Material.cpp:11-72)
    float G = ggx_vis(nv, vh, m.rough) * ggx_vis(nl, lh, m.rough);
    V3 f = fresnel(m, wi, h);
    if (nl * nv > 0.0f) {
        V3 spec = v3s(0.0f);
        if (G != 0.0f) {
            spec = divs(mul(mul(f, D), G), (float)(4.0 * (double)fabs_(nv)));
            if (!kCos) spec = divs(spec, fabs_(nl));
        }
        V3 diff = v3s(0.0f);
        if (m.type == TPT_DIELETRIC) {
            diff = divs(m.kd * (v3s(1.0f) - f), kPi);
            if (kCos) diff = mul(diff, saturate(nl));
        }
        f_out = diff + spec;
        return;
    }
    if (m.type != TPT_TRANSPARENT) return;
    float ior_i, ior_o;
    if (nv < 0.0f) { ior_i = 1.0f; ior_o = m.ior_d; }
    else { ior_i = m.ior_d; ior_o = 1.0f; }
    float pa = fabs_(vh) * fabs_(lh) / (fabs_(nv));
    if (!kCos) pa /= fabs_(nl);
    float pb = ior_o * ior_o * (1.0f - f.x) * G * D;
    if (pa * pb == 0.0f) return;
    float pc = ior_i * lh + ior_o * vh;
    pc *= pc;
    f_out = v3s(pa * pb / pc);
}

TPT_D void bsdf_pdf(const Mat& m, V3 wo, V3 wi, V3 N, V3& f_out, float& pdf_out) {
    bsdf_pdf_t<false>(m, wo, wi, N, (float)dot3(N, wo), f_out, pdf_out);
}

// Material::sample (Material.cpp:150-214).  kLateH (BDPT's gen; PT measured 0.8 %
// slower with it, 43.55 vs 43.2 ms): the Dieletric branch makes its GGX half vector
// after the coin.
#ifndef TPT_MAT_TAIL_MERGE
#define TPT_MAT_TAIL_MERGE 1  // Dieletric pdf tail once per wave (PT: 40.35-40.57 -> 39.50-39.66 ms, configs[3] -2.2 %
                              // same-box; PT-indirect keeps the branch form, 553 vs 574 ms)
#endif
template <bool kLateH = false, bool kTail = TPT_MAT_TAIL_MERGE>
TPT_D V3 mat_sample(const Mat& m, V3 wo, const Shade& sh, float* pdf, uint32_t& rs) {
    const V3 n = sh.n;
    if (kLateH && m.type == TPT_DIELETRIC) {
        // The same draws in the same order (the half vector's two, then the coin), but
        // the GGX half vector and everything derived from it are made only in the
        // branch that uses them: the cosine branch replaces H, so across the branches
        // only the two draws stay live (they kept mat_sample's f64 temporaries in
        // scratch).
        const float d1 = rng_float(rs), d2 = rng_float(rs);
        if (xorshift32(rs) < kCoinHalf) {  // rng_float(rs) < 0.5f
            const V3 H = ggx_h(sh, m.rough, d1, d2);
            const V3 wis = reflect(wo, H);
            const float pdf_h = ggx_half_pdf(n, H, m.rough);
            const float jr = safe_div(1.0f, 4.0f * fabs_((float)dot3(wo, H)));
            const float pd = cosine_pdf(n, wis);
            *pdf = (pdf_h * jr + pd) * 0.5f;
            if ((double)sh.nv * dot3(wis, n) < 0.0f) *pdf = 0.0f;
            return wis;
        }
        float pd;
        V3 wid = cosine_sample(sh, pd, rs);
        const V3 H = normalized(wid + wo);
        const float avh = fabs_((float)dot3(wo, H));
        const float pdf_h = ggx_half_pdf(n, H, m.rough);
        const float jr = safe_div(1.0f, 4.0f * avh);
        *pdf = (pdf_h * jr + pd) * 0.5f;
        if ((double)sh.nv * dot3(wid, n) < 0.0f) *pdf = 0.0f;
        return wid;
    }
    if (kTail && m.type == TPT_DIELETRIC) {
        // (round 6) the half vector first (its two draws, then the coin: the reference's
        // order), each branch makes only its direction, and the pdf tail that both
        // branches share -- the GGX half-vector pdf, the Jacobian, the mix -- runs once
        // for the wave instead of once per branch; per lane the same float ops as below
        V3 H = ggx_sample_h(sh, m.rough, rs);
        V3 wi;
        float pd;
        if (xorshift32(rs) < kCoinHalf) {  // rng_float(rs) < 0.5f
            wi = reflect(wo, H);
            pd = cosine_pdf(n, wi);
        } else {
            wi = cosine_sample(sh, pd, rs);
            H = normalized(wi + wo);
        }
        const float pdf_h = ggx_half_pdf(n, H, m.rough);
        const float jr = safe_div(1.0f, 4.0f * fabs_((float)dot3(wo, H)));
        *pdf = (pdf_h * jr + pd) * 0.5f;
        if ((double)sh.nv * dot3(wi, n) < 0.0f) *pdf = 0.0f;
        return wi;
    }
    V3 H = ggx_sample_h(sh, m.rough, rs);
    V3 wis = reflect(wo, H);
    float pdf_h = ggx_half_pdf(n, H, m.rough);
    float vn = sh.nv;  // (float)DotProduct(wo, n)
    float vh = (float)dot3(wo, H);
    float avh = fabs_(vh);
    float jr = safe_div(1.0f, 4.0f * avh);
    if (m.type == TPT_METAL) {
        *pdf = pdf_h * jr;
        if ((double)vn * dot3(wis, n) < 0.0f) *pdf = 0.0f;
        return wis;
    }
    if (m.type == TPT_DIELETRIC) {
        if (xorshift32(rs) < kCoinHalf) {  // rng_float(rs) < 0.5f
            float pd = cosine_pdf(n, wis);
            *pdf = (pdf_h * jr + pd) * 0.5f;
            if ((double)vn * dot3(wis, n) < 0.0f) *pdf = 0.0f;
            return wis;
        }
        float pd;
        V3 wid = cosine_sample(sh, pd, rs);
        H = normalized(wid + wo);
        vh = (float)dot3(wo, H);
        avh = fabs_(vh);
        pdf_h = ggx_half_pdf(n, H, m.rough);
        jr = safe_div(1.0f, 4.0f * avh);
        *pdf = (pdf_h * jr + pd) * 0.5f;
        if ((double)vn * dot3(wid, n) < 0.0f) *pdf = 0.0f;
        return wid;
    }
    V3 f = fresnel(m, wo, H);
    if (rng_float(rs) < f.x) {
        *pdf = pdf_h * f.x * jr;
        if ((double)vn * dot3(wis, n) < 0.0f) *pdf = 0.0f;
        return wis;
    }
    V3 wr = refract(wo, H, m.ior_d);
    float ior_i, ior_o;
    inout_ior(n, wr, vn, m.ior_d, ior_i, ior_o);
    float lh = (float)dot3(wr, H);
    float den = ior_i * lh + ior_o * vh;
    float jt = safe_div(ior_o * ior_o * avh, den * den);
    *pdf = pdf_h * (1.0f - f.x) * jt;
    if ((double)vn * dot3(wr, n) > 0.0f) *pdf = 0.0f;
    return wr;
}
template <bool kLateH = false>
TPT_D V3 mat_sample(const Mat& m, V3 wo, V3 n, float* pdf, uint32_t& rs) {
    return mat_sample<kLateH>(m, wo, make_shade(n, wo), pdf, rs);
}

// ---------------------------------------------------------- light objects --
// Object::Sample: BVHAccel::Sample / getSample (BVH.cpp:145-159) + Triangle::Sample
// (Triangle.hpp:31-36); Sphere::Sample (Sphere.cpp:48-55).
TPT_D void object_sample(const DScene& s, const DObj& o, V3& pc, V3& pn, int& prim, uint32_t& rs) {
    if (o.kind == TPT_OBJ_MESH) {
        float p = sqrt_f(rng_float(rs)) * o.root_area;
        int ni = o.root;
        for (;;) {
            const DNode n = s.nodes[ni];
            if (n.a < 0) break;
            const float la = s.node_area[n.a];
            if (p < la) ni = n.a;
            else { p = p - la; ni = n.b; }
        }
        const int t = -1 - s.nodes[ni].a;
        const DTri tri = s.tris[t];
        const DTriX tx = s.trix[t];
        float x = sqrt_f(rng_float(rs)), y = rng_float(rs);
        pc = mul(v3(tri.v0[0], tri.v0[1], tri.v0[2]), 1.0f - x) + mul(v3(tx.v1[0], tx.v1[1], tx.v1[2]), x * (1.0f - y)) +
             mul(v3(tx.v2[0], tx.v2[1], tx.v2[2]), x * y);
        pn = tri_normal(tri);
        prim = t;
    } else {
        const DSphere sp = s.sph[o.sphere_prim - s.ntri];
        float theta = (float)(2.0 * (double)kPi * (double)rng_float(rs));
        float phi = (float)(kPi * rng_float(rs));
        float sph, cph, sth, cth;
        tpt_sincosf(phi, &sph, &cph);
        tpt_sincosf(theta, &sth, &cth);
        V3 dir = v3(cph, sph * cth, sph * sth);
        pc = v3(sp.c[0], sp.c[1], sp.c[2]) + mul(dir, sp.r);
        pn = dir;
        prim = o.sphere_prim;
    }
}

// Object::GetIntersection for one emitter object, evaluating two culling modes on
// one ray in a single traversal (the box tests do not depend on culling; the
// culling test is the first step of each primitive test, Triangle.cpp:81-88).
struct Hit2 {
    Hit a, b;
};
// NoCull and CullBack closest hits of one ray against one emitter object, one
// traversal (same node order, same strict `>` tie rule for each result).
template <bool kFin>
TPT_D void mesh_hit_nocull_back(const DScene& s, int root, const Ray& r, Hit& hn, Hit& hb) {
    int cur = root;  // a mesh subtree ends in kMeshExit
    while (cur >= 0) {
        const DNode n = s.tnodes[cur];
        int nxt = n.b;
        if (box_hit_t<kFin>(n, r)) {
            if (n.a >= 0) {
                nxt = n.a;
            } else if (n.a != kEmptyLeaf) {
                const int prim = -1 - n.a;
                const DTri t = s.tris[prim];
                double d;
                if (tri_test(t, r, TPT_NO_CULL, d)) {  // culling is the test's first step
                    if (hn.prim < 0 || hn.dist > d) { hn.prim = prim; hn.dist = d; }
                    if (!(dot3(r.d, tri_normal(t)) > 0) && (hb.prim < 0 || hb.dist > d)) { hb.prim = prim; hb.dist = d; }
                }
            }
        }
        cur = nxt;
    }
}
TPT_D void object_hit_nocull_back(const DScene& s, const DObj& o, const Ray& r, Hit& hn, Hit& hb) {
    hn.prim = hb.prim = -1;
    hn.dist = hb.dist = 0.0;
    if (o.kind != TPT_OBJ_MESH) {
        double d;
        const DSphere sp = s.sph[o.sphere_prim - s.ntri];
        if (sphere_test(sp, r, TPT_NO_CULL, d)) { hn.prim = o.sphere_prim; hn.dist = d; }
        if (sphere_test(sp, r, TPT_CULL_BACK, d)) { hb.prim = o.sphere_prim; hb.dist = d; }
        return;
    }
    if (o.root < 0) return;
    if (wave_finite(r)) mesh_hit_nocull_back<true>(s, o.root, r, hn, hb);
    else mesh_hit_nocull_back<false>(s, o.root, r, hn, hb);
}

TPT_D Hit object_hit(const DScene& s, const DObj& o, const Ray& r, int cull) {
    if (o.kind == TPT_OBJ_MESH) return traverse(s, o.root, r, cull);
    Hit h;
    h.prim = -1;
    h.dist = 0.0;
    double dist;
    if (sphere_test(s.sph[o.sphere_prim - s.ntri], r, cull, dist)) { h.prim = o.sphere_prim; h.dist = dist; }
    return h;
}

// ------------------------------------------------------------------- PT ---
// The camera hit and its material are invariant over a pixel's spp loop.  Held in
// registers across the loop they cost ~25 VGPRs at every point of the sample body
// and push the kernel into scratch spills; instead each lane parks them in LDS
// ([slot][kBlock] floats, conflict-free) and re-reads them where they are used.  The
// empty asm makes the lane offset opaque, so the compiler can neither hoist the
// reads out of the loop nor keep one read alive across the sample body.
// The material's constants are not parked: they are read from the material table
// (staged in LDS with the scene) by the parked index.  Parked too (26 slots instead
// of 18) they made the occlusion and refractive-ball scenes 7 % slower and Standard
// 0.3 % faster (same-box A/B: 47.6 / 54.7 / 50.6 ms vs 44.2 / 51.0 / 50.8 ms).
enum PixSlot {
    kPxMat = 0,  // the material type is read from the LDS material table by this index
    kPxX,
    kPxN = kPxX + 3,
    kPxWo = kPxN + 3,
    kPxT = kPxWo + 3,  // Shade of the camera hit: tangent, bitangent, n.wo
    kPxB = kPxT + 3,
    kPxNv = kPxB + 3,
    kPixSlots
};
struct PixPark {
    float* base;  // kPixSlots x kBlock floats of LDS
    TPT_D const float* lane() const {
        unsigned off = threadIdx.x;
        asm volatile("" : "+v"(off));
        return base + off;
    }
    TPT_D V3 v(int k) const {
        const float* p = lane();
        return v3(p[k * kBlock], p[(k + 1) * kBlock], p[(k + 2) * kBlock]);
    }
    TPT_D int mat_index() const { return __float_as_int(lane()[kPxMat * kBlock]); }
    TPT_D int type(const DScene& s) const { return s.mats[mat_index()].type; }
    TPT_D Shade shade() const {
        Shade f;
        f.n = v(kPxN);
        f.t = v(kPxT);
        f.b = v(kPxB);
        f.nv = lane()[kPxNv * kBlock];
        return f;
    }
    TPT_D Mat mat(const DScene& s) const {
        const DMat& d = s.mats[mat_index()];
        Mat m;
        m.type = d.type;
        m.ior_d = d.ior_d;
        m.rough = d.rough;
        const float* kdm = m.type == TPT_METAL ? d.ior_m : d.kd;  // each type reads only its own
        m.kd = v3(kdm[0], kdm[1], kdm[2]);
        m.ior_m = m.kd;
        m.ior_m_k = v3(d.ior_m_k[0], d.ior_m_k[1], d.ior_m_k[2]);
        m.em = v3s(0.0f);  // emission is read from the scene where it is used
        return m;
    }
    TPT_D void put(int k, float x) { base[k * kBlock + threadIdx.x] = x; }
    TPT_D void put3(int k, V3 a) {
        put(k, a.x);
        put(k + 1, a.y);
        put(k + 2, a.z);
    }
    TPT_D void park(V3 x, V3 n, V3 wo, int mi, const Mat& m) {
        put(kPxMat, __int_as_float(mi));
        put3(kPxX, x);
        put3(kPxN, n);
        put3(kPxWo, wo);
        const Shade f = make_shade(n, wo);
        put3(kPxT, f.t);
        put3(kPxB, f.b);
        put(kPxNv, f.nv);
    }
};

// PathTrace at HEAD (PathTracer.cpp:44-134): emission of the camera hit + MIS
// direct lighting from every emitter, then the unconditional `break` (:109).
// The camera hit is the same for every sample of a pixel (no jitter,
// SceneRenderingHelper.cpp:16-22): the caller computes it once and parks it in `px`.
// A copy of `a` the compiler cannot see through: values derived from it (the f64
// conversions of a dot product) are computed after this point, not hoisted out of
// the emitter loop and held (spilled) across the queries in between.
TPT_D V3 opaque(V3 a) {
    asm volatile("" : "+v"(a.x), "+v"(a.y), "+v"(a.z));
    return a;
}
TPT_D V3 pt_sample(const DScene& s, PixPark px, uint32_t& rs, uint64_t cone = ~0ull) {
    V3 result = v3s(0.0f);
    {
        const DMat& dm = s.mats[px.mat_index()];
        if (dm.has_em) result = result + v3(dm.em[0], dm.em[1], dm.em[2]);
    }
    float pdf_b0;
    const V3 wib0 = mat_sample(px.mat(s), px.v(kPxWo), px.shade(), &pdf_b0, rs);
    for (int li = 0; li < s.n_emitters; ++li) {
        // opaque per-iteration copies of the BSDF sample: what the body derives from it
        // (the ray's reciprocals, f64 conversions) is made here, not hoisted out of the
        // emitter loop and held (spilled) across its queries -- Standard has one emitter
        const V3 wib = opaque(wib0);
        float pdf_b = pdf_b0;
        asm volatile("" : "+v"(pdf_b));
        const DObj o = s.objs[s.emitters[li]];
        // DirectLightSampler::sample (PathTracer.cpp:26-40)
        V3 pc, pn;
        int pp;
        object_sample(s, o, pc, pn, pp, rs);
        V3 wil = pc - px.v(kPxX);
        float d2 = (float)dot3(wil, wil);
        wil = normalized(wil);
        float ct = (float)dot3(pn, -wil);
        float pll = (float)((double)o.pdf * d2 / (double)fabs_(ct));
        V3 ev = v3s(0.0f);
        {
            // DirectLightSampler::pdf (PathTracer.cpp:14-24) on the BSDF direction
            const V3 hx0 = px.v(kPxX);
            Ray rb = make_ray(hx0, wib);
            Hit hnc, hb;
            object_hit_nocull_back(s, o, rb, hnc, hb);
            float pbl = 0.0f;
            if (hnc.prim >= 0) {
                V3 hx, hn;
                hit_geometry(s, rb, hnc, hx, hn);
                float ld2 = (float)dot3(hx - hx0, hx - hx0);
                float c = (float)dot3(hn, -opaque(wib));
                if (c != 0.0f) pbl = (float)((double)o.pdf * ld2 / (double)fabs_(c));
            }
            if (pdf_b + pbl > 0.0f) {
                if (hb.prim >= 0) {
                    V3 hx, hn;
                    hit_geometry(s, rb, hb, hx, hn);
                    const bool sh = shadow_ray(s, hx, px.v(kPxX), TPT_CULL_BACK, cone, true);  // hx: a hit on the emitter
                    if (!sh)
                        ev = ev + divs(eval_bsdf(px.mat(s), px.v(kPxWo), opaque(wib), px.shade(), true),
                                       1e-4f + pdf_b + pbl);
                }
            }
        }
        // the light branch (PathTracer.cpp:95-106); plb is pure, so it is computed here
        // Material::pdf and evalGivenSample(.., true) of wil together (one half vector)
        float plb;
        V3 fl;
        {
            const Shade sh = px.shade();
            bsdf_pdf_t<true>(px.mat(s), px.v(kPxWo), wil, sh.n, sh.nv, fl, plb);
        }
        if (pll + plb > 0.0f) {
            Ray rl = make_ray(px.v(kPxX), wil);
            Hit hl = object_hit(s, o, rl, TPT_CULL_BACK);
            V3 hx = v3s(0.0f), hn;  // default Intersection::coords when missed (Intersection.hpp:14-21)
            if (hl.prim >= 0) hit_geometry(s, rl, hl, hx, hn);
            const bool sh = shadow_ray(s, hx, px.v(kPxX), TPT_CULL_BACK, cone, hl.prim >= 0);
            if (!sh) ev = ev + divs(fl, 1e-4f + pll + plb);
        }
        result = result + ev * load_mat(s, o.mat).em;
    }
    return result;
}

// ------------------------------------------------ PT, indirect bounce on ---
// TPT_MODE_PT_INDIRECT: PathTracer.cpp:44-134 with the `break` at :109 removed.
// One iteration of the loop body after its closest hit `v` (:64-131): emission on
// the first hit only (lastBounceExplicitSampledLight is false only until the first
// light loop, :50/:80), MIS direct lighting from every emitter weighted by the
// throughput alpha, then the BSDF-sampled continuation with Russian roulette after
// five bounces (the coin is drawn only then, :122-123).  Updates the ray, alpha,
// radiance, bounce count and culling flip in place; false when the path ends.
struct PtiPath {
    Ray r;
    V3 alpha, res;
    int nb;     // outBounces
    bool flip;  // lastBounceFlipCulling
};
TPT_D bool pti_step(const DScene& s, const PTV& v, PtiPath& p, uint32_t& rs) {
    const int mi = prim_mat(s, v.prim);
    const Mat m = load_mat(s, mi);
    if (p.nb == 0 && s.mats[mi].has_em) p.res = p.res + p.alpha * m.em;  // :64-68
    const V3 x = v.x, wo = -p.r.d;
    const Shade sh = make_shade(v.N, wo);
    float pdf_b;
    const V3 wib = mat_sample<false, false>(m, wo, sh, &pdf_b, rs);  // :76 (the per-branch form: faster here)
    for (int li = 0; li < s.n_emitters; ++li) {        // :82-106, as pt_sample
        const DObj o = s.objs[s.emitters[li]];
        V3 pc, pn;
        int pp;
        object_sample(s, o, pc, pn, pp, rs);
        V3 wil = pc - x;
        const float d2 = (float)dot3(wil, wil);
        wil = normalized(wil);
        const float ct = (float)dot3(pn, -wil);
        const float pll = (float)((double)o.pdf * d2 / (double)fabs_(ct));
        V3 ev = v3s(0.0f);
        {
            const Ray rb = make_ray(x, wib);
            Hit hnc, hb;
            object_hit_nocull_back(s, o, rb, hnc, hb);
            float pbl = 0.0f;
            if (hnc.prim >= 0) {
                V3 hx, hn;
                hit_geometry(s, rb, hnc, hx, hn);
                const float ld2 = (float)dot3(hx - x, hx - x);
                const float c = (float)dot3(hn, -wib);
                if (c != 0.0f) pbl = (float)((double)o.pdf * ld2 / (double)fabs_(c));
            }
            if (pdf_b + pbl > 0.0f && hb.prim >= 0) {
                V3 hx, hn;
                hit_geometry(s, rb, hb, hx, hn);
                if (!shadow_ray(s, hx, x, TPT_CULL_BACK))
                    ev = ev + divs(eval_bsdf(m, wo, wib, sh, true), 1e-4f + pdf_b + pbl);
            }
        }
        const float plb = mat_pdf(m, wo, sh, wil);
        if (pll + plb > 0.0f) {
            const Ray rl = make_ray(x, wil);
            const Hit hl = object_hit(s, o, rl, TPT_CULL_BACK);
            V3 hx = v3s(0.0f), hn;  // default Intersection::coords when missed
            if (hl.prim >= 0) hit_geometry(s, rl, hl, hx, hn);
            if (!shadow_ray(s, hx, x, TPT_CULL_BACK))
                ev = ev + divs(eval_bsdf(m, wo, wil, sh, true), 1e-4f + pll + plb);
        }
        p.res = p.res + p.alpha * ev * load_mat(s, o.mat).em;  // :105
    }
    V3 weight = v3s(0.0f);  // :111-114
    if (pdf_b > 0.0f) weight = divs(eval_bsdf(m, wo, wib, sh, true), 1e-4f + pdf_b);
    p.r = make_ray(x, wib);             // :116
    p.flip = dot3(v.N, wib) < 0.0;      // :117-120
    const bool rr = p.nb > 4;           // :122
    if (!rr || rng_float(rs) < 0.8f) {  // :123-127
        p.alpha = divs(p.alpha * weight, rr ? 0.8f : 1.0f);
        p.nb += 1;
        return true;
    }
    return false;
}

// Camera (SceneRenderingHelper.cpp:16-22); scale is host-computed CalculateScale.
TPT_D V3 pixel_ray(int px, int py, int w, int h, float scale) {
    float aspect = (float)(w / h);
    float x = (float)((2 * ((double)px + 0.5) / (double)(float)w - 1) * (double)aspect * (double)scale);
    float y = (float)((1 - 2 * ((double)py + 0.5) / (double)(float)h) * (double)scale);
    return normalized(v3(-x, y, 1));
}

}  // namespace tpt
