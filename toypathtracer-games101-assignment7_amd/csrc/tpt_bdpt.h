// tpt_bdpt.h -- bidirectional path tracing sample on gfx950 (BDPT.cpp:17-351,
// BDPT.hpp:15-169), arithmetic-identical to the reference.
//
// GPU restructuring (results unchanged, see tests/test_gpu_parity.py):
//  * BDPTPath::PathWeight (BDPT.cpp:173-259) copies a 3.6 KB path and re-Appends
//    the other subpath vertex by vertex to obtain reverse pdfs.  Append only reads
//    the appended vertex, the current last vertex and the one before it, and the
//    throughput it computes is never read by PathWeight.  So the k-th appended
//    vertex's pdf depends on the (s,t) connection only for k = 0, 1; for k >= 2 it
//    is a function of one subpath alone and is computed once
//    per path (`rev`), then multiplied by the same RR factor (count > 4 ? .8 : 1)
//    and folded into the same sequential cur_pdf / weightdenominator chain with the
//    same cur_pdf == 0 early exit.
//  * FillPathUsingRussianRoulette (BDPT.cpp:92-118) draws the RR random number
//    right after Material::sample; SampleNextVertex's intersection and BSDF
//    evaluation draw nothing, so they are skipped when the RR draw ends the path
//    and the BSDF evaluation is skipped when the pdf test ends it.
//    For k >= 2 the factor folded into cur_pdf is safe_div(rev * rr, pdf) with rr
//    either 1 or .8, so both variants are precomputed per vertex (`q1`, `q8`): the
//    O(n^3) chain then costs a select and a multiply per step, same float ops in the
//    same order.
//  * The camera vertices v0, v1 are the same for every sample (no jitter) and are
//    computed once per pixel.
//  * t = 1 splats (DrawToImage, SceneRenderingHelper.cpp:30-55) are fp32 atomics;
//    zero contributions are skipped (adding +-0 never changes an fp32 sum here).
#pragma once

#include "tpt_device.h"

namespace tpt {

constexpr int kMaxLen = 16;                   // MAX_BDPT_PATH_LENGTH (BDPT.hpp:8)
constexpr float kCamZeroPdf = (float)1e10;    // CAMERA_ZERO_PDF (BDPT.cpp:7)
constexpr float kCamRayPdf = (float)10.0;     // CAMERA_RAY_PDF (BDPT.cpp:8)

// BDPTPath::InternalPathVertex (BDPT.hpp:16-21) + cached reverse pdf.
struct BVert {
    V3 x, N;
    int type, prim;
    int mat;       // material of prim (-1 for the camera / background), resolved once at generation
    float pdf;
    V3 alpha;
    float q1, q8;  // safe_div(rev * rr, pdf) for rr = 1 and rr = .8 (rev: reverse pdf)
};

TPT_D PTV as_ptv(const BVert& b) {
    PTV v;
    v.x = b.x; v.N = b.N; v.type = b.type; v.prim = b.prim;
    return v;
}
TPT_D V3 normal_of(int type, V3 N) { return type == T_CAM ? v3(0.0f, 0.0f, 1.0f) : N; }  // BDPT.hpp:91-95

// SrpdfToAreaPdf (SampleHelperFunctions.hpp:122-131)
TPT_D float srpdf_to_area(float sr, int t1, V3 x1, V3 n1, int t2, V3 x2, V3 n2) {
    float d2;
    V3 w = normalize_len2(x2 - x1, &d2);
    float c1 = t1 == T_CAM ? 1.0f : (float)dabs_(dot3(w, n1));
    float c2 = t2 == T_CAM ? 1.0f : (float)dabs_(dot3(-w, n2));
    return sr * fabs_(c1 * c2 / d2);
}

// PathVertex::EvalPdfOnSolidAngle (BDPT.cpp:332-351); `pre` = Pre().Position()
TPT_D float eval_pdf_sa(const DScene& s, int type, int mat, V3 x, V3 N, V3 pre, V3 dir) {
    const V3 n = normal_of(type, N);
    float c = (float)dabs_(dot3(dir, n));
    if (type == T_LIGHT) return safe_div(cosine_pdf(n, dir), c);
    if (type == T_CAM) return kCamRayPdf;
    if (c == 0.0f) return 0.0f;
    V3 wo = normalized(pre - x);
    return safe_div(mat_pdf(load_mat(s, mat), wo, n, dir), c);
}
// PathVertex::EvalBsdfOnSolidAngle (BDPT.cpp:317-330)
TPT_D V3 eval_bsdf_sa(const DScene& s, int type, int mat, V3 x, V3 N, V3 pre, V3 dir) {
    if (type == T_LIGHT || type == T_CAM) return v3s(1.0f);
    return eval_bsdf(load_mat(s, mat), normalized(pre - x), dir, normal_of(type, N), false);
}
// eval_bsdf_sa and eval_pdf_sa of the same vertex and direction together (bsdf_pdf).
TPT_D void eval_pair_sa(const DScene& s, int type, int mat, V3 x, V3 N, V3 pre, V3 dir, V3& f, float& sr) {
    const V3 n = normal_of(type, N);
    float c = (float)dabs_(dot3(dir, n));
    if (type == T_LIGHT || type == T_CAM) {
        f = v3s(1.0f);
        sr = type == T_LIGHT ? safe_div(cosine_pdf(n, dir), c) : kCamRayPdf;
        return;
    }
    const V3 wo = normalized(pre - x);
    float pdf;
    bsdf_pdf(load_mat(s, mat), wo, dir, n, f, pdf);
    sr = c == 0.0f ? 0.0f : safe_div(pdf, c);
}
// Append's pdf for `v` appended after `last` (whose predecessor is at `pre`), before
// the RR factor (BDPT.cpp:154-158).
TPT_D float append_pdf(const DScene& s, int ltype, int lmat, V3 lx, V3 lN, V3 pre, int vtype, V3 vx, V3 vN) {
    float d2;
    V3 wi = normalize_len2(vx - lx, &d2);
    float sr = eval_pdf_sa(s, ltype, lmat, lx, lN, pre, wi);
    return srpdf_to_area(sr, ltype, lx, lN, vtype, vx, vN);
}
TPT_D float rr_of(int count) { return count > 4 ? .8f : 1.f; }

// Object::pdf() of a primitive (Triangle::pdf / Sphere::pdf), for Append(count==0)
TPT_D float prim_pdf(const DScene& s, int prim) {
    return prim < s.ntri ? 1.0f / s.trix[prim].area : 1.0f / s.sph[prim - s.ntri].area;
}

// Scene::ShadowCheck(const PTVertex&, const PTVertex&) (Scene.cpp:50-83), the part
// before the ray query: false when the reference answers "not shadowed" without a
// query (Scene.cpp:71-78), otherwise the culling mode of the query (Scene.cpp:58-68).
TPT_D bool shadow_query(const DScene& s, const BVert& v1, const BVert& v2, int& cull) {
    V3 atob = v2.x - v1.x;
    cull = TPT_CULL_BACK;
    if (v1.prim >= 0 && v2.prim != v1.prim && s.mats[v1.mat].type == TPT_TRANSPARENT) {
        if (dot3(atob, v1.N) < 0.0f) cull = TPT_CULL_FRONT;
        return true;
    }
    if (v1.prim >= 0 && dot3(atob, v1.N) < 0.0f) return false;  // fast path "not shadowed" (Scene.cpp:71-74)
    if (v2.prim >= 0 && dot3(-atob, v2.N) < 0.0f) return false;  // Scene.cpp:75-78
    return true;
}
TPT_D bool shadow_v(const DScene& s, const BVert& v1, const BVert& v2) {
    int cull;
    return shadow_query(s, v1, v2, cull) && shadow_ray(s, v1.x, v2.x, cull);
}

// BDPTPath::PathWeight (BDPT.cpp:173-259) for light sub-length sl, camera sub-length tl.
// Paths are read through an accessor P: P::cam(j), P::lit(j) return vertex records,
// P::camq / P::litq the cached MIS factors (rr .8 when `r8`).
// kCls >= 0: the caller's strategies are all of one task class (tpt_bdpt_scatter_kernel's
// runs: 0 s = 0, 1 t > 1 and s > 1, 2 t > 1 and s = 1, 3 t = 1), so the branches of the
// other classes fold away (the same float ops in the same order for the strategies run).
// kDS: the shadow query is not made here; *need is set when the strategy needs it (a
// non-zero unshadowed contribution with sl != 0) and the caller makes it (the queued
// connect, tpt_capi.hip): the result is then this value or 0.
template <int kCls = -1, bool kDS = false, class P>
TPT_D V3 path_weight(const DScene& s, const P& paths, int sl, int tl, bool* need = nullptr) {
    if constexpr (kCls == 0) __builtin_assume(sl == 0 && tl >= 2);
    if constexpr (kCls == 1) __builtin_assume(sl >= 2 && tl >= 2);
    if constexpr (kCls == 2) __builtin_assume(sl == 1 && tl >= 2);
    if constexpr (kCls == 3) __builtin_assume(tl == 1 && sl >= 1);
    const int z = tl - 1;
    const BVert cz = paths.cam(z);
    if (cz.type == T_BG) return sl == 0 ? cz.alpha * v3(s.bg[0], s.bg[1], s.bg[2]) : v3s(0.0f);
    const BVert ly = sl >= 1 ? paths.lit(sl - 1) : cz;
    if (sl != 0 && ly.type == T_BG) return v3s(0.0f);
    const V3 cpre = z >= 1 ? paths.cam(z - 1).x : cz.x;
    const V3 lpre = sl >= 2 ? paths.lit(sl - 2).x : ly.x;
    V3 cst;
    float srA0 = 0.0f, srB0 = 0.0f;  // set when sl >= 1
    if (sl == 0) {
        V3 wi = normalized(cpre - cz.x);
        V3 em = v3s(0.0f);  // PathVertex::Emission (BDPT.hpp:119-128)
        if (cz.prim >= 0) em = load_mat(s, cz.mat).em;
        cst = mul(em, (float)dot3(normal_of(cz.type, cz.N), wi));
        if (dot3(em, em) == 0.0f) return v3s(0.0f);
    } else {
        float d2;
        V3 dir = normalize_len2(cz.x - ly.x, &d2);
        // Scene::ShadowCheck (BDPT.cpp:205) is deferred to the end: a shadowed
        // strategy returns 0, so the test only matters when the unshadowed result is
        // not 0 (about a quarter of the tested strategies are 0 anyway).
        // each vertex's BSDF toward the other and the solid-angle pdf that Append
        // computes for the same pair in loops A/B at k = 0 (ly -> cz: dir; cz -> ly:
        // normalize(ly - cz) == -dir bit for bit), evaluated together
        V3 fl, fc;
        eval_pair_sa(s, ly.type, ly.mat, ly.x, ly.N, lpre, dir, fl, srB0);
        eval_pair_sa(s, cz.type, cz.mat, cz.x, cz.N, cpre, -dir, fc, srA0);
        cst = mul(fl * fc, (float)dabs_(dot3(normal_of(ly.type, ly.N), dir) * dot3(normal_of(cz.type, cz.N), -dir) / (double)d2));
    }
    float wd = 1.0f;
#ifndef TPT_DIAG_NO_MIS
#define TPT_DIAG_NO_MIS 0  // diagnostics builds only (timing attribution; wrong images): no MIS chains
#endif
    // loop A: camera prefix C[0..tl), append L[sl-1], ..., L[0]
    float cur = 1.0f;
    for (int k = 0; k < (TPT_DIAG_NO_MIS ? 0 : sl); ++k) {
        const int j = sl - 1 - k;
        if (k >= 2) {
            cur *= paths.litq(j, tl + k > 4);
        } else {
            const BVert v = k == 0 ? ly : paths.lit(j);
            float pdf;
            if (k == 0) pdf = srpdf_to_area(srA0, cz.type, cz.x, cz.N, v.type, v.x, v.N);  // append_pdf(cz -> ly)
            else pdf = append_pdf(s, ly.type, ly.mat, ly.x, ly.N, cz.x, v.type, v.x, v.N);
            pdf *= rr_of(tl + k);
            cur *= safe_div(pdf, v.pdf);
        }
        wd += cur * cur;
        if (cur == 0.0f) break;
    }
    // loop B: light prefix L[0..sl), append C[tl-1], ..., C[0]
    cur = 1.0f;
    for (int k = 0; k < (TPT_DIAG_NO_MIS ? 0 : tl); ++k) {
        const int j = tl - 1 - k;
        const int count = sl + k;
        if (k >= 2) {
            cur *= paths.camq(j, count > 4);
        } else {
            const BVert v = k == 0 ? cz : paths.cam(j);
            float pdf;
            if (count == 0) {
                pdf = prim_pdf(s, v.prim);  // Append(count==0): vertex.obj->pdf(), no RR factor
            } else {
                if (k == 0) {
                    pdf = srpdf_to_area(srB0, ly.type, ly.x, ly.N, v.type, v.x, v.N);  // append_pdf(ly -> cz), sl >= 1
                } else {
                    // last = C[tl-1] as appended (type Light when it opened the path, BDPT.cpp:240-242)
                    const int at = sl == 0 ? T_LIGHT : cz.type;
                    pdf = append_pdf(s, at, cz.mat, cz.x, cz.N, sl >= 1 ? ly.x : cz.x, v.type, v.x, v.N);
                }
                pdf *= rr_of(count);
            }
            cur *= safe_div(pdf, v.pdf);
        }
        wd += cur * cur;
        if (cur == 0.0f) break;
    }
    V3 lt = sl == 0 ? v3s(1.0f) : ly.alpha;
    V3 uc = lt * cz.alpha * cst;
    const V3 res = divs(uc, wd);
    if (sl != 0) {
        // Zero after the clamp either way (NaN compares false and is tested): +0 and
        // -0 sum identically into the pixel (its sum starts at +0) and t = 1 splats
        // skip zeros, so returning +0 without the test is exact.
        const V3 c = vmax0(res);
        if (c.x == 0.0f && c.y == 0.0f && c.z == 0.0f) return v3s(0.0f);
#ifndef TPT_DIAG_NO_CONN_SHADOW
#define TPT_DIAG_NO_CONN_SHADOW 0  // diagnostics builds only (timing attribution; wrong images)
#endif
        if constexpr (kDS) {
            *need = true;
        } else {
            if (!TPT_DIAG_NO_CONN_SHADOW && shadow_v(s, cz, ly)) return v3s(0.0f);
        }
    }
    return res;
}

// DrawToImage (SceneRenderingHelper.cpp:24-55), BlendMode::Additive, fp32 atomics,
// for the splats of a whole wave (call with every lane of the wave that is still in
// the loop; `want` marks the lanes that have a splat).  Same float ops per tap as
// the reference (zero contributions skipped), but the adds are regrouped: a splat touches a 3x3 block of
// pixels = three row segments of 9 contiguous floats (rgb), so 27 lanes add one
// splat with ONE atomic wave-instruction (two splats per instruction: lanes 0-26
// and 32-58).  A per-lane form issues 64 adds to 64 scattered rows per
// instruction, which the memory-side atomic unit serves ~17x slower per byte
// (MI355X_MICROARCH.md, Global float atomics).  Only the summation order changes,
// and fp32 atomics have no fixed order anyway.
TPT_D void splat_wave(const DScene& s, bool want, V3 light, V3 cam, V3 value, float* splat) {
    want = want && !(value.x == 0.0f && value.y == 0.0f && value.z == 0.0f);
    float cx = 0.0f, cy = 0.0f;
    if (want) {
        V3 d = normalized(light - cam);
        d = divs(d, d.z);
        float aspect = (float)(s.width / s.height);
        V3 t = v3(-d.x / s.scale / aspect, -d.y / s.scale, 0.0f);
        V3 uv = mul(t + v3s(1.0f), 0.5f);
        cx = uv.x * s.width;
        cy = uv.y * s.height;
    }
    unsigned long long m = __ballot(want);
    const int l = (int)__lane_id();
    const int half = l >> 5, j = l & 31;
    const int tap = j / 3, comp = j - 3 * tap;
    const int ox = tap % 3 - 1, oy = tap / 3 - 1;
    while (m != 0) {
        const int a = __builtin_ctzll(m);
        m &= m - 1;
        const bool two = m != 0;  // a second splat for the upper half-wave
        const int b = two ? __builtin_ctzll(m) : a;
        if (two) m &= m - 1;
        auto pick = [&](float v) {
            const int va = __builtin_amdgcn_readlane(__float_as_int(v), a);
            const int vb = __builtin_amdgcn_readlane(__float_as_int(v), b);
            return __int_as_float(half ? vb : va);
        };
        const float px = pick(cx), py = pick(cy), vr = pick(value.x), vg = pick(value.y), vb = pick(value.z);
        if (j < 27 && (!half || two)) {
            const int ix = (int)px + ox, iy = (int)py + oy;
            if (ix >= 0 && iy >= 0 && ix < s.width && iy < s.height) {
                float dx = fabs_(px - (ix + 0.5f)), dy = fabs_(py - (iy + 0.5f));
                float w = smax(0.0f, 1.0f - dx) * smax(0.0f, 1.0f - dy);
                const float c = (comp == 0 ? vr : comp == 1 ? vg : vb) * w;
                if (c != 0.0f) atomicAdd(splat + 3 * ((int64_t)ix + (int64_t)s.height * iy) + comp, c);
            }
        }
    }
}

// GenerateCameraPath's v0 (BDPT.cpp:41-47): the camera, the same for every pixel; made
// where used (an opaque copy of the eye: hoisted out of a persistent loop it spilled).
TPT_D BVert camera_v0(const DScene& s) {
    // every field through an opaque copy: the constants too (as VGPR vectors hoisted
    // out of the loop they were spilled)
    float ex = s.eye[0], ey = s.eye[1], ez = s.eye[2], z = 0.0f, one = 1.0f, pdf = kCamZeroPdf;
    int m = -1;
    asm volatile("" : "+v"(ex), "+v"(ey), "+v"(ez), "+v"(z), "+v"(one), "+v"(pdf), "+v"(m));
    BVert c0;
    c0.x = v3(ex, ey, ez); c0.N = v3s(z); c0.type = T_CAM; c0.prim = m; c0.mat = m;
    c0.pdf = pdf; c0.alpha = v3s(one); c0.q1 = c0.q8 = z;
    return c0;
}
// GenerateCameraPath's v0/v1 (BDPT.cpp:41-59): identical for every sample of a pixel.
TPT_D void camera_vertices(const DScene& s, int64_t i, BVert& c0, BVert& c1) {
    const int px = (int)(i % s.width), py = (int)(i / s.width);
    // opaque copies: the f64 conversions of width, height, aspect and scale are made
    // here, not hoisted out of gen's persistent loop and spilled across it
    int w = s.width, h = s.height;
    float sc = s.scale;
    asm volatile("" : "+v"(w), "+v"(h), "+v"(sc));
    const V3 dir = pixel_ray(px, py, w, h, sc);
    const V3 eye = v3(s.eye[0], s.eye[1], s.eye[2]);
    c0.x = eye; c0.N = v3s(0.0f); c0.type = T_CAM; c0.prim = -1; c0.mat = -1;
    c0.pdf = kCamZeroPdf; c0.alpha = v3s(1.0f); c0.q1 = c0.q8 = 0.0f;
    PTV h1 = scene_intersect(s, make_ray(eye, dir), TPT_CULL_BACK);
    c1.x = h1.x; c1.N = h1.N; c1.type = h1.type; c1.prim = h1.prim;
    c1.mat = h1.prim >= 0 ? prim_mat(s, h1.prim) : -1;
    c1.pdf = srpdf_to_area(kCamRayPdf, T_CAM, c0.x, c0.N, h1.type, h1.x, h1.N);
    c1.alpha = v3s(1.0f);
    c1.q1 = c1.q8 = 0.0f;
}

// ------------------------------------------------------------ wavefront --
// A wavefront holds `nb` consecutive sample iterations of n pixel streams: its items
// are (iteration b, pixel k), item = b * n + k.  For every item:
//   gen:     generate both subpaths and write them to HBM as vertex records; one lane
//            runs its pixel's nb samples back to back (the RNG stream is sequential
//            per pixel), so a small shard still fills a wavefront as large as a full
//            frame's and the per-wavefront tail is paid once per nb iterations;
//   scan:    inclusive prefix sums of the strategy counts per item;
//   scatter: task[g] = (item, t, s) for every strategy, in four class runs, so a
//            wave holds one kind (4 B per task; the result slot is the task's index);
//   connect: ONE LANE PER STRATEGY (PathWeight), so a wave's work is 64 strategies
//            instead of the longest lane's cn*(ln+1) (measured 18 mean vs 73 max);
//            t = 1 splats go straight to the splat buffer;
//   fold:    per pixel, for b = 0 .. nb-1 in order: result += w over the item's
//            strategies in (t, s) order (t > 1), fb += (1/spp) * result -- the
//            reference's summation order.
// One vertex record = 64 B = four float4: (x, type|prim) (N, pdf) (alpha, mat) (q1, q8, -, -),
// laid out [item][slot] so a vertex is one contiguous line segment (4 x 16-B accesses).
constexpr int kRecV = 4;  // float4 per vertex record
struct WfState {
    float4* rec;          // items * 32 * kRecV float4
    int* cnt;             // per item: cn | ln << 16
    // strategies per pixel in four classes (task runs, see tpt_bdpt_scatter_kernel):
    //   np  = (s = 0: cn - 1) | (t > 1, s > 1: (cn - 1)(ln - 1)) << 32
    //   np2 = (t > 1, s = 1: cn - 1) | (t = 1: ln) << 32
    unsigned long long* np;
    unsigned long long* incl;   // inclusive scan of np (both halves at once)
    unsigned long long* np2;
    unsigned long long* incl2;  // inclusive scan of np2
    unsigned* task;       // strategy -> item | t << 22 | s << 27 (item < kWfChunk)
    float* res;           // 3 floats per strategy, in task order
    float* isum;          // 3 floats per item: its result (nb > 1 folds in two passes)
    // Per pixel stream: (wavefronts completed) << 32 | XorShift32 state.  Consecutive
    // wavefronts' gen kernels run concurrently (two streams): the lane that finishes
    // pixel k's samples of wavefront f publishes seq f + 1 with the state in ONE 64-bit
    // agent-scope atomic store, and gen(f + 1) starts pixel k once it reads seq f + 1.
    unsigned long long* rngseq;
    int* stall;           // set when a gen lane gave up waiting (watchdog); never in a good run
    unsigned stall_ticks; // the watchdog's limit (100 MHz real-time counter ticks)
    int drop_k;           // diagnostics builds (TPT_DIAG_HOOKS): pixel ordinal whose wavefront-1
                          // publication gen skips, to drive the watchdog path; -1 otherwise
    int conc;             // 1: consecutive wavefronts' gen kernels run concurrently (two streams)
    int cam_nb;           // items (b, k) with b < cam_nb of this buffer already hold the camera vertices
                          // (an earlier wavefront of the chunk in the same buffer wrote them)
    float* acc;           // 3 floats per pixel
    const int64_t* list;  // pixel list (or null: begin + k*stride)
    int64_t begin, stride, n;  // n: pixel streams
    int nb;                    // sample iterations in this wavefront (items = nb * n)
    int64_t ni;                // items = nb * n
    unsigned long long* bounces;
};
// One wavefront holds at most kWfChunk items (launch() splits larger shards, and sizes
// nb so that nb * n <= kWfChunk): the task record keeps the item in 22 bits and the
// per-class scans count in 32.
constexpr int64_t kWfChunk = int64_t(1) << 22;
constexpr unsigned kTaskPixelMask = (unsigned)kWfChunk - 1;
static_assert(kMaxLen < 32, "task records keep t and s in 5 bits each");
static_assert(kWfChunk * (kMaxLen * (kMaxLen + 1)) < (int64_t(1) << 32), "per-class scan halves are 32-bit");
TPT_D int64_t wf_pixel(const WfState& w, int64_t k) { return w.list ? w.list[k] : w.begin + k * w.stride; }
TPT_D int tp_pack(int type, int prim) { return (prim + 1) * 4 + type; }
TPT_D float4* rec_at(float4* rec, int64_t k, int slot) { return rec + ((k * (2 * kMaxLen) + slot) * kRecV); }
// Stores of the wavefront state (plain stores, published by the kernel's end).
// kZ (the walk-scene gen kernel): the record's unused pad zeros are made at the store --
// hoisted out of gen<2>'s persistent loop as a register quad they were spilled and
// reloaded at every store (gen<1> keeps the constant form: the opaque one costs it 12
// B/lane of scratch)
#ifndef TPT_GEN_REC_Z
#define TPT_GEN_REC_Z 1
#endif
template <bool kZ = false>
TPT_D void rec_store(const WfState& w, int slot, int64_t k, const BVert& v) {
    float4* r = rec_at(w.rec, k, slot);
    r[0] = make_float4(v.x.x, v.x.y, v.x.z, __builtin_bit_cast(float, tp_pack(v.type, v.prim)));
    r[1] = make_float4(v.N.x, v.N.y, v.N.z, v.pdf);
    r[2] = make_float4(v.alpha.x, v.alpha.y, v.alpha.z, __builtin_bit_cast(float, v.mat));
    if constexpr (kZ) {
        float z = 0.0f;
        asm volatile("" : "+v"(z));
        r[3] = make_float4(v.q1, v.q8, z, z);
    } else {
        r[3] = make_float4(v.q1, v.q8, 0.0f, 0.0f);
    }
}
TPT_D void rec_store_q(const WfState& w, int slot, int64_t k, float q1, float q8) {
    *reinterpret_cast<float2*>(rec_at(w.rec, k, slot) + 3) = make_float2(q1, q8);
}

// One generation step of a lane's sample, for the persistent gen kernel: either
// GenerateLightPath's start (phase 1: light vertex l0 from m_emissionObjects[0] and
// the first bounce l1, BDPT.cpp:61-90) or one iteration of
// FillPathUsingRussianRoulette's loop (BDPT.cpp:92-118 with SampleNextVertex,
// :261-279).  Both end in ONE closest-hit query, so a wave whose lanes are in
// different phases traces a single query.  Vertices stream into the HBM records as
// they are made; vertex j's reverse pdf (Append(P[j]) after last = P[j+1], Pre =
// P[j+2], folded into q1 / q8) is written as soon as P[j+2] exists, so only a
// three-vertex window is live.  Same draws, vertices and float ops as the reference.
// Returns false when the current subpath has ended: its vertex count is then i + 1.
// Deferred walks (round 4; walk-group scenes).  A lane whose extension ray passes the
// walk group's box walks the mesh's tree; in a wave of persistent gen lanes only a few
// need that at any one step, and the whole wave waits on their walks.  With kDefer a
// lane that needs the walk while fewer than TPT_GEN_DEFER_MIN lanes of its wave do
// parks the step half done -- the ray direction, the pdf and culling, and its closest
// hit over the flat groups before the walk group (the DFS order) -- in its LDS slot
// (GenDefer) and makes no progress this iteration; the parked lanes walk together a
// few iterations later (when enough lanes want a walk, when one has waited
// TPT_GEN_DEFER_MAX iterations, or when no other lane is active), then fold the flat
// groups after the walk group and finish the step.  The lane's draws, operands, fold
// order and stores are exactly the undeferred step's: only the time differs.
#ifndef TPT_GEN_DEFER
#define TPT_GEN_DEFER 1
#endif
#ifndef TPT_GEN_DEFER_MIN
#define TPT_GEN_DEFER_MIN 12  // lanes wanting a walk before a wave walks (round 6, with the stealing walks and
                              // the compiler changes, bunny 256 spp 24 / 20 / 16 / 12 / 8 -> 624.4 / 619.1 /
                              // 617.0 / 616.3 / 619.5 ms, 1/8 shard 93.2 / 92.6 / 91.8 / 91.6 / 91.0 ms)
#endif
#ifndef TPT_GEN_DEFER_MAX
#define TPT_GEN_DEFER_MAX 3  // iterations a parked lane waits at most
#endif
enum { kGdDx, kGdDy, kGdDz, kGdSr, kGdCl, kGdPrim, kGdDlo, kGdDhi, kGenDeferSlots };
struct GenDefer {  // [slot][lane] in LDS
    float* base;
    TPT_D float& at(int slot) const { return base[slot * kBlock + threadIdx.x]; }
};

// Deferred walks with work stealing (round 5, TPT_WALK_STEAL).  A wave's deferred walk
// ran as long as its longest lane's (46 steps against 16.9 on average, ~20 of 64 lanes
// walking): the other lanes idled.  Here every lane of the wave that reached the walk
// takes part.  A lane whose walk has ended (or that had none) takes the bottom entry
// of another lane's pending stack -- a whole subtree of that lane's ray -- and walks it
// with the owner's ray (rebuilt from the owner's LDS slots: the same make_ray, so the
// same bits).  Each job (a subtree) folds its triangles in its own DFS order with
// BVHAccel::Intersect's strict `>` (BVH.cpp:103-143), which keeps the job's nearest hit
// of smallest DFS rank; the jobs' hits are then merged per ray by (distance, DFS rank)
// (HostScene::grank), which is exactly the sequential fold's answer: its first
// minimum.  (The merge is a wave-uniform scan of the list by each owner; a version
// with LDS atomic minima lost hits -- why: DESIGN.md §5.2 -- and was not kept;
// tests/test_steal_walk.py runs this function on an emulated wave.)  The walk group's leaves all follow the flat groups before it in the DFS
// order and precede the ones after, so the caller folds the merged hit into `best`
// with the same strict `>`.  Distances are finite (finite rays, |det| >= 1e-4), and
// -0.0 ties +0.0 as in the reference (the key clears the sign; the winner's own bits
// are returned).  Only the time differs from the per-lane walk.
#ifndef TPT_WALK_STEAL
#define TPT_WALK_STEAL 1
#endif
// the origin's slots while a walk runs (their parked values are in registers by then)
enum { kGdOx = kGdPrim, kGdOy = kGdDlo, kGdOz = kGdDhi };
constexpr int kStealList = kQC - 64;  // jobs per walk at most, so the stolen jobs' hit list fits QScratch::res
TPT_D unsigned long long dist_key(double d) { return (unsigned long long)__double_as_longlong(d) & 0x7fffffffffffffffull; }
// Does hit a come before hit b in the walk's fold (strict `>` in DFS order): a nearer
// distance, or the same distance (key: -0.0 ties +0.0) and a lower DFS rank?  The
// ranks are read only on a tie.
TPT_D bool hit_before(const DScene& s, const Hit& a, const Hit& b) {
    if (b.prim < 0) return true;
    const unsigned long long ka = dist_key(a.dist), kb = dist_key(b.dist);
    if (ka != kb) return ka < kb;
    return s.grank[a.prim] < s.grank[b.prim];
}
TPT_D Ray owner_ray(const GenDefer& dl, int l, int& cl) {
    const float* b = dl.base + ((int)threadIdx.x & ~63) + l;
    cl = __float_as_int(b[kGdCl * kBlock]);
    return make_ray(v3(b[kGdOx * kBlock], b[kGdOy * kBlock], b[kGdOz * kBlock]),
                    v3(b[kGdDx * kBlock], b[kGdDy * kBlock], b[kGdDz * kBlock]));
}
// `need` lanes walk the group whose 4-wide root is qnodes[root] with their ray (r, cl),
// which they have stored in their dl slots; returns each need lane's first-minimum hit
// in the group (prim -1: none).  Every active lane must call it (wave-synchronous).
TPT_D Hit walk4_steal(const DScene& s, int root, bool need, Ray r, int cl, const GenDefer& dl) {
    QScratch* qs = wave_qs(s);
    const int lane = (int)__lane_id();
    uint16_t* st = s.ws + threadIdx.x;  // [slot][lane]
    int sb = 0, sp = 0, cur = root, owner = lane;
    bool job = need;
    Hit jb;
    jb.prim = -1;
    jb.dist = 0.0;
    int ncnt = 0, jobs = __popcll(__ballot(need));
    Hit own;  // the merged hits of this lane's own ray's jobs that this lane walked
    own.prim = -1;
    own.dist = 0.0;
    for (;;) {
        bool done = false;
        if (job) {  // one step of the job's walk (walk4's)
            if (cur < 0) {
                const int prim = -1 - cur;
                double dist;
                if (tri_test(load_gtri(s.gtris + prim), r, cl, dist) && (jb.prim < 0 || jb.dist > dist)) {
                    jb.dist = dist;
                    jb.prim = prim;
                }
                if (sp == sb) done = true;
                else cur = (int)(int16_t)st[kBlock * --sp];
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
        // an ended job's hit: into the lane's own result when the ray is its own, else
        // onto the wave's list
        if (done && jb.prim >= 0 && owner == lane && hit_before(s, jb, own)) own = jb;
        const uint64_t fm = __ballot(done && jb.prim >= 0 && owner != lane);
        if (fm != 0) {
            if (done && jb.prim >= 0 && owner != lane) {
                const int e = ncnt + mbcnt64(fm);
                qs->res[e] = jb.dist;
                qs->prim[e] = jb.prim;
                qs->pair[e] = (uint16_t)owner;
            }
            ncnt += __popcll(fm);
        }
        if (done) job = false;
        const uint64_t jm = __ballot(job);
        if (jm == 0) break;
        // idle lanes take the bottom entries of lanes with pending entries (k-th idle
        // lane from the k-th such lane, through a mailbox)
        const uint64_t vm = __ballot(job && sp > sb);
        const uint64_t im = __ballot(!job);
        int m = __popcll(im) < __popcll(vm) ? __popcll(im) : __popcll(vm);
        if (m > kStealList - jobs) m = kStealList - jobs;
        if (m > 0) {
            if (job && sp > sb) {
                const int rv = mbcnt64(vm);
                if (rv < m) {
                    qs->flag[rv] = (uint32_t)st[kBlock * sb] | (uint32_t)owner << 16;
                    ++sb;
                }
            }
            wave_lds_sync();
            if (!job) {
                const int ri = mbcnt64(im);
                if (ri < m) {
                    const uint32_t mb = qs->flag[ri];
                    cur = (int)(int16_t)(mb & 0xffffu);
                    owner = (int)(mb >> 16);
                    r = owner_ray(dl, owner, cl);
                    job = true;
                    sb = sp = 0;
                    jb.prim = -1;
                    jb.dist = 0.0;
                }
            }
            jobs += m;
            wave_lds_sync();  // the mailbox is reused
        }
    }
    // per ray: the least (distance key, DFS rank) over its own result and its list entries
    wave_lds_sync();
    Hit out = own;
    for (int e = 0; e < ncnt; ++e) {
        if (need && (int)qs->pair[e] == lane) {
            Hit h;
            h.dist = qs->res[e];
            h.prim = qs->prim[e];
            if (hit_before(s, h, out)) out = h;
        }
    }
    wave_lds_sync();  // QScratch is reused by the next query
    return out;
}

#ifndef TPT_GEN_STATS
#define TPT_GEN_STATS 0
#endif
#if TPT_GEN_STATS
// diagnostics only: [0] wave-ticks inside deferred-step walks, [1] such walks, [2] lanes
// walking in them, [3] wave-ticks inside whole gen steps, [4] steps (100 MHz ticks)
TPT_TU_STATIC __device__ unsigned long long tpt_walkstat[8];
#endif
#ifndef TPT_GEN_MERGE
#define TPT_GEN_MERGE 1  // one call site for both phases' cosine-weighted samples (gen_step_t)
#endif
// One generation step (see the comment above gen_step's callers).  Returns 1 when the
// subpath continues, 0 when it has ended (its vertex count is then i + 1), 2 when the
// step was deferred (kDefer only; `pend` counts the iterations it has waited).
template <bool kDefer>
TPT_D int gen_step_t(const DScene& s, const WfState& w, int64_t k, int& phase, BVert& prev, BVert& cur, int& i,
                     uint32_t& rs, int& pend, GenDefer dl, int gw) {
    const bool start = phase == 1;
    bool go = true;
    Ray ray;
    int cl = TPT_CULL_BACK;
    float sr = 0.0f;
    Hit best;
    best.prim = -1;
    best.dist = 0.0;
    const bool resumed = kDefer && pend != 0;
    if (resumed) {
        sr = dl.at(kGdSr);
        cl = __float_as_int(dl.at(kGdCl));
        best.prim = __float_as_int(dl.at(kGdPrim));
        best.dist = __hiloint2double(__float_as_int(dl.at(kGdDhi)), __float_as_int(dl.at(kGdDlo)));
        ray = make_ray(cur.x, v3(dl.at(kGdDx), dl.at(kGdDy), dl.at(kGdDz)));  // the same Ray as when parked
    } else if (TPT_GEN_MERGE) {
        // Both phases' cosine-weighted samples in ONE call site (round 6): the light start's
        // (GenerateLightPath, BDPT.cpp:61-90) and the Dieletric extension's diffuse branch
        // (Material::sample, Material.cpp:150-214).  In a wave of persistent lanes both
        // kinds are nearly always present, and as two call sites the f64 sin/cos ran twice
        // per step with a few lanes each.  Per lane the same draws in the same order (the
        // light sample's three, or the GGX pair and the coin, before the cosine pair) and
        // the same float operations; only the SIMD schedule changes.
        BVert l0;
        V3 wo = v3s(0.0f), wi = v3s(0.0f), H = v3s(0.0f);
        float pdfv = 0.0f;
        Shade csh;
        bool wantc = false, diel = false, spec = false;
        float rough = 0.0f;
        if (start) {
            const DObj lo = s.objs[s.emitters[0]];
            V3 pc, pn;
            int pp;
            object_sample(s, lo, pc, pn, pp, rs);
            l0.x = pc; l0.N = pn; l0.type = T_LIGHT; l0.prim = pp; l0.mat = lo.mat;
            l0.pdf = lo.pdf;
            l0.alpha = divs(load_mat(s, lo.mat).em, l0.pdf);
            l0.q1 = l0.q8 = 0.0f;
            csh = make_shade(pn, pn);
            wantc = true;
        } else {
            go = !(i >= kMaxLen - 1 || cur.type == T_BG);
            if (go) {
                wo = normalized(prev.x - cur.x);
                const Mat m = load_mat(s, cur.mat);
                if (m.type == TPT_DIELETRIC) {
                    diel = true;
                    rough = m.rough;
                    csh = make_shade(cur.N, wo);
                    const float d1 = rng_float(rs), d2 = rng_float(rs);
                    spec = xorshift32(rs) < kCoinHalf;  // rng_float(rs) < 0.5f
                    if (spec) {
                        H = ggx_h(csh, rough, d1, d2);
                        wi = reflect(wo, H);
                    } else {
                        wantc = true;
                    }
                } else {
                    wi = mat_sample<true>(m, wo, cur.N, &pdfv, rs);
                }
            }
        }
        float pdc = 0.0f;
        if (wantc) wi = cosine_sample(csh, pdc, rs);
        if (start) {
            const float ct = (float)dot3(l0.N, wi);
            sr = safe_div(pdc, ct);
            ray = make_ray(l0.x, wi);
            rec_store<kDefer && TPT_GEN_REC_Z>(w, kMaxLen, k, l0);
            cur = l0;
        } else if (go) {
            if (diel) {  // Material::sample's Dieletric tail, either branch (mat_sample<true>)
                const V3 n = csh.n;
                if (!spec) H = normalized(wi + wo);
                const float pdf_h = ggx_half_pdf(n, H, rough);
                const float jr = safe_div(1.0f, 4.0f * fabs_((float)dot3(wo, H)));
                const float pd = spec ? cosine_pdf(n, wi) : pdc;
                pdfv = (pdf_h * jr + pd) * 0.5f;
                if ((double)csh.nv * dot3(wi, n) < 0.0f) pdfv = 0.0f;
            }
            const float rr = i > 4 ? .8f : 1.f;
            go = !(rng_float(rs) > rr);
            if (go) {
                const float ct = (float)dabs_(dot3(cur.N, wi));
                sr = safe_div(pdfv, ct);
                ray = make_ray(cur.x, wi);
                cl = dot3(cur.N, wi) > 0.0f ? TPT_CULL_BACK : TPT_CULL_FRONT;
            }
        }
    } else if (start) {
        const DObj lo = s.objs[s.emitters[0]];
        V3 pc, pn;
        int pp;
        object_sample(s, lo, pc, pn, pp, rs);
        BVert l0;
        l0.x = pc; l0.N = pn; l0.type = T_LIGHT; l0.prim = pp; l0.mat = lo.mat;
        l0.pdf = lo.pdf;
        l0.alpha = divs(load_mat(s, lo.mat).em, l0.pdf);
        l0.q1 = l0.q8 = 0.0f;
        float pdf1;
        const V3 wi = cosine_sample(pn, pdf1, rs);
        const float ct = (float)dot3(l0.N, wi);
        sr = safe_div(pdf1, ct);
        ray = make_ray(l0.x, wi);
        rec_store<kDefer && TPT_GEN_REC_Z>(w, kMaxLen, k, l0);
        cur = l0;
    } else {
        go = !(i >= kMaxLen - 1 || cur.type == T_BG);
        if (go) {
            const V3 wo = normalized(prev.x - cur.x);
            float raw;
            const V3 wi = mat_sample<true>(load_mat(s, cur.mat), wo, cur.N, &raw, rs);  // same draws, fewer live values
            const float rr = i > 4 ? .8f : 1.f;
            go = !(rng_float(rs) > rr);
            if (go) {
                const float ct = (float)dabs_(dot3(cur.N, wi));
                sr = safe_div(raw, ct);
                ray = make_ray(cur.x, wi);
                cl = dot3(cur.N, wi) > 0.0f ? TPT_CULL_BACK : TPT_CULL_FRONT;
            }
        }
    }
    if (!go) return 0;
    PTV it;
    if (!kDefer || gw < 0 || !(s.flat & kFlatHit) || !wave_finite(ray)) {
        // Scene::Intersect as a whole (a parked lane's ray is finite, but another lane's
        // may not be: the threaded walk then answers every lane, parked ones included,
        // with the same result)
        it = scene_intersect(s, ray, cl);
        if (kDefer) pend = 0;
    } else {
        if (!resumed) closest_groups_c(s, 0, gw, ray, cl, best);  // the groups before the walk group
        const DNode gn = s.groups[gw];
        const bool need =
            resumed || slab_hit_finite(gn.bmin[0], gn.bmin[1], gn.bmin[2], gn.bmax[0], gn.bmax[1], gn.bmax[2], ray);
        const uint64_t nm = __ballot(need);
        const bool walk_now = __popcll(nm) >= TPT_GEN_DEFER_MIN || __ballot(resumed && pend >= TPT_GEN_DEFER_MAX) != 0 ||
                              __ballot(!need) == 0;
        if (need && !walk_now) {
            if (!resumed) {
                dl.at(kGdDx) = ray.d.x; dl.at(kGdDy) = ray.d.y; dl.at(kGdDz) = ray.d.z;
                dl.at(kGdSr) = sr;
                dl.at(kGdCl) = __int_as_float(cl);
                dl.at(kGdPrim) = __int_as_float(best.prim);
                dl.at(kGdDlo) = __int_as_float(__double2loint(best.dist));
                dl.at(kGdDhi) = __int_as_float(__double2hiint(best.dist));
            }
            pend = resumed ? pend + 1 : 1;
            return 2;
        }
#if TPT_GEN_STATS
        const unsigned long long tw0 = __builtin_amdgcn_s_memrealtime();
        const unsigned long long wl = __ballot(need);
        int wit = 0;
        if (need) group_closest(s, gn, ray, cl, best, &wit);
        int wmax = 0, wsum = 0;
        for (unsigned long long m = wl; m; m &= m - 1) {
            const int v = __builtin_amdgcn_readlane(wit, __builtin_ctzll(m));
            wmax = max(wmax, v);
            wsum += v;
        }
        if (wl && lane_id() == (unsigned)__builtin_ctzll(__ballot(true))) {
            atomicAdd(&tpt_walkstat[0], __builtin_amdgcn_s_memrealtime() - tw0);
            atomicAdd(&tpt_walkstat[1], 1ull);
            atomicAdd(&tpt_walkstat[2], (unsigned long long)__popcll(wl));
            atomicAdd(&tpt_walkstat[5], (unsigned long long)wsum);
            atomicAdd(&tpt_walkstat[6], (unsigned long long)wmax);
        }
#else
        if (TPT_WALK_STEAL && gn.b <= -2 && s.ws) {
            if (need) {  // the owner's ray, for the lanes that take part of its walk
                dl.at(kGdDx) = ray.d.x; dl.at(kGdDy) = ray.d.y; dl.at(kGdDz) = ray.d.z;
                dl.at(kGdCl) = __int_as_float(cl);
                dl.at(kGdOx) = ray.o.x; dl.at(kGdOy) = ray.o.y; dl.at(kGdOz) = ray.o.z;
            }
            const Hit wh = walk4_steal(s, -2 - gn.b, need, ray, cl, dl);
            if (wh.prim >= 0 && (best.prim < 0 || best.dist > wh.dist)) best = wh;
        } else if (need) {
            group_closest(s, gn, ray, cl, best);
        }
#endif
        pend = 0;
        closest_groups_c(s, gw + 1, s.ngroup, ray, cl, best);  // ... and after it
        it = ptv_bg();
        if (best.prim >= 0) {
            hit_geometry(s, ray, best, it.x, it.N);
            it.type = T_MID;
            it.prim = best.prim;
        }
    }
    const float pdf = srpdf_to_area(sr, cur.type, cur.x, cur.N, it.type, it.x, it.N);
    BVert nx;
    nx.x = it.x; nx.N = it.N; nx.type = it.type; nx.prim = it.prim;
    nx.mat = it.prim >= 0 ? prim_mat(s, it.prim) : -1;
    nx.q1 = nx.q8 = 0.0f;
    if (start) {
        nx.pdf = pdf;
        nx.alpha = v3s(0.0f);  // fresh InternalPathVertex (BDPT.hpp:19)
        if (sr != 0.0f) nx.alpha = safe_div(cur.alpha, sr);
        rec_store<kDefer && TPT_GEN_REC_Z>(w, kMaxLen + 1, k, nx);
        prev = cur;
        cur = nx;
        i = 1;
        phase = 2;
        return !(sr == 0.0f && it.type == T_BG) ? 1 : 0;
    }
    if (pdf == 0.0f) return 0;
    const V3 wo = normalized(prev.x - cur.x);
    const Mat m = load_mat(s, cur.mat);
    const float rr = i > 4 ? .8f : 1.f;
    const V3 bsdf = eval_bsdf(m, wo, ray.d, cur.N, false);
    nx.pdf = pdf * rr;
    nx.alpha = divs(cur.alpha * safe_div(bsdf, sr), rr);
    const int base = phase == 0 ? 0 : kMaxLen;
    rec_store<kDefer && TPT_GEN_REC_Z>(w, base + i + 1, k, nx);
    // path_rev for j = i - 1: Append(P[j]) after last = P[i], Pre = P[i+1]
    const float rev = append_pdf(s, cur.type, cur.mat, cur.x, cur.N, nx.x, prev.type, prev.x, prev.N);
    rec_store_q(w, base + i - 1, k, safe_div(rev * 1.f, prev.pdf), safe_div(rev * .8f, prev.pdf));
    prev = cur;
    cur = nx;
    ++i;
    return 1;
}
TPT_D bool gen_step(const DScene& s, const WfState& w, int64_t k, int& phase, BVert& prev, BVert& cur, int& i,
                    uint32_t& rs) {
    int pend = 0;
    return gen_step_t<false>(s, w, k, phase, prev, cur, i, rs, pend, GenDefer{nullptr}, -1) != 0;
}

struct GlobPaths {  // one pixel's paths in the HBM records
    const float4* rec;  // this pixel's 32 vertex records
    TPT_D BVert load(int slot) const {
        const float4* r = rec + slot * kRecV;
        const float4 a = r[0], b = r[1], c = r[2];
        const float2 q = *reinterpret_cast<const float2*>(r + 3);
        BVert v;
        v.x = v3(a.x, a.y, a.z);
        const int tp = __builtin_bit_cast(int, a.w);
        v.type = tp & 3;
        v.prim = (tp >> 2) - 1;
        v.N = v3(b.x, b.y, b.z);
        v.pdf = b.w;
        v.alpha = v3(c.x, c.y, c.z);
        v.mat = __builtin_bit_cast(int, c.w);
        v.q1 = q.x;
        v.q8 = q.y;
        return v;
    }
    TPT_D float q(int slot, bool r8) const {
        const float* r = reinterpret_cast<const float*>(rec + slot * kRecV + 3);
        return r8 ? r[1] : r[0];
    }
    TPT_D BVert cam(int j) const { return load(j); }
    TPT_D BVert lit(int j) const { return load(kMaxLen + j); }
    TPT_D float camq(int j, bool r8) const { return q(j, r8); }
    TPT_D float litq(int j, bool r8) const { return q(kMaxLen + j, r8); }
};

}  // namespace tpt
