// oracle/tpt_oracle.cpp -- CPU RESTATEMENT OF THE REFERENCE'S HOT PATH.
//
// TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg may load this library, and only as the checker / CPU
// baseline -- never as the product path (the product is libtpt.so, HIP only).
//
// What it restates (reference = yangrc1234/ToyPathTracer-GAMES101-Assignment7,
// file:line relative to that repository):
//   RNG               global.cpp:5-22, Random.cpp:5
//   vector math       Vector.hpp:13-113 (DotProduct in double), Ray.hpp:12-15
//   camera / splat    SceneRenderingHelper.cpp:12-55
//   BVH build         BVH.cpp:30-99 (median split, std::sort tie order), :161-169
//   BVH traversal     BVH.cpp:103-143, Bounds3.hpp:92-115
//   light sampling    BVH.cpp:145-159, Triangle.hpp:31-40,58-60, Sphere.cpp:48-55
//   primitives        Triangle.cpp:77-118 (f64 Moller-Trumbore), Sphere.cpp:4-41,
//                     SampleHelperFunctions.cpp:4-18
//   scene queries     Scene.cpp:21-83
//   materials         Material.cpp:11-252, GGX.hpp:8-59,
//                     SampleHelperFunctions.{hpp,cpp}
//   PT integrator     PathTracer.cpp:6-134 (HEAD: direct lighting only, `break` :109)
//   BDPT integrator   BDPT.cpp:17-351, BDPT.hpp:15-169
//   render driver     Renderer.cpp:32-127
//
// Numerics contract: abs() on float/double is the
// float/double abs (MSVC semantics, the reference is built with `using std::abs`
// for the oracle); every implicit float<->double conversion of the reference is
// spelled out below; compiled with -ffp-contract=off.  Pinned bit-exact against
// oracle/_ref/libref.so (the reference itself) by tests/test_oracle_pinning.py.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <limits>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "../include/tpt.h"

namespace orc {

// ----------------------------------------------------------------- RNG ---
// global.cpp:5-13 (shifts 13, 17, 15), :15-17, :19-22.  thread_local state as
// Random.cpp:5.
static thread_local uint32_t rnd_state = 1;
// Traversal counters behind SURVEY.md §8(d)'s algorithmic bytes: BVH nodes popped
// (top + mesh BVHs, BVH.cpp:113) and triangle tests (Triangle.cpp:77).  Read by
// oracle_traversal_counts only.
static thread_local uint64_t cnt_nodes = 0, cnt_tris = 0;
static inline uint32_t xorshift32() {
    uint32_t x = rnd_state;
    x ^= x << 13;
    x ^= x >> 17;
    x ^= x << 15;
    rnd_state = x;
    return x;
}
static inline void reset_random(int seed) { rnd_state = (uint32_t)seed; }
static inline float rand_float() { return (float)((double)xorshift32() / 4294967295.0); }

// ---------------------------------------------------------------- math ---
static const float PI_F = 3.141592653589793f;  // global.hpp:7-8 (float M_PI)
static const float EPS = 1e-4f;                // Renderer.cpp:19

struct V3 {
    float x, y, z;
    V3() : x(0), y(0), z(0) {}
    V3(float a) : x(a), y(a), z(a) {}
    V3(float a, float b, float c) : x(a), y(b), z(c) {}
};
static inline V3 operator+(V3 a, V3 b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline V3 operator-(V3 a, V3 b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline V3 operator*(V3 a, V3 b) { return V3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline V3 operator/(V3 a, V3 b) { return V3(a.x / b.x, a.y / b.y, a.z / b.z); }
static inline V3 operator-(V3 a) { return V3(-a.x, -a.y, -a.z); }
static inline V3 mul(V3 a, float r) { return V3(a.x * r, a.y * r, a.z * r); }   // Vector.hpp:25, :48
static inline V3 divs(V3 a, float r) { return V3(a.x / r, a.y / r, a.z / r); }  // Vector.hpp:26
static inline double dot(V3 a, V3 b) {                                            // Vector.hpp:103-104
    return (double)a.x * b.x + (double)a.y * b.y + (double)a.z * b.z;
}
static inline V3 cross(V3 a, V3 b) {                                              // Vector.hpp:106-113
    return V3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline V3 normalized(V3 a) {                                               // Vector.hpp:31-34
    float n = std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z);
    return V3(a.x / n, a.y / n, a.z / n);
}
static inline float magnitude(V3 a) { return std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }
static inline V3 normalize_len2(V3 a, float* len2) {                              // Vector.hpp:36-39
    *len2 = (float)dot(a, a);
    return divs(a, std::sqrt(*len2));
}
static inline V3 vmin(V3 a, V3 b) { return V3(std::min(a.x, b.x), std::min(a.y, b.y), std::min(a.z, b.z)); }
static inline V3 vmax(V3 a, V3 b) { return V3(std::max(a.x, b.x), std::max(a.y, b.y), std::max(a.z, b.z)); }
static inline float comp(V3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }

struct Ray {                                                                      // Ray.hpp:12-15
    V3 o, d, inv;
    Ray(V3 oo, V3 dd) : o(oo), d(dd) {
        inv = V3((float)(1. / dd.x), (float)(1. / dd.y), (float)(1. / dd.z));
    }
};

template <typename T>
static inline T safe_div(T v, float p) {                                          // SampleHelperFunctions.hpp:24-32
    if (p == 0.0f) return T(0.0f);
    return v / p;
}
static inline V3 safe_div(V3 v, float p) {
    if (p == 0.0f) return V3(0.0f);
    return divs(v, p);
}
static inline float saturate(float t) { return std::clamp(t, 0.0f, 1.0f); }

// ------------------------------------------------------------- Bounds3 ---
struct Bounds {                                                                   // Bounds3.hpp:11-24
    V3 mn, mx;
    Bounds() {
        mx = V3(std::numeric_limits<float>::lowest());
        mn = V3(std::numeric_limits<float>::max());
    }
};
static inline Bounds unite(const Bounds& a, const Bounds& b) {                     // Bounds3.hpp:117-123
    Bounds r; r.mn = vmin(a.mn, b.mn); r.mx = vmax(a.mx, b.mx); return r;
}
static inline Bounds unite(const Bounds& a, V3 p) {                                // Bounds3.hpp:125-131
    Bounds r; r.mn = vmin(a.mn, p); r.mx = vmax(a.mx, p); return r;
}
static inline Bounds bounds2(V3 p1, V3 p2) {                                       // Bounds3.hpp:24-28
    Bounds r;
    r.mn = V3(std::fmin(p1.x, p2.x), std::fmin(p1.y, p2.y), std::fmin(p1.z, p2.z));
    r.mx = V3(std::fmax(p1.x, p2.x), std::fmax(p1.y, p2.y), std::fmax(p1.z, p2.z));
    return r;
}
static inline V3 centroid(const Bounds& b) { return mul(b.mn, 0.5f) + mul(b.mx, 0.5f); }  // Bounds3.hpp:48
static inline int max_extent(const Bounds& b) {                                    // Bounds3.hpp:31-40
    V3 d = b.mx - b.mn;
    if (d.x > d.y && d.x > d.z) return 0;
    else if (d.y > d.z) return 1;
    return 2;
}
static inline bool box_hit(const Bounds& b, const Ray& r) {                        // Bounds3.hpp:92-115
    float nmin = std::numeric_limits<float>::min(), nmax = std::numeric_limits<float>::max();
    for (int a = 0; a < 3; ++a) {
        float o = comp(r.o, a), invD = comp(r.inv, a);
        float t1 = (comp(b.mn, a) - o) * invD;
        float t2 = (comp(b.mx, a) - o) * invD;
        if (t1 > t2) std::swap(t1, t2);
        nmin = std::max(nmin, t1);
        nmax = std::min(nmax, t2);
    }
    return nmax > 0.0f && nmin <= nmax;
}

// ---------------------------------------------------------- materials ---
enum { DIELETRIC = 0, METAL = 1, TRANSPARENT = 2 };
struct Material {
    int type = DIELETRIC;
    V3 emission;
    float ior_d = 1.5f;
    V3 ior_m = V3(0.13100f, 0.55758f, 1.4561f), ior_m_k = V3(4.0624f, 2.2039f, 1.9541f);
    V3 kd = V3(0.5f);
    float rough = 0.2f;
    bool has_emission() const { return emission.x > 0.0f || emission.y > 0.0f || emission.z > 0.0f; }
};
static inline float smooth_to_rough(float s) { return std::max(0.002f, (1.0f - s) * (1.0f - s)); }  // GGX.hpp:38-40

// SampleHelperFunctions.cpp:51-67
static V3 any_perp(V3 i) {
    if (i.z == 0.0f) {
        if (i.y == 0.0f) return V3(0.0f, 1.0f, 0.0f);
        return normalized(V3(1.0f, -i.x / i.y, 0.0f));
    }
    return normalized(V3(0.0f, 1.0f, -1.0f * i.y / i.z));
}
// SampleHelperFunctions.hpp:46-54
static inline V3 to_world(V3 a, V3 n) {
    V3 t = any_perp(n), b = cross(n, t);
    return V3(a.x * t.x + a.y * b.x + a.z * n.x, a.x * t.y + a.y * b.y + a.z * n.y, a.x * t.z + a.y * b.z + a.z * n.z);
}
// SampleHelperFunctions.cpp:21-25
static inline V3 reflect(V3 I, V3 N) {
    I = -I;
    return I - mul(N, (float)(2 * dot(I, N)));
}
// SampleHelperFunctions.cpp:38-49
static inline V3 refract(V3 I, V3 N, float ior) {
    I = -I;
    float cosi = (float)std::clamp(dot(I, N), -1.0, 1.0);
    float etai = 1, etat = ior;
    V3 n = N;
    if (cosi < 0) cosi = -cosi;
    else { std::swap(etai, etat); n = -N; }
    float eta = etai / etat;
    float k = 1 - eta * eta * (1 - cosi * cosi);
    return k < 0 ? V3(0) : normalized(mul(I, eta) + mul(n, eta * cosi - sqrtf(k)));
}
// SampleHelperFunctions.cpp:4-18 (a, b, c are float parameters)
static bool solve_quadratic(float a, float b, float c, float& x0, float& x1) {
    double discr = (double)b * b - 4.0 * a * c;
    if (discr < 0) return false;
    else if (discr == 0) x0 = x1 = (float)(-0.5 * b / a);
    else {
        float q = (b > 0) ? (float)(-0.5 * (b + std::sqrt(discr))) : (float)(-0.5 * (b - std::sqrt(discr)));
        x0 = q / a;
        x1 = c / q;
    }
    if (x0 > x1) std::swap(x0, x1);
    return true;
}
// SampleHelperFunctions.hpp:57-73
static inline void inout_ior(V3 N, V3 wi, V3 wo, float mior, float& ior_i, float& ior_o) {
    float nl = (float)dot(N, wi), nv = (float)dot(N, wo);
    ior_i = nl < 0.0f ? mior : 1.0f;
    ior_o = nv < 0.0f ? mior : 1.0f;
}
// SampleHelperFunctions.hpp:79-102
static inline V3 half_dir(V3 N, V3 wi, V3 wo, float mior) {
    float nl = (float)dot(N, wi), nv = (float)dot(N, wo);
    if (nl == 0.0f || nv == 0.0f) return V3(0.0f);
    V3 h;
    if (nl * nv > 0.0f) {
        h = normalized(wi + wo);
        if (nv < 0.0f) h = -h;
    } else if (nv < 0.0f) {
        h = -normalized(mul(wo, mior) + wi);
    } else {
        h = -normalized(wo + mul(wi, mior));
    }
    return h;
}
// SampleHelperFunctions.hpp:105-115.  `cos`/`sin` are unqualified with a float
// argument: under libstdc++ only ::cos(double) is visible there, so they run in
// double and r * cos(theta) is a double product rounded to float.
static inline V3 cosine_sample(V3 N, float& pdf) {
    float u1 = rand_float();
    float r = std::sqrt(u1);
    float theta = 2 * PI_F * rand_float();
    float x = (float)(r * ::cos((double)theta)), y = (float)(r * ::sin((double)theta));
    V3 wi = normalized(to_world(V3(x, y, std::sqrt(1.0f - u1)), N));
    pdf = (float)(dot(wi, N) / (double)PI_F);
    return wi;
}
// SampleHelperFunctions.hpp:118-120
static inline float cosine_pdf(V3 N, V3 wi) { return saturate((float)dot(wi, N)) / PI_F; }
// SampleHelperFunctions.hpp:122-131 (types: 0 bg, 1 intermediate, 2 light, 3 camera)
enum { T_BG = 0, T_MID = 1, T_LIGHT = 2, T_CAM = 3 };
struct PTV {
    int type = T_BG;
    V3 x, N;
    int prim = -1;  // Object* (Triangle* / Sphere*) -> primitive index, -1 = nullptr
};
static inline float srpdf_to_area(float srpdf, const PTV& v1, const PTV& v2) {
    float d2;
    V3 w = normalize_len2(v2.x - v1.x, &d2);
    float c1 = v1.type == T_CAM ? 1.0f : (float)std::fabs(dot(w, v1.N));
    float c2 = v2.type == T_CAM ? 1.0f : (float)std::fabs(dot(-w, v2.N));
    return srpdf * std::fabs(c1 * c2 / d2);
}

// GGX.hpp:8-14
static inline float ggx_vis(float vn, float vh, float r) {
    if (vh * vn <= 0.0f) return 0.0f;
    float vh2 = vh * vh;
    float tan2 = (1.0f - vh2) / vh2;
    return 2.0f / (1 + std::sqrt(1.0f + r * r * tan2));
}
// GGX.hpp:17-30
static inline float ggx_d(float c, float r) {
    float a2 = r * r;
    float c2 = c * c;
    float c4 = c2 * c2;
    float t2 = (1.0f - c2) / c2;
    float b = a2 + t2;
    b = b * b;
    return a2 / (PI_F * c4 * b);
}
// GGX.hpp:33-35: GGXTerm(float(|d|)) * |d| evaluated in double, returned as float
static inline float ggx_half_pdf(V3 n, V3 h, float r) {
    double d = std::fabs(dot(n, h));
    return (float)((double)ggx_d((float)d, r) * d);
}
// GGX.hpp:46-59
static inline V3 ggx_sample_h(V3 N, float r) {
    float d1 = rand_float(), d2 = rand_float();
    float theta = std::atan2(r * std::sqrt(d1), std::sqrt(1.0f - d1));
    float phi = 2.0f * PI_F * d2;
    V3 local(std::sin(theta) * std::cos(phi), std::sin(theta) * std::sin(phi), std::cos(theta));
    return normalized(to_world(local, N));
}

// Material.cpp:221-252
static V3 fresnel(const Material& m, V3 I, V3 N) {
    if (m.type == METAL) {
        float c = (float)dot(I, N);
        float c2 = c * c;
        V3 two = mul(mul(m.ior_m, 2.0f), c);
        V3 t0 = m.ior_m * m.ior_m + m.ior_m_k * m.ior_m_k;
        V3 t1 = mul(t0, c2);
        V3 Rs = (t0 - two + V3(c2)) / (t0 + two + V3(c2));
        V3 Rp = (t1 - two + V3(1.0f)) / (t1 + two + V3(1.0f));
        return mul(Rp + Rs, 0.5f);
    }
    I = -I;
    float cosi = (float)std::clamp(dot(I, N), -1., 1.);
    float etai = 1, etat = m.ior_d;
    if (cosi > 0) std::swap(etai, etat);
    float sint = etai / etat * sqrtf(std::max(0.f, 1 - cosi * cosi));
    if (sint >= 1) return V3(1.0f);
    float cost = sqrtf(std::max(0.f, 1 - sint * sint));
    cosi = fabsf(cosi);
    float Rs = ((etat * cosi) - (etai * cost)) / ((etat * cosi) + (etai * cost));
    float Rp = ((etai * cosi) - (etat * cost)) / ((etai * cosi) + (etat * cost));
    return V3((Rs * Rs + Rp * Rp) / 2);
}

// Material.cpp:11-72
static V3 eval_bsdf(const Material& m, V3 wo, V3 wi, V3 N, bool cosine) {
    float nl = (float)dot(N, wi);
    float nv = (float)dot(N, wo);
    if (nl == 0.0f || nv == 0.0f) return V3(0.0f);
    V3 h = half_dir(N, wi, wo, m.ior_d);
    float nh = (float)dot(N, h);
    float lh = (float)dot(wi, h);
    float vh = (float)dot(wo, h);
    float D = ggx_d(nh, m.rough);
    float G = ggx_vis(nv, vh, m.rough) * ggx_vis(nl, lh, m.rough);
    V3 f = fresnel(m, wi, h);
    if (nl * nv > 0.0f) {
        V3 spec(0.0f);
        if (G != 0.0f) {
            spec = divs(mul(mul(f, D), G), (float)(4.0 * (double)std::fabs(nv)));
            if (!cosine) spec = divs(spec, std::fabs(nl));
        }
        V3 diff(0.0f);
        if (m.type == DIELETRIC) {
            diff = divs(m.kd * (V3(1.0f) - f), PI_F);
            if (cosine) diff = mul(diff, saturate(nl));
        }
        return diff + spec;
    }
    if (m.type != TRANSPARENT) return V3(0.0f);
    float ior_i, ior_o;
    if (nv < 0.0f) { ior_i = 1.0f; ior_o = m.ior_d; }
    else { ior_i = m.ior_d; ior_o = 1.0f; }
    float pa = std::fabs(vh) * std::fabs(lh) / (std::fabs(nv));
    if (!cosine) pa /= std::fabs(nl);
    float pb = ior_o * ior_o * (1.0f - f.x) * G * D;
    if (pa * pb == 0.0f) return V3(0.0f);
    float pc = ior_i * lh + ior_o * vh;
    pc *= pc;
    return V3(pa * pb / pc);
}

// Material.cpp:105-147
static float mat_pdf(const Material& m, V3 wo, V3 n, V3 wi) {
    float nv = (float)dot(n, wo), nl = (float)dot(n, wi);
    if (nv == 0.0f || nl == 0.0f) return 0.0f;
    V3 h = half_dir(n, wi, wo, m.ior_d);
    V3 f = fresnel(m, wo, h);
    float pdf_h = ggx_half_pdf(n, h, m.rough);
    float vh = (float)dot(wo, h);
    float avh = std::fabs(vh);
    float lh = (float)dot(wi, h);
    float ior_i, ior_o;
    inout_ior(n, wi, wo, m.ior_d, ior_i, ior_o);
    if (nv * nl < 0.0f) {
        float den = ior_i * lh + ior_o * vh;
        float jac = safe_div(ior_o * ior_o * avh, den * den);
        if (m.type != TRANSPARENT) return 0.0f;
        return pdf_h * (1.0f - f.x) * jac;
    } else if (nv * nl > 0.0f) {
        float jac = safe_div(1.0f, 4.0f * avh);
        float diff = cosine_pdf(n, wi);
        if (m.type == METAL) return pdf_h * jac;
        if (m.type == DIELETRIC) return (diff + pdf_h * jac) * 0.5f;
        return pdf_h * f.x * jac;
    }
    return 0.0f;
}

// Material.cpp:150-214
static V3 mat_sample(const Material& m, V3 wo, V3 n, float* pdf) {
    V3 H = ggx_sample_h(n, m.rough);
    V3 wis = reflect(wo, H);
    float pdf_h = ggx_half_pdf(n, H, m.rough);
    float vn = (float)dot(wo, n);
    float vh = (float)dot(wo, H);
    float avh = std::fabs(vh);
    float jr = safe_div(1.0f, 4.0f * avh);
    if (m.type == METAL) {
        *pdf = pdf_h * jr;
        if ((double)vn * dot(wis, n) < 0.0f) *pdf = 0.0f;
        return wis;
    }
    if (m.type == DIELETRIC) {
        if (rand_float() < 0.5f) {
            float pd = cosine_pdf(n, wis);
            *pdf = (pdf_h * jr + pd) * 0.5f;
            if ((double)vn * dot(wis, n) < 0.0f) *pdf = 0.0f;
            return wis;
        }
        float pd;
        V3 wid = cosine_sample(n, pd);
        H = normalized(wid + wo);
        vh = (float)dot(wo, H);
        avh = std::fabs(vh);
        pdf_h = ggx_half_pdf(n, H, m.rough);
        jr = safe_div(1.0f, 4.0f * avh);
        *pdf = (pdf_h * jr + pd) * 0.5f;
        if ((double)vn * dot(wid, n) < 0.0f) *pdf = 0.0f;
        return wid;
    }
    V3 f = fresnel(m, wo, H);
    if (rand_float() < f.x) {
        *pdf = pdf_h * f.x * jr;
        if ((double)vn * dot(wis, n) < 0.0f) *pdf = 0.0f;
        return wis;
    }
    V3 wr = refract(wo, H, m.ior_d);
    float ior_i, ior_o;
    inout_ior(n, wr, wo, m.ior_d, ior_i, ior_o);
    float lh = (float)dot(wr, H);
    float den = ior_i * lh + ior_o * vh;
    float jt = safe_div(ior_o * ior_o * avh, den * den);
    *pdf = pdf_h * (1.0f - f.x) * jt;
    if ((double)vn * dot(wr, n) > 0.0f) *pdf = 0.0f;
    return wr;
}

// --------------------------------------------------------------- scene ---
enum { P_TRI = 0, P_SPHERE = 1 };
struct Prim {
    int kind = P_TRI;
    int mat = 0;
    int object = 0;
    // Triangle (Triangle.hpp:15-51)
    V3 v0, v1, v2, e1, e2, normal;
    float area = 0;
    // Sphere (Sphere.hpp:11-31)
    V3 center;
    float radius = 0, radius2 = 0;
    Bounds bounds() const {
        if (kind == P_TRI) return unite(bounds2(v0, v1), v2);                      // Triangle.hpp:29
        return bounds2(V3(center.x - radius, center.y - radius, center.z - radius),  // Sphere.cpp:43-46
                       V3(center.x + radius, center.y + radius, center.z + radius));
    }
};
struct Node {
    Bounds b;
    int left = -1, right = -1;
    int item = -1;  // primitive (mesh BVH) or object (scene BVH); -1 = interior
    float area = 0;
};
struct Hit {
    bool happened = false;
    V3 coords, normal;
    double distance = 0;
    int prim = -1;
};

struct Scene;
struct Object {
    int kind = 0;  // 0 mesh, 1 sphere
    int mat = 0;
    std::vector<Node> nodes;  // mesh BVH (BVHAccel per MeshTriangle, Triangle.cpp:74)
    Bounds bbox;
    float area = 0;           // MeshTriangle::area (sequential sum, Triangle.cpp:70-73)
    int sphere_prim = -1;
};

struct Scene {
    int width = 784, height = 784;
    double fov = 40;
    V3 eye, bg;
    std::vector<Material> mats;
    std::vector<Prim> prims;
    std::vector<Object> objects;
    std::vector<Node> top;     // Scene::bvh
    std::vector<int> emitters; // m_emissionObjects (Scene.cpp:14-18)

    Bounds item_bounds(bool scene_level, int it) const {
        if (!scene_level) return prims[it].bounds();
        const Object& o = objects[it];
        return o.kind == 0 ? o.bbox : prims[o.sphere_prim].bounds();
    }
    float item_area(bool scene_level, int it) const {
        if (!scene_level) return prims[it].area;
        const Object& o = objects[it];
        return o.kind == 0 ? o.area : prims[o.sphere_prim].area;
    }
    // BVH.cpp:30-99
    int build(std::vector<Node>& nodes, std::vector<int> items, bool sl) {
        int idx = (int)nodes.size();
        nodes.push_back(Node());
        Bounds bb;
        for (int it : items) bb = unite(bb, item_bounds(sl, it));
        if (items.size() == 1) {
            nodes[idx].b = item_bounds(sl, items[0]);
            nodes[idx].item = items[0];
            nodes[idx].area = item_area(sl, items[0]);
            return idx;
        }
        if (items.size() == 2) {
            int l = build(nodes, {items[0]}, sl);
            int r = build(nodes, {items[1]}, sl);
            nodes[idx].left = l; nodes[idx].right = r;
            nodes[idx].b = unite(nodes[l].b, nodes[r].b);
            nodes[idx].area = nodes[l].area + nodes[r].area;
            return idx;
        }
        Bounds cb;
        for (int it : items) cb = unite(cb, centroid(item_bounds(sl, it)));
        int dim = max_extent(cb);
        std::sort(items.begin(), items.end(), [&](int a, int b) {
            return comp(centroid(item_bounds(sl, a)), dim) < comp(centroid(item_bounds(sl, b)), dim);
        });
        size_t mid = items.size() / 2;
        std::vector<int> L(items.begin(), items.begin() + mid), R(items.begin() + mid, items.end());
        int l = build(nodes, L, sl);
        int r = build(nodes, R, sl);
        nodes[idx].left = l; nodes[idx].right = r;
        nodes[idx].b = unite(nodes[l].b, nodes[r].b);
        nodes[idx].area = nodes[l].area + nodes[r].area;
        return idx;
    }

    // Triangle.cpp:77-118
    Hit tri_hit(int pi, const Ray& ray, int cull) const {
        const Prim& t = prims[pi];
        Hit h;
        if (cull == TPT_CULL_BACK) { if (dot(ray.d, t.normal) > 0) return h; }
        else if (cull == TPT_CULL_FRONT) { if (dot(ray.d, t.normal) < 0) return h; }
        V3 pvec = cross(ray.d, t.e2);
        double det = dot(t.e1, pvec);
        if (std::fabs(det) < EPS) return h;
        double det_inv = 1. / det;
        V3 tvec = ray.o - t.v0;
        double u = dot(tvec, pvec) * det_inv;
        if (u < 0 || u > 1) return h;
        V3 qvec = cross(tvec, t.e1);
        double v = dot(ray.d, qvec) * det_inv;
        if (v < 0 || u + v > 1) return h;
        double tt = dot(t.e2, qvec) * det_inv;
        if (tt < 0.0f) return h;
        h.distance = tt;
        h.coords = ray.o + mul(ray.d, (float)tt);
        h.prim = pi;
        h.normal = t.normal;
        h.happened = true;
        return h;
    }
    // Sphere.cpp:4-41
    Hit sphere_hit(int pi, const Ray& ray, int cull) const {
        const Prim& s = prims[pi];
        Hit h;
        V3 L = ray.o - s.center;
        double a = dot(ray.d, ray.d);
        double b = 2.0 * dot(ray.d, L);
        double c = dot(L, L) - s.radius2;
        float t0, t1;
        if (!solve_quadratic((float)a, (float)b, (float)c, t0, t1)) return h;
        float tk;
        if (cull == TPT_CULL_BACK) tk = t0;
        else if (cull == TPT_CULL_FRONT) tk = t1;
        else tk = t0 <= 0 ? t1 : t0;
        if (tk > 0.0f) {
            h.happened = true;
            h.coords = ray.o + mul(ray.d, tk);
            h.normal = normalized(h.coords - s.center);
            h.prim = pi;
            h.distance = tk;
        }
        return h;
    }
    // BVH.cpp:103-143 over a mesh BVH
    Hit mesh_hit(int oi, const Ray& ray, int cull) const {
        const std::vector<Node>& nodes = objects[oi].nodes;
        Hit best;
        if (nodes.empty()) return best;
        int stack[64];
        int sp = 0;
        stack[sp++] = 0;
        while (sp) {
            const Node& n = nodes[stack[--sp]];
            ++cnt_nodes;
            if (!box_hit(n.b, ray)) continue;
            if (n.item >= 0) {
                ++cnt_tris;
                Hit t = tri_hit(n.item, ray, cull);
                if (t.happened && (!best.happened || best.distance > t.distance)) best = t;
            } else if (sp + 2 < 64) {
                stack[sp++] = n.left;
                stack[sp++] = n.right;
            }
        }
        return best;
    }
    Hit object_hit(int oi, const Ray& ray, int cull) const {
        const Object& o = objects[oi];
        return o.kind == 0 ? mesh_hit(oi, ray, cull) : sphere_hit(o.sphere_prim, ray, cull);
    }
    Hit scene_hit(const Ray& ray, int cull) const {
        Hit best;
        if (top.empty()) return best;
        int stack[64];
        int sp = 0;
        stack[sp++] = 0;
        while (sp) {
            const Node& n = top[stack[--sp]];
            ++cnt_nodes;
            if (!box_hit(n.b, ray)) continue;
            if (n.item >= 0) {
                Hit t = object_hit(n.item, ray, cull);
                if (t.happened && (!best.happened || best.distance > t.distance)) best = t;
            } else if (sp + 2 < 64) {
                stack[sp++] = n.left;
                stack[sp++] = n.right;
            }
        }
        return best;
    }
    // Scene.cpp:21-35
    PTV intersect(const Ray& ray, int cull = TPT_CULL_BACK) const {
        Hit t = scene_hit(ray, cull);
        PTV r;
        if (t.happened) { r.prim = t.prim; r.N = t.normal; r.type = T_MID; r.x = t.coords; }
        else r.type = T_BG;
        return r;
    }
    // Scene.cpp:37-48
    bool shadow(V3 lc, V3 x, int cull = TPT_CULL_BACK) const {
        double ld2 = dot(lc - x, lc - x);
        PTV s = intersect(Ray(lc, normalized(x - lc)), cull);
        double sd2 = dot(s.x - lc, s.x - lc);
        return s.type != T_BG && sd2 < ld2 - 1.0f;
    }
    const Material& mat_of(int prim) const { return mats[prims[prim].mat]; }
    // Scene.cpp:50-83
    bool shadow(const PTV& v1, const PTV& v2) const {
        V3 atob = v2.x - v1.x;
        if (v1.prim >= 0 && v2.prim != v1.prim && mat_of(v1.prim).type == TRANSPARENT) {
            if (dot(atob, v1.N) < 0.0f) return shadow(v1.x, v2.x, TPT_CULL_FRONT);
            return shadow(v1.x, v2.x);
        }
        if (v1.prim >= 0 && dot(atob, v1.N) < 0.0f) return false;
        if (v2.prim >= 0 && dot(-atob, v2.N) < 0.0f) return false;
        return shadow(v1.x, v2.x);
    }
    // Object::pdf(): Triangle 1/area, MeshTriangle 1/root-area, Sphere 1/area
    float prim_pdf(int pi) const { return 1.0f / prims[pi].area; }
    float object_pdf(int oi) const {
        const Object& o = objects[oi];
        if (o.kind == 0) return 1.0f / o.nodes[0].area;
        return 1.0f / prims[o.sphere_prim].area;
    }
    // Object::Sample: MeshTriangle -> BVHAccel::Sample (BVH.cpp:145-159) -> Triangle::Sample
    // (Triangle.hpp:31-36); Sphere::Sample (Sphere.cpp:48-55).
    void object_sample(int oi, V3& coords, V3& normal, int& prim) const {
        const Object& o = objects[oi];
        if (o.kind == 0) {
            float p = std::sqrt(rand_float()) * o.nodes[0].area;
            int ni = 0;
            for (;;) {
                const Node& n = o.nodes[ni];
                if (n.left < 0 || n.right < 0) break;
                if (p < o.nodes[n.left].area) ni = n.left;
                else { p = p - o.nodes[n.left].area; ni = n.right; }
            }
            const Prim& t = prims[o.nodes[ni].item];
            float x = std::sqrt(rand_float()), y = rand_float();
            coords = mul(t.v0, 1.0f - x) + mul(t.v1, x * (1.0f - y)) + mul(t.v2, x * y);
            normal = t.normal;
            prim = o.nodes[ni].item;
        } else {
            const Prim& s = prims[o.sphere_prim];
            float theta = (float)(2.0 * PI_F * rand_float()), phi = (float)(PI_F * rand_float());
            V3 dir(std::cos(phi), std::sin(phi) * std::cos(theta), std::sin(phi) * std::sin(theta));
            coords = s.center + mul(dir, s.radius);
            normal = dir;
            prim = o.sphere_prim;
        }
    }
};

// ---------------------------------------------------------------- PT -----
// PathTracer.cpp:14-24
static float light_pdf(const Scene& sc, int L, V3 x, V3 wi) {
    Hit h = sc.object_hit(L, Ray(x, wi), TPT_NO_CULL);
    if (!h.happened) return 0.0f;
    float d2 = (float)dot(h.coords - x, h.coords - x);
    float raw = sc.object_pdf(L);
    float ct = (float)dot(h.normal, -wi);
    if (ct == 0.0f) return 0.0f;
    return (float)((double)raw * d2 / std::fabs(ct));
}
// PathTracer.cpp:26-40
static V3 light_sample(const Scene& sc, int L, V3 x, float* pdf) {
    V3 pc, pn; int pp;
    sc.object_sample(L, pc, pn, pp);
    V3 wi = pc - x;
    float d2 = (float)dot(wi, wi);
    wi = normalized(wi);
    float raw = sc.object_pdf(L);
    float ct = (float)dot(pn, -wi);
    *pdf = (float)((double)raw * d2 / std::fabs(ct));
    return wi;
}
// PathTracer.cpp:44-134 (HEAD: one iteration, then `break`)
static V3 path_trace(const Scene& sc, const Ray& ray, int& bounces) {
    bounces = 0;
    V3 result(0.0f);
    PTV it = sc.intersect(ray, TPT_CULL_BACK);
    if (it.type == T_BG) return result;
    const Material& m = sc.mat_of(it.prim);
    if (m.has_emission()) result = result + m.emission;  // alpha == 1
    V3 x = it.x, wo = -ray.d, n = it.N;
    float pdf_b;
    V3 wib = mat_sample(m, wo, n, &pdf_b);
    for (int L : sc.emitters) {
        float pll, pbl, plb;
        V3 wil = light_sample(sc, L, x, &pll);
        plb = mat_pdf(m, wo, n, wil);
        pbl = light_pdf(sc, L, x, wib);
        V3 ev(0.0f);
        if (pdf_b + pbl > 0.0f) {
            Hit h = sc.object_hit(L, Ray(x, wib), TPT_CULL_BACK);
            if (h.happened && !sc.shadow(h.coords, x))
                ev = ev + divs(eval_bsdf(m, wo, wib, n, true), EPS + pdf_b + pbl);
        }
        if (pll + plb > 0.0f) {
            Hit h = sc.object_hit(L, Ray(x, wil), TPT_CULL_BACK);
            if (!sc.shadow(h.coords, x))
                ev = ev + divs(eval_bsdf(m, wo, wil, n, true), EPS + pll + plb);
        }
        result = result + ev * sc.mats[sc.objects[L].mat].emission;  // alpha == 1
    }
    return result;
}

// PathTracer.cpp:44-134 with the `break` at :109 removed (TPT_MODE_PT_INDIRECT,
// the reference's dead indirect-bounce code re-enabled; its
// oracle is the reference built with that one line dropped, oracle/build_ref.sh).
static V3 path_trace_indirect(const Scene& sc, const Ray& ray, int& bounces) {
    bounces = 0;
    Ray cur = ray;
    V3 alpha(1.0f), result(0.0f);
    bool explicit_light = false, flip = false;
    for (;;) {
        if (alpha.x == 0.0f && alpha.y == 0.0f && alpha.z == 0.0f) break;               // :54-55
        PTV it = sc.intersect(cur, flip ? TPT_CULL_FRONT : TPT_CULL_BACK);             // :56
        if (it.type == T_BG) break;                                                    // :58-62
        const Material& m = sc.mat_of(it.prim);
        if (m.has_emission() && !explicit_light) result = result + alpha * m.emission;  // :64-68
        V3 x = it.x, wo = -cur.d, n = it.N;
        float pdf_b;
        V3 wib = mat_sample(m, wo, n, &pdf_b);                                         // :76
        explicit_light = true;                                                         // :80
        for (int L : sc.emitters) {                                                    // :82-106
            float pll, pbl, plb;
            V3 wil = light_sample(sc, L, x, &pll);
            plb = mat_pdf(m, wo, n, wil);
            pbl = light_pdf(sc, L, x, wib);
            V3 ev(0.0f);
            if (pdf_b + pbl > 0.0f) {
                Hit h = sc.object_hit(L, Ray(x, wib), TPT_CULL_BACK);
                if (h.happened && !sc.shadow(h.coords, x))
                    ev = ev + divs(eval_bsdf(m, wo, wib, n, true), EPS + pdf_b + pbl);
            }
            if (pll + plb > 0.0f) {
                Hit h = sc.object_hit(L, Ray(x, wil), TPT_CULL_BACK);
                if (!sc.shadow(h.coords, x))
                    ev = ev + divs(eval_bsdf(m, wo, wil, n, true), EPS + pll + plb);
            }
            result = result + alpha * ev * sc.mats[sc.objects[L].mat].emission;
        }
        V3 weight(0.0f);                                                               // :111-114
        if (pdf_b > 0.0f) weight = divs(eval_bsdf(m, wo, wib, n, true), EPS + pdf_b);
        cur = Ray(x, wib);                                                             // :116
        flip = dot(n, wib) < 0.0f;                                                     // :117-120
        const bool rr = bounces > 4;                                                   // :122-131
        if (!rr || rand_float() < 0.8f) {
            alpha = divs(alpha * weight, rr ? 0.8f : 1.0f);
            bounces += 1;
            continue;
        }
        break;
    }
    return result;
}

// --------------------------------------------------------------- BDPT ----
// BDPT.hpp:8-9, BDPT.cpp:7-8
static const int MAXLEN = 16;
static const float CAM_ZERO_PDF = (float)10000000000.0;
static const float CAM_RAY_PDF = (float)10.0;

struct PVert {          // BDPTPath::InternalPathVertex (BDPT.hpp:16-21)
    PTV v;
    float pdf = 0;
    V3 alpha;
    bool shadowed = false;
};
struct Path {           // BDPTPath (BDPT.hpp:15-60)
    int count = 0;
    PVert verts[MAXLEN * 2];
    const Scene* sc;
    explicit Path(const Scene* s) : sc(s) {}

    // PathVertex accessors (BDPT.hpp:87-128)
    V3 pos(int i) const { return verts[i].v.x; }
    V3 nrm(int i) const { return verts[i].v.type == T_CAM ? V3(0.0f, 0.0f, 1.0f) : verts[i].v.N; }
    int type(int i) const { return verts[i].v.type; }
    const Material* material(int i) const { return verts[i].v.prim >= 0 ? &sc->mat_of(verts[i].v.prim) : nullptr; }
    V3 emission(int i) const {
        const Material* m = material(i);
        if (!m) return V3(0.0f);
        if (type(i) == T_BG) return sc->bg;
        return m->emission;
    }
    // BDPT.cpp:317-330
    V3 eval_bsdf_sa(int i, V3 dir) const {
        if (type(i) == T_LIGHT || type(i) == T_CAM) return V3(1.0f);
        return eval_bsdf(*material(i), normalized(pos(i - 1) - pos(i)), dir, nrm(i), false);
    }
    // BDPT.cpp:332-351
    float eval_pdf_sa(int i, V3 dir) const {
        float c = (float)std::fabs(dot(dir, nrm(i)));
        if (type(i) == T_LIGHT) return safe_div(cosine_pdf(nrm(i), dir), c);
        if (type(i) == T_CAM) return CAM_RAY_PDF;
        if (c == 0.0f) return 0.0f;
        V3 wo = normalized(pos(i - 1) - pos(i));
        return safe_div(mat_pdf(*material(i), wo, nrm(i), dir), c);
    }
    // BDPT.cpp:41-59
    void gen_camera(const Ray& ray) {
        verts[0].v = PTV(); verts[0].v.type = T_CAM; verts[0].v.x = ray.o;
        verts[0].pdf = CAM_ZERO_PDF; verts[0].alpha = V3(1.0f); verts[0].shadowed = false;
        verts[1].v = sc->intersect(ray);
        verts[1].pdf = srpdf_to_area(CAM_RAY_PDF, verts[0].v, verts[1].v);
        verts[1].alpha = V3(1.0f); verts[1].shadowed = false;
        if (verts[1].v.type == T_BG) { count = 2; return; }
        fill(1);
    }
    // BDPT.cpp:61-90
    void gen_light(int L) {
        V3 c, n; int p;
        sc->object_sample(L, c, n, p);
        verts[0].v.x = c; verts[0].v.type = T_LIGHT; verts[0].v.prim = p; verts[0].v.N = n;
        verts[0].shadowed = false;
        verts[0].pdf = sc->object_pdf(L);
        verts[0].alpha = divs(sc->mats[sc->objects[L].mat].emission, verts[0].pdf);
        float pdf1;
        V3 wi = cosine_sample(n, pdf1);
        float ct = (float)dot(verts[0].v.N, wi);
        pdf1 = safe_div(pdf1, ct);
        verts[1].v = sc->intersect(Ray(verts[0].v.x, wi));
        verts[1].shadowed = false;
        verts[1].pdf = srpdf_to_area(pdf1, verts[0].v, verts[1].v);
        if (pdf1 != 0.0f) verts[1].alpha = safe_div(verts[0].alpha, pdf1);
        else if (verts[1].v.type == T_BG) { count = 2; return; }
        fill(1);
    }
    // BDPT.cpp:261-279
    PVert sample_next(const PVert& vx, V3 wo) const {
        const Material& m = sc->mat_of(vx.v.prim);
        float raw;
        V3 wi = mat_sample(m, wo, vx.v.N, &raw);
        float ct = (float)std::fabs(dot(vx.v.N, wi));
        float sr = safe_div(raw, ct);
        PTV it = sc->intersect(Ray(vx.v.x, wi), dot(vx.v.N, wi) > 0.0f ? TPT_CULL_BACK : TPT_CULL_FRONT);
        V3 bsdf = eval_bsdf(m, wo, wi, vx.v.N, false);
        PVert r;
        r.shadowed = false;
        r.v = it;
        r.alpha = safe_div(bsdf, sr);
        r.pdf = srpdf_to_area(sr, vx.v, r.v);
        return r;
    }
    // BDPT.cpp:92-118
    void fill(int start) {
        count = start + 1;
        for (int i = start; i < MAXLEN - 1; i++) {
            if (verts[i].v.type == T_BG) break;
            V3 wo = normalized(verts[i - 1].v.x - verts[i].v.x);
            verts[i + 1] = sample_next(verts[i], wo);
            float rr = i > 4 ? .8f : 1.f;
            if (rand_float() > rr) break;
            if (verts[i + 1].pdf == 0.0f) break;
            verts[i + 1].pdf *= rr;
            verts[i + 1].alpha = divs(verts[i].alpha * verts[i + 1].alpha, rr);
            count++;
        }
    }
    // BDPT.cpp:125-171 (always called with dontcheckshadow = true)
    void append(const PTV& vertex) {
        if (count == 0) {
            verts[0].v = vertex; verts[0].shadowed = false;
            verts[0].pdf = sc->prim_pdf(vertex.prim);
            if (vertex.type == T_LIGHT) verts[0].alpha = divs(sc->mat_of(vertex.prim).emission, verts[0].pdf);
            else verts[0].alpha = V3(1.0f);
            count++;
            return;
        }
        int li = count - 1;
        PVert& e = verts[count];
        e.v = vertex;
        e.shadowed = false;
        float d2;
        V3 wi = normalize_len2(vertex.x - pos(li), &d2);
        float sr = eval_pdf_sa(li, wi);
        e.pdf = srpdf_to_area(sr, verts[li].v, e.v);
        V3 a = safe_div(eval_bsdf_sa(li, wi), sr);
        e.alpha = verts[li].alpha * a;
        float rr = count > 4 ? .8f : 1.f;
        e.pdf *= rr;
        e.alpha = safe_div(e.alpha, rr);
        count++;
    }
};

// BDPT.cpp:173-259.  lp/s = light path & its sub-length, cp/t = camera path & sub-length.
static V3 path_weight(const Path& lp, int s, const Path& cp, int t) {
    const Scene* sc = lp.sc;
    int z1 = t - 1;
    if (cp.type(z1) == T_BG) {
        if (s == 0) return cp.verts[z1].alpha * sc->bg;
        return V3(0.0f);
    }
    if (s != 0 && lp.type(s - 1) == T_BG) return V3(0.0f);
    V3 cst;
    if (s == 0) {
        V3 wi = normalized(cp.pos(z1 - 1) - cp.pos(z1));
        V3 em = cp.emission(z1);
        cst = mul(em, (float)dot(cp.nrm(z1), wi));
        if (dot(em, em) == 0.0f) return V3(0.0f);
    } else if (t == 0) {
        return V3(0.0f);
    } else {
        float d2;
        V3 dir = normalize_len2(cp.pos(z1) - lp.pos(s - 1), &d2);
        if (sc->shadow(cp.verts[z1].v, lp.verts[s - 1].v)) return V3(0.0f);
        cst = mul(lp.eval_bsdf_sa(s - 1, dir) * cp.eval_bsdf_sa(z1, -dir),
                  (float)std::fabs(dot(lp.nrm(s - 1), dir) * dot(cp.nrm(z1), -dir) / d2));
    }
    float wd = 1.0f;
    Path tmp = cp;
    tmp.count = t;
    float cur = 1.0f;
    for (int i = s - 1; i >= 0; i--) {
        tmp.append(lp.verts[i].v);
        float pdf = tmp.verts[tmp.count - 1].pdf;
        cur *= safe_div(pdf, lp.verts[i].pdf);
        wd += cur * cur;
        if (cur == 0.0f) break;
    }
    tmp = lp;
    tmp.count = s;
    cur = 1.0f;
    for (int i = t - 1; i >= 0; i--) {
        if (tmp.count == 0) {
            PTV ta = cp.verts[i].v;
            ta.type = T_LIGHT;
            tmp.append(ta);
        } else {
            tmp.append(cp.verts[i].v);
        }
        float pdf = tmp.verts[tmp.count - 1].pdf;
        cur *= safe_div(pdf, cp.verts[i].pdf);
        wd += cur * cur;
        if (cur == 0.0f) break;
    }
    V3 lt = s == 0 ? V3(1.0f) : lp.verts[s - 1].alpha;
    V3 uc = lt * cp.verts[z1].alpha * cst;
    return divs(uc, wd);
}

// SceneRenderingHelper.cpp:24-55 (Additive)
static void draw_to_image(const Scene& sc, float scale, V3 lo, V3 ld, V3* buf, V3 value) {
    (void)lo;
    ld = divs(ld, ld.z);
    float aspect = (float)(sc.width / sc.height);
    V3 t(-ld.x / scale / aspect, -ld.y / scale, 0.0f);
    V3 uv = mul(t + V3(1.0f), 0.5f);
    V3 cs(uv.x * sc.width, uv.y * sc.height, 0.0f);
    int cx = (int)cs.x, cy = (int)cs.y;
    for (int ix = cx - 1; ix <= cx + 1; ix++)
        for (int iy = cy - 1; iy <= cy + 1; iy++) {
            if (ix < 0 || iy < 0 || ix >= sc.width || iy >= sc.height) continue;
            float dx = std::fabs(cs.x - (ix + 0.5f)), dy = std::fabs(cs.y - (iy + 0.5f));
            float w = std::max(0.0f, 1.0f - dx) * std::max(0.0f, 1.0f - dy);
            V3& b = buf[ix + sc.height * iy];
            b = b + mul(value, w);
        }
}

// BDPT.cpp:282-315
static V3 bdpt(const Scene& sc, float scale, const Ray& ray, int& bounces, V3* splat) {
    Path lp(&sc), cp(&sc);
    cp.gen_camera(ray);
    lp.gen_light(sc.emitters[0]);
    bounces = cp.count + lp.count;
    V3 result(0.0f);
    for (int t = 1; t <= cp.count; t++)
        for (int s = 0; s <= lp.count; s++) {
            if (t + s < 2) continue;
            V3 w = path_weight(lp, s, cp, t);
            w = vmax(w, V3(0.0f));
            if (t > 1) result = result + w;
            else if (splat) {
                V3 l = lp.pos(s - 1), c = cp.pos(0);
                draw_to_image(sc, scale, l, normalized(l - c), splat, w);
            }
        }
    return result;
}

// ------------------------------------------------------------- camera ----
// SceneRenderingHelper.cpp:12-14
static float camera_scale(double fov) {
    float half = (float)(fov * 0.5);
    float rad = (float)(half * PI_F / 180.0);
    return (float)std::tan((double)rad);
}
// SceneRenderingHelper.cpp:16-22
static V3 pixel_ray(int px, int py, int w, int h, float scale) {
    float aspect = (float)(w / h);
    float x = (float)((2 * (px + 0.5) / (float)w - 1) * aspect * scale);
    float y = (float)((1 - 2 * (py + 0.5) / (float)h) * scale);
    return normalized(V3(-x, y, 1));
}

// ----------------------------------------------------- scene assembly ----
static void finalize(Scene& sc) {
    // per-mesh BVHs (Triangle.cpp:67-74), then the scene BVH (Scene.cpp:11-19)
    for (size_t oi = 0; oi < sc.objects.size(); ++oi) {
        Object& o = sc.objects[oi];
        if (o.kind != 0) continue;
        std::vector<int> items;
        for (size_t p = 0; p < sc.prims.size(); ++p)
            if (sc.prims[p].object == (int)oi && sc.prims[p].kind == P_TRI) items.push_back((int)p);
        if (!items.empty()) sc.build(o.nodes, items, false);
    }
    std::vector<int> objs;
    for (size_t i = 0; i < sc.objects.size(); ++i) objs.push_back((int)i);
    if (!objs.empty()) sc.build(sc.top, objs, true);
    for (size_t i = 0; i < sc.objects.size(); ++i)
        if (sc.mats[sc.objects[i].mat].has_emission()) sc.emitters.push_back((int)i);
}

static Prim make_tri(V3 a, V3 b, V3 c, int mat, int obj) {  // Triangle.hpp:18-25
    Prim t;
    t.kind = P_TRI; t.mat = mat; t.object = obj;
    t.v0 = a; t.v1 = b; t.v2 = c;
    t.e1 = b - a; t.e2 = c - a;
    t.normal = normalized(cross(t.e1, t.e2));
    t.area = magnitude(cross(t.e1, t.e2)) * 0.5f;
    return t;
}

static void add_mesh(Scene& sc, const std::vector<V3>& soup, int mat) {  // Triangle.cpp:32-75
    Object o;
    o.kind = 0; o.mat = mat;
    int oi = (int)sc.objects.size();
    V3 mn(std::numeric_limits<float>::max()), mx(-std::numeric_limits<float>::max());
    for (size_t i = 0; i + 2 < soup.size(); i += 3) {
        for (int j = 0; j < 3; ++j) {
            V3 v = soup[i + j];
            mn = V3(std::min(mn.x, v.x), std::min(mn.y, v.y), std::min(mn.z, v.z));
            mx = V3(std::max(mx.x, v.x), std::max(mx.y, v.y), std::max(mx.z, v.z));
        }
        sc.prims.push_back(make_tri(soup[i], soup[i + 1], soup[i + 2], mat, oi));
    }
    o.bbox = bounds2(mn, mx);
    o.area = 0;
    for (size_t p = 0; p < sc.prims.size(); ++p)
        if (sc.prims[p].object == oi) o.area += sc.prims[p].area;
    sc.objects.push_back(o);
}

static void add_sphere(Scene& sc, V3 c, float r, int mat) {  // Sphere.hpp:16
    Object o;
    o.kind = 1; o.mat = mat;
    int oi = (int)sc.objects.size();
    Prim s;
    s.kind = P_SPHERE; s.mat = mat; s.object = oi;
    s.center = c; s.radius = r; s.radius2 = r * r;
    s.area = 4 * PI_F * r * r;
    o.sphere_prim = (int)sc.prims.size();
    sc.prims.push_back(s);
    sc.objects.push_back(o);
}

// Minimal triangle-only OBJ reader: `v x y z` (std::stof == strtof) and `f a b c`
// (1-based, negative = relative), emitting the per-face vertex soup the
// reference's objl loader produces for triangle faces (OBJ_Loader.hpp:533-590).
static bool load_obj(const std::string& path, std::vector<V3>& soup) {
    std::ifstream f(path);
    if (!f) return false;
    std::vector<V3> pos;
    std::string line;
    while (std::getline(f, line)) {
        std::istringstream ss(line);
        std::string tok;
        if (!(ss >> tok)) continue;
        if (tok == "v") {
            std::string a, b, c;
            ss >> a >> b >> c;
            pos.push_back(V3(std::strtof(a.c_str(), nullptr), std::strtof(b.c_str(), nullptr), std::strtof(c.c_str(), nullptr)));
        } else if (tok == "f") {
            std::string w;
            while (ss >> w) {
                long idx = std::strtol(w.c_str(), nullptr, 10);
                size_t k = idx < 0 ? pos.size() + idx : (size_t)(idx - 1);
                soup.push_back(pos[k]);
            }
        }
    }
    return true;
}

static Scene* from_desc(const tpt_scene_desc* d) {
    Scene* sc = new Scene();
    sc->width = d->width; sc->height = d->height; sc->fov = d->fov;
    sc->eye = V3(d->eye[0], d->eye[1], d->eye[2]);
    sc->bg = V3(d->background[0], d->background[1], d->background[2]);
    for (int i = 0; i < d->num_materials; ++i) {
        const tpt_material& m = d->materials[i];
        Material mm;
        mm.type = m.type;
        mm.emission = V3(m.emission[0], m.emission[1], m.emission[2]);
        mm.ior_d = m.ior_d;
        mm.ior_m = V3(m.ior_m[0], m.ior_m[1], m.ior_m[2]);
        mm.ior_m_k = V3(m.ior_m_k[0], m.ior_m_k[1], m.ior_m_k[2]);
        mm.kd = V3(m.kd[0], m.kd[1], m.kd[2]);
        mm.rough = m.rough;
        sc->mats.push_back(mm);
    }
    for (int i = 0; i < d->num_objects; ++i) {
        const tpt_object& o = d->objects[i];
        if (o.kind == TPT_OBJ_MESH) {
            std::vector<V3> soup;
            for (int t = 0; t < o.num_triangles; ++t)
                for (int j = 0; j < 3; ++j) {
                    const float* v = d->vertices + 3 * (3 * (int64_t)(o.first_triangle + t) + j);
                    soup.push_back(V3(v[0], v[1], v[2]));
                }
            add_mesh(*sc, soup, o.material);
        } else {
            add_sphere(*sc, V3(o.center[0], o.center[1], o.center[2]), o.radius, o.material);
        }
    }
    finalize(*sc);
    return sc;
}

// Presets: main.cpp:49-103 and SURVEY.md §8(d).
static Scene* preset(const std::string& dir, const std::string& p, int w, int h) {
    Scene* sc = new Scene();
    sc->width = w; sc->height = h;
    sc->eye = V3(278, 278, -800);
    // main.cpp:51 sets the background to 0; "background" keeps Scene.hpp:23's default
    sc->bg = p == "background" ? V3(0.235294f, 0.67451f, 0.843137f) : V3(0.0f);
    auto mat = [&](int type, V3 e) { Material m; m.type = type; m.emission = e; m.kd = V3(0.5f, 0.5f, 0.5f); sc->mats.push_back(m); return (int)sc->mats.size() - 1; };
    int red = mat(DIELETRIC, V3(0.0f)); sc->mats[red].kd = V3(0.63f, 0.065f, 0.05f);
    int green = mat(DIELETRIC, V3(0.0f)); sc->mats[green].kd = V3(0.14f, 0.45f, 0.091f);
    int white = mat(DIELETRIC, V3(0.0f)); sc->mats[white].kd = V3(0.725f, 0.71f, 0.68f);
    sc->mats[white].rough = smooth_to_rough(p == "smooth_dielectric" ? 0.7f : .1f);
    V3 le = mul(V3(0.747f + 0.058f, 0.747f + 0.258f, 0.747f), 8.0f) + mul(V3(0.740f + 0.287f, 0.740f + 0.160f, 0.740f), 15.6f) +
            mul(V3(0.737f + 0.642f, 0.737f + 0.159f, 0.737f), 18.4f);
    int light = mat(DIELETRIC, le); sc->mats[light].kd = V3(0.65f);
    int silver = mat(METAL, V3(0.0f));
    sc->mats[silver].ior_m = V3(0.041000f, 0.53285f, 0.049317f);
    sc->mats[silver].ior_m_k = V3(4.8025f, 3.4101f, 2.8545f);
    sc->mats[silver].rough = smooth_to_rough(1.f);
    int glass = mat(TRANSPARENT, V3(0.0f)); sc->mats[glass].ior_d = 1.5f; sc->mats[glass].rough = smooth_to_rough(.9f);
    int lightball = mat(DIELETRIC, V3(3.0f, 2.4f, 1.5f)); sc->mats[lightball].kd = V3(0.65f);
    int boxes;
    if (p == "silver") boxes = silver;
    else if (p == "standard" || p == "refractive_ball" || p == "occlusion" || p == "smooth_dielectric" || p == "bunny" ||
             p == "multi_light" || p == "emissive_sphere" || p == "background") boxes = white;
    else { delete sc; return nullptr; }
    auto mesh = [&](const char* f, int m) {
        std::vector<V3> soup;
        if (!load_obj(dir + "/" + f, soup)) return false;
        add_mesh(*sc, soup, m);
        return true;
    };
    bool ok = true;
    if (p == "bunny") {
        ok &= mesh("floor.obj", white); ok &= mesh("left.obj", red); ok &= mesh("right.obj", green);
        ok &= mesh("light.obj", light); ok &= mesh("bunny_cornell.obj", white);
    } else {
        ok &= mesh("floor.obj", boxes); ok &= mesh("shortbox.obj", boxes); ok &= mesh("tallbox.obj", boxes);
        ok &= mesh("left.obj", red); ok &= mesh("right.obj", green);
        // "emissive_sphere": the glowing ball is m_emissionObjects[0] (BDPT.cpp:287)
        if (p == "emissive_sphere") add_sphere(*sc, V3(420.0f, 60.0f, 150.0f), 60.0f, lightball);
        ok &= mesh("light.obj", light);
        if (p == "multi_light") { ok &= mesh("light2.obj", light); ok &= mesh("light3.obj", light); }
        if (p == "refractive_ball") add_sphere(*sc, V3(278.0f, 278.0f, 200.0f), 50.0f, glass);
        if (p == "occlusion") ok &= mesh("lightocculuder.obj", white);
    }
    if (!ok) { delete sc; return nullptr; }
    finalize(*sc);
    return sc;
}

// Renderer.cpp:32-63 for one pixel.
static void trace_pixel(const Scene& sc, float scale, int mode, int spp, int64_t i, float* out, V3* splat, int64_t* bounces) {
    int px = (int)(i % sc.width), py = (int)(i / sc.width);
    reset_random((int)i + 1);
    V3 acc(0.0f);
    int64_t nb = 0;
    for (int s = 0; s < spp; ++s) {
        V3 dir = pixel_ray(px, py, sc.width, sc.height, scale);
        int b = 0;
        V3 L = mode == TPT_MODE_BDPT          ? bdpt(sc, scale, Ray(sc.eye, dir), b, splat)
               : mode == TPT_MODE_PT_INDIRECT ? path_trace_indirect(sc, Ray(sc.eye, dir), b)
                                              : path_trace(sc, Ray(sc.eye, dir), b);
        acc = acc + mul(L, 1.0f / spp);
        nb += b;
    }
    out[0] = acc.x; out[1] = acc.y; out[2] = acc.z;
    if (bounces) *bounces = nb;
}

// TPT_FLAG_SAMPLE_SEED (include/tpt.h): not the reference's seeding -- sample j of
// pixel i starts its own XorShift32 stream (SplitMix64 finalizer of ((i+1) << 32 | j),
// folded to 32 bits, never 0); everything else is the reference's per-sample
// estimator.  `lanes` = how the library spreads a pixel's samples: 1 sums (1/spp) * L
// in sample order (PT), L > 1 sums per lane q over samples j = q, q + L, ... and then
// the L partial sums in lane order (PT-indirect with TPT_PT_LANES lanes).
static uint32_t sample_seed(int64_t i, int j) {
    uint64_t z = ((uint64_t)(i + 1) << 32 | (uint32_t)j) + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    const uint32_t r = (uint32_t)z ^ (uint32_t)(z >> 32);
    return r ? r : 0x6B43A9B5u;
}
static void trace_pixel_seeded(const Scene& sc, float scale, int mode, int spp, int64_t i, int lanes, float* out,
                               int64_t* bounces) {
    int px = (int)(i % sc.width), py = (int)(i / sc.width);
    V3 acc(0.0f);
    int64_t nb = 0;
    for (int q = 0; q < lanes; ++q) {
        V3 part(0.0f);
        for (int s = q; s < spp; s += lanes) {
            rnd_state = sample_seed(i, s);
            V3 dir = pixel_ray(px, py, sc.width, sc.height, scale);
            int b = 0;
            V3 L = mode == TPT_MODE_PT_INDIRECT ? path_trace_indirect(sc, Ray(sc.eye, dir), b) : path_trace(sc, Ray(sc.eye, dir), b);
            part = part + mul(L, 1.0f / spp);
            nb += b;
        }
        acc = lanes == 1 ? part : acc + part;
    }
    out[0] = acc.x; out[1] = acc.y; out[2] = acc.z;
    if (bounces) *bounces = nb;
}

}  // namespace orc

using namespace orc;

extern "C" {

void* oracle_preset(const char* models_dir, const char* name, int w, int h) { return preset(models_dir, name, w, h); }
void* oracle_create(const tpt_scene_desc* d) { return from_desc(d); }
void oracle_destroy(void* s) { delete (Scene*)s; }
float oracle_camera_scale(double fov) { return camera_scale(fov); }

// Scene description export (so tests can hand the oracle's own preset to libtpt).
// Returns counts; arrays may be null to query sizes.
int oracle_scene_counts(void* h, int* n_mat, int* n_obj, int64_t* n_tri, int* n_top_nodes, int* n_emitters) {
    Scene* s = (Scene*)h;
    *n_mat = (int)s->mats.size(); *n_obj = (int)s->objects.size();
    int64_t nt = 0;
    for (auto& p : s->prims) nt += p.kind == P_TRI;
    *n_tri = nt; *n_top_nodes = (int)s->top.size(); *n_emitters = (int)s->emitters.size();
    return 0;
}

void oracle_trace_pixels(void* h, int mode, int spp, const int64_t* pix, int64_t n, float* out, float* splat, int64_t* bounces) {
    Scene* s = (Scene*)h;
    float scale = camera_scale(s->fov);
    std::vector<V3> em;
    if (mode == TPT_MODE_BDPT) em.assign((size_t)s->width * s->height, V3(0.0f));
    for (int64_t k = 0; k < n; ++k)
        trace_pixel(*s, scale, mode, spp, pix[k], out + 3 * k, em.empty() ? nullptr : em.data(), bounces ? bounces + k : nullptr);
    if (splat && !em.empty())
        for (size_t i = 0; i < em.size(); ++i) {
            // Renderer.cpp:59 `emissionBuffer[i] * 1.0f / spp`
            V3 e(em[i].x * 1.0f / spp, em[i].y * 1.0f / spp, em[i].z * 1.0f / spp);
            splat[3 * i] = e.x; splat[3 * i + 1] = e.y; splat[3 * i + 2] = e.z;
        }
}

// TPT_FLAG_SAMPLE_SEED restated (see trace_pixel_seeded); PT / PT-indirect only.
void oracle_trace_pixels_seeded(void* h, int mode, int spp, const int64_t* pix, int64_t n, int lanes, float* out,
                                int64_t* bounces) {
    Scene* s = (Scene*)h;
    float scale = camera_scale(s->fov);
    for (int64_t k = 0; k < n; ++k)
        trace_pixel_seeded(*s, scale, mode, spp, pix[k], lanes, out + 3 * k, bounces ? bounces + k : nullptr);
}
uint32_t oracle_sample_seed(int64_t i, int j) { return sample_seed(i, j); }

// Renderer::Render (Renderer.cpp:68-127): `threads` workers on the interleaved
// pixel split, per-thread splat buffers merged in thread order.  Used as the
// CPU baseline ("port") in bench.py.  pixel_limit > 0 renders only pixels < limit
// (bounded CPU sample).  Returns wall milliseconds.
double oracle_render(void* h, int mode, int spp, int threads, int64_t pixel_limit, float* out) {
    Scene* s = (Scene*)h;
    float scale = camera_scale(s->fov);
    int64_t np = (int64_t)s->width * s->height;
    int64_t lim = pixel_limit > 0 ? std::min(pixel_limit, np) : np;
    if (threads < 1) threads = 1;
    std::vector<std::vector<V3>> em(threads);
    std::memset(out, 0, sizeof(float) * 3 * np);
    auto t0 = std::chrono::steady_clock::now();
    auto work = [&](int off) {
        if (mode == TPT_MODE_BDPT) em[off].assign(np, V3(0.0f));
        for (int64_t i = off; i < lim; i += threads)
            trace_pixel(*s, scale, mode, spp, i, out + 3 * i, mode == TPT_MODE_BDPT ? em[off].data() : nullptr, nullptr);
        if (mode == TPT_MODE_BDPT)
            for (auto& e : em[off]) e = V3(e.x * 1.0f / spp, e.y * 1.0f / spp, e.z * 1.0f / spp);
    };
    std::vector<std::thread> th;
    for (int t = 1; t < threads; ++t) th.emplace_back(work, t);
    work(0);
    for (auto& t : th) t.join();
    if (mode == TPT_MODE_BDPT)
        for (int64_t j = 0; j < np; ++j)
            for (int t = 0; t < threads; ++t) {
                out[3 * j] += em[t][j].x; out[3 * j + 1] += em[t][j].y; out[3 * j + 2] += em[t][j].z;
            }
    auto t1 = std::chrono::steady_clock::now();
    return std::chrono::duration<double, std::milli>(t1 - t0).count();
}

// SURVEY.md §8(d) B_alg: node pops and triangle tests of the reference traversal
// over the given pixels at `spp` (the oracle is single-threaded here).  out[0] =
// nodes, out[1] = triangle tests, both totals.
void oracle_traversal_counts(void* h, int mode, int spp, const int64_t* pix, int64_t n, uint64_t* out) {
    std::vector<float> rgb(3 * (size_t)n), splat;
    Scene* s = (Scene*)h;
    if (mode == TPT_MODE_BDPT) splat.resize(3 * (size_t)s->width * s->height);
    cnt_nodes = cnt_tris = 0;
    oracle_trace_pixels(h, mode, spp, pix, n, rgb.data(), splat.empty() ? nullptr : splat.data(), nullptr);
    out[0] = cnt_nodes; out[1] = cnt_tris;
}

void oracle_rng(uint32_t seed, int n, uint32_t* u, float* f) {
    reset_random((int)seed);
    for (int i = 0; i < n; ++i) u[i] = xorshift32();
    reset_random((int)seed);
    for (int i = 0; i < n; ++i) f[i] = rand_float();
}

// ordinal = primitive index (triangles of each mesh in soup order, spheres in place)
void oracle_intersect(void* h, const float* rays, int64_t n, int cull, float* out) {
    Scene* s = (Scene*)h;
    for (int64_t k = 0; k < n; ++k) {
        const float* r = rays + 6 * k;
        PTV v = s->intersect(Ray(V3(r[0], r[1], r[2]), V3(r[3], r[4], r[5])), cull);
        float* o = out + 8 * k;
        o[0] = v.type == T_BG ? 0.f : 1.f;
        o[1] = v.x.x; o[2] = v.x.y; o[3] = v.x.z;
        o[4] = v.N.x; o[5] = v.N.y; o[6] = v.N.z;
        o[7] = (float)v.prim;
    }
}

static Material mat_from(const float* m) {
    Material mat;
    mat.type = (int)m[0];
    mat.ior_d = m[1];
    mat.ior_m = V3(m[2], m[3], m[4]);
    mat.ior_m_k = V3(m[5], m[6], m[7]);
    mat.kd = V3(m[8], m[9], m[10]);
    mat.rough = m[11];
    return mat;
}
// Same layout as ref_material_kat (oracle/ref_harness.cpp).
void oracle_material_kat(const float* m, const float* in, int n, float* out) {
    Material mat = mat_from(m);
    for (int k = 0; k < n; ++k) {
        const float* c = in + 10 * k;
        V3 wo(c[0], c[1], c[2]), nn(c[3], c[4], c[5]), wi(c[6], c[7], c[8]);
        uint32_t seed; std::memcpy(&seed, &c[9], 4);
        float* o = out + 17 * k;
        reset_random((int)seed);
        float sp = 0.f;
        V3 sm = mat_sample(mat, wo, nn, &sp);
        o[0] = sm.x; o[1] = sm.y; o[2] = sm.z; o[3] = sp;
        o[4] = mat_pdf(mat, wo, nn, wi);
        V3 e1 = eval_bsdf(mat, wo, wi, nn, true), e2 = eval_bsdf(mat, wo, wi, nn, false);
        o[5] = e1.x; o[6] = e1.y; o[7] = e1.z; o[8] = e2.x; o[9] = e2.y; o[10] = e2.z;
        V3 f = fresnel(mat, wi, nn);
        o[11] = f.x; o[12] = f.y; o[13] = f.z;
        float cp = 0.f;
        V3 cw = cosine_sample(nn, cp);
        o[14] = cw.x; o[15] = cw.y; o[16] = cp;
    }
}
void oracle_helper_kat(const float* in, int n, float* out) {
    for (int k = 0; k < n; ++k) {
        const float* c = in + 8 * k;
        V3 a(c[0], c[1], c[2]), b(c[3], c[4], c[5]);
        float* o = out + 16 * k;
        V3 r = reflect(a, b), rf = refract(a, b, c[6]), ap = any_perp(a);
        o[0] = r.x; o[1] = r.y; o[2] = r.z; o[3] = rf.x; o[4] = rf.y; o[5] = rf.z;
        o[6] = ap.x; o[7] = ap.y; o[8] = ap.z;
        o[9] = ggx_vis(c[6], c[7], 0.3f);
        o[10] = ggx_d(c[6], 0.3f);
        float x0 = 0, x1 = 0;
        bool ok = solve_quadratic(c[6], c[7], c[0], x0, x1);
        o[11] = ok ? 1.f : 0.f; o[12] = ok ? x0 : 0.f; o[13] = ok ? x1 : 0.f;
        o[14] = smooth_to_rough(c[6]);
        o[15] = (float)dot(a, b);
    }
}
}
