// tpt_devmath.h -- scalar / vector math of the reference's hot path, written for
// gfx950 device code (also compiles as plain host C++ so the libm replicas can be
// checked exhaustively against glibc on the CPU: tests/test_devmath.py).
//
// Numerics contract: the reference is fp32 with selected
// fp64 steps; every kernel TU is compiled with -ffp-contract=off so float
// expressions round exactly like the reference's x86-64 build.  Deliberate
// exceptions, all provably identical:
//   * dot3(): the reference's DotProduct (Vector.hpp:103-104) sums three products
//     of floats in double.  A float*float product is exact in double (48 bits), so
//     fma(a, b, p) == p + a*b rounded once == the reference's add.  We use 1 mul +
//     2 fma instead of 3 mul + 2 add.
//   * rng_float(): (double)x / 4294967295.0 rounded to float equals
//     (double)x * (1/4294967295.0) rounded to float for all 2^32 x (checked
//     exhaustively, tests/test_devmath.py).
//   * sinf/cosf/atan2f: the reference calls glibc's float versions, which are not
//     correctly rounded (1.3% / 18.6% of inputs differ from the correctly rounded
//     result).  tpt_sinf / tpt_cosf / tpt_atan2f restate glibc 2.35's algorithms
//     (sysdeps/ieee754/flt-32: s_sinf.c + sincosf_data.c, s_atanf.c + e_atan2f.c)
//     and agree with glibc bit-for-bit on every float of the domains the hot path
//     uses ([0, 2pi] for sin/cos, all finite non-negative floats for atan).
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define TPT_HD __host__ __device__ __forceinline__
#else
#include <cmath>
#include <cstring>
#define TPT_HD inline
#endif

namespace tpt {

#if defined(__HIPCC__)
TPT_HD uint32_t f2u(float f) { return __builtin_bit_cast(uint32_t, f); }
TPT_HD float u2f(uint32_t u) { return __builtin_bit_cast(float, u); }
#else
TPT_HD uint32_t f2u(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
TPT_HD float u2f(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }
#endif

TPT_HD float fabs_(float x) { return u2f(f2u(x) & 0x7fffffffu); }
TPT_HD double dabs_(double x) { return x < 0 ? -x : (x == 0 ? 0.0 : x); }
// std::min / std::max semantics: min(a,b) = (b < a) ? b : a ; max(a,b) = (a < b) ? b : a
TPT_HD float smin(float a, float b) { return (b < a) ? b : a; }
TPT_HD float smax(float a, float b) { return (a < b) ? b : a; }

// --------------------------------------------------------------- vectors --
struct V3 {
    float x, y, z;
};
TPT_HD V3 v3(float a, float b, float c) { V3 r; r.x = a; r.y = b; r.z = c; return r; }
TPT_HD V3 v3s(float a) { return v3(a, a, a); }
TPT_HD V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
TPT_HD V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
TPT_HD V3 operator*(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
TPT_HD V3 operator/(V3 a, V3 b) { return v3(a.x / b.x, a.y / b.y, a.z / b.z); }
TPT_HD V3 operator-(V3 a) { return v3(-a.x, -a.y, -a.z); }
TPT_HD V3 mul(V3 a, float r) { return v3(a.x * r, a.y * r, a.z * r); }   // Vector.hpp:25,48
TPT_HD V3 divs(V3 a, float r) { return v3(a.x / r, a.y / r, a.z / r); }  // Vector.hpp:26

// Vector.hpp:103-104 (see header note on the fma form)
TPT_HD double dot3(V3 a, V3 b) {
#if defined(__HIPCC__) && defined(__HIP_DEVICE_COMPILE__)
    double p = (double)a.x * (double)b.x;
    p = __builtin_fma((double)a.y, (double)b.y, p);
    return __builtin_fma((double)a.z, (double)b.z, p);
#else
    return (double)a.x * b.x + (double)a.y * b.y + (double)a.z * b.z;
#endif
}
TPT_HD V3 cross(V3 a, V3 b) {  // Vector.hpp:106-113
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
TPT_HD float sqrt_f(float x) {
#if defined(__HIPCC__)
    return __builtin_sqrtf(x);
#else
    return std::sqrt(x);
#endif
}
TPT_HD double sqrt_d(double x) {
#if defined(__HIPCC__)
    return __builtin_sqrt(x);
#else
    return std::sqrt(x);
#endif
}
TPT_HD V3 normalized(V3 a) {  // Vector.hpp:31-34
    float n = sqrt_f(a.x * a.x + a.y * a.y + a.z * a.z);
    return v3(a.x / n, a.y / n, a.z / n);
}
TPT_HD V3 normalize_len2(V3 a, float* len2) {  // Vector.hpp:36-39
    *len2 = (float)dot3(a, a);
    return divs(a, sqrt_f(*len2));
}
TPT_HD V3 vmax0(V3 a) { return v3(smax(a.x, 0.0f), smax(a.y, 0.0f), smax(a.z, 0.0f)); }  // Vector3f::Max(v, 0)

// ------------------------------------------------------------------- RNG --
// XorShift32 with shifts 13, 17, 15 (global.cpp:5-13); seed = pixel + 1
// (Renderer.cpp:42); GetRandomFloat (global.cpp:19-22).
TPT_HD uint32_t xorshift32(uint32_t& s) {
    uint32_t x = s;
    x ^= x << 13;
    x ^= x >> 17;
    x ^= x << 15;
    s = x;
    return x;
}
TPT_HD float rng_float(uint32_t& s) {
    return (float)((double)xorshift32(s) * (1.0 / 4294967295.0));
}

// --------------------------------------------------- glibc float libm -----
// sinf / cosf: glibc 2.35 flt-32 s_sinf.c / s_cosf.c; polynomial table
// __sincosf_table (values read from this image's libm.so.6).  The |x| < 120
// paths only (the hot path calls them on [0, 2pi]).
struct SinCosTab {
    double sign[4], hpi_inv, hpi, c0, c1, s1, c2, s2, c3, s3, c4;
};
#if defined(__HIPCC__)
__device__ __constant__
#endif
static const SinCosTab kSinCos[2] = {
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0, 0x1p0, -0x1.ffffffd0c621cp-2,
     -0x1.555545995a603p-3, 0x1.55553e1068f19p-5, 0x1.1107605230bc4p-7, -0x1.6c087e89a359dp-10,
     -0x1.994eb3774cf24p-13, 0x1.99343027bf8c3p-16},
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0, -0x1p0, 0x1.ffffffd0c621cp-2,
     -0x1.555545995a603p-3, -0x1.55553e1068f19p-5, 0x1.1107605230bc4p-7, 0x1.6c087e89a359dp-10,
     -0x1.994eb3774cf24p-13, -0x1.99343027bf8c3p-16},
};
TPT_HD uint32_t abstop12(float x) { return (f2u(x) >> 20) & 0x7ff; }
TPT_HD double fma_d(double a, double b, double c) {
#if defined(__HIPCC__)
    return __builtin_fma(a, b, c);
#else
    return std::fma(a, b, c);
#endif
}
// sinf_poly (sincosf.h); the FMA-contracted form of glibc's x86-64 FMA ifunc build.
// The plain (mul+add) form gives identical results on the hot path's domain
// (both checked exhaustively); the fma form is cheaper on gfx950.
TPT_HD float sincos_poly(double x, double x2, const SinCosTab* p, int n) {
    if ((n & 1) == 0) {
        double x3 = x * x2;
        double s1 = fma_d(x2, p->s3, p->s2);
        double x7 = x3 * x2;
        double s = fma_d(x3, p->s1, x);
        return (float)fma_d(x7, s1, s);
    }
    double x4 = x2 * x2;
    double c2 = fma_d(x2, p->c4, p->c3);
    double c1 = fma_d(x2, p->c1, p->c0);
    double x6 = x4 * x2;
    double c = fma_d(x4, p->c2, c1);
    return (float)fma_d(x6, c2, c);
}
TPT_HD double reduce_fast(double x, const SinCosTab* p, int* np) {
    double r = x * p->hpi_inv;
    int n = ((int32_t)r + 0x800000) >> 24;
    *np = n;
    return fma_d(-(double)n, p->hpi, x);
}
TPT_HD float tpt_sinf(float y) {
    double x = y;
    const SinCosTab* p = &kSinCos[0];
    if (abstop12(y) < abstop12(0x1.921fb6p-1f)) {
        double s = x * x;
        if (abstop12(y) < abstop12(0x1p-12f)) return y;
        return sincos_poly(x, s, p, 0);
    }
    int n;
    x = reduce_fast(x, p, &n);
    double s = p->sign[n & 3];
    if (n & 2) p = &kSinCos[1];
    return sincos_poly(x * s, x * x, p, n);
}
TPT_HD float tpt_cosf(float y) {
    double x = y;
    const SinCosTab* p = &kSinCos[0];
    if (abstop12(y) < abstop12(0x1.921fb6p-1f)) {
        double x2 = x * x;
        if (abstop12(y) < abstop12(0x1p-12f)) return 1.0f;
        return sincos_poly(x, x2, p, 1);
    }
    int n;
    x = reduce_fast(x, p, &n);
    double s = p->sign[n & 3];
    if (n & 2) p = &kSinCos[1];
    return sincos_poly(x * s, x * x, p, n ^ 1);
}

// atanf / atan2f: fdlibm-derived glibc 2.35 flt-32 s_atanf.c / e_atan2f.c (float
// arithmetic).  tpt_atan2f covers the hot path's domain (finite y >= 0, x >= 0).
TPT_HD float tpt_atanf(float x) {
    const float atanhi[4] = {4.6364760399e-01f, 7.8539812565e-01f, 9.8279368877e-01f, 1.5707962513e+00f};
    const float atanlo[4] = {5.0121582440e-09f, 3.7748947079e-08f, 3.4473217170e-08f, 7.5497894159e-08f};
    const float aT0 = 3.3333334327e-01f, aT1 = -2.0000000298e-01f, aT2 = 1.4285714924e-01f,
                aT3 = -1.1111110449e-01f, aT4 = 9.0908870101e-02f, aT5 = -7.6918758452e-02f,
                aT6 = 6.6610731184e-02f, aT7 = -5.8335702866e-02f, aT8 = 4.9768779427e-02f,
                aT9 = -3.6531571299e-02f, aT10 = 1.6285819933e-02f;
    int32_t hx = (int32_t)f2u(x);
    int32_t ix = hx & 0x7fffffff;
    int id;
    if (ix >= 0x4c000000) {
        if (ix > 0x7f800000) return x + x;
        return hx > 0 ? atanhi[3] + atanlo[3] : -atanhi[3] - atanlo[3];
    }
    if (ix < 0x3ee00000) {
        if (ix < 0x31000000) return x;
        id = -1;
    } else {
        x = fabs_(x);
        if (ix < 0x3f980000) {
            if (ix < 0x3f300000) { id = 0; x = (2.0f * x - 1.0f) / (2.0f + x); }
            else { id = 1; x = (x - 1.0f) / (x + 1.0f); }
        } else {
            if (ix < 0x401c0000) { id = 2; x = (x - 1.5f) / (1.0f + 1.5f * x); }
            else { id = 3; x = -1.0f / x; }
        }
    }
    float z = x * x;
    float w = z * z;
    float s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
    float s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
    if (id < 0) return x - x * (s1 + s2);
    float r = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
    return hx < 0 ? -r : r;
}
TPT_HD float tpt_atan2f(float y, float x) {
    const float pi_o_2 = 1.5707963705e+00f, pi_lo = -8.7422776573e-08f;
    uint32_t hx = f2u(x), hy = f2u(y);
    uint32_t ix = hx & 0x7fffffffu, iy = hy & 0x7fffffffu;
    if (ix > 0x7f800000u || iy > 0x7f800000u) return x + y;
    if (hx == 0x3f800000u) return tpt_atanf(y);
    if (iy == 0) return y;                  // y == +-0, x > 0 (domain: x >= 0)
    if (ix == 0) return pi_o_2 + 1.0e-30f;  // x == 0, y > 0
    int k = ((int32_t)iy - (int32_t)ix) >> 23;
    if (k > 26) return pi_o_2 + 0.5f * pi_lo;
    return tpt_atanf(fabs_(y / x));
}

// Unqualified cos/sin on a float in SampleHelperFunctions.hpp:110 bind to the
// double ::cos/::sin under libstdc++; only the float-rounded product r*cos(theta)
// is kept, so a faithfully rounded double cos suffices for that float result
// except within ~2^-29 of a float rounding boundary.
TPT_HD double cos_d(double x) { return ::cos(x); }  // ocml f64 on the device, glibc on the host
TPT_HD double sin_d(double x) { return ::sin(x); }

static const float kPi = 3.141592653589793f;  // global.hpp:7-8 (float M_PI)

}  // namespace tpt
