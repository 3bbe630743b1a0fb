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

// Three correctly rounded float quotients a.{x,y,z} / r sharing one denominator
// (Vector.hpp:26 operator/, and Normalized's x/n, y/n, z/n), from ONE f64
// reciprocal: y = two Newton steps from the estimate y0, then RN32(RN64(a * y)).
// Exact: for floats a, r the quotient a/r is never a midpoint of two adjacent
// floats and lies at least 2^-49 (relative) from every midpoint (a = m*r would need
// a 49-bit product to have 24 significant bits), while y is within ~2^-52 of 1/r
// once y0 is within 2^-20 (v_rcp_f64 is far closer), so RN64(a*y) is within
// 2^-51 of a/r and rounds to the same float -- denormal results included (the
// absolute error, < 2^-177, is below their 2^-150 midpoint spacing).  Needs r finite
// and non-zero (the caller falls back to the plain quotient otherwise).  Checked
// against IEEE division with a deliberately poor y0 (relative error 2^-20) on
// random and near-midpoint operands: tests/native/devmath_check.cpp.
TPT_HD V3 div3_rcp(V3 a, float r, double y0) {
    const double d = (double)r;
    double e = __builtin_fma(-d, y0, 1.0);
    double y = __builtin_fma(y0, e, y0);
    e = __builtin_fma(-d, y, 1.0);
    y = __builtin_fma(y, e, y);
    return v3((float)((double)a.x * y), (float)((double)a.y * y), (float)((double)a.z * y));
}
TPT_HD V3 divs(V3 a, float r) {  // Vector.hpp:26
#if defined(__HIPCC__) && defined(__HIP_DEVICE_COMPILE__)
    if (__builtin_expect(r != 0.0f && __builtin_fabsf(r) <= 3.40282347e+38f, 1))
        return div3_rcp(a, r, __builtin_amdgcn_rcp((double)r));
#endif
    return v3(a.x / r, a.y / r, a.z / r);
}

// 1.0f / x from v_rcp_f32 and one Newton correction (e = 1 - x*y exactly by fma,
// y + e*y): equal to the IEEE quotient for every x with 2^-126 <= |x| <= 2^126
// (rcp_fast_ok), checked on the GPU over all 2^32 floats (tests/native/rcpf_check.hip).
#if defined(__HIPCC__)
__device__ __forceinline__ float rcp_fast_f32(float x) {
    const float y = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, y, 1.0f);
    return __builtin_fmaf(e, y, y);
}
#endif
TPT_HD bool rcp_fast_ok(float x) {
    const float a = fabs_(x);
    return a >= 1.17549435e-38f && a <= 8.50705917e+37f;  // [2^-126, 2^126]
}

// Vector.hpp:103-104 (see header note on the fma form)
#ifndef TPT_DOT_OPAQUE
#define TPT_DOT_OPAQUE 0
#endif
TPT_HD double dot3(V3 a, V3 b) {
#if defined(__HIPCC__) && defined(__HIP_DEVICE_COMPILE__)
#if TPT_DOT_OPAQUE
    // opaque operands: the f64 conversions are made at each dot product instead of
    // being shared between dot products and held (spilled) across the code in between
    asm volatile("" : "+v"(a.x), "+v"(a.y), "+v"(a.z), "+v"(b.x), "+v"(b.y), "+v"(b.z));
#endif
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
    return divs(a, n);  // x / n, y / n, z / n
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
// rng_float is non-decreasing in the XorShift32 output x, so rng_float(s) >= 0.5f
// exactly when x >= kCoinHalf, the smallest x whose float is 0.5f (x = kCoinHalf - 1
// gives 0.49999997f; tests/native/devmath_check.cpp checks all 2^32 outputs).
constexpr uint32_t kCoinHalf = 0x7fffffc0u;
// TPT_FLAG_SAMPLE_SEED (include/tpt.h): sample j of pixel i starts its own stream.
// SplitMix64's finalizer of ((i + 1) << 32 | j), folded to 32 bits, never 0
// (a zero XorShift32 state stays zero).  Not the reference's seeding.
TPT_HD uint32_t sample_seed(int64_t i, int j) {
    uint64_t z = ((uint64_t)(i + 1) << 32 | (uint32_t)j) + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    const uint32_t s = (uint32_t)z ^ (uint32_t)(z >> 32);
    return s ? s : 0x6B43A9B5u;
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

// sinf and cosf of the same argument share glibc's reduction (s_sinf.c and
// s_cosf.c run the same reduce_fast / table selection and differ only in the
// polynomial parity), so computing both from one reduction is bit-identical.
TPT_HD void tpt_sincosf(float y, float* sn, float* cs) {
    double x = y;
    const SinCosTab* p = &kSinCos[0];
    if (abstop12(y) < abstop12(0x1.921fb6p-1f)) {
        double x2 = x * x;
        if (abstop12(y) < abstop12(0x1p-12f)) { *sn = y; *cs = 1.0f; return; }
        *sn = sincos_poly(x, x2, p, 0);
        *cs = sincos_poly(x, x2, p, 1);
        return;
    }
    int n;
    x = reduce_fast(x, p, &n);
    double s = p->sign[n & 3];
    if (n & 2) p = &kSinCos[1];
    *sn = sincos_poly(x * s, x * x, p, n);
    *cs = sincos_poly(x * s, x * x, p, n ^ 1);
}

// atanf / atan2f: fdlibm-derived glibc 2.35 flt-32 s_atanf.c / e_atan2f.c (float
// arithmetic).  tpt_atan2f covers the hot path's domain (finite y >= 0, x >= 0).
// The five argument ranges of s_atanf.c differ only in the reduction
// x' = (A x + B) / (C x + D) with A,C in {0, 1, 1.5, 2} (products exact or rounded
// exactly as fdlibm's) -- so the range is selected by coefficients and ONE divide,
// branch-free (lanes of a wave fall in different ranges).  Domain: x >= 0, finite;
// equal to glibc atanf on every such float (tests/test_devmath.py).
TPT_HD float tpt_atanf(float x) {
    const float aT0 = 3.3333334327e-01f, aT1 = -2.0000000298e-01f, aT2 = 1.4285714924e-01f,
                aT3 = -1.1111110449e-01f, aT4 = 9.0908870101e-02f, aT5 = -7.6918758452e-02f,
                aT6 = 6.6610731184e-02f, aT7 = -5.8335702866e-02f, aT8 = 4.9768779427e-02f,
                aT9 = -3.6531571299e-02f, aT10 = 1.6285819933e-02f;
    const uint32_t ix = f2u(x) & 0x7fffffffu;
    const int id = ix < 0x3ee00000u ? -1 : ix < 0x3f300000u ? 0 : ix < 0x3f980000u ? 1 : ix < 0x401c0000u ? 2 : 3;
    const float A = id == 0 ? 2.0f : (id == 3 ? 0.0f : 1.0f);
    const float B = id == 2 ? -1.5f : -1.0f;
    const float C = id == 2 ? 1.5f : 1.0f;
    const float D = id == 0 ? 2.0f : (id == 3 ? 0.0f : 1.0f);
    const float xr = id < 0 ? x : (A * x + B) / (C * x + D);
    const float z = xr * xr, w = z * z;
    const float s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
    const float s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
    const float hi = id <= 0 ? 4.6364760399e-01f : id == 1 ? 7.8539812565e-01f : id == 2 ? 9.8279368877e-01f
                                                                                           : 1.5707962513e+00f;
    const float lo = id <= 0 ? 5.0121582440e-09f : id == 1 ? 3.7748947079e-08f : id == 2 ? 3.4473217170e-08f
                                                                                           : 7.5497894159e-08f;
    float r = id < 0 ? xr - xr * (s1 + s2) : hi - ((xr * (s1 + s2) - lo) - xr);
    if (ix < 0x31000000u) r = x;                          // |x| < 2^-29
    if (ix >= 0x4c000000u) r = 1.5707962513e+00f + 7.5497894159e-08f;  // |x| >= 2^25
    return r;
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
// double ::cos/::sin under libstdc++; only the float-rounded product r*cos(theta) is
// kept.  tpt_sincos_d: fdlibm k_sin/k_cos kernels after a 3-part pi/2 reduction
// (0 <= x <= ~8), within 1 ulp (double) of glibc on every float in [0, 2pi]; the
// float products r*cos / r*sin then agree with glibc's (0 mismatches in 3.8e7
// checks at the differing inputs, tests/test_devmath.py).  One shared reduction
// for both functions, ~40 f64 ops instead of two ocml calls.
TPT_HD double rint_d(double x) {
#if defined(__HIPCC__)
    return __builtin_rint(x);
#else
    return std::nearbyint(x);
#endif
}
TPT_HD void tpt_sincos_d(double x, double* sn, double* cs) {
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03, S3 = -1.98412698298579493134e-04,
                 S4 = 2.75573137070700676789e-06, S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03, C3 = 2.48015872894767294178e-05,
                 C4 = -2.75573143513906633035e-07, C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    const double invpio2 = 6.36619772367581382433e-01, pio2_1 = 1.57079632673412561417e+00,
                 pio2_2 = 6.07710050630396597660e-11, pio2_2t = 2.02226624879595063154e-21;
    const double fn = rint_d(x * invpio2);
    const int n = (int)fn;
    double r = x - fn * pio2_1;
    const double t = r;
    double w = fn * pio2_2;
    r = t - w;
    w = fn * pio2_2t - ((t - r) - w);
    const double y0 = r - w;
    const double y1 = (r - y0) - w;
    const double z = y0 * y0, v = z * y0;
    const double rr = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    const double ks = y0 - ((z * (0.5 * y1 - v * rr) - y1) - v * S1);
    const double rc = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    const double hz = 0.5 * z, ww = 1.0 - hz;
    const double kc = ww + (((1.0 - ww) - hz) + (z * rc - y0 * y1));
    const int q = n & 3;
    *sn = q == 0 ? ks : q == 1 ? kc : q == 2 ? -ks : -kc;
    *cs = q == 0 ? kc : q == 1 ? -ks : q == 2 ? -kc : ks;
}

static const float kPi = 3.141592653589793f;  // global.hpp:7-8 (float M_PI)

}  // namespace tpt
