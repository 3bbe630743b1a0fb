// Exhaustive host check of csrc/tpt_devmath.h's glibc replicas and RNG form
// against this image's glibc (run by tests/test_devmath.py).
// usage: devmath_check [stride]   (stride 1 = every float of each domain)
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include "../../toypathtracer-games101-assignment7_amd/csrc/tpt_devmath.h"
using namespace tpt;
int main(int argc, char** argv) {
    uint32_t stride = argc > 1 ? (uint32_t)atol(argv[1]) : 1;
    long bad = 0, n = 0;
    uint32_t hi = f2u(6.2831855f);
    for (uint32_t u = 0; u <= hi; u += stride) {
        float x = u2f(u);
        n++;
        if (f2u(sinf(x)) != f2u(tpt_sinf(x))) bad++;
        if (f2u(cosf(x)) != f2u(tpt_cosf(x))) bad++;
        float s2, c2;
        tpt_sincosf(x, &s2, &c2);
        if (f2u(s2) != f2u(sinf(x)) || f2u(c2) != f2u(cosf(x))) bad++;
    }
    printf("sincos n=%ld bad=%ld\n", n, bad);
    long bad2 = 0, n2 = 0;
    for (uint32_t u = 0; u < 0x7f800000u; u += stride) {
        float x = u2f(u);
        n2++;
        if (f2u(atanf(x)) != f2u(tpt_atanf(x))) bad2++;
    }
    printf("atanf n=%ld bad=%ld\n", n2, bad2);
    long bad3 = 0, n3 = 0;
    const float roughs[] = {0.81f, 0.002f, 0.01f, 0.2f, 0.09f, 1.0f};
    for (float r : roughs)
        for (uint32_t k = 0; k <= (1u << 24); k += stride) {
            float d1 = (float)k / (float)(1u << 24);
            float y = r * std::sqrt(d1), x = std::sqrt(1.0f - d1);
            n3++;
            if (f2u(std::atan2(y, x)) != f2u(tpt_atan2f(y, x))) bad3++;
        }
    printf("atan2f n=%ld bad=%ld\n", n3, bad3);
    long bad4 = 0, n4 = 0;
    for (uint64_t x = 0; x <= 0xffffffffull; x += stride) {
        uint32_t s = (uint32_t)x;
        // rng_float advances the state; reproduce the single-step value directly
        float a = (float)((double)s / 4294967295.0);
        float b = (float)((double)s * (1.0 / 4294967295.0));
        n4++;
        if (f2u(a) != f2u(b)) bad4++;
    }
    printf("rng n=%ld bad=%ld\n", n4, bad4);
    // f64 sincos: float(r*cos), float(r*sin) as used by GetCosineWeightedSample
    long bad5 = 0, n5 = 0;
    for (uint32_t u = 0; u <= hi; u += stride) {
        float th = u2f(u);
        double sd, cd;
        tpt_sincos_d((double)th, &sd, &cd);
        double gs = std::sin((double)th), gc = std::cos((double)th);
        for (int k = 1; k <= 4; ++k) {
            float r = std::sqrt((float)k / 5.0f);
            n5++;
            if (f2u((float)(r * cd)) != f2u((float)(r * gc)) || f2u((float)(r * sd)) != f2u((float)(r * gs))) bad5++;
        }
    }
    printf("sincos_d-products n=%ld bad=%ld\n", n5, bad5);
    // div3_rcp (the device's shared-denominator division) against IEEE float
    // division, with a reciprocal estimate 2^-20 off (v_rcp_f64 is much closer):
    // random bit patterns over all finite operands, and operands built so that the
    // exact quotient sits next to a rounding midpoint.
    long bad6 = 0, n6 = 0;
    {
        std::mt19937_64 g(7);
        std::uniform_real_distribution<double> pert(-std::ldexp(1.0, -20), std::ldexp(1.0, -20));
        const long iters = 20000000L * 61 / (long)stride;
        for (long i = 0; i < iters; ++i) {
            const float x = u2f((uint32_t)g()), r = u2f((uint32_t)g());
            if (!std::isfinite(x) || !std::isfinite(r) || r == 0.0f) continue;
            const V3 q = div3_rcp(v3(x, -x, x), r, (1.0 / (double)r) * (1.0 + pert(g)));
            const float w = x / r;
            n6++;
            if (f2u(q.x) != f2u(w) || f2u(q.y) != f2u(-x / r)) bad6++;
        }
        std::uniform_int_distribution<uint32_t> mant(0, (1u << 23) - 1);
        std::uniform_int_distribution<int> ex(-60, 60);
        for (long i = 0; i < iters / 4; ++i) {
            const float r = std::ldexp(1.0f + mant(g) / 8388608.0f, ex(g));
            const float q = std::ldexp(1.0f + mant(g) / 8388608.0f, ex(g));
            const double mid = (double)q + std::ldexp(1.0, std::ilogb(q) - 24);
            const float x0 = (float)(mid * (double)r);
            for (int k = -2; k <= 2; ++k) {
                const float x = u2f(f2u(x0) + k);
                if (!std::isfinite(x)) continue;
                n6++;
                if (f2u(div3_rcp(v3(x, x, x), r, (1.0 / (double)r) * (1.0 + pert(g))).x) != f2u(x / r)) bad6++;
            }
        }
    }
    printf("div3_rcp n=%ld bad=%ld\n", n6, bad6);
    // the integer coin of the PT stream skip: rng_float >= 0.5f <=> x >= kCoinHalf,
    // every 32-bit output (stride ignored: an integer compare and one product each)
    long bad7 = 0, n7 = 0;
    for (uint64_t x = 0; x <= 0xffffffffull; ++x) {
        const bool a = (float)((double)(uint32_t)x * (1.0 / 4294967295.0)) >= 0.5f;
        n7++;
        if (a != ((uint32_t)x >= kCoinHalf)) bad7++;
    }
    printf("coin n=%ld bad=%ld\n", n7, bad7);
    return (bad || bad2 || bad3 || bad4 || bad5 || bad6 || bad7) ? 1 : 0;
}
