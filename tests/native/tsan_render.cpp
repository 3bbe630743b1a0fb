// tests/native/tsan_render.cpp -- TEST INFRASTRUCTURE: the CPU restatement's threaded
// Renderer::Render (oracle/tpt_oracle.cpp oracle_render, mirroring Renderer.cpp:86-114:
// interleaved pixel split over std::thread workers, thread_local XorShift state,
// per-thread splat buffers merged after the join) built with -fsanitize=thread and run
// on 8 threads (SURVEY.md §5 "Race detection": "Run the CPU restatement under TSan").
// It also checks the threaded frames against the 1-thread ones: PT bit-identical (the
// split is a pure partition), BDPT radiance + splats within the merge-order rounding.
//   usage: tsan_render MODELS_DIR   (exit 0 = clean; ThreadSanitizer exits 66 on a race)
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

extern "C" {
void* oracle_preset(const char* models_dir, const char* name, int w, int h);
void oracle_destroy(void* s);
double oracle_render(void* h, int mode, int spp, int threads, int64_t pixel_limit, float* out);
}

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    const int W = 64, H = 64;
    void* s = oracle_preset(argv[1], "standard", W, H);
    if (!s) { std::fprintf(stderr, "preset failed\n"); return 2; }
    std::vector<float> a(W * H * 3), b(W * H * 3);
    int bad = 0;
    for (int mode : {0, 1}) {  // TPT_MODE_PT, TPT_MODE_BDPT
        const int spp = mode == 0 ? 8 : 2;
        oracle_render(s, mode, spp, 8, 0, a.data());
        oracle_render(s, mode, spp, 1, 0, b.data());
        double num = 0, den = 0;
        int diff = 0;
        for (size_t k = 0; k < a.size(); ++k) {
            diff += std::memcmp(&a[k], &b[k], 4) != 0;
            num += (double)(a[k] - b[k]) * (a[k] - b[k]);
            den += (double)b[k] * b[k];
        }
        const double rel = den > 0 ? std::sqrt(num / den) : 0.0;
        std::printf("mode %d spp %d: 8 threads vs 1: %d floats differ, relL2 %.3g\n", mode, spp, diff, rel);
        if (mode == 0 ? diff != 0 : rel > 1e-5) bad = 1;
    }
    oracle_destroy(s);
    return bad;
}
