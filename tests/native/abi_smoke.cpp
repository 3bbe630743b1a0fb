// Minimal C++ caller of the C ABI: preset -> upload -> closest hit -> 1-spp PT frame.
// Built by tests/test_abi.py::test_abi_smoke_builds, run by tests/test_gpu_parity.py::test_cli_and_abi_smoke.
// Prints a backtrace on SIGSEGV.
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../../include/tpt.h"
#include "../../include/tpt_host.h"
static void on_segv(int) {
    void* bt[64];
    int n = backtrace(bt, 64);
    backtrace_symbols_fd(bt, n, 2);
    _exit(139);
}
int main(int argc, char** argv) {
    signal(SIGSEGV, on_segv);
    const char* models = argc > 1 ? argv[1] : "toypathtracer-games101-assignment7_amd/models";
    tpt_preset* p = nullptr;
    if (tpt_preset_load(models, "standard", 784, 784, &p)) { std::puts("preset failed"); return 1; }
    tpt_ctx* c = nullptr;
    int rc = tpt_create(0, &c);
    std::printf("create %d\n", rc); std::fflush(stdout);
    if (rc) return 1;
    rc = tpt_upload_scene(c, tpt_preset_desc(p));
    std::printf("upload %d %s\n", rc, tpt_last_error(c)); std::fflush(stdout);
    if (rc) return 1;
    float ray[6] = {278, 278, -800, 0, 0, 1}, out[8];
    rc = tpt_intersect(c, ray, 1, TPT_CULL_BACK, out);
    std::printf("intersect %d %s hit=%g x=%g %g %g prim=%g\n", rc, tpt_last_error(c), out[0], out[1], out[2], out[3], out[7]);
    std::vector<float> rgb(784 * 784 * 3);
    tpt_render_params rp = {1, TPT_MODE_PT, 0, 1, 0, 0};
    tpt_stats st;
    rc = tpt_render(c, &rp, rgb.data(), nullptr, &st);
    double s = 0; for (float v : rgb) s += v;
    std::printf("render %d %s sum=%g kernel_ms=%g\n", rc, tpt_last_error(c), s, st.kernel_ms);
    if (rc) return 1;
    tpt_destroy(c);
    tpt_preset_free(p);
    return 0;
}
