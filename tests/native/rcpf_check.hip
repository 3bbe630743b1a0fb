// GPU check of rcp_exact_f32 (csrc/tpt_devmath.h) against IEEE 1.0f / x, bit for
// bit, over all 2^32 float bit patterns.  Prints the number of mismatches among the
// inputs the fast path accepts (rcp_fast_ok) and over all inputs; exit status 1 if the
// accepted inputs have any.
#include <cstdio>
#include <cstdint>

#include "../../toypathtracer-games101-assignment7_amd/csrc/tpt_devmath.h"

__global__ void check(uint32_t hi_bits, unsigned long long* bad) {
    const uint32_t u = hi_bits | (blockIdx.x * blockDim.x + threadIdx.x);
    const float x = __uint_as_float(u);
    const float want = 1.0f / x;
    const float got = tpt::rcp_fast_f32(x);
    const bool ok = tpt::rcp_fast_ok(x);
    if (__float_as_uint(want) != __float_as_uint(got) && !(want != want && got != got)) {
        atomicAdd(&bad[ok ? 0 : 1], 1ull);
        if (ok && atomicAdd(&bad[2], 1ull) == 0ull) bad[3] = u;
    }
}

int main() {
    unsigned long long* bad;
    if (hipMalloc(&bad, 4 * sizeof(*bad)) != hipSuccess) return 2;
    (void)hipMemset(bad, 0, 4 * sizeof(*bad));
    for (uint32_t h = 0; h < 16; ++h) check<<<(1u << 28) / 256, 256>>>(h << 28, bad);
    if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 2; }
    unsigned long long hb[4];
    (void)hipMemcpy(hb, bad, sizeof(hb), hipMemcpyDeviceToHost);
    printf("rcpf_check: 2^32 floats, %llu mismatches where the fast path is taken (first %#llx), %llu outside it\n",
           hb[0], hb[0] ? hb[3] : 0ull, hb[1]);
    return hb[0] ? 1 : 0;
}
