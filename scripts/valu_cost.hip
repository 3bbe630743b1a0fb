// valu_cost.hip -- measures the VALU issue cost (SIMD cycles per wave64 instruction)
// of each instruction class the rocprofv3 SQ_INSTS_VALU_* counters split a kernel
// into, on the MI355X this runs on.  MEASUREMENT TOOL ONLY (not product code): the
// cost table it prints turns the PT / BDPT kernels' per-class instruction counts
// into the VALU-issue roofline that bench.py reports.
//
// Method: every CU runs W waves per SIMD (W = 1, 2, 4, 8; 256-thread workgroups,
// W workgroups per CU).  Each lane keeps 8 independent accumulators and issues the
// instruction under test on each of them, 8 x kUnroll times per loop trip, through
// inline asm (nothing the compiler can fold).  Each wave stamps s_memtime (shader
// clock) around its loop; with W co-resident waves per SIMD the SIMD's throughput is
// W * instructions / cycles, so
//     cycles per wave-instruction = median(delta s_memtime) / (W * instructions per wave).
// The in-kernel clock is delta s_memtime / delta s_memrealtime * 100 MHz.
//
//   hipcc --offload-arch=gfx950 -O3 -o scripts/valu_cost scripts/valu_cost.hip
//   scripts/valu_cost            -> one JSON line per (instruction, W)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CHECK(x)                                                                     \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
            std::exit(1);                                                            \
        }                                                                            \
    } while (0)

constexpr int kUnroll = 4;
constexpr int kAcc = 8;

// One instruction per accumulator; F32 ops read/write a float VGPR, F64 a pair.
#define OP_F32(name, text)                                                             \
    struct name {                                                                      \
        using T = float;                                                               \
        static const char* id() { return #name; }                                      \
        static __device__ __forceinline__ void op(float& a, float b, float c) {        \
            asm volatile(text : "+v"(a) : "v"(b), "v"(c));                             \
        }                                                                              \
    };
#define OP_F64(name, text)                                                             \
    struct name {                                                                      \
        using T = double;                                                              \
        static const char* id() { return #name; }                                      \
        static __device__ __forceinline__ void op(double& a, double b, double c) {     \
            asm volatile(text : "+v"(a) : "v"(b), "v"(c));                             \
        }                                                                              \
    };

OP_F32(v_add_f32, "v_add_f32 %0, %0, %1")
OP_F32(v_mul_f32, "v_mul_f32 %0, %0, %1")
OP_F32(v_fma_f32, "v_fma_f32 %0, %0, %1, %2")
OP_F32(v_rcp_f32, "v_rcp_f32 %0, %0")
OP_F32(v_sqrt_f32, "v_sqrt_f32 %0, %0")
OP_F32(v_div_fixup_f32, "v_div_fixup_f32 %0, %0, %1, %2")
OP_F32(v_add_u32, "v_add_u32 %0, %0, %1")
OP_F32(v_mad_u32_u24, "v_mad_u32_u24 %0, %0, %1, %2")
OP_F32(v_and_b32, "v_and_b32 %0, %0, %1")
OP_F32(v_mov_b32, "v_mov_b32 %0, %1")
struct v_cndmask_b32 {  // v_cmp_lt_f32 (writes VCC) + v_cndmask_b32
    using T = float;
    static const char* id() { return "v_cmp_lt_f32+v_cndmask_b32"; }
    static __device__ __forceinline__ void op(float& a, float b, float c) {
        asm volatile("v_cmp_lt_f32 vcc, %0, %1\n\tv_cndmask_b32 %0, %1, %2, vcc" : "+v"(a) : "v"(b), "v"(c) : "vcc");
    }
};
OP_F32(v_max_f32, "v_max_f32 %0, %0, %1")
OP_F64(v_add_f64, "v_add_f64 %0, %0, %1")
OP_F64(v_mul_f64, "v_mul_f64 %0, %0, %1")
OP_F64(v_fma_f64, "v_fma_f64 %0, %0, %1, %2")
OP_F64(v_rcp_f64, "v_rcp_f64 %0, %0")
OP_F64(v_sqrt_f64, "v_sqrt_f64 %0, %0")
OP_F64(v_lshlrev_b64, "v_lshlrev_b64 %0, 1, %0")
// conversions: write a float from a double and back (two instructions per op)
struct v_cvt_f64_f32 {
    using T = double;
    static const char* id() { return "v_cvt_f64_f32+v_cvt_f32_f64"; }
    static __device__ __forceinline__ void op(double& a, double, double) {
        float t;
        asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(t) : "v"(a));
        asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(a) : "v"(t));
    }
};

template <class Op>
__global__ __launch_bounds__(256) void bench_kernel(typename Op::T* out, long long* stamps, int trips) {
    using T = typename Op::T;
    T acc[kAcc];
    const T b = (T)(1.0 + 1e-7 * threadIdx.x), c = (T)0.5;
#pragma unroll
    for (int k = 0; k < kAcc; ++k) acc[k] = (T)(1.0 + 0.01 * k + 1e-6 * threadIdx.x);
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    const long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < trips; ++i) {
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
#pragma unroll
            for (int k = 0; k < kAcc; ++k) Op::op(acc[k], b, c);
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    const long long r1 = __builtin_amdgcn_s_memrealtime();
    T s = acc[0];
#pragma unroll
    for (int k = 1; k < kAcc; ++k) s = s + acc[k];
    const int gw = (blockIdx.x * blockDim.x + threadIdx.x) / 64;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) {  // vector stores of the wave's stamps
        stamps[2 * gw] = t1 - t0;
        stamps[2 * gw + 1] = r1 - r0;
    }
}

template <class Op>
void run(int num_cu, int W, int trips, int insts_per_op) {
    using T = typename Op::T;
    const int blocks = num_cu * W;  // 256 threads = one wave per SIMD per block
    const int waves = blocks * 4;
    T* out = nullptr;
    long long* st = nullptr;
    CHECK(hipMalloc(&out, sizeof(T) * blocks * 256));
    CHECK(hipMalloc(&st, sizeof(long long) * 2 * waves));
    hipLaunchKernelGGL(bench_kernel<Op>, dim3(blocks), dim3(256), 0, 0, out, st, trips / 8);  // warm-up
    CHECK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(bench_kernel<Op>, dim3(blocks), dim3(256), 0, 0, out, st, trips);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipDeviceSynchronize());
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<long long> h(2 * waves);
    CHECK(hipMemcpy(h.data(), st, sizeof(long long) * 2 * waves, hipMemcpyDeviceToHost));
    std::vector<double> cyc(waves), clk(waves);
    for (int w = 0; w < waves; ++w) {
        cyc[w] = (double)h[2 * w];
        clk[w] = h[2 * w + 1] > 0 ? (double)h[2 * w] / (double)h[2 * w + 1] * 100.0 : 0.0;  // MHz
    }
    std::sort(cyc.begin(), cyc.end());
    std::sort(clk.begin(), clk.end());
    const double per_wave = (double)trips * kUnroll * kAcc * insts_per_op;  // wave-instructions per wave
    const double cpi = cyc[waves / 2] / (W * per_wave);
    // event-time cross-check: SIMD-cycles available / wave-instructions issued, at the median clock
    const double total = per_wave * waves;
    const double cpi_ev = (double)ms * 1e-3 * clk[waves / 2] * 1e6 * (num_cu * 4) / total;
    std::printf("{\"inst\": \"%s\", \"waves_per_simd\": %d, \"cycles_per_wave_inst\": %.3f, "
                "\"cycles_per_wave_inst_event\": %.3f, \"clock_mhz\": %.0f, \"kernel_ms\": %.3f}\n",
                Op::id(), W, cpi / 1.0, cpi_ev, clk[waves / 2], ms);
    std::fflush(stdout);
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
    CHECK(hipFree(out));
    CHECK(hipFree(st));
}

template <class Op>
void sweep(int num_cu, int trips, int insts_per_op = 1) {
    for (int W : {1, 2, 4, 8}) run<Op>(num_cu, W, trips, insts_per_op);
}

int main(int argc, char** argv) {
    int num_cu = 0;
    CHECK(hipDeviceGetAttribute(&num_cu, hipDeviceAttributeMultiprocessorCount, 0));
    const int trips = argc > 1 ? std::atoi(argv[1]) : 4096;
    sweep<v_add_f32>(num_cu, trips);
    sweep<v_mul_f32>(num_cu, trips);
    sweep<v_fma_f32>(num_cu, trips);
    sweep<v_max_f32>(num_cu, trips);
    sweep<v_rcp_f32>(num_cu, trips);
    sweep<v_sqrt_f32>(num_cu, trips);
    sweep<v_div_fixup_f32>(num_cu, trips);
    sweep<v_add_u32>(num_cu, trips);
    sweep<v_mad_u32_u24>(num_cu, trips);
    sweep<v_and_b32>(num_cu, trips);
    sweep<v_mov_b32>(num_cu, trips);
    sweep<v_cndmask_b32>(num_cu, trips, 2);
    sweep<v_add_f64>(num_cu, trips);
    sweep<v_mul_f64>(num_cu, trips);
    sweep<v_fma_f64>(num_cu, trips);
    sweep<v_rcp_f64>(num_cu, trips);
    sweep<v_sqrt_f64>(num_cu, trips);
    sweep<v_lshlrev_b64>(num_cu, trips);
    sweep<v_cvt_f64_f32>(num_cu, trips, 2);
    return 0;
}
