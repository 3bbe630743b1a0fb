// tpt_capi.hip -- gfx950 kernels of the integration loop + the C ABI (include/tpt.h).
//
// Kernel geometry (replay mode): one lane per pixel stream, serial spp loop, which
// is what the reference's RNG contract requires -- ResetRandom(i+1) once per pixel
// and ONE XorShift stream through all spp samples (Renderer.cpp:42-52), with a
// data-dependent number of draws per sample, so sample k of a pixel can only be
// produced after samples 0..k-1.  784x784 = 614,656 streams =
// 9,604 wave64s: ~9 waves per SIMD on 256 CUs, enough to fill the chip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/tpt.h"
#include "tpt_bdpt.h"
#include "tpt_device.h"
#include "tpt_scene_build.h"

using namespace tpt;

// ------------------------------------------------------------------ kernels --
// PT: Renderer.cpp:38-52 for TPT_MODE_PT.  Pixels are {begin + k*stride} or
// list[k]; rgb row = pixel index (full frame) or k (list).
__global__ __launch_bounds__(kBlock) void tpt_pt_kernel(DScene s, int spp, int64_t begin, int64_t stride,
                                                        int64_t count, const int64_t* __restrict__ list,
                                                        float* __restrict__ out) {
    __shared__ int stack[kStackCap * kBlock];
    int* stk = stack + threadIdx.x;
    const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k >= count) return;
    const int64_t i = list ? list[k] : begin + k * stride;
    const int64_t row = list ? k : i;
    const int px = (int)(i % s.width), py = (int)(i / s.width);
    const V3 dir = pixel_ray(px, py, s.width, s.height, s.scale);
    const V3 eye = v3(s.eye[0], s.eye[1], s.eye[2]);
    const Ray r = make_ray(eye, dir);
    PTV v = scene_intersect(s, r, TPT_CULL_BACK, stk);
    V3 acc = v3s(0.0f);
    if (v.type != T_BG) {
        uint32_t rs = (uint32_t)((int)i + 1);
        PTHit h;
        h.x = v.x;
        h.n = v.N;
        h.wo = -dir;
        h.mat = prim_mat(s, v.prim);
        const Mat m = load_mat(s, h.mat);
        const float inv = 1.0f / spp;
        for (int j = 0; j < spp; ++j) acc = acc + mul(pt_sample(s, h, m, rs, stk), inv);
    }
    out[3 * row + 0] = acc.x;
    out[3 * row + 1] = acc.y;
    out[3 * row + 2] = acc.z;
}

// BDPT: Renderer.cpp:38-52 + :58-60 for TPT_MODE_BDPT.  t=1 strategies splat into
// `splat` with fp32 atomics (the reference sums per-thread buffers instead,
// Renderer.cpp:98-114: same values, different summation order).
__global__ __launch_bounds__(kBlock) void tpt_bdpt_kernel(DScene s, int spp, int64_t begin, int64_t stride,
                                                          int64_t count, const int64_t* __restrict__ list,
                                                          float* __restrict__ out, float* __restrict__ splat,
                                                          unsigned long long* __restrict__ bounces) {
    __shared__ int stack[kStackCap * kBlock];
    int* stk = stack + threadIdx.x;
    const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k >= count) return;
    const int64_t i = list ? list[k] : begin + k * stride;
    const int64_t row = list ? k : i;
    V3 acc = v3s(0.0f);
    unsigned long long nb = 0;
    bdpt_pixel(s, i, spp, acc, splat, nb, stk);
    out[3 * row + 0] = acc.x;
    out[3 * row + 1] = acc.y;
    out[3 * row + 2] = acc.z;
    if (bounces) atomicAdd(bounces, nb);
}

__global__ void tpt_scale_kernel(float* __restrict__ buf, int64_t n, float spp) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n) buf[k] = buf[k] * 1.0f / spp;  // Renderer.cpp:59 `e * 1.0f / spp`
}

// Closest-hit queries (Scene::Intersect) for tpt_intersect.
__global__ __launch_bounds__(kBlock) void tpt_intersect_kernel(DScene s, const float* __restrict__ rays, int64_t n,
                                                               int cull, float* __restrict__ out) {
    __shared__ int stack[kStackCap * kBlock];
    int* stk = stack + threadIdx.x;
    const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k >= n) return;
    const float* q = rays + 6 * k;
    Ray r = make_ray(v3(q[0], q[1], q[2]), v3(q[3], q[4], q[5]));
    PTV v = scene_intersect(s, r, cull, stk);
    float* o = out + 8 * k;
    o[0] = v.type == T_BG ? 0.f : 1.f;
    o[1] = v.x.x; o[2] = v.x.y; o[3] = v.x.z;
    o[4] = v.N.x; o[5] = v.N.y; o[6] = v.N.z;
    o[7] = (float)v.prim;
}

// ------------------------------------------------------------------ C ABI --
struct tpt_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    std::string err;
    bool has_scene = false;
    HostScene hs;
    DScene ds{};
    void* blob = nullptr;
    float* rgb = nullptr;
    float* splat = nullptr;
    int64_t fb_floats = 0;
    int64_t* list = nullptr;
    int64_t list_cap = 0;
    float* rows = nullptr;
    int64_t rows_cap = 0;
    unsigned long long* counters = nullptr;
};

namespace {

int fail(tpt_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    return code;
}
#define HIP_TRY(c, expr)                                                                     \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            return fail((c), TPT_E_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

float camera_scale(double fov) {  // SceneRenderingHelper.cpp:12-14 (deg2rad in float, tan in double)
    float half = (float)(fov * 0.5);
    float rad = (float)(half * 3.141592653589793f / 180.0);
    return (float)std::tan((double)rad);
}

template <typename T>
size_t push_array(std::vector<char>& blob, const std::vector<T>& v) {
    size_t off = (blob.size() + 255) & ~(size_t)255;
    blob.resize(off + std::max<size_t>(v.size() * sizeof(T), 16));
    if (!v.empty()) std::memcpy(blob.data() + off, v.data(), v.size() * sizeof(T));
    return off;
}

int ensure_fb(tpt_ctx* c) {
    int64_t need = (int64_t)c->hs.width * c->hs.height * 3;
    if (c->fb_floats >= need) return TPT_OK;
    if (c->rgb) (void)hipFree(c->rgb);
    if (c->splat) (void)hipFree(c->splat);
    c->rgb = c->splat = nullptr;
    c->fb_floats = 0;
    HIP_TRY(c, hipMalloc(&c->rgb, need * sizeof(float)));
    HIP_TRY(c, hipMalloc(&c->splat, need * sizeof(float)));
    c->fb_floats = need;
    return TPT_OK;
}

int64_t shard_count(int64_t npix, int64_t begin, int64_t stride) {
    if (begin >= npix) return 0;
    return (npix - begin + stride - 1) / stride;
}

// Launch the integration kernel for `count` pixels; rows/splat are device buffers.
int launch(tpt_ctx* c, int mode, int spp, int64_t begin, int64_t stride, int64_t count, const int64_t* dlist,
           float* drows, float* dsplat, tpt_stats* st) {
    if (count <= 0) return TPT_OK;
    const int64_t blocks = (count + kBlock - 1) / kBlock;
    HIP_TRY(c, hipMemsetAsync(c->counters, 0, sizeof(unsigned long long) * 4, c->stream));
    HIP_TRY(c, hipEventRecord(c->ev0, c->stream));
    if (mode == TPT_MODE_PT) {
        hipLaunchKernelGGL(tpt_pt_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, c->stream, c->ds, spp, begin,
                           stride, count, dlist, drows);
    } else {
        hipLaunchKernelGGL(tpt_bdpt_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, c->stream, c->ds, spp, begin,
                           stride, count, dlist, drows, dsplat, c->counters);
    }
    HIP_TRY(c, hipGetLastError());
    HIP_TRY(c, hipEventRecord(c->ev1, c->stream));
    if (mode == TPT_MODE_BDPT && dsplat) {
        int64_t n = (int64_t)c->hs.width * c->hs.height * 3;
        hipLaunchKernelGGL(tpt_scale_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream, dsplat, n,
                           (float)spp);
        HIP_TRY(c, hipGetLastError());
    }
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (st) {
        float ms = 0.f;
        HIP_TRY(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
        st->kernel_ms = ms;
        st->pixels = count;
        st->samples = count * (int64_t)spp;
        unsigned long long nb = 0;
        HIP_TRY(c, hipMemcpy(&nb, c->counters, sizeof(nb), hipMemcpyDeviceToHost));
        st->bounces = (int64_t)nb;
    }
    return TPT_OK;
}

int check_render_args(tpt_ctx* c, int spp, int mode) {
    if (!c) return TPT_E_INVALID;
    if (!c->has_scene) return fail(c, TPT_E_NOSCENE, "no scene uploaded");
    if (spp <= 0) return fail(c, TPT_E_INVALID, "spp must be positive");
    if (mode != TPT_MODE_PT && mode != TPT_MODE_BDPT) return fail(c, TPT_E_INVALID, "unknown mode");
    if (mode == TPT_MODE_BDPT && c->hs.emitters.empty())
        return fail(c, TPT_E_INVALID, "BDPT needs an emitter (BDPT.cpp:287 uses m_emissionObjects[0])");
    return TPT_OK;
}

}  // namespace

extern "C" {

int tpt_abi_version(void) { return TPT_ABI_VERSION; }
float tpt_camera_scale(double fov) { return camera_scale(fov); }

int tpt_create(int device, tpt_ctx** out) {
    if (!out) return TPT_E_INVALID;
    *out = nullptr;
    tpt_ctx* c = new tpt_ctx();
    c->device = device;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) {
        delete c;
        return TPT_E_DEVICE;
    }
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
        hipMalloc(&c->counters, sizeof(unsigned long long) * 4) != hipSuccess) {
        delete c;
        return TPT_E_DEVICE;
    }
    *out = c;
    return TPT_OK;
}

void tpt_destroy(tpt_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (void* p : {(void*)c->blob, (void*)c->rgb, (void*)c->splat, (void*)c->list, (void*)c->rows, (void*)c->counters})
        if (p) (void)hipFree(p);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

const char* tpt_last_error(const tpt_ctx* c) { return c ? c->err.c_str() : "null context"; }

int tpt_upload_scene(tpt_ctx* c, const tpt_scene_desc* d) {
    if (!c) return TPT_E_INVALID;
    HIP_TRY(c, hipSetDevice(c->device));
    HostScene hs;
    int rc = build_host_scene(d, hs, c->err);
    if (rc != TPT_OK) return rc;
    if (hs.max_stack > kStackCap)
        return fail(c, TPT_E_UNSUPPORTED, "BVH deeper than the LDS traversal stack (" + std::to_string(hs.max_stack) + ")");
    if (hs.nodes.size() > (size_t)0x7fffffff) return fail(c, TPT_E_UNSUPPORTED, "too many BVH nodes");
    std::vector<char> blob;
    size_t o_nodes = push_array(blob, hs.nodes), o_area = push_array(blob, hs.node_area),
           o_tris = push_array(blob, hs.tris), o_trix = push_array(blob, hs.trix), o_sph = push_array(blob, hs.sph),
           o_mats = push_array(blob, hs.mats), o_objs = push_array(blob, hs.objs),
           o_em = push_array(blob, hs.emitters);
    if (c->blob) { (void)hipFree(c->blob); c->blob = nullptr; }
    HIP_TRY(c, hipMalloc(&c->blob, blob.size()));
    HIP_TRY(c, hipMemcpy(c->blob, blob.data(), blob.size(), hipMemcpyHostToDevice));
    char* b = (char*)c->blob;
    DScene ds;
    std::memset(&ds, 0, sizeof(ds));
    ds.nodes = (const DNode*)(b + o_nodes);
    ds.node_area = (const float*)(b + o_area);
    ds.tris = (const DTri*)(b + o_tris);
    ds.trix = (const DTriX*)(b + o_trix);
    ds.sph = (const DSphere*)(b + o_sph);
    ds.mats = (const DMat*)(b + o_mats);
    ds.objs = (const DObj*)(b + o_objs);
    ds.emitters = (const int32_t*)(b + o_em);
    ds.n_emitters = (int)hs.emitters.size();
    ds.ntri = (int)hs.tris.size();
    ds.nsph = (int)hs.sph.size();
    ds.nnodes = (int)hs.nodes.size();
    ds.nobj = (int)hs.objs.size();
    ds.width = hs.width;
    ds.height = hs.height;
    ds.scale = camera_scale(hs.fov);
    for (int k = 0; k < 3; ++k) { ds.eye[k] = hs.eye[k]; ds.bg[k] = hs.bg[k]; }
    ds.max_stack = hs.max_stack;
    c->ds = ds;
    c->hs = std::move(hs);
    c->has_scene = true;
    return ensure_fb(c);
}

int tpt_render_device(tpt_ctx* c, const tpt_render_params* p, float* rgb_dev, float* splat_dev, tpt_stats* st) {
    if (!c || !p) return TPT_E_INVALID;
    int rc = check_render_args(c, p->spp, p->mode);
    if (rc) return rc;
    if (p->pixel_begin < 0 || p->pixel_stride < 1) return fail(c, TPT_E_INVALID, "bad pixel shard");
    if (!rgb_dev || (p->mode == TPT_MODE_BDPT && !splat_dev)) return fail(c, TPT_E_INVALID, "null output buffer");
    HIP_TRY(c, hipSetDevice(c->device));
    auto t0 = std::chrono::steady_clock::now();
    const int64_t npix = (int64_t)c->hs.width * c->hs.height;
    HIP_TRY(c, hipMemsetAsync(rgb_dev, 0, npix * 3 * sizeof(float), c->stream));
    if (p->mode == TPT_MODE_BDPT) HIP_TRY(c, hipMemsetAsync(splat_dev, 0, npix * 3 * sizeof(float), c->stream));
    const int64_t count = shard_count(npix, p->pixel_begin, p->pixel_stride);
    rc = launch(c, p->mode, p->spp, p->pixel_begin, p->pixel_stride, count, nullptr, rgb_dev,
                p->mode == TPT_MODE_BDPT ? splat_dev : nullptr, st);
    if (rc) return rc;
    if (st) st->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return TPT_OK;
}

int tpt_render(tpt_ctx* c, const tpt_render_params* p, float* rgb, float* splat, tpt_stats* st) {
    if (!c || !p || !rgb) return TPT_E_INVALID;
    int rc = check_render_args(c, p->spp, p->mode);
    if (rc) return rc;
    auto t0 = std::chrono::steady_clock::now();
    rc = tpt_render_device(c, p, c->rgb, c->splat, st);
    if (rc) return rc;
    const int64_t n = (int64_t)c->hs.width * c->hs.height * 3;
    HIP_TRY(c, hipMemcpy(rgb, c->rgb, n * sizeof(float), hipMemcpyDeviceToHost));
    if (p->mode == TPT_MODE_BDPT && splat) HIP_TRY(c, hipMemcpy(splat, c->splat, n * sizeof(float), hipMemcpyDeviceToHost));
    if (st) st->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return TPT_OK;
}

int tpt_render_pixels(tpt_ctx* c, int32_t spp, int32_t mode, const int64_t* pixels, int64_t n, float* rgb,
                      float* splat, tpt_stats* st) {
    int rc = check_render_args(c, spp, mode);
    if (rc) return rc;
    if (n < 0 || (n > 0 && (!pixels || !rgb))) return fail(c, TPT_E_INVALID, "bad pixel list");
    const int64_t npix = (int64_t)c->hs.width * c->hs.height;
    for (int64_t k = 0; k < n; ++k)
        if (pixels[k] < 0 || pixels[k] >= npix) return fail(c, TPT_E_INVALID, "pixel index out of range");
    HIP_TRY(c, hipSetDevice(c->device));
    auto t0 = std::chrono::steady_clock::now();
    if (n > c->list_cap) {
        if (c->list) (void)hipFree(c->list);
        if (c->rows) (void)hipFree(c->rows);
        c->list = nullptr; c->rows = nullptr; c->list_cap = 0;
        HIP_TRY(c, hipMalloc(&c->list, n * sizeof(int64_t)));
        HIP_TRY(c, hipMalloc(&c->rows, n * 3 * sizeof(float)));
        c->list_cap = n;
    }
    if (n > 0) HIP_TRY(c, hipMemcpyAsync(c->list, pixels, n * sizeof(int64_t), hipMemcpyHostToDevice, c->stream));
    if (mode == TPT_MODE_BDPT) HIP_TRY(c, hipMemsetAsync(c->splat, 0, npix * 3 * sizeof(float), c->stream));
    rc = launch(c, mode, spp, 0, 1, n, c->list, c->rows, mode == TPT_MODE_BDPT ? c->splat : nullptr, st);
    if (rc) return rc;
    if (n > 0) HIP_TRY(c, hipMemcpy(rgb, c->rows, n * 3 * sizeof(float), hipMemcpyDeviceToHost));
    if (mode == TPT_MODE_BDPT && splat)
        HIP_TRY(c, hipMemcpy(splat, c->splat, npix * 3 * sizeof(float), hipMemcpyDeviceToHost));
    if (st) st->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return TPT_OK;
}

int tpt_intersect(tpt_ctx* c, const float* rays, int64_t n, int32_t cull, float* out) {
    if (!c) return TPT_E_INVALID;
    if (!c->has_scene) return fail(c, TPT_E_NOSCENE, "no scene uploaded");
    if (n <= 0) return TPT_OK;
    if (!rays || !out || cull < 0 || cull > 2) return fail(c, TPT_E_INVALID, "bad intersect arguments");
    HIP_TRY(c, hipSetDevice(c->device));
    float *dr = nullptr, *dout = nullptr;
    HIP_TRY(c, hipMalloc(&dr, n * 6 * sizeof(float)));
    hipError_t e = hipMalloc(&dout, n * 8 * sizeof(float));
    if (e != hipSuccess) { (void)hipFree(dr); return fail(c, TPT_E_ALLOC, "intersect buffers"); }
    int rc = TPT_OK;
    if (hipMemcpy(dr, rays, n * 6 * sizeof(float), hipMemcpyHostToDevice) != hipSuccess) rc = TPT_E_DEVICE;
    if (!rc) {
        hipLaunchKernelGGL(tpt_intersect_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                           c->stream, c->ds, dr, n, cull, dout);
        if (hipGetLastError() != hipSuccess || hipStreamSynchronize(c->stream) != hipSuccess ||
            hipMemcpy(out, dout, n * 8 * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess)
            rc = TPT_E_DEVICE;
    }
    (void)hipFree(dr);
    (void)hipFree(dout);
    if (rc) c->err = "intersect kernel failed";
    return rc;
}

}  // extern "C"
