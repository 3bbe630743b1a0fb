// tpt_multi.cpp -- tpt_multi_* / tpt_render_multi (include/tpt.h): one frame sharded
// over the GPUs of one node, merged with ONE RCCL reduce over xGMI.
//
// Replaces the reference's worker split and merge (Renderer.cpp:86-114):
//   * the reference gives thread t the pixels i = t, t + j, t + 2j, ... (:38); here
//     device r of n renders pixel shard {pixel_begin = r, pixel_stride = n} through
//     its own libtpt context (tpt_render_device), into a zeroed full-size [rgb; splat]
//     buffer on that device.  Every pixel's XorShift stream starts at ResetRandom(i+1)
//     (:42) whichever device renders it, so the frame does not depend on n;
//   * each device's splat buffer is already scaled by 1/spp (:59) when the reduce sums
//     the n [rgb; splat] buffers onto the first device (ncclReduce, sum, fp32; for PT,
//     which splats nothing, the rgb half alone); the radiance shards are disjoint
//     (x + 0 = x: bit-identical to one GPU) and the splats are a genuine sum, the
//     reference's per-thread merge (:98-114).
// The devices render concurrently (one host thread each: tpt_render_device is
// synchronous); the reduce runs on a stream per device after every render returned.
//
// RCCL is opened at tpt_multi_create time (dlopen "librccl.so.1"), so libtpt.so
// itself has no load-time dependency on it; a process that already has RCCL loaded
// (torch) shares that copy.
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <exception>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/tpt.h"

namespace {

struct Rccl {
    void* h = nullptr;
    ncclResult_t (*init_all)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, int, ncclComm_t,
                           hipStream_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
    const char* (*err)(ncclResult_t) = nullptr;

    bool open(std::string& why) {
        if (h) return true;
        for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
            h = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
            if (h) break;
        }
        if (!h) { why = std::string("cannot load RCCL: ") + dlerror(); return false; }
        init_all = reinterpret_cast<decltype(init_all)>(dlsym(h, "ncclCommInitAll"));
        destroy = reinterpret_cast<decltype(destroy)>(dlsym(h, "ncclCommDestroy"));
        reduce = reinterpret_cast<decltype(reduce)>(dlsym(h, "ncclReduce"));
        group_start = reinterpret_cast<decltype(group_start)>(dlsym(h, "ncclGroupStart"));
        group_end = reinterpret_cast<decltype(group_end)>(dlsym(h, "ncclGroupEnd"));
        err = reinterpret_cast<decltype(err)>(dlsym(h, "ncclGetErrorString"));
        if (!init_all || !destroy || !reduce || !group_start || !group_end || !err) {
            why = "RCCL library lacks the collective entry points";
            return false;
        }
        return true;
    }
};
Rccl g_rccl;

// tpt_multi_last_error(NULL): why the calling thread's last tpt_multi_create failed
// (the group does not exist then, so the reason cannot live in it).
thread_local std::string g_create_err;

// Restores the calling thread's current HIP device on every return path: the group
// switches devices per rank, and a caller (torch) in the same thread must not find
// itself on another GPU afterwards.
struct DeviceGuard {
    int dev = -1;
    DeviceGuard() {
        if (hipGetDevice(&dev) != hipSuccess) dev = -1;
    }
    ~DeviceGuard() {
        if (dev >= 0) (void)hipSetDevice(dev);
    }
};

}  // namespace

struct tpt_multi {
    std::vector<int> dev;
    std::vector<tpt_ctx*> ctx;
    std::vector<ncclComm_t> comm;
    std::vector<hipStream_t> stream;
    std::vector<float*> fb;  // per device: [rgb; splat], 2 * W*H*3 floats
    int64_t fb_floats = 0;   // W*H*3
    std::string err;
    bool has_scene = false;
};

namespace {

int mfail(tpt_multi* m, int code, const std::string& msg) {
    if (m) m->err = msg;
    return code;
}

void release(tpt_multi* m) {
    for (size_t r = 0; r < m->dev.size(); ++r) {
        (void)hipSetDevice(m->dev[r]);
        if (r < m->stream.size() && m->stream[r]) (void)hipStreamSynchronize(m->stream[r]);
        if (r < m->fb.size() && m->fb[r]) (void)hipFree(m->fb[r]);
        if (r < m->stream.size() && m->stream[r]) (void)hipStreamDestroy(m->stream[r]);
    }
    for (ncclComm_t c : m->comm)
        if (c && g_rccl.destroy) (void)g_rccl.destroy(c);
    for (tpt_ctx* c : m->ctx)
        if (c) tpt_destroy(c);
    m->fb.clear();
    m->stream.clear();
    m->comm.clear();
    m->ctx.clear();
}


int create_fail(tpt_multi* m, int code, const std::string& why) {
    g_create_err = why;
    if (m) {
        release(m);
        delete m;
    }
    return code;
}

int multi_create(int ngpu, const int* devices, tpt_multi** out) {
    int avail = 0;
    if (hipGetDeviceCount(&avail) != hipSuccess) return create_fail(nullptr, TPT_E_DEVICE, "hipGetDeviceCount failed");
    if (ngpu < 1 || ngpu > avail)
        return create_fail(nullptr, TPT_E_INVALID,
                           "ngpu " + std::to_string(ngpu) + " outside 1.." + std::to_string(avail));
    tpt_multi* m = new tpt_multi();
    for (int r = 0; r < ngpu; ++r) {
        const int d = devices ? devices[r] : r;
        if (d < 0 || d >= avail || std::count(m->dev.begin(), m->dev.end(), d))
            return create_fail(m, TPT_E_INVALID, "bad or repeated device id " + std::to_string(d));
        m->dev.push_back(d);
    }
    std::string why;
    if (!g_rccl.open(why)) return create_fail(m, TPT_E_UNSUPPORTED, why);
    for (int r = 0; r < ngpu; ++r) {
        tpt_ctx* c = nullptr;
        int rc = tpt_create(m->dev[r], &c);
        m->ctx.push_back(c);
        hipStream_t s = nullptr;
        if (rc == TPT_OK && (hipSetDevice(m->dev[r]) != hipSuccess ||
                             hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess))
            rc = TPT_E_DEVICE;
        m->stream.push_back(s);
        if (rc != TPT_OK) return create_fail(m, rc, "device " + std::to_string(m->dev[r]) + ": context or stream");
    }
    m->comm.assign(ngpu, nullptr);
    const ncclResult_t e = g_rccl.init_all(m->comm.data(), ngpu, m->dev.data());
    if (e != ncclSuccess) {
        m->comm.assign(ngpu, nullptr);
        return create_fail(m, TPT_E_DEVICE, std::string("ncclCommInitAll: ") + g_rccl.err(e));
    }
    *out = m;
    g_create_err.clear();
    return TPT_OK;
}

}  // namespace

extern "C" {

int tpt_multi_create(int ngpu, const int* devices, tpt_multi** out) {
    if (!out) return TPT_E_INVALID;
    *out = nullptr;
    DeviceGuard guard;
    try {
        return multi_create(ngpu, devices, out);
    } catch (const std::bad_alloc&) {
        g_create_err = "host allocation failed";
        return TPT_E_ALLOC;
    } catch (const std::exception& x) {
        g_create_err = x.what();
        return TPT_E_DEVICE;
    } catch (...) {
        g_create_err = "unknown exception";
        return TPT_E_DEVICE;
    }
}

void tpt_multi_destroy(tpt_multi* m) {
    if (!m) return;
    DeviceGuard guard;
    release(m);
    delete m;
}

// With m == NULL: the reason the calling thread's last tpt_multi_create failed.
const char* tpt_multi_last_error(const tpt_multi* m) { return m ? m->err.c_str() : g_create_err.c_str(); }

}  // extern "C"

namespace {

int multi_upload(tpt_multi* m, const tpt_scene_desc* d) {
    m->has_scene = false;
    for (size_t r = 0; r < m->ctx.size(); ++r) {
        int rc = tpt_upload_scene(m->ctx[r], d);
        if (rc) return mfail(m, rc, "device " + std::to_string(m->dev[r]) + ": " + tpt_last_error(m->ctx[r]));
    }
    const int64_t n = (int64_t)d->width * d->height * 3;
    if (n != m->fb_floats) {
        for (size_t r = 0; r < m->fb.size(); ++r) {
            (void)hipSetDevice(m->dev[r]);
            if (m->fb[r]) (void)hipFree(m->fb[r]);
        }
        m->fb.assign(m->dev.size(), nullptr);
        m->fb_floats = 0;
        for (size_t r = 0; r < m->dev.size(); ++r) {
            if (hipSetDevice(m->dev[r]) != hipSuccess || hipMalloc(&m->fb[r], 2 * n * sizeof(float)) != hipSuccess)
                return mfail(m, TPT_E_ALLOC, "frame buffers");
        }
        m->fb_floats = n;
    }
    m->has_scene = true;
    return TPT_OK;
}

int multi_render(tpt_multi* m, const tpt_render_params* p, float* rgb, float* splat, tpt_stats* st) {
    if (!m->has_scene) return mfail(m, TPT_E_NOSCENE, "no scene uploaded");
    if (p->pixel_begin != 0 || p->pixel_stride != 1)
        return mfail(m, TPT_E_INVALID, "tpt_render_multi shards the whole frame itself: pixel_begin 0, stride 1");
    const auto t0 = std::chrono::steady_clock::now();
    const int n = (int)m->dev.size();
    const int64_t nf = m->fb_floats;
    const bool bdpt = p->mode == TPT_MODE_BDPT;
    std::vector<int> rc(n, TPT_OK);
    std::vector<tpt_stats> part(n);
    {
        std::vector<std::thread> th;
        th.reserve(n);
        try {
            for (int r = 0; r < n; ++r) {
                th.emplace_back([&, r]() {
                    tpt_render_params q = *p;
                    q.pixel_begin = r;  // Renderer.cpp:38: i = off; i += j
                    q.pixel_stride = n;
                    // rgb (and splat for BDPT) are zeroed by tpt_render_device: pixels
                    // outside the shard stay 0.  PT splats nothing and its splat half is
                    // neither written nor reduced.
                    rc[r] = tpt_render_device(m->ctx[r], &q, m->fb[r], bdpt ? m->fb[r] + nf : nullptr, &part[r]);
                });
            }
        } catch (...) {  // std::system_error: join what started, then report
            for (auto& t : th) t.join();
            return mfail(m, TPT_E_DEVICE, "cannot start a render thread");
        }
        for (auto& t : th) t.join();
    }
    for (int r = 0; r < n; ++r)
        if (rc[r]) return mfail(m, rc[r], "device " + std::to_string(m->dev[r]) + ": " + tpt_last_error(m->ctx[r]));
    // ONE collective: sum the n buffers onto the first device (Renderer.cpp:98-114):
    // [rgb; splat] (2 W*H*3 floats) for BDPT, the rgb half alone for PT / PT-indirect.
    // With one device it is RCCL's in-place single-rank reduce (a no-op), kept so the
    // one-GPU box exercises the same code path as the 8-GPU node.
    const size_t count = (size_t)(bdpt ? 2 * nf : nf);
    {
        if (g_rccl.group_start() != ncclSuccess) return mfail(m, TPT_E_DEVICE, "ncclGroupStart");
        ncclResult_t e = ncclSuccess;
        bool dev_ok = true;
        for (int r = 0; r < n && e == ncclSuccess && dev_ok; ++r) {
            dev_ok = hipSetDevice(m->dev[r]) == hipSuccess;
            if (dev_ok) e = g_rccl.reduce(m->fb[r], m->fb[r], count, ncclFloat32, ncclSum, 0, m->comm[r], m->stream[r]);
        }
        const ncclResult_t e2 = g_rccl.group_end();  // always closes the group
        if (!dev_ok) return mfail(m, TPT_E_DEVICE, "hipSetDevice");
        if (e != ncclSuccess || e2 != ncclSuccess)
            return mfail(m, TPT_E_DEVICE, std::string("ncclReduce: ") + g_rccl.err(e != ncclSuccess ? e : e2));
    }
    for (int r = 0; r < n; ++r) {
        if (hipSetDevice(m->dev[r]) != hipSuccess || hipStreamSynchronize(m->stream[r]) != hipSuccess)
            return mfail(m, TPT_E_DEVICE, "reduce did not complete");
    }
    if (hipSetDevice(m->dev[0]) != hipSuccess ||
        hipMemcpy(rgb, m->fb[0], nf * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess ||
        (splat && bdpt && hipMemcpy(splat, m->fb[0] + nf, nf * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess))
        return mfail(m, TPT_E_DEVICE, "copy of the reduced frame");
    if (st) {
        for (int r = 0; r < n; ++r) {
            st->pixels += part[r].pixels;
            st->samples += part[r].samples;
            st->bounces += part[r].bounces;
            st->nonfinite += part[r].nonfinite;  // shards are disjoint
            st->nonfinite_splat += part[r].nonfinite_splat;
            st->kernel_ms = std::max(st->kernel_ms, part[r].kernel_ms);
        }
        if (splat && bdpt && n > 1) {
            // splats of several devices land on the same pixels: count the reduced buffer
            int64_t bad = 0;
            for (int64_t p = 0; p < nf / 3; ++p)
                bad += !(std::isfinite(splat[3 * p]) && std::isfinite(splat[3 * p + 1]) && std::isfinite(splat[3 * p + 2]));
            st->nonfinite_splat = bad;
        }
        st->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    return TPT_OK;
}

// No C++ exception crosses the ABI (tpt.h): map them to status codes.
template <typename F>
int guarded(tpt_multi* m, F&& f) {
    try {
        return f();
    } catch (const std::bad_alloc&) {
        return mfail(m, TPT_E_ALLOC, "host allocation failed");
    } catch (const std::exception& x) {
        return mfail(m, TPT_E_DEVICE, x.what());
    } catch (...) {
        return mfail(m, TPT_E_DEVICE, "unknown exception");
    }
}

}  // namespace

extern "C" {

int tpt_multi_upload_scene(tpt_multi* m, const tpt_scene_desc* d) {
    if (!m || !d) return TPT_E_INVALID;
    DeviceGuard guard;
    return guarded(m, [&] { return multi_upload(m, d); });
}

int tpt_render_multi(tpt_multi* m, const tpt_render_params* p, float* rgb, float* splat, tpt_stats* st) {
    if (!m || !p || !rgb) return TPT_E_INVALID;
    if (st) std::memset(st, 0, sizeof(*st));
    DeviceGuard guard;
    return guarded(m, [&] { return multi_render(m, p, rgb, splat, st); });
}

}  // extern "C"
