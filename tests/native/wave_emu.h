// wave_emu.h -- host emulation of ONE 64-lane wavefront, so that device code of the hot
// path (csrc/tpt_device.h, csrc/tpt_bdpt.h) can run unmodified on the CPU in tests.
//
// Each lane is a fiber of one OS thread (a minimal x86-64 SysV stack switch: the
// callee-saved registers and the stack pointer; ucontext's swapcontext made a system call
// per switch and took 30 s of the test).  Lanes run one after the other up to
// their next wave-collective (a ballot, a shuffle, readfirstlane, a wave barrier); when
// the last active lane arrives the collective completes and every lane resumes with its
// result, in lane order.  This is SIMT lockstep for code whose collectives are reached
// by every active lane in the same order -- which device code that calls __ballot must
// satisfy anyway (tpt_bdpt.h's walk4_steal: "every active lane must call it").  Between
// collectives each lane runs its own (possibly divergent) code, as the hardware's
// exec-masked execution would; LDS is ordinary host memory visible to all lanes, and a
// wave barrier orders it like wave_lds_sync() does.
//
// Include this BEFORE the device headers; define TPT_HOST_EMU.  Tests only.
#pragma once
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <vector>

extern "C" void wemu_swap(void** save_sp, void* load_sp);
asm(R"(
    .text
    .globl wemu_swap
    .type wemu_swap, @function
wemu_swap:
    pushq %rbp
    pushq %rbx
    pushq %r12
    pushq %r13
    pushq %r14
    pushq %r15
    movq %rsp, (%rdi)
    movq %rsi, %rsp
    popq %r15
    popq %r14
    popq %r13
    popq %r12
    popq %rbx
    popq %rbp
    ret
    .size wemu_swap, .-wemu_swap
)");

namespace wemu {
constexpr int kLanes = 64;
struct Wave {
    void* main_ctx = nullptr;
    void* ctx[kLanes];
    std::vector<char> stack[kLanes];
    bool done[kLanes];
    int cur = 0, active = 0, arrived = 0;
    unsigned long long gen = 0, collectives = 0;
    uint64_t dep[kLanes], snap[kLanes];
    uint64_t in_mask = 0, snap_mask = 0;  // lanes that deposited in the current / last collective
    const char* site = nullptr;           // call site of the current collective (all lanes must match)
    std::function<void(int)> body;
};
inline Wave*& wave() {
    static Wave* w = nullptr;
    return w;
}
inline void switch_from(int me) {  // run the next lane that has not finished (or return to main)
    Wave& w = *wave();
    for (int k = 1; k <= kLanes; ++k) {
        const int j = (me + k) % kLanes;
        if (!w.done[j]) {
            if (j == me) return;
            w.cur = j;
            wemu_swap(&w.ctx[me], w.ctx[j]);
            w.cur = me;
            return;
        }
    }
    wemu_swap(&w.ctx[me], w.main_ctx);
}
inline void complete() {
    Wave& w = *wave();
    w.site = nullptr;
    std::memcpy(w.snap, w.dep, sizeof(w.dep));
    w.snap_mask = w.in_mask;
    w.in_mask = 0;
    w.arrived = 0;
    ++w.gen;
    ++w.collectives;
}
// Deposit v, wait for every active lane; returns the snapshot of all lanes' deposits.
// Every active lane must reach the SAME collective (`site`): a collective inside code
// that only some lanes execute (the hardware's exec mask) is not modelled, and is
// reported instead of being merged with another site's.
inline const uint64_t* exchange_at(uint64_t v, const char* site) {
    Wave& w = *wave();
    const int me = w.cur;
    if (w.site == nullptr) {
        w.site = site;
    } else if (std::strcmp(w.site, site) != 0) {
        std::fprintf(stderr, "wave_emu: lanes at different collectives (%s vs %s): divergent collective\n", w.site, site);
        std::abort();
    }
    w.dep[me] = v;
    w.in_mask |= 1ull << me;
    const unsigned long long g = w.gen;
    if (++w.arrived == w.active) complete();
    while (w.gen == g) switch_from(me);
    return w.snap;
}
#define WEMU_STR2(x) #x
#define WEMU_STR(x) WEMU_STR2(x)
#define WEMU_SITE __FILE__ ":" WEMU_STR(__LINE__)
[[noreturn]] inline void entry() {
    Wave& w = *wave();
    const int me = w.cur;
    w.body(me);
    w.done[me] = true;
    --w.active;
    if (w.active > 0 && w.arrived == w.active) complete();  // the others waited on this lane
    switch_from(me);
    std::abort();  // a finished lane is never resumed
}
// Run body(lane) on all 64 lanes of one emulated wave.
inline unsigned long long run(const std::function<void(int)>& body) {
    static Wave* pool = new Wave;  // one wave and its fiber stacks, reused by every run
    Wave* w = pool;
    w->cur = w->active = w->arrived = 0;
    w->gen = w->collectives = 0;
    w->in_mask = w->snap_mask = 0;
    w->site = nullptr;
    wave() = w;
    w->body = body;
    w->active = kLanes;
    for (int l = 0; l < kLanes; ++l) {
        w->done[l] = false;
        if (w->stack[l].empty()) w->stack[l].resize(1 << 20);
        // a fresh fiber's stack: six zero registers for wemu_swap's pops, then entry as
        // its return address (entered with rsp = 8 mod 16, as after a call)
        uintptr_t top = ((uintptr_t)(w->stack[l].data() + w->stack[l].size())) & ~(uintptr_t)15;
        void** sp = (void**)top;
        *--sp = nullptr;                 // entry's (never used) return address
        *--sp = (void*)&entry;
        for (int r = 0; r < 6; ++r) *--sp = nullptr;
        w->ctx[l] = sp;
    }
    w->cur = 0;
    wemu_swap(&w->main_ctx, w->ctx[0]);
    for (int l = 0; l < kLanes; ++l)
        if (!w->done[l]) { std::fprintf(stderr, "wave_emu: lane %d did not finish\n", l); std::abort(); }
    const unsigned long long n = w->collectives;
    wave() = nullptr;
    return n;
}
inline int lane() { return wave()->cur; }
inline uint64_t ballot(bool p, const char* site) {
    exchange_at(p ? 1 : 0, site);
    uint64_t m = 0;
    const Wave& w = *wave();
    for (int l = 0; l < kLanes; ++l)
        if (((w.snap_mask >> l) & 1) && w.snap[l]) m |= 1ull << l;
    return m;
}
inline uint32_t bits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
inline float fbits(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }
template <class T>
inline T shfl(T v, int src, const char* site) {  // __shfl: lane src's value (mod 64) if it took part, else its own
    uint64_t u = 0;
    std::memcpy(&u, &v, sizeof(T));
    const uint64_t* s = exchange_at(u, site);
    src &= 63;
    uint64_t r = ((wave()->snap_mask >> src) & 1) ? s[src] : u;
    T out;
    std::memcpy(&out, &r, sizeof(T));
    return out;
}
inline int readfirstlane(int v, const char* site) {
    const uint64_t* s = exchange_at((uint32_t)v, site);
    const uint64_t m = wave()->snap_mask;
    return (int)(uint32_t)s[__builtin_ctzll(m)];
}
inline int readlane(int v, int l, const char* site) { return (int)(uint32_t)exchange_at((uint32_t)v, site)[l & 63]; }
struct Tid {
    unsigned x;
};
}  // namespace wemu

// ---- the device intrinsics the hot-path headers use, on the emulated wave ----------
#define __ballot(p) wemu::ballot((p), WEMU_SITE)
#define __lane_id() ((unsigned)wemu::lane())
#define __shfl(v, l) wemu::shfl((v), (l), WEMU_SITE)
#define __shfl_xor(v, o) wemu::shfl((v), wemu::lane() ^ (o), WEMU_SITE)
#define threadIdx (wemu::Tid{(unsigned)wemu::lane()})
#define __builtin_amdgcn_readfirstlane(v) wemu::readfirstlane((v), WEMU_SITE)
#define __builtin_amdgcn_readlane(v, l) wemu::readlane((v), (l), WEMU_SITE)
#define __builtin_amdgcn_mbcnt_lo(m, a) ((unsigned)__builtin_popcount((unsigned)(m) & ((wemu::lane() >= 32) ? ~0u : ((1u << wemu::lane()) - 1u))) + (a))
#define __builtin_amdgcn_mbcnt_hi(m, a) ((unsigned)__builtin_popcount((unsigned)(m) & ((wemu::lane() < 32) ? 0u : ((wemu::lane() == 32) ? 0u : ((1u << (wemu::lane() - 32)) - 1u)))) + (a))
#define __builtin_amdgcn_fence(...) ((void)0)
#define __builtin_amdgcn_wave_barrier() ((void)wemu::exchange_at(0, WEMU_SITE))
#define __builtin_amdgcn_s_memrealtime() 0ull
#define __builtin_amdgcn_s_sleep(n) ((void)0)
// the fast reciprocals: rcp_fast_f32 equals the IEEE quotient on rcp_fast_ok's range
// (tests/native/rcpf_check.hip, all 2^32 floats on the GPU), and div3_rcp's Newton steps
// give the correctly rounded quotient from any estimate this close (tpt_devmath.h)
#define __builtin_amdgcn_rcpf(x) (1.0f / (x))
#define __builtin_amdgcn_rcp(x) (1.0 / (x))
static inline int __popcll(unsigned long long m) { return __builtin_popcountll(m); }
static inline float __int_as_float(int i) { float f; std::memcpy(&f, &i, 4); return f; }
static inline int __float_as_int(float f) { int i; std::memcpy(&i, &f, 4); return i; }
static inline unsigned __float_as_uint(float f) { unsigned i; std::memcpy(&i, &f, 4); return i; }
static inline float __uint_as_float(unsigned i) { float f; std::memcpy(&f, &i, 4); return f; }
static inline long long __double_as_longlong(double d) { long long i; std::memcpy(&i, &d, 8); return i; }
static inline double __longlong_as_double(long long i) { double d; std::memcpy(&d, &i, 8); return d; }
static inline int __double2loint(double d) { return (int)(uint32_t)__double_as_longlong(d); }
static inline int __double2hiint(double d) { return (int)(uint32_t)((unsigned long long)__double_as_longlong(d) >> 32); }
static inline double __hiloint2double(int hi, int lo) {
    return __longlong_as_double((long long)((unsigned long long)(uint32_t)hi << 32 | (uint32_t)lo));
}
template <class T, class U>
static inline T atomicAdd(T* p, U v) { T o = *p; *p = o + (T)v; return o; }
template <class T, class U>
static inline T atomicOr(T* p, U v) { T o = *p; *p = o | (T)v; return o; }
// tpt_devmath.h defines rcp_fast_f32 for HIP builds only; on the host the IEEE quotient,
// which it equals wherever make_ray uses it (rcp_fast_ok)
namespace tpt {
inline float rcp_fast_f32(float x) { return 1.0f / x; }
}  // namespace tpt
