// tpt_capi.hip -- gfx950 kernels of the integration loop + the C ABI (include/tpt.h).
//
// Replay contract: ResetRandom(i+1) once per pixel and ONE XorShift stream through
// all spp samples (Renderer.cpp:42-52).  BDPT's draws per sample depend on the
// geometry, so a BDPT pixel stream is one lane with a serial spp loop (784x784 =
// 9,604 wave64s).  PT's draws per sample do not, so PT spreads a pixel's samples
// over Q lanes (see tpt_pt_kernel).
#include <hip/hip_runtime.h>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/tpt.h"
#include "tpt_bdpt.h"
#include "tpt_device.h"
#include "tpt_genseq.h"
#include "tpt_scene_build.h"

using namespace tpt;

// ------------------------------------------------------------------ kernels --
extern __shared__ __align__(16) unsigned char tpt_smem[];

// Workgroup prologue: LDS = [tnodes][tris][mats][leaves][groups][ftris].  With kLds
// the scene's node and triangle arrays are copied into LDS (16 B per lane per step)
// and the kernel's DScene is pointed at them, so every traversal fetch is a ds_read
// instead of a dependent L1/L2 load.  Returns the first LDS byte after the scene.
// kSc: 0 no LDS (tree walks only), 1 LDS + a flat list of primitives only, 2 LDS + a
// flat list with treelets or walk groups.  s.big is set to the constant kSc == 2 so
// the compiler drops the large-scene branches from the small-scene kernels.
template <int kSc>
TPT_D unsigned char* stage_scene(DScene& s) {
    s.big = kSc == 2;
    if (kSc == 0) return tpt_smem;
    unsigned char* base = tpt_smem;
    const bool full = s.lds_full != 0;  // else only the flat-query arrays (+ ftris at the end)
    const int nb = full ? s.nnodes * (int)sizeof(DNode) : 0, tb = full ? s.ntri * (int)sizeof(DTri) : 0,
              mb = s.nmats * (int)sizeof(DMat);
    const uint4* gn = reinterpret_cast<const uint4*>(s.tnodes);
    const uint4* gt = reinterpret_cast<const uint4*>(s.tris);
    uint4* ln = reinterpret_cast<uint4*>(base);
    uint4* lt = reinterpret_cast<uint4*>(base + nb);
    for (int i = threadIdx.x; i < nb / 16; i += kBlock) ln[i] = gn[i];
    for (int i = threadIdx.x; i < tb / 16; i += kBlock) lt[i] = gt[i];
    const uint4* gm = reinterpret_cast<const uint4*>(s.mats);
    uint4* lm = reinterpret_cast<uint4*>(base + nb + tb);
    for (int i = threadIdx.x; i < (mb + 15) / 16; i += kBlock) lm[i] = gm[i];  // 72-B records: round up
    const int lo = nb + tb + ((mb + 15) & ~15), lb = s.nleaf * (int)sizeof(DNode);
    const uint4* gl = reinterpret_cast<const uint4*>(s.leaves);
    uint4* ll = reinterpret_cast<uint4*>(base + lo);
    for (int i = threadIdx.x; i < lb / 16; i += kBlock) ll[i] = gl[i];
    const int go = lo + lb, gb = s.ngroup * (int)sizeof(DNode);
    const uint4* gg = reinterpret_cast<const uint4*>(s.groups);
    uint4* lg = reinterpret_cast<uint4*>(base + go);
    for (int i = threadIdx.x; i < gb / 16; i += kBlock) lg[i] = gg[i];
    const int fo = go + gb, fb = full ? 0 : s.nleaf * (int)sizeof(DTri);
    const uint4* gf = reinterpret_cast<const uint4*>(s.ftris);
    uint4* lf = reinterpret_cast<uint4*>(base + fo);
    for (int i = threadIdx.x; i < fb / 16; i += kBlock) lf[i] = gf[i];
    __syncthreads();
    s.leaves = reinterpret_cast<const DNode*>(base + lo);
    s.groups = reinterpret_cast<const DNode*>(base + go);
    s.mats = reinterpret_cast<const DMat*>(base + nb + tb);
    if (full) {
        s.tnodes = reinterpret_cast<const DNode*>(base);  // the binary `nodes` stay in L1/L2 (light sampling)
        s.tris = reinterpret_cast<const DTri*>(base + nb);
        s.ftris = s.tris;
    } else {
        s.ftris = reinterpret_cast<const DTri*>(base + fo);
    }
    return base + s.lds_bytes;
}

#ifndef TPT_PT_JUMP
#define TPT_PT_JUMP 1  // jump tables for the PT stream skip (see build_jump)
#endif
#ifndef TPT_PT_MINWAVES
#define TPT_PT_MINWAVES 5  // waves per SIMD the PT kernel's register budget must allow (measured: 4 / 5 / 6 = 52.9 / 50.8 / 57.1 ms; 5 spills 112 B/lane and still wins)
#endif

// PT (Renderer.cpp:38-52 with PathTrace), replay-exact, Q lanes per pixel.
//
// PathTrace at HEAD draws, per sample: 2 (GGX half vector) + 1 coin (Dieletric,
// Transparent) + 2 more iff a Dieletric coin >= 0.5 (cosine sample) + 3 per mesh
// emitter / 2 per sphere emitter (light sampling) -- a count that depends only on
// the first-hit material and the coin value, never on geometry (Material.cpp:150-214,
// PathTracer.cpp:76-86, BVH.cpp:156, Triangle.hpp:32).  So the XorShift state at the
// start of sample k of a pixel is reached by stepping the stream without tracing.
// Lane q of the Q lanes that share a pixel takes samples q, q+Q, q+2Q, ... and skips
// the Q-1 samples in between (~45 VALU ops per skipped sample vs ~4,800 per traced
// one); after every round the Q radiances are folded into the pixel in sample order,
// `fb[i] += (1.0f/spp) * L` exactly as Renderer.cpp:49-51.  Q = 1 is one lane per
// pixel stream; Q > 1 multiplies the parallelism (multi-GPU shards, small frames).
// The first hit is identical for every sample (no jitter) and is hoisted.
TPT_D uint32_t skip_samples(uint32_t st, int type, int light_draws, int n) {
    for (int j = 0; j < n; ++j) {
        xorshift32(st);
        xorshift32(st);
        if (type == TPT_DIELETRIC) {
            if (xorshift32(st) >= kCoinHalf) { xorshift32(st); xorshift32(st); }  // rng_float(st) >= 0.5f
        } else if (type == TPT_TRANSPARENT) {
            xorshift32(st);
        }
        for (int d = 0; d < light_draws; ++d) xorshift32(st);
    }
    return st;
}

// Jump tables for the stream skip of a Dieletric or Transparent camera hit.  XorShift32
// is linear over GF(2)^32, so n steps map x to XOR_k T_n[k][byte k of x] with
// T_n[k][b] = the state n steps from b << 8k.  A skipped Dieletric sample draws 3 + L
// numbers, 2 more when its coin (the 3rd) is >= 0.5 (skip_samples), so from one
// sample's coin state the next sample's coin state is L + 3 or L + 5 steps away: one
// table jump per skipped sample instead of 5-7 XorShift steps (a Transparent sample
// always draws 3 + L).  Word [k][b][far] of the table (8 KB of LDS): far = 0 for
// L + 3 steps, 1 for L + 5.
constexpr int kJumpWords = 4 * 256 * 2;
constexpr size_t kLdsGranule = 1280;  // LDS allocation unit (measured, see launch())
TPT_D void build_jump(uint32_t* jt, int light_draws) {
    for (int e = threadIdx.x; e < 4 * 256; e += kBlock) {
        uint32_t x = (uint32_t)(e & 255) << (8 * (e >> 8));
        for (int i = 0; i < light_draws + 3; ++i) xorshift32(x);
        jt[2 * e] = x;
        xorshift32(x);
        xorshift32(x);
        jt[2 * e + 1] = x;
    }
}
TPT_D uint32_t jump(const uint32_t* jt, uint32_t x, bool coin) {
    const uint32_t far = coin && x >= kCoinHalf ? 1u : 0u;  // a Dieletric coin: rng_float(x) >= 0.5f
    return jt[(x & 255u) << 1 | far] ^ jt[512 + ((x >> 8 & 255u) << 1 | far)] ^
           jt[1024 + ((x >> 16 & 255u) << 1 | far)] ^ jt[1536 + ((x >> 24) << 1 | far)];
}
// skip_samples through the jump table, n >= 1 samples, for a Dieletric hit (the chain
// runs over the skipped samples' coin states) or a Transparent one (3 + L draws per
// sample, always: the chain runs over sample starts with far = 0).
TPT_D uint32_t skip_jump(uint32_t st, const uint32_t* jt, int light_draws, int n, bool diel) {
    if (diel) {
        xorshift32(st);
        xorshift32(st);
        xorshift32(st);  // the first skipped sample's coin state
    }
    for (int j = 1; j < n; ++j) st = jump(jt, st, diel);
    if (!diel) return jump(jt, st, false);
    if (st >= kCoinHalf) { xorshift32(st); xorshift32(st); }
    for (int d = 0; d < light_draws; ++d) xorshift32(st);
    return st;
}

#ifndef TPT_PT_LANES
#define TPT_PT_LANES 8  // Q lanes per PT pixel stream (1, 2, 4, 8 or 16; 8 measured best on one MI355X)
#endif
constexpr int kQ = TPT_PT_LANES;
static_assert(kQ == 1 || kQ == 2 || kQ == 4 || kQ == 8 || kQ == 16, "Q must be a power of two dividing the wave");
#ifndef TPT_PT_SMALL_PIXELS
// PT shards of at most this many pixel streams run 16 lanes per stream instead of
// kQ (same-box shard model, Standard 1024 spp: 1/2, 1/4, 1/8 of the frame 24.3 /
// 13.5 / 7.6 ms with 8 lanes, 23.7 / 12.5 / 6.9 ms with 16; the whole frame 45.3 vs
// 45.8 ms).
#define TPT_PT_SMALL_PIXELS 400000  // 32 lanes at 1/8 of the frame: 0.77 of linear vs 0.82 with 16
#endif
#ifndef TPT_PT_TAIL_WAVES
#define TPT_PT_TAIL_WAVES 1  // pixel streams of the grid's 64-lane tail tier, in resident waves (round 4:
                             // 1 / 2 / 3 / 4 -> 1/8 shard 6.638 / 6.695 / 6.846 / 6.936 ms, whole frame
                             // unchanged)
#endif

#ifndef TPT_PT_CONE
#define TPT_PT_CONE 1  // PT's shadow queries skip the leaves outside the wave's shadow cone (pt_cone_mask)
#endif
#ifndef TPT_PT_DPP
#define TPT_PT_DPP 1
#endif
// acc += L of lane (this + jj) for jj = J, J + 1, ... < n (n <= Q <= 16), in that order.
template <int J, int Q>
TPT_D void fold_dpp(V3& acc, V3 L, int n) {
    if constexpr (J < Q && J < 16) {
        if (J < n) {
            if (J == 0) {
                acc = acc + L;
            } else {
                constexpr int ctrl = 0x100 + J;  // DPP row_shl:J
                acc.x = acc.x + __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, L.x), ctrl, 0xf, 0xf, false));
                acc.y = acc.y + __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, L.y), ctrl, 0xf, 0xf, false));
                acc.z = acc.z + __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, L.z), ctrl, 0xf, 0xf, false));
            }
            fold_dpp<J + 1, Q>(acc, L, n);
        }
    }
}

#ifndef TPT_PT_WAVETIME
#define TPT_PT_WAVETIME 0  // diagnostics only: per-wave start / end times of the PT kernel
#endif
#if TPT_PT_WAVETIME
constexpr int kWaveTimeMax = 1 << 17;
TPT_TU_STATIC __device__ unsigned long long tpt_wavetime[3 * kWaveTimeMax];  // start, end, hw id per wave
#endif

// kSeeded: TPT_FLAG_SAMPLE_SEED -- each sample seeds its own stream (sample_seed), so
// no lane steps past the other lanes' samples.
// One tier of the PT grid: pixel ordinals [k0, k1) of the shard / list with kQP lanes
// per pixel stream, `blk` the workgroup's index within the tier.
template <int kSc, bool kSeeded, int kQP>
TPT_D void pt_tier(const DScene& s, unsigned char* lds_free, const uint32_t* jt, int spp, int64_t begin,
                   int64_t stride, int64_t k0, int64_t k1, int64_t blk, const int64_t* __restrict__ list,
                   float* __restrict__ out, int use_jump) {
    V3 acc = v3s(0.0f);
    {
        const int64_t gl = blk * kBlock + threadIdx.x;
        const int64_t k = k0 + gl / kQP;  // pixel ordinal in the shard / list
        const int q = (int)(gl % kQP);  // this lane's sample phase
        const bool on = k < k1;
        const int64_t i = on ? (list ? list[k] : begin + k * stride) : 0;
        const int px = (int)(i % s.width), py = (int)(i / s.width);
        const V3 dir = pixel_ray(px, py, s.width, s.height, s.scale);
        const Ray r = make_ray(v3(s.eye[0], s.eye[1], s.eye[2]), dir);
        PTV v = scene_intersect(s, r, TPT_CULL_BACK);
        // the wave's shadow-cone mask (pt_cone_mask): the OR of its pixels' masks, with
        // every lane of the wave here; wave-uniform (SGPRs) across the sample loop
        uint64_t cone = ~0ull;
        if (TPT_PT_CONE && (s.flat & (kFlatShadow | kFlatNoCone)) == kFlatShadow && s.nleaf <= 64 && s.n_emitters > 0) {
            const uint64_t cm = on && v.type != T_BG ? pt_cone_mask(s, v.x) : 0ull;
            uint32_t lo = (uint32_t)cm, hi = (uint32_t)(cm >> 32);
            for (int o = 1; o < 64; o <<= 1) {
                lo |= (uint32_t)__shfl_xor((int)lo, o);
                hi |= (uint32_t)__shfl_xor((int)hi, o);
            }
            cone = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)lo) |
                   (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)hi) << 32;
        }
        if (on && v.type != T_BG) {
            const int mi = prim_mat(s, v.prim);
            const Mat m = load_mat(s, mi);
            PixPark px;
            px.base = reinterpret_cast<float*>(lds_free);
            px.park(v.x, v.N, -dir, mi, m);
            const float inv = 1.0f / spp;
            uint32_t rs = (uint32_t)((int)i + 1);  // ResetRandom(i + 1), Renderer.cpp:42
            if (!kSeeded) rs = skip_samples(rs, m.type, s.light_draws, q);
            // Only acc, rs and the loop counter stay live across the sample loop: the
            // lane's phase, the material type (parked) and the output row are
            // recomputed where they are used, so nothing spills around the loop.
            for (int j0 = 0; j0 < spp; j0 += kQP) {
                unsigned ln = threadIdx.x;  // opaque: the lane's phase and shuffle base are
                asm volatile("" : "+v"(ln));  // recomputed per round, not hoisted and spilled
                const int qq = (int)(ln & (kQP - 1));  // == q: blocks hold whole pixels
                V3 L = v3s(0.0f);
                if (j0 + qq < spp) {
                    if (kSeeded) {
                        const int64_t kk = k0 + (blk * kBlock + ln) / kQP;
                        rs = sample_seed(list ? list[kk] : begin + kk * stride, j0 + qq);
                    }
                    L = mul(pt_sample(s, px, rs, cone), inv);
                    if (kQP > 1 && !kSeeded) {
                        const int ty = px.type(s);
                        rs = kQP > 2 && use_jump && ty != TPT_METAL
                                 ? skip_jump(rs, jt, s.light_draws, kQP - 1, ty == TPT_DIELETRIC)
                                 : skip_samples(rs, ty, s.light_draws, kQP - 1);
                    }
                }
                if (kQP == 1) {
                    acc = acc + L;
                } else if (kQP >= 8 && TPT_PT_DPP) {
                    // The fold through DPP row shifts: lane i reads L of lane i + jj of its
                    // 16-lane row, so the first lane of each pixel (i = 0 mod kQP) adds its
                    // pixel's samples in sample order (other lanes' acc is never read);
                    // past 16 lanes the other rows' samples follow through shuffles.
                    const int n = spp - j0 < kQP ? spp - j0 : kQP;
                    fold_dpp<0, kQP>(acc, L, n < 16 ? n : 16);
                    if (kQP > 16) {
                        const int l0 = lane_id();
                        for (int jj = 16; jj < n; ++jj) {
                            acc.x = acc.x + __shfl(L.x, l0 + jj);
                            acc.y = acc.y + __shfl(L.y, l0 + jj);
                            acc.z = acc.z + __shfl(L.z, l0 + jj);
                        }
                    }
                } else {
                    const int base = (int)(ln & 63) - qq;  // first lane of this pixel
                    const int n = spp - j0 < kQP ? spp - j0 : kQP;
                    for (int jj = 0; jj < n; ++jj) {
                        acc.x = acc.x + __shfl(L.x, base + jj);
                        acc.y = acc.y + __shfl(L.y, base + jj);
                        acc.z = acc.z + __shfl(L.z, base + jj);
                    }
                }
            }
        }
    }
    unsigned tid = threadIdx.x;
    asm volatile("" : "+v"(tid));  // recomputed, not kept alive across the loop
    const int64_t gl = blk * kBlock + tid;
    const int64_t k = k0 + gl / kQP;
    if (k < k1 && gl % kQP == 0) {
        const int64_t row = list ? k : begin + k * stride;
        out[3 * row + 0] = acc.x;
        out[3 * row + 1] = acc.y;
        out[3 * row + 2] = acc.z;
    }
}

// The PT grid in two tiers: pixels [0, k_tail) with kQP lanes per pixel stream (8 for a
// frame; 16 for shards of a frame -- half as long waves, so the tail of a small grid is
// half as long; launch()), then pixels [k_tail, count) with kQT = 64 lanes each (one
// wave per pixel stream, a quarter of a 16-lane wave's time).  Workgroups are
// dispatched in order, so the short waves of the last tier are what is left to run
// while the long ones drain: they fill the grid's tail.  A pixel's result does not
// depend on its tier (the same samples, folded in sample order).
#ifndef TPT_PT_KQT
#define TPT_PT_KQT 64  // lanes per pixel stream of the tail tier
#endif
constexpr int kQT = TPT_PT_KQT;
template <int kSc, bool kSeeded, int kQP>
__global__ __launch_bounds__(kBlock, TPT_PT_MINWAVES) void tpt_pt_kernel(DScene s, int spp, int64_t begin,
                                                                        int64_t stride, int64_t count,
                                                                        const int64_t* __restrict__ list,
                                                                        float* __restrict__ out, int use_jump,
                                                                        int64_t k_tail, int64_t b_tail) {
#if TPT_PT_WAVETIME
    const unsigned long long wt0 = __builtin_amdgcn_s_memrealtime();
#endif
    unsigned char* lds_free = stage_scene<kSc>(s);
    uint32_t* jt = reinterpret_cast<uint32_t*>(lds_free + kPixSlots * kBlock * sizeof(float));
    if (!kSeeded && kQP > 2 && use_jump) {
        build_jump(jt, s.light_draws);
        __syncthreads();
    }
    s.qs = nullptr;  // coherent rays: the per-leaf flat loops (the compacted form's code folds away)
    s.ws = nullptr;  // and the binary walks for walk groups (no LDS left for stacks at 5 blocks/CU)
    if ((int64_t)blockIdx.x < b_tail)
        pt_tier<kSc, kSeeded, kQP>(s, lds_free, jt, spp, begin, stride, 0, k_tail, blockIdx.x, list, out, use_jump);
    else
        pt_tier<kSc, kSeeded, kQT>(s, lds_free, jt, spp, begin, stride, k_tail, count, blockIdx.x - b_tail, list, out,
                                   use_jump);
#if TPT_PT_WAVETIME
    const int wv = (int)(blockIdx.x * (kBlock / 64) + threadIdx.x / 64);
    if (lane_id() == 0 && wv < kWaveTimeMax) {
        tpt_wavetime[3 * wv] = wt0;
        tpt_wavetime[3 * wv + 1] = __builtin_amdgcn_s_memrealtime();
        // HW_REG_HW_ID1 (23) in the low word, HW_REG_XCC_ID (20, 4 bits) above it
        tpt_wavetime[3 * wv + 2] = (unsigned long long)(unsigned)__builtin_amdgcn_s_getreg(23 | (31 << 11)) |
                                   (unsigned long long)(unsigned)__builtin_amdgcn_s_getreg(20 | (3 << 11)) << 32;
    }
#endif
}

#ifndef TPT_PTI_MINWAVES
#define TPT_PTI_MINWAVES 4
#endif
// Generous bound on one path's bounces so that every lane provably leaves its loop.
// A path continues past bounce 5 only on a draw < 0.8 (PathTracer.cpp:122-123); the
// longest run of such draws in XorShift32's whole period is ~100, so the bound is
// never reached and results are the reference's.
constexpr int kPtiMaxBounces = 1 << 16;

// TPT_MODE_PT_INDIRECT (Renderer.cpp:38-52 with PathTrace minus the :109 `break`).
// Draws per sample depend on the geometry the path meets, so a pixel's stream is
// one lane.  The lane runs its spp samples back to back as ONE loop of bounces: a
// sample that ends (miss, alpha == 0, Russian roulette) is folded into the pixel and
// the next sample starts in the same iteration, so lanes of a wave never wait for
// one another's long paths until the pixel's last sample (per-lane regeneration,
// in registers).
//
// kSeeded (TPT_FLAG_SAMPLE_SEED): samples are independent, so kQ lanes share a pixel:
// lane q runs samples q, q + kQ, ... back to back (each from sample_seed), sums its
// own (1/spp) * L, and the kQ partial sums are added in lane order at the end.
template <int kSc, bool kSeeded>
__global__ __launch_bounds__(kBlock, TPT_PTI_MINWAVES) void tpt_pti_kernel(DScene s, int spp, int64_t begin,
                                                                          int64_t stride, int64_t count,
                                                                          const int64_t* __restrict__ list,
                                                                          float* __restrict__ out,
                                                                          unsigned long long* __restrict__ bounces) {
    stage_scene<kSc>(s);
#ifndef TPT_PTI_COMPACT
#define TPT_PTI_COMPACT 1  // same-box A/B, Standard 1024 spp: 737 -> 708 ms
#endif
#if TPT_PTI_COMPACT
    __shared__ QScratch qsm[kBlock / 64];  // incoherent bounce rays: compacted flat queries
    s.qs = qsm;
#else
    s.qs = nullptr;
#endif
    s.ws = nullptr;
    if constexpr (kSc == 2) {
        __shared__ uint16_t wst[kWalkStack * kBlock];
        s.ws = wst;
    }
    constexpr int kL = kSeeded ? kQ : 1;  // lanes per pixel
    const int64_t gl = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t k = gl / kL;
    const int q = (int)(gl % kL);
    const bool on = k < count;
    const int64_t i = on ? (list ? list[k] : begin + k * stride) : 0;
    const V3 eye = v3(s.eye[0], s.eye[1], s.eye[2]);
    const V3 dir = pixel_ray((int)(i % s.width), (int)(i / s.width), s.width, s.height, s.scale);
    const float inv = 1.0f / spp;
    uint32_t rs = kSeeded ? sample_seed(i, q) : (uint32_t)((int)i + 1);  // ResetRandom(i + 1), Renderer.cpp:42
    V3 acc = v3s(0.0f);
    PtiPath p;
    p.r = make_ray(eye, dir);
    p.alpha = v3s(1.0f);
    p.res = v3s(0.0f);
    p.nb = 0;
    p.flip = false;
    unsigned long long nbt = 0;
    for (int j = on ? q : spp; j < spp;) {
        bool live = !(p.alpha.x == 0.0f && p.alpha.y == 0.0f && p.alpha.z == 0.0f) && p.nb < kPtiMaxBounces;  // :54-55
        if (live) {
            const PTV v = scene_intersect(s, p.r, p.flip ? TPT_CULL_FRONT : TPT_CULL_BACK);  // :56
            live = v.type != T_BG && pti_step(s, v, p, rs);                                   // :58-131
        }
        if (!live) {
            acc = acc + mul(p.res, inv);  // Renderer.cpp:49 `fb[i] += (1.0f / spp) * L`
            nbt += (unsigned long long)p.nb;
            j += kL;
            if (kSeeded && j < spp) rs = sample_seed(i, j);
            p.r = make_ray(eye, dir);
            p.alpha = v3s(1.0f);
            p.res = v3s(0.0f);
            p.nb = 0;
            p.flip = false;
        }
    }
    if (kSeeded) {  // the pixel's kL partial sums, in lane order (blocks hold whole pixels)
        const int base = lane_id() - q;
        V3 t = v3s(0.0f);
        for (int jj = 0; jj < kL; ++jj) {
            t.x = t.x + __shfl(acc.x, base + jj);
            t.y = t.y + __shfl(acc.y, base + jj);
            t.z = t.z + __shfl(acc.z, base + jj);
        }
        acc = t;
    }
    if (on && q == 0) {
        const int64_t row = list ? k : i;
        out[3 * row + 0] = acc.x;
        out[3 * row + 1] = acc.y;
        out[3 * row + 2] = acc.z;
    }
    for (int o = 32; o >= 1; o >>= 1) nbt += __shfl_xor(nbt, o);
    if (lane_id() == 0) atomicAdd(bounces, nbt);
}

// ---- wavefront BDPT kernels (see tpt_bdpt.h, "wavefront") --------------------
#ifndef TPT_GEN_MINWAVES
#define TPT_GEN_MINWAVES 4  // waves per SIMD (measured: 4 beats 3 and 5)
#endif
#ifndef TPT_CONN_MINWAVES
#define TPT_CONN_MINWAVES 4  // waves per SIMD (measured: 4 beats 2, 3 and 5)
#endif

#ifndef TPT_GEN_STATS
#define TPT_GEN_STATS 0  // diagnostics only: per-wave loop statistics of the gen kernels
#endif
#if TPT_GEN_STATS
constexpr int kGenStatMax = 1 << 16;
// per wave: kernel (0: gen) | launch ordinal << 8, step iterations, lane-steps, idle
// iterations, real-time ticks (100 MHz)
TPT_TU_STATIC __device__ unsigned long long tpt_genstats[5 * kGenStatMax];
TPT_TU_STATIC __device__ unsigned tpt_genstat_n;
struct GenStat {
    unsigned long long it = 0, ls = 0, idle = 0, t0 = 0;
    TPT_D void begin() { t0 = __builtin_amdgcn_s_memrealtime(); }
    TPT_D void step(unsigned long long run) {
        if (run) { ++it; ls += (unsigned long long)__popcll(run); } else { ++idle; }
    }
    TPT_D void end(int kind, int batch) {
        if (lane_id() != 0) return;
        const unsigned slot = atomicAdd(&tpt_genstat_n, 1u);
        if (slot >= (unsigned)kGenStatMax) return;
        unsigned long long* o = tpt_genstats + 5 * (size_t)slot;
        o[0] = (unsigned long long)kind | ((unsigned long long)batch << 8);
        o[1] = it; o[2] = ls; o[3] = idle; o[4] = __builtin_amdgcn_s_memrealtime() - t0;
    }
};
#endif
#ifndef TPT_WF_BUFS
#define TPT_WF_BUFS 3  // BDPT wavefront buffers in flight.  Same-box shard model, 2 / 3 / 4:
// 1/8-frame shards Standard BDPT 0.814 / 0.849 / 0.849 of linear, bunny 0.859 / 0.900 /
// 0.898; whole frames unchanged (bunny 256 spp 1112 / 1089 / 1091 ms)
#endif
constexpr int kWfBufs = TPT_WF_BUFS;

// Path generation, persistent: each lane runs a pixel's nb samples (the wavefront's
// iterations) as a sequence of steps (start, camera-path vertex..., light start,
// light-path vertex..., then the next sample of the same pixel) and takes the next
// pixel from its shard's queue as soon as it is done, so a wave stays full although
// path lengths differ per lane (a lane-per-pixel grid ran at 44 % lane efficiency).
// Per-pixel order -- and so every RNG draw -- is unchanged.  Queues: one counter per
// shard of pixels, shard = blockIdx.x % 8 (blocks b and b + 8 are dealt to the same
// XCD; speed only).  `batch`: this wavefront's ordinal in the chunk (0: the streams
// start at ResetRandom(i + 1); >= 2: this buffer already holds the camera vertices).
//
// Wavefront f's gen runs beside wavefront f - 1's (another stream): a lane that claims
// pixel k waits, inside the persistent loop, until gen(f - 1) has published k's stream
// state (WfState::rngseq), so gen(f)'s tail of long paths no longer idles the chip
// until gen(f + 1) may start.  gen(f - 1) never waits on gen(f), so it always drains.
// A watchdog (kStallTicks of the 100 MHz real-time counter) ends a wait that cannot
// finish -- never expected -- by flagging w.stall and giving the pixel no strategies,
// so a broken pipeline is reported as an error instead of hanging the GPU.
#ifndef TPT_WATCHDOG
#define TPT_WATCHDOG 1
#endif
#ifndef TPT_STALL_TICKS
#define TPT_STALL_TICKS 2000000000u  // 20 s at 100 MHz (32-bit differences wrap at 42 s)
#endif
constexpr uint32_t kStallTicks = TPT_STALL_TICKS;
#ifndef TPT_DIAG_HOOKS
// 1: diagnostics build (libtpt_diag.so, tests only): each BDPT render reads
// TPT_DIAG_DROP_PUBLISH (a pixel ordinal whose stream state gen(1) does not publish, so
// gen(2) waits on it until the watchdog fires) and TPT_DIAG_STALL_TICKS (the watchdog's
// limit) from the environment.  The production library has neither.
#define TPT_DIAG_HOOKS 0
#endif
// The base pointer passes through an opaque SGPR copy at each use, so the compiler does
// not keep a VGPR copy of it alive (and spilled) across gen's persistent loop.
TPT_D unsigned long long load_rngseq(const unsigned long long* base, int k) {
    asm volatile("" : "+s"(base));
    return __hip_atomic_load(base + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
TPT_D void store_rngseq(unsigned long long* base, int k, unsigned long long v) {
    asm volatile("" : "+s"(base));
    __hip_atomic_store(base + k, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
#ifndef TPT_GEN_PRIO
#define TPT_GEN_PRIO 0  // gen waves' issue priority (s_setprio) over connect's
#endif
template <int kSc>
__global__ __launch_bounds__(kBlock, TPT_GEN_MINWAVES) void tpt_bdpt_gen_kernel(DScene s, WfState w, int batch,
                                                                               unsigned* __restrict__ queue) {
    if (TPT_GEN_PRIO) __builtin_amdgcn_s_setprio(TPT_GEN_PRIO);
    stage_scene<kSc>(s);
    __shared__ QScratch qsm[kBlock / 64];  // compacted flat queries (tpt_device.h)
    s.qs = qsm;
    s.ws = nullptr;
    if constexpr (kSc == 2) {  // walk groups: per-lane stacks of the 4-wide walks
        __shared__ uint16_t wst[kWalkStack * kBlock];
        s.ws = wst;
    }
    // deferred walks (gen_step_t): scenes with exactly one walk group
    constexpr bool kDef = kSc == 2 && TPT_GEN_DEFER;
    GenDefer dl{nullptr};
    int gw = -1;
    if constexpr (kDef) {
        __shared__ float gdl[kGenDeferSlots * kBlock];
        dl.base = gdl;
        int nw = 0;
        for (int gi = 0; gi < s.ngroup; ++gi)
            if (s.groups[gi].b < 0) {
                gw = gi;
                ++nw;
            }
        if (nw != 1) gw = -1;
    }
    int pend = 0;  // iterations this lane's step has been parked (0: none)
    const int shard = blockIdx.x & 7;
    // pixel ordinals and items are < kWfChunk = 2^22: 32-bit indices in the loop
    const int nn = (int)w.n;
    const int k_lo = (int)(w.n * shard / 8), k_hi = (int)(w.n * (shard + 1) / 8);
    unsigned* q = queue + shard * 16;  // 64 B apart
    int k = -1;       // this lane's pixel ordinal (-1: none)
    int b = 0;        // its current sample in the wavefront (item b * n + k)
    int phase = 0;    // 0: camera path, 1: light start pending, 2: light path
    int i = 0, cn = 0;
    uint32_t rs = 0;
    unsigned long long nbounce = 0;
    bool drained = false;
    BVert prev, cur;
    // The camera vertices v0 / v1 of item (b, k): GenerateCameraPath's first two
    // vertices (BDPT.cpp:41-59) do not depend on the sample (no jitter).  Items (b, k)
    // with b < w.cam_nb were written by an earlier wavefront of the chunk in this buffer
    // and their slots 0/1 still hold them (their q1/q8 may be stale; those of vertices
    // cn-2, cn-1 are never read); otherwise sample 0 traces them (or finds them in
    // item (0, k)) and the later samples copy them from item (0, k).
    auto start_sample = [&]() {
        const int it = b * nn + k;
        BVert c0, c1;
        const bool cached = b < w.cam_nb;
        if (cached || b > 0) {
            GlobPaths P;
            P.rec = rec_at(w.rec, cached ? it : k, 0);
            c0 = P.cam(0);
            c1 = P.cam(1);
        } else {
            camera_vertices(s, wf_pixel(w, k), c0, c1);
        }
        if (!cached) {
            rec_store<kDef && TPT_GEN_REC_Z>(w, 0, it, c0);
            rec_store<kDef && TPT_GEN_REC_Z>(w, 1, it, c1);
        }
        prev = c0;
        cur = c1;
        i = 1;
        phase = 0;
    };
#if TPT_GEN_STATS
    GenStat gst;
    gst.begin();
#endif
    bool ready = false;                 // k's stream state is in rs (its previous wavefront is done)
    bool fresh = false;                 // sample b of k starts at the top of the next step
    uint32_t wait_t0 = 0;               // when this lane started waiting for k (low 32 bits | 1; 0: not yet)
    for (;;) {
        const bool need = k < 0 && !drained;
        const unsigned long long nm = __ballot(need);
        if (nm != 0) {
            const int leader = __builtin_ctzll(nm);
            unsigned base = 0;
            if (lane_id() == leader) {
                unsigned* qa = q;  // opaque: used from SGPRs here, not held in VGPRs across the loop
                asm volatile("" : "+s"(qa));
                base = atomicAdd(qa, (unsigned)__popcll(nm));
            }
            base = __shfl(base, leader);
            if (need) {
                const int kk = k_lo + (int)base + __popcll(nm & ((1ull << lane_id()) - 1));
                if (kk < k_hi) {
                    k = kk;
                    b = 0;
                    ready = false;
                    wait_t0 = 0;
                } else {
                    drained = true;
                }
            }
        }
        if (k >= 0 && !ready) {
            if (batch == 0) {
                rs = (uint32_t)((int)wf_pixel(w, k) + 1);  // ResetRandom(i + 1), Renderer.cpp:42
                float z = 0.0f;  // opaque: the zeros are made here, not held (spilled) across the loop
                asm volatile("" : "+v"(z));
                w.acc[3 * k] = z; w.acc[3 * k + 1] = z; w.acc[3 * k + 2] = z;
                ready = true;
            } else {
                // one gen stream: gen(f - 1) completed before this kernel started, so a
                // plain load sees its state; two: wait for its publication
                const unsigned long long v = w.conc ? load_rngseq(w.rngseq, k) : w.rngseq[k];
                if (seq_ready(v, batch)) {
                    rs = seq_state(v);
                    ready = true;
                } else if (wait_t0 == 0) {
                    wait_t0 = (uint32_t)__builtin_amdgcn_s_memrealtime() | 1u;  // the wait starts
                } else if (TPT_WATCHDOG && (uint32_t)__builtin_amdgcn_s_memrealtime() - wait_t0 > w.stall_ticks) {
                    // watchdog: give up on k, publish it so later wavefronts do not wait
                    // too, and report it.  Its items keep older contents, which are
                    // always a complete sample's (ensure_wf zeroes the arrays when it
                    // allocates them), so the scan, scatter and connect stay in bounds.
                    store_rngseq(w.rngseq, k, seq_give_up(batch));
                    atomicOr(w.stall, 1);
                    k = -1;
                }
            }
            fresh = ready;
        }
        if (fresh) {  // one call site: camera_vertices (a closest-hit query) is inlined once
            start_sample();
            fresh = false;
        }
        if (__ballot(k >= 0) == 0) break;  // every lane idle and its shard drained
        const bool run = k >= 0 && ready;
#if TPT_GEN_STATS
        gst.step(__ballot(run));
#endif
        // The whole wave waits on gen(f - 1): back off.  (No `continue` on this uniform
        // branch: that form of the loop spilled 120 B/lane instead of 52.)
        if (__ballot(run) == 0) __builtin_amdgcn_s_sleep(8);
        if (!run) continue;
        const int it = b * nn + k;
        int ln = -1;  // >= 0: the pixel's sample is complete
#if TPT_GEN_STATS
        const unsigned long long ts0 = __builtin_amdgcn_s_memrealtime();
#endif
        const int gsr = gen_step_t<kDef>(s, w, it, phase, prev, cur, i, rs, pend, dl, gw);
#if TPT_GEN_STATS
        if (lane_id() == (unsigned)__builtin_ctzll(__ballot(true))) {
            atomicAdd(&tpt_walkstat[3], __builtin_amdgcn_s_memrealtime() - ts0);
            atomicAdd(&tpt_walkstat[4], 1ull);
        }
#endif
        if (gsr == 0) {
            if (phase == 0) {
                cn = i + 1;
                phase = 1;
            } else {
                ln = i + 1;
            }
        }
        if (ln >= 0) {
            w.cnt[it] = cn | (ln << 16);
            w.np[it] = (unsigned long long)(cn - 1) | ((unsigned long long)((cn - 1) * (ln - 1)) << 32);
            w.np2[it] = (unsigned long long)(cn - 1) | ((unsigned long long)ln << 32);
            nbounce += (unsigned long long)(cn + ln);
            if (++b < w.nb) {
                fresh = true;  // the pixel's next sample, same stream, from the next step
            } else {
                const unsigned long long v = seq_publish(batch, rs);
                if (TPT_DIAG_HOOKS && batch == 1 && k == w.drop_k) {
                    // diagnostics: k's state is never published, gen(2)'s watchdog takes over
                } else if (w.conc) {
                    store_rngseq(w.rngseq, k, v);
                } else {
                    w.rngseq[k] = v;
                }
                k = -1;
                ready = false;
            }
        }
    }
#if TPT_GEN_STATS
    gst.end(0, batch);
#endif
    atomicAdd(w.bounces, nbounce);
}


// Task runs.  A strategy's cost depends on its class: s = 0 (emission only), and
// for connections whether the light-side vertex is the light itself (s = 1: no BSDF
// there) and whether the camera-side one is the camera (t = 1: no BSDF, a splat).
// The task list holds four runs, each pixel-major in (t, s) order:
//   [s = 0][t > 1, s > 1][t > 1, s = 1][t = 1]
// so a wave's 64 strategies are (nearly always) of one class and take the same
// branches through PathWeight.  Results still land in their canonical (t, s) slots.
struct StratRange {
    int64_t b[4];        // the pixel's start in each run (absolute task index)
    int ln, np;          // light vertices, strategies
};
TPT_D StratRange strat_range(const WfState& w, int64_t k) {  // k: item
    const unsigned long long e1 = w.incl[k], c1 = w.np[k], e2 = w.incl2[k], c2 = w.np2[k];
    const unsigned long long t1 = w.incl[w.ni - 1], t2 = w.incl2[w.ni - 1];
    const int64_t totA = (int64_t)(t1 & 0xffffffffull), totE = (int64_t)(t1 >> 32), totD = (int64_t)(t2 & 0xffffffffull);
    const int64_t xA = (int64_t)(e1 & 0xffffffffull) - (int64_t)(c1 & 0xffffffffull);
    const int64_t xE = (int64_t)(e1 >> 32) - (int64_t)(c1 >> 32);
    const int64_t xD = (int64_t)(e2 & 0xffffffffull) - (int64_t)(c2 & 0xffffffffull);
    const int64_t xT = (int64_t)(e2 >> 32) - (int64_t)(c2 >> 32);
    StratRange r;
    r.b[0] = xA;
    r.b[1] = totA + xE;
    r.b[2] = totA + totE + xD;
    r.b[3] = totA + totE + totD + xT;
    r.ln = w.cnt[k] >> 16;
    r.np = (int)(c1 & 0xffffffffull) + (int)(c1 >> 32) + (int)(c2 & 0xffffffffull) + (int)(c2 >> 32);
    return r;
}
TPT_D int64_t total_tasks(const WfState& w) {
    const unsigned long long t1 = w.incl[w.ni - 1], t2 = w.incl2[w.ni - 1];
    return (int64_t)(t1 & 0xffffffffull) + (int64_t)(t1 >> 32) + (int64_t)(t2 & 0xffffffffull) + (int64_t)(t2 >> 32);
}

#if !TPT_TU_CONN2
__global__ __launch_bounds__(kBlock) void tpt_bdpt_scatter_kernel(WfState w, unsigned* __restrict__ queue) {
    const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;  // item
    if (k < 8) queue[k * 16] = 0;  // gen of the next wavefront (same stream, after this kernel) starts its shards at 0
    if (k >= w.ni) return;
    const StratRange r = strat_range(w, k);
    const int ln = r.ln, cn = w.cnt[k] & 0xffff;
    const unsigned kk = (unsigned)k;
    for (int sl = 1; sl <= ln; ++sl) w.task[r.b[3] + (sl - 1)] = kk | 1u << 22 | (unsigned)sl << 27;  // t = 1
    for (int t = 2; t <= cn; ++t) {
        const unsigned kt = kk | (unsigned)t << 22;
        w.task[r.b[0] + (t - 2)] = kt;                 // s = 0
        w.task[r.b[2] + (t - 2)] = kt | 1u << 27;      // s = 1
        const int64_t g1 = r.b[1] + (int64_t)(t - 2) * (ln - 1) - 2;
        for (int sl = 2; sl <= ln; ++sl) w.task[g1 + sl] = kt | (unsigned)sl << 27;
    }
}
#endif

// One strategy (task g) of connect: PathWeight, the result at its task index (t > 1)
// or the splat of the wave (t = 1; call with every lane of the wave).
template <int kCls = -1>
TPT_D void conn_task(const DScene& s, const WfState& w, float* __restrict__ splat, int64_t g, bool on, V3 eye) {
    V3 v = v3s(0.0f), lx = eye;
    bool sp = false;
    if (on) {
        const unsigned tk = w.task[g];
        const int64_t k = (int64_t)(tk & kTaskPixelMask);
        const int t = (int)((tk >> 22) & 31), sl = (int)(tk >> 27);
        GlobPaths P;
        P.rec = rec_at(w.rec, k, 0);
        v = vmax0(path_weight<kCls>(s, P, sl, t));
        if (t > 1) {  // the result stays in task order; fold finds it from (t, s)
            w.res[3 * g] = v.x;
            w.res[3 * g + 1] = v.y;
            w.res[3 * g + 2] = v.z;
        } else if (splat) {
            sp = true;
            lx = P.lit(sl - 1).x;
        }
    }
    // t = 1: DrawToImage of the light vertex (BDPT.cpp:303-305), whole wave
    if (kCls < 0 || kCls == 3)
        if (splat) splat_wave(s, sp, lx, eye, v, splat);
}

// Queued shadow queries (round 6, TPT_CONN_QUEUE).  A strategy's shadow query
// (BDPT.cpp:205) is needed only when its unshadowed contribution is not 0, so in a wave of
// 64 strategies only some lanes make it, and the others idle through it (for walk-group
// scenes: through the bunny walks).  Here PathWeight runs without it (path_weight<.., kDS>)
// and stores the unshadowed result at the task's index; the tasks that need the query go
// into a per-wave LDS queue, and the queries run 64 at a time, dense: a shadowed
// strategy's result is overwritten with 0 (t > 1) or its splat is dropped (t = 1; the
// splat is added only after the query, from the stored value).  Same queries on the
// same vertices, same results; splats are fp32 atomics in another order.
#ifndef TPT_CONN_QUEUE
#define TPT_CONN_QUEUE 1  // small flat scenes, wavefronts of < 8 iterations (whole frames): Standard BDPT 256 spp
                          // 423.5-425.2 -> 414.7-417.1 ms same-box; its 1/8 shard 60.3 -> 60.7 ms, so shards keep
                          // the in-place queries.  Walk-group scenes keep them too (bunny 256 spp -0.5 %, and this
                          // compiler crashed building the partitioned kernel with the queue and the AMDGPU trackers)
#endif
#ifndef TPT_CONN_QUEUE_WALK
#define TPT_CONN_QUEUE_WALK 0  // walk-group scenes: the queue behind the walker partition (OFF: bunny 256 spp
                               // 609.1-610.4 -> 610.1-614.3 ms same-box, c5 pins green)
#endif
constexpr int kShQ = 128;  // per-wave queue slots (<= 63 left over + 64 appended)
struct ShadowQueue {
    uint32_t* q;  // this wave's kShQ task indices (LDS)
    int n;        // queued (wave-uniform)
};
// PathWeight of task g without the shadow query; true when the query is needed.
TPT_D bool conn_unshadowed(const DScene& s, const WfState& w, int64_t g, bool on) {
    bool need = false;
    if (on) {
        const unsigned tk = w.task[g];
        const int64_t k = (int64_t)(tk & kTaskPixelMask);
        const int t = (int)((tk >> 22) & 31), sl = (int)(tk >> 27);
        GlobPaths P;
        P.rec = rec_at(w.rec, k, 0);
        const V3 v = vmax0(path_weight<-1, true>(s, P, sl, t, &need));
        w.res[3 * g] = v.x;
        w.res[3 * g + 1] = v.y;
        w.res[3 * g + 2] = v.z;
    }
    return need;
}
// The queries of queue entries [0, cnt) (cnt <= 64, lane i takes entry i); every lane of
// the wave calls it.
TPT_D void conn_shadow_round(const DScene& s, const WfState& w, float* __restrict__ splat, const uint32_t* q, int cnt,
                             V3 eye) {
    const int lane = (int)lane_id();
    bool want = false;
    V3 v = v3s(0.0f), lx = eye;
    if (lane < cnt) {
        const int64_t g = (int64_t)q[lane];
        const unsigned tk = w.task[g];
        const int64_t k = (int64_t)(tk & kTaskPixelMask);
        const int t = (int)((tk >> 22) & 31), sl = (int)(tk >> 27);
        GlobPaths P;
        P.rec = rec_at(w.rec, k, 0);
        const BVert cz = P.cam(t - 1), ly = P.lit(sl - 1);
        const bool sh = !TPT_DIAG_NO_CONN_SHADOW && shadow_v(s, cz, ly);
        if (t > 1) {
            if (sh) {
                w.res[3 * g] = 0.0f;
                w.res[3 * g + 1] = 0.0f;
                w.res[3 * g + 2] = 0.0f;
            }
        } else if (splat && !sh) {
            want = true;
            lx = ly.x;
            v = v3(w.res[3 * g], w.res[3 * g + 1], w.res[3 * g + 2]);
        }
    }
    if (splat) splat_wave(s, want, lx, eye, v, splat);
}
// Append this round's needing lanes (task g) and run the full rounds of 64.
TPT_D void conn_queue_push(const DScene& s, const WfState& w, float* __restrict__ splat, ShadowQueue& sq, bool need,
                           int64_t g, V3 eye) {
    const uint64_t m = __ballot(need);
    if (need) sq.q[sq.n + mbcnt64(m)] = (uint32_t)g;
    sq.n += __popcll(m);
    wave_lds_sync();
    if (sq.n >= 64) {
        conn_shadow_round(s, w, splat, sq.q, 64, eye);
        wave_lds_sync();
        const int lane = (int)lane_id();
        const uint32_t rest = lane + 64 < sq.n ? sq.q[lane + 64] : 0u;
        wave_lds_sync();
        if (lane + 64 < sq.n) sq.q[lane] = rest;
        sq.n -= 64;
        wave_lds_sync();
    }
}
TPT_D void conn_queue_flush(const DScene& s, const WfState& w, float* __restrict__ splat, ShadowQueue& sq, V3 eye) {
    if (sq.n > 0) {
        conn_shadow_round(s, w, splat, sq.q, sq.n, eye);
        sq.n = 0;
        wave_lds_sync();
    }
}

// Walker partition (round 4).  For a scene with walk groups the shadow query of a
// strategy (BDPT.cpp:205), from the camera-side vertex toward the light-side one,
// walks the mesh's tree when its ray passes the walk group's box; dealt pixel-major,
// a wave of 64 strategies almost always holds a few such lanes, and the whole wave
// waits on their walks.  So each wave takes kSortN = 64 R consecutive tasks, marks
// the ones whose ray passes the box (a cheap approximate slab test: the mark only
// decides which lanes run together), and runs them in R rounds with the unmarked
// tasks first and the marked ones last, each group in task order (a stable
// partition through ballots; the permutation sits in LDS).  Every task still writes
// its result at its own task index (fold is unchanged) and splats are fp32 atomics
// in any order, so results are unchanged.
#ifndef TPT_CONN_SORT
#define TPT_CONN_SORT 1  // 1: scenes with walk groups, 2: every scene, 0: off
#endif
#ifndef TPT_CONN_SORT_R
#define TPT_CONN_SORT_R 16  // rounds of 64 tasks per partitioned chunk (4 / 8 -> bunny 256 spp 745.7 / 735.6 ms,
                            // 1/8 shard 109.4 / 107.5 ms; at six-frame wavefronts 4 / 8 / 16 -> 740.6 / 725.3 /
                            // 718.0 ms, 1/8 shard 8 / 16 -> 109.6 / 107.8 ms)
#endif
constexpr int kSortR = TPT_CONN_SORT_R;
constexpr int kSortN = 64 * kSortR;
static_assert(kSortR >= 1 && kSortR <= 16, "chunk of 64 R tasks");
// Does task g's shadow ray (camera-side vertex toward the light-side one) pass the box
// of walk group gi?  False for s = 0 (no shadow query).
TPT_D bool conn_marked(const DScene& s, const WfState& w, int64_t g, int gi) {
    const unsigned tk = w.task[g];
    const int t = (int)((tk >> 22) & 31), sl = (int)(tk >> 27);
    if (sl == 0) return false;
    const DNode gn = s.groups[gi];
    const float4* r = rec_at(w.rec, (int64_t)(tk & kTaskPixelMask), 0);
    const float4 a = r[(t - 1) * kRecV], b = r[(kMaxLen + sl - 1) * kRecV];
    const float ix = __builtin_amdgcn_rcpf(b.x - a.x), iy = __builtin_amdgcn_rcpf(b.y - a.y),
                iz = __builtin_amdgcn_rcpf(b.z - a.z);
    const float ax = (gn.bmin[0] - a.x) * ix, cx = (gn.bmax[0] - a.x) * ix;
    const float ay = (gn.bmin[1] - a.y) * iy, cy = (gn.bmax[1] - a.y) * iy;
    const float az = (gn.bmin[2] - a.z) * iz, cz = (gn.bmax[2] - a.z) * iz;
    const float t0 = fmaxf(fmaxf(0.0f, fminf(ax, cx)), fmaxf(fminf(ay, cy), fminf(az, cz)));
    const float t1 = fminf(fmaxf(ax, cx), fminf(fmaxf(ay, cy), fmaxf(az, cz)));
    return t0 <= t1;
}

// One lane per strategy, grid-stride in wave-sized steps so that every lane of a
// wave stays in the loop until the wave is done (splat_wave needs the whole wave).
template <int kSc, bool kQueue = false>
__global__ __launch_bounds__(kBlock, TPT_CONN_MINWAVES) void tpt_bdpt_conn_kernel(DScene s, WfState w, float* __restrict__ splat) {
    stage_scene<kSc>(s);
    __shared__ QScratch qsm[kBlock / 64];
    s.qs = qsm;
    s.ws = nullptr;
    if constexpr (kSc == 2) {
        __shared__ uint16_t wst[kWalkStack * kBlock];
        s.ws = wst;
    }
    const int64_t total = total_tasks(w);
    const V3 eye = v3(s.eye[0], s.eye[1], s.eye[2]);
    constexpr bool kPart = TPT_CONN_SORT == 2 || (TPT_CONN_SORT == 1 && kSc == 2);
    if constexpr (!kPart && kQueue) {  // queued shadow queries (small flat scenes, whole frames)
        __shared__ uint32_t shq_all[kBlock / 64][kShQ];
        ShadowQueue sq{shq_all[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)], 0};
        for (int64_t g0 = (int64_t)blockIdx.x * kBlock + (threadIdx.x & ~63); g0 < total;
             g0 += (int64_t)gridDim.x * kBlock) {
            const int64_t g = g0 + lane_id();
            conn_queue_push(s, w, splat, sq, conn_unshadowed(s, w, g, g < total), g, eye);
        }
        conn_queue_flush(s, w, splat, sq, eye);
    } else if constexpr (!kPart) {
        for (int64_t g0 = (int64_t)blockIdx.x * kBlock + (threadIdx.x & ~63); g0 < total;
             g0 += (int64_t)gridDim.x * kBlock) {
            const int64_t g = g0 + lane_id();
            conn_task(s, w, splat, g, g < total, eye);
        }
    } else {
        __shared__ uint16_t srt_all[kBlock / 64][kSortN];
        const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        uint16_t* srt = srt_all[wv];
        __shared__ uint32_t shq_p[kQueue ? kBlock / 64 : 1][kQueue ? kShQ : 1];
        ShadowQueue sq{shq_p[kQueue ? wv : 0], 0};
        int box = -1;  // the first walk group
        for (int gi = s.ngroup - 1; gi >= 0; --gi)
            if (s.groups[gi].b < 0) box = gi;
        for (int64_t c0 = ((int64_t)blockIdx.x * (kBlock / 64) + wv) * kSortN; c0 < total;
             c0 += (int64_t)gridDim.x * kBlock * kSortR) {
            unsigned mk = 0;  // bit r: the lane's task of round r is marked
            int nu = 0;       // unmarked tasks of the chunk (wave-uniform)
            for (int r = 0; r < kSortR; ++r) {
                const int64_t g = c0 + r * 64 + lane_id();
                const bool m = box >= 0 && g < total && conn_marked(s, w, g, box);
                mk |= (m ? 1u : 0u) << r;
                nu += 64 - __popcll(__ballot(m));
            }
            int pu = 0, pm = nu;  // next slot of each group
            for (int r = 0; r < kSortR; ++r) {
                const bool m = (mk >> r) & 1u;
                const uint64_t bm = __ballot(m);
                const int before = mbcnt64(m ? bm : ~bm);
                srt[(m ? pm : pu) + before] = (uint16_t)(r * 64 + lane_id());
                pm += __popcll(bm);
                pu += 64 - __popcll(bm);
            }
            wave_lds_sync();
            for (int j0 = 0; j0 < kSortN; j0 += 64) {
                const int64_t g = c0 + (int64_t)srt[j0 + lane_id()];
                if constexpr (kQueue) conn_queue_push(s, w, splat, sq, conn_unshadowed(s, w, g, g < total), g, eye);
                else conn_task(s, w, splat, g, g < total, eye);
            }
            wave_lds_sync();  // the next chunk reuses srt
        }
        if constexpr (kQueue) conn_queue_flush(s, w, splat, sq, eye);
    }
}

// The walk-group scenes' connect (kSc = 2) is compiled in tpt_conn2.hip, without the
// AMDGPU register-pressure trackers: with them this compiler segfaults in its machine
// scheduler on that kernel for some code shapes (round 6: the queued walker partition,
// the uncapped connect stealing), and the bunny measures the same without them.
extern template __global__ void tpt_bdpt_conn_kernel<2, TPT_CONN_QUEUE_WALK != 0>(DScene, WfState, float*);
#if !TPT_TU_CONN2

// Class kernels (round 6, TPT_CONN_CLASS, small flat scenes; OFF: measured slower).  The
// emission-only run (s = 0: no connection, no shadow query, one MIS chain) needs 58
// VGPRs where the other classes need 128 (PathWeight compiled per class,
// path_weight<kCls>: the s = 1 and t = 1 forms even spill 32 / 92 B/lane at 128), so it
// can run in a launch of its own at TPT_CONN_W0 waves per SIMD beside the generic kernel
// for the other three runs.  Same tasks, same results at the same task indices, same
// splats (the c3 pins passed on the GPU), but Standard BDPT 256 spp went 429.6-430.9 ->
// 435.1-436.5 ms (8 waves; 6 waves 436.3-437.1 ms): the second launch's drain per
// wavefront costs more than the emission strategies' occupancy gains.
#ifndef TPT_CONN_CLASS
#define TPT_CONN_CLASS 0
#endif
#ifndef TPT_CONN_W0
#define TPT_CONN_W0 8  // waves per SIMD of the s = 0 launch
#endif
// [begin, end) of task run c (0 .. 3) of the wavefront's task list; c = -2: runs 1 .. 3
TPT_D void class_range(const WfState& w, int c, int64_t& b, int64_t& e) {
    const unsigned long long t1 = w.incl[w.ni - 1], t2 = w.incl2[w.ni - 1];
    const int64_t n[4] = {(int64_t)(t1 & 0xffffffffull), (int64_t)(t1 >> 32), (int64_t)(t2 & 0xffffffffull),
                          (int64_t)(t2 >> 32)};
    const int c0 = c < 0 ? 1 : c, c1 = c < 0 ? 3 : c;
    b = 0;
    for (int i = 0; i < c0; ++i) b += n[i];
    e = b;
    for (int i = c0; i <= c1; ++i) e += n[i];
}
template <int kSc, int kCls>
__global__ __launch_bounds__(kBlock, kCls == 0 ? TPT_CONN_W0 : TPT_CONN_MINWAVES) void tpt_bdpt_conn_cls_kernel(
        DScene s, WfState w, float* __restrict__ splat) {
    stage_scene<kSc>(s);
    __shared__ QScratch qsm[kBlock / 64];
    s.qs = qsm;
    s.ws = nullptr;
    int64_t b, e;
    class_range(w, kCls, b, e);
    const V3 eye = v3(s.eye[0], s.eye[1], s.eye[2]);
    for (int64_t g0 = b + (int64_t)blockIdx.x * kBlock + (threadIdx.x & ~63); g0 < e; g0 += (int64_t)gridDim.x * kBlock) {
        const int64_t g = g0 + lane_id();
        conn_task<kCls < 0 ? -1 : kCls>(s, w, splat, g, g < e, eye);
    }
}

#ifndef TPT_FLAT_DEFAULT
#define TPT_FLAT_DEFAULT 3  // kFlatShadow | kFlatHit; measured: BDPT 882 -> 812 ms, PT 64.0 -> 61.3 ms
#endif
// BDPT.cpp:289-311's `result` of item it: its t > 1 strategies in (t, s) order (t = 1
// ones were splatted), each read from its place in the task runs -- the same positions
// tpt_bdpt_scatter_kernel wrote.
TPT_D V3 item_result(const WfState& w, int64_t it) {
    const StratRange r = strat_range(w, it);
    const int ln = r.ln, cn = w.cnt[it] & 0xffff;
    V3 res = v3s(0.0f);  // BDPT.cpp:289 `Vector3f result;`
    auto add = [&](int64_t g) { res = res + v3(w.res[3 * g], w.res[3 * g + 1], w.res[3 * g + 2]); };
    for (int t = 2; t <= cn; ++t) {
        add(r.b[0] + (t - 2));  // s = 0
        add(r.b[2] + (t - 2));  // s = 1
        const int64_t g1 = r.b[1] + (int64_t)(t - 2) * (ln - 1) - 2;
        for (int sl = 2; sl <= ln; ++sl) add(g1 + sl);
    }
    return res;
}

// One wavefront of one iteration (nb = 1): per pixel, acc += (1/spp) * result.
__global__ __launch_bounds__(kBlock) void tpt_bdpt_fold_kernel(WfState w, float inv) {
    const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;  // pixel
    if (k >= w.n) return;
    V3 acc = v3(w.acc[3 * k], w.acc[3 * k + 1], w.acc[3 * k + 2]);
    for (int b = 0; b < w.nb; ++b) acc = acc + mul(item_result(w, (int64_t)b * w.n + k), inv);  // Renderer.cpp:49
    w.acc[3 * k] = acc.x;
    w.acc[3 * k + 1] = acc.y;
    w.acc[3 * k + 2] = acc.z;
}

// nb > 1 in two passes, so the strategy sums run one thread per item instead of nb
// items per pixel thread: tpt_bdpt_isum_kernel writes every item's result, then
// tpt_bdpt_fold_items_kernel adds a pixel's nb results in sample order
// (Renderer.cpp:49 `fb[i] += (1.0f / spp) * BDPT(...)`, the same float ops).
__global__ __launch_bounds__(kBlock) void tpt_bdpt_isum_kernel(WfState w) {
    const int64_t it = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (it >= w.ni) return;
    const V3 r = item_result(w, it);
    w.isum[3 * it] = r.x;
    w.isum[3 * it + 1] = r.y;
    w.isum[3 * it + 2] = r.z;
}
__global__ __launch_bounds__(kBlock) void tpt_bdpt_fold_items_kernel(WfState w, float inv) {
    const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;  // pixel
    if (k >= w.n) return;
    V3 acc = v3(w.acc[3 * k], w.acc[3 * k + 1], w.acc[3 * k + 2]);
    for (int b = 0; b < w.nb; ++b) {
        const int64_t it = (int64_t)b * w.n + k;
        acc = acc + mul(v3(w.isum[3 * it], w.isum[3 * it + 1], w.isum[3 * it + 2]), inv);
    }
    w.acc[3 * k] = acc.x;
    w.acc[3 * k + 1] = acc.y;
    w.acc[3 * k + 2] = acc.z;
}

__global__ __launch_bounds__(kBlock) void tpt_bdpt_out_kernel(WfState w, float* __restrict__ out, int rows) {
    const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k >= w.n) return;
    const int64_t row = rows ? k : wf_pixel(w, k);
    out[3 * row] = w.acc[3 * k];
    out[3 * row + 1] = w.acc[3 * k + 1];
    out[3 * row + 2] = w.acc[3 * k + 2];
}

// Splat accumulation in stages (round 4).  t = 1 splats (DrawToImage) are fp32 atomics;
// summed straight into one buffer over a 4096-spp frame, a bright pixel's sum reaches
// ~1.4e5 and contributions below half an ulp of it (~0.004) are lost, a bias that grows
// with spp: configs[4]'s frame came out 0.16 % low overall and 0.27 % low at the light
// against the reference's own per-worker sums.  (The reference sums each worker's
// splats in its own float buffer and merges the buffers after the join,
// Renderer.cpp:86-114; the fold below does the same across groups of sample
// iterations.)  Connect splats into a partial buffer, and every TPT_SPLAT_FOLD_SPP
// iterations (and at the end) the partial sums are added into the caller's buffer and
// cleared, in iteration order on the connect stream.
__global__ void tpt_splat_fold_kernel(float* __restrict__ acc, float* __restrict__ part, int64_t n) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
        acc[k] = acc[k] + part[k];
        part[k] = 0.0f;
    }
}

__global__ void tpt_scale_kernel(float* __restrict__ buf, int64_t n, float spp) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n) buf[k] = buf[k] * 1.0f / spp;  // Renderer.cpp:59 `e * 1.0f / spp`
}

// tpt_stats.nonfinite / nonfinite_splat: rows (pixels) of `buf` with a non-finite
// component, one atomic per wave.  The reference traps NaN only in MSVC _DEBUG builds
// (Vector.hpp:19-22); a release build carries a NaN sample into its pixel silently.
__global__ __launch_bounds__(kBlock) void tpt_count_nonfinite_kernel(const float* __restrict__ buf, int64_t rows,
                                                                     unsigned long long* __restrict__ out) {
    unsigned long long n = 0;
    for (int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x; k - lane_id() < rows;
         k += (int64_t)gridDim.x * kBlock) {
        bool bad = false;
        if (k < rows) {
            const float x = buf[3 * k], y = buf[3 * k + 1], z = buf[3 * k + 2];
            bad = !(__builtin_isfinite(x) && __builtin_isfinite(y) && __builtin_isfinite(z));
        }
        n += (unsigned long long)__popcll(__ballot(bad));
    }
    if (lane_id() == 0 && n) atomicAdd(out, n);
}

// Closest-hit queries (Scene::Intersect) for tpt_intersect.
__global__ __launch_bounds__(kBlock) void tpt_intersect_kernel(DScene s, const float* __restrict__ rays, int64_t n,
                                                               int cull, float* __restrict__ out) {
    __shared__ QScratch qsm[kBlock / 64];
    s.qs = qsm;
    __shared__ uint16_t wst[kWalkStack * kBlock];
    s.ws = wst;
    const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k >= n) return;
    const float* q = rays + 6 * k;
    Ray r = make_ray(v3(q[0], q[1], q[2]), v3(q[3], q[4], q[5]));
    PTV v = scene_intersect(s, r, cull);
    float* o = out + 8 * k;
    o[0] = v.type == T_BG ? 0.f : 1.f;
    o[1] = v.x.x; o[2] = v.x.y; o[3] = v.x.z;
    o[4] = v.N.x; o[5] = v.N.y; o[6] = v.N.z;
    o[7] = (float)v.prim;
}

// ------------------------------------------------------------------ C ABI --
#ifndef TPT_BDPT_SERIAL
#define TPT_BDPT_SERIAL 0  // 1: connect / fold on the gen stream (per-kernel timing builds only)
#endif

// per wavefront buffer: gen's 8 shard counters, 64 B apart
constexpr size_t kQueueBytes = kWfBufs * 8 * 64;
static_assert(kWfBufs >= 2 && kWfBufs <= 4, "2 to 4 wavefront buffers");

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
    float* splat_part = nullptr;  // BDPT: the splats of the last few wavefronts (folded into the caller's buffer)
    int64_t part_floats = 0;
    int64_t* list = nullptr;
    int64_t list_cap = 0;
    float* rows = nullptr;
    int64_t rows_cap = 0;
    unsigned long long* counters = nullptr;
    unsigned* queue = nullptr;  // persistent gen: 8 shard counters, 64 B apart, per wavefront buffer
    int num_cu = 0;
    int sc = 0;  // kernel scene class (stage_scene): 0 no LDS, 1 small flat scene, 2 flat + treelets / walk groups
    // wavefront BDPT state (sized for wf_cap pixels)
    void* wf_mem = nullptr;
    int64_t wf_cap = 0;
    int64_t wf_stride = 0;            // bytes from one wavefront buffer's arrays to the next one's
    int64_t wf_failed = 0;            // a wavefront allocation of this many items failed (0: none);
                                      // later renders of the same shard size do not retry it
    int64_t wf_failed_count = 0;      // ... for shards of this many pixel streams
    WfState wf[kWfBufs]{};            // kWfBufs wavefront buffers: gen(f+1..) overlaps connect(f)
    hipStream_t stream2 = nullptr;    // connect + fold
    hipStream_t stream3 = nullptr;    // gen / scan / scatter of the odd wavefronts (even ones: stream)
    hipEvent_t ev_gen[kWfBufs]{}, ev_fold[kWfBufs]{}, ev_start = nullptr;
    unsigned stall_ticks = kStallTicks;  // gen watchdog limit (TPT_DIAG_HOOKS builds: per render from the env)
    int drop_k = -1;                     // TPT_DIAG_HOOKS builds only (see there)
    void* scan_tmp = nullptr;         // two scratch areas: the gen streams scan concurrently
    void* scan_tmp_g[2]{};            // per gen stream
    size_t scan_bytes = 0;
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

// The partial splat buffer (W * H * 3 floats, zero between folds).
int ensure_part(tpt_ctx* c) {
    const int64_t need = (int64_t)c->hs.width * c->hs.height * 3;
    if (c->part_floats < need) {
        if (c->splat_part) (void)hipFree(c->splat_part);
        c->splat_part = nullptr;
        c->part_floats = 0;
        HIP_TRY(c, hipMalloc(&c->splat_part, need * sizeof(float)));
        c->part_floats = need;
    }
    // cleared at the start of every render (before its first kernel, on the stream every
    // launch follows): a render that failed between a connect and its fold must not leave
    // partial splats behind for the next one (~7 MB, negligible beside a frame)
    HIP_TRY(c, hipMemsetAsync(c->splat_part, 0, need * sizeof(float), c->stream));
    return TPT_OK;
}

// Wavefront BDPT buffers for n items (iteration, pixel stream): path records (2 KB per
// item) and the strategy list (<= 271 strategies per item: cn, ln <= 16).  The per-pixel
// rng / acc arrays are sized for n pixels too (a wavefront never has more pixels than
// items).
int ensure_wf(tpt_ctx* c, int64_t n) {
    if (n <= c->wf_cap) return TPT_OK;
#if TPT_DIAG_HOOKS
    // diagnostics: refuse wavefront buffers above TPT_DIAG_WF_ITEMS_MAX items, as a failed
    // hipMalloc would (drives launch()'s fallback to one iteration per wavefront)
    if (const char* lim = std::getenv("TPT_DIAG_WF_ITEMS_MAX"))
        if (*lim && n > std::atoll(lim)) return fail(c, TPT_E_ALLOC, "diagnostics: wavefront items above the limit");
#endif
    if (c->wf_mem) (void)hipFree(c->wf_mem);
    if (c->scan_tmp) (void)hipFree(c->scan_tmp);
    c->wf_mem = c->scan_tmp = nullptr;
    c->wf_cap = 0;
    const int64_t maxs = (int64_t)kMaxLen * (kMaxLen + 1) - 1;
    auto al = [](int64_t b) { return (b + 255) & ~(int64_t)255; };
    const int64_t b_rec = al(2 * kMaxLen * kRecV * n * 16), b_i = al(n * 4), b_l = al(n * 8),
                  b_own = al(n * maxs * 4), b_res = al(n * maxs * 12), b_acc = al(n * 12);
    // per buffer: a multiple of one item's records (2 KB)
    const int64_t rec_item = 2 * kMaxLen * kRecV * 16;
    const int64_t per_buf = (b_rec + b_i + 4 * b_l + b_own + b_res + b_acc + rec_item - 1) / rec_item * rec_item;
    const int64_t total = kWfBufs * per_buf + b_l + b_acc;
    HIP_TRY(c, hipMalloc(&c->wf_mem, total));

    char* p = (char*)c->wf_mem;
    c->wf_stride = per_buf;
    for (int b = 0; b < kWfBufs; ++b) {
        WfState& w = c->wf[b];
        p = (char*)c->wf_mem + b * per_buf;
        w.rec = (float4*)p; p += b_rec;
        w.cnt = (int*)p; p += b_i;
        w.np = (unsigned long long*)p; p += b_l;
        w.incl = (unsigned long long*)p; p += b_l;
        w.np2 = (unsigned long long*)p; p += b_l;
        w.incl2 = (unsigned long long*)p; p += b_l;
        w.task = (unsigned*)p; p += b_own;
        w.res = (float*)p; p += b_res;
        w.isum = (float*)p; p += b_acc;
    }
    p = (char*)c->wf_mem + kWfBufs * per_buf;
    for (int b = 0; b < kWfBufs; ++b) c->wf[b].rngseq = (unsigned long long*)p;
    p += b_l;
    // Every item's (cnt, np, np2) starts as a valid empty sample, so a wavefront whose
    // gen watchdog fired (a lane gave up on its pixel) still scans and scatters in
    // bounds.  Per array (each < 32 MB per wavefront buffer at a frame's size), on the
    // context's stream ahead of the first launch.
    for (int b = 0; b < kWfBufs; ++b) {
        HIP_TRY(c, hipMemsetAsync(c->wf[b].cnt, 0, n * sizeof(int), c->stream));
        HIP_TRY(c, hipMemsetAsync(c->wf[b].np, 0, n * sizeof(unsigned long long), c->stream));
        HIP_TRY(c, hipMemsetAsync(c->wf[b].np2, 0, n * sizeof(unsigned long long), c->stream));
    }
    for (int b = 0; b < kWfBufs; ++b) c->wf[b].acc = (float*)p;
    const WfState& w = c->wf[0];
    size_t bytes = 0;
    HIP_TRY(c, rocprim::inclusive_scan(nullptr, bytes, w.np, w.incl, (size_t)n, rocprim::plus<unsigned long long>(),
                                       c->stream));
    bytes = (bytes + 255) & ~(size_t)255;
    HIP_TRY(c, hipMalloc(&c->scan_tmp, 2 * bytes));
    c->scan_tmp_g[0] = c->scan_tmp;
    c->scan_tmp_g[1] = (char*)c->scan_tmp + bytes;
    c->scan_bytes = bytes;
    c->wf_cap = n;
    return TPT_OK;
}

int64_t shard_count(int64_t npix, int64_t begin, int64_t stride) {
    if (begin >= npix) return 0;
    return (npix - begin + stride - 1) / stride;
}

#ifndef TPT_WF_ITEMS
// Items a BDPT wavefront aims for: a shard of n pixel streams runs
// nb = max(1, TPT_WF_ITEMS / n) sample iterations per wavefront (at most spp /
// TPT_WF_MIN_FRONTS), so a small shard (1/8 of a frame on each of 8 GPUs) launches and
// drains as few wavefronts as a whole frame does.  Default: two 784 x 784 frames'
// worth, ~24 GB of wavefront buffers.  Same-box shard model (Standard BDPT 256 spp,
// whole frame / 1/8 shard): one frame 457.9 / 64.3 ms, two 445.6 / 61.9, three 442.5 /
// 62.0, four 438.7 / 62.9 ms (47 GB); bunny BDPT 256 spp whole frame 940 / 933 / 928 /
// 926 ms.  Round 4: four frames (bunny 256 spp 801 -> 788 ms with the partition), then
// six (~70 GB; same-box A/B at build b7f5ad7: bunny 256 spp 738.9 -> 729.8 ms, Standard
// 435.9 -> 435.6 ms, bunny 4096 spp 1/8 shard 1621.8 -> 1621.7 ms).  Must stay < kWfChunk.
#define TPT_WF_ITEMS 3687936
#endif
#if TPT_WF_ITEMS > (1 << 22)
#error "TPT_WF_ITEMS must not exceed kWfChunk (32-bit item indices)"
#endif
#ifndef TPT_WF_MIN_FRONTS
// ... and at least this many wavefronts where spp allows (a wavefront's fill and drain
// do not overlap with another's): 1/8 shards run 16 iterations per wavefront.
#define TPT_WF_MIN_FRONTS 16
#endif
#ifndef TPT_GEN_GRID_Q
// gen's persistent grid, in 32nds of what fits on the chip at once.  A full grid
// occupies every CU until the queue drains, so connect (other stream) only runs in
// gen's tail; a third of the chip leaves room for both.  Same-box sweep, Standard
// BDPT 256 spp / bunny BDPT 256 spp: 32 -> 601 ms / -, 8 -> 592 / 1275, 9 -> 564 /
// 1173, 10 -> 553 / 1131, 11 -> 556 / 1108, 12 -> 567 / -, 16 -> 585 / -.  Round 3,
// wavefronts of two iterations: 10 -> 445.0 / 929.5, 11 -> 447.2 / 933.6, 12 -> 449.9 /
// 932.6 ms.
#define TPT_GEN_GRID_Q 9  // round 4, four-iteration wavefronts on two gen streams: 8 / 9 / 10 / 11 / 12 ->
                          // 433.4 / 432.4 / 434.4 / 435.7 / 435.8 ms (Standard BDPT 256 spp); 9 took the
                          // 1/8 shard from 61.6 to 63.9 ms, so 10 stayed.  Round 6 (the faster kernels):
                          // 9 / 10 / 11 -> 422.2 / 424.5-425.5 / 424.3-425.9 ms whole frame, 1/8 shard
                          // 61.8 / 60.5 ms: 9 for whole frames, 10 for shards (TPT_GEN_GRID_Q_SHARD)
#endif
#ifndef TPT_GEN_GRID_Q_SHARD
#define TPT_GEN_GRID_Q_SHARD 10  // ... small flat scenes, wavefronts of >= 8 iterations (shards of a frame)
#endif
#ifndef TPT_GEN_GRID_Q_WALK
// ... for scenes with walk groups (the bunny), whose connect runs the walker partition:
// connect got 21 % cheaper (serialised kernel trace, bunny BDPT 64 spp: 4.55 -> 3.60 ms
// per wavefront), so gen, which now bounds the frame, takes a larger share.  Same-box
// sweep, bunny BDPT 256 spp with the partition: 10 -> 925, 11 -> 866, 12 -> 799,
// 13 -> 798, 14 -> 813 ms (no partition, 10: 917 ms).
#define TPT_GEN_GRID_Q_WALK 12
#endif
#ifndef TPT_GEN_GRID_Q_WALK2
#define TPT_GEN_GRID_Q_WALK2 8  // ... when two gen kernels run at once (wavefronts of >= 3 iterations: whole
                                // frames since round 4).  With the deferred walks, bunny 256 spp, 9 / 10 /
                                // 11 / 12 -> 742.0 / 742.1 / 753.9 / 760.4 ms; with the stealing walks (round
                                // 5) 6 / 7 / 8 / 10 -> 659 / 651 / 651 / 684 ms (means of two), configs[4]'s
                                // 4096-spp frame 7 / 8 / 10 -> 10.39 / 10.38 / 10.93 s
#endif
#ifndef TPT_GEN_GRID_Q_WALK_SHARD
#define TPT_GEN_GRID_Q_WALK_SHARD 11  // ... and for wavefronts of >= 8 iterations (shards of a frame, whose gen
                                      // lanes run many samples each): 1/8 shard 9 / 10 / 11 / 12 -> 110.2 /
                                      // 108.5 / 106.8 / 107.5 ms
#endif
#ifndef TPT_SPLAT_FOLD_SPP
#define TPT_SPLAT_FOLD_SPP 64  // sample iterations per partial splat sum (tpt_splat_fold_kernel); one
                               // buffer over 256 spp was within 1.4e-5 of the reference (frame_c5r)
#endif
#ifndef TPT_GEN2_MIN_NB
#define TPT_GEN2_MIN_NB 3  // two gen streams when a wavefront holds >= this many iterations (whole frames,
                           // 2 iterations: one stream, bunny BDPT 256 spp 931.7 -> 919.2 ms, Standard 440.8 either way)
#endif
int wf_iters(int64_t count, int spp) {
    const int64_t nb = std::max<int64_t>(1, std::min<int64_t>((int64_t)TPT_WF_ITEMS, kWfChunk) / std::max<int64_t>(count, 1));
    return (int)std::min<int64_t>(nb, std::max(1, spp / TPT_WF_MIN_FRONTS));
}

#ifndef TPT_WF_RAMP
#define TPT_WF_RAMP 2  // ramp steps at each end of the wavefront schedule (0: uniform; 2 / 3 / 4 -> bunny BDPT 256 spp
                       // 718.1 -> 715.2 / 716.2 / 715.9 ms, Standard 432.1 -> 430.1 / 431.0 / 429.8 ms, same box)
#endif
// Sample iterations of each wavefront of a chunk.  Connect(f) starts only when gen(f)
// is complete, so the first gen runs with nothing beside it and the last connect runs
// alone.  With TPT_WF_RAMP = R the schedule starts and ends with wavefronts of nb >> R,
// ..., nb >> 1 iterations (the pipeline fills and drains in short steps), and the
// iterations in between are split into wavefronts of at most nb, as even as possible.
// Uniform (nb, ..., nb, remainder) when R = 0 or spp is too small for the ramps.
std::vector<int> wf_schedule(int spp, int nb) {
    std::vector<int> ramp;
    for (int r = TPT_WF_RAMP; r >= 1; --r) {
        const int v = std::max(1, nb >> r);
        if (v < nb && (ramp.empty() || v > ramp.back())) ramp.push_back(v);
    }
    int rs = 0;
    for (int v : ramp) rs += 2 * v;
    std::vector<int> out;
    if (ramp.empty() || spp < rs + nb) {
        for (int it0 = 0; it0 < spp; it0 += nb) out.push_back(std::min(nb, spp - it0));
        return out;
    }
    out = ramp;
    const int mid = spp - rs, m = (mid + nb - 1) / nb;
    for (int j = 0; j < m; ++j) out.push_back(mid / m + (j < mid % m ? 1 : 0));
    out.insert(out.end(), ramp.rbegin(), ramp.rend());
    return out;
}

#ifndef TPT_CONN_GRID
#define TPT_CONN_GRID 16384  // connect's grid-stride grid, small flat scenes (Standard BDPT 256 spp: 8192 / 16384 -> 445.4 / 441.2 ms)
#endif
#ifndef TPT_CONN_GRID_WALK
#define TPT_CONN_GRID_WALK 8192  // ... and scenes with walk groups (round 3, bunny BDPT 256 spp: 8192 / 16384 -> 928 / 935 ms;
                                 // round 5, with the partition: 716.3 / 715.5 ms, its 1/8 shard at 4096 spp 1597 / 1577 ms;
                                 // with the stealing gen walks and gen at 8/32: 643 / 655 ms, shard 1351 / 1393 ms,
                                 // configs[4]'s frame 10.19 / 10.31 s; 8,192 with 8-round partition chunks: 654 ms)
#endif

// The BDPT sample loop over `count` (<= kWfChunk) pixel streams, as wavefronts of
// nb = wf_iters(count, spp) sample iterations each.
int launch_bdpt_chunk(tpt_ctx* c, int spp, int64_t begin, int64_t stride, int64_t count, const int64_t* dlist,
                      float* drows, float* dsplat) {
    const size_t shmem = (size_t)c->ds.lds_bytes;
    // Two streams: gen/scan/scatter of wavefront f on c->stream, connect/fold on
    // c->stream2, with the wavefront state double-buffered so gen(f+1) runs beside
    // connect(f) and fills the tail of each.  Ordering per pixel is kept: gen is
    // sequential on one stream (RNG state), fold is sequential on the other (acc,
    // splat), and buffer b is rewritten by gen(f+2) only after fold(f).
    // Streams: gen / scan / scatter of wavefront f on gs[f & 1] (the two gen streams let
    // gen(f + 1) start while gen(f) drains its long paths; they hand each pixel's
    // stream state over through WfState::rngseq), connect / fold of every wavefront on
    // s2.  The wavefront state is double-buffered: buffer f & 1 is rewritten by
    // gen(f + 2) only after fold(f).  Per pixel the order is kept: gen(f) samples after
    // gen(f - 1) (rngseq), fold is sequential on s2 (acc, splat).
    const int nb = (int)std::min<int64_t>(wf_iters(count, spp), std::max<int64_t>(1, c->wf_cap / count));
    hipStream_t s2 = TPT_BDPT_SERIAL ? c->stream : c->stream2;
    // The second gen stream only where wavefronts hold several iterations (small
    // shards: a lane runs nb samples of one pixel, so gen's tail is long).  For a
    // frame-sized shard (nb = 1) gen(f + 1)'s lanes would mostly sit waiting on
    // gen(f)'s pixels and take slots from connect: same-box 452 vs 477 ms (Standard
    // BDPT 256 spp); at 1/8 of the frame the two streams win, 0.72 -> 0.81 of linear.
    const bool two_gen = !TPT_BDPT_SERIAL && nb >= TPT_GEN2_MIN_NB;
    hipStream_t gs[2] = {c->stream, two_gen ? c->stream3 : c->stream};
    // both gen streams start after everything queued so far; the pixel states and the
    // queue counters of both buffers start at 0
    HIP_TRY(c, hipMemsetAsync(c->wf[0].rngseq, 0, count * sizeof(unsigned long long), c->stream));
    HIP_TRY(c, hipMemsetAsync(c->queue, 0, kQueueBytes, c->stream));
    HIP_TRY(c, hipEventRecord(c->ev_start, c->stream));
    HIP_TRY(c, hipStreamWaitEvent(s2, c->ev_start, 0));
    if (gs[1] != gs[0]) HIP_TRY(c, hipStreamWaitEvent(gs[1], c->ev_start, 0));
    const unsigned pblocks = (unsigned)((count + kBlock - 1) / kBlock);
    const int gen_q = c->sc != 2 ? (nb >= 8 ? TPT_GEN_GRID_Q_SHARD : TPT_GEN_GRID_Q)
                      : !two_gen  ? TPT_GEN_GRID_Q_WALK
                      : nb >= 8   ? TPT_GEN_GRID_Q_WALK_SHARD
                                  : TPT_GEN_GRID_Q_WALK2;
    // persistent gen grid: as many workgroups as are resident at once, a multiple of
    // the 8 queue shards, and no more than the pixels need
    const auto gen_k = c->sc == 2 ? tpt_bdpt_gen_kernel<2> : c->sc == 1 ? tpt_bdpt_gen_kernel<1> : tpt_bdpt_gen_kernel<0>;
    const bool qconn = TPT_CONN_QUEUE && nb < 8;
    const auto conn_k = c->sc == 2 ? tpt_bdpt_conn_kernel<2, TPT_CONN_QUEUE_WALK != 0>
                        : c->sc == 1 ? (qconn ? tpt_bdpt_conn_kernel<1, true> : tpt_bdpt_conn_kernel<1>)
                                     : (qconn ? tpt_bdpt_conn_kernel<0, true> : tpt_bdpt_conn_kernel<0>);
    int per_cu = 0;
    HIP_TRY(c, hipOccupancyMaxActiveBlocksPerMultiprocessor(
                   &per_cu, (const void*)gen_k, kBlock, shmem));
    int64_t gb = (int64_t)std::max(per_cu, 1) * std::max(c->num_cu, 1) * gen_q / 32;
    gb = std::min<int64_t>(gb, ((int64_t)pblocks + 7) / 8 * 8);
    const unsigned gblocks = (unsigned)std::max<int64_t>(8, gb / 8 * 8);
    // The two-stream hand-off (gen(f) waits, lane by lane, on gen(f - 1)'s publications)
    // cannot deadlock only while gen(f - 1) can always be scheduled: gen(f) spins on at
    // most its own grid, so each gen grid must leave at least half of the chip's
    // resident workgroups to the other kernels.  (connect never waits; it frees its
    // slots as it finishes.)
    const int64_t resident = (int64_t)std::max(per_cu, 1) * std::max(c->num_cu, 1);
    if (two_gen && !gen_grid_ok((long long)gblocks, (long long)resident))
        return fail(c, TPT_E_DEVICE, "BDPT: gen grid of " + std::to_string(gblocks) + " workgroups exceeds half of the " +
                                         std::to_string(resident) + " resident ones (two-stream hand-off invariant)");
    const float inv = 1.0f / spp;
    const std::vector<int> sched = wf_schedule(spp, nb);
    int cam_nb[kWfBufs] = {};  // per buffer: leading iterations whose items hold the camera vertices
    for (int f = 0, it0 = 0; it0 < spp; it0 += sched[f], ++f) {
        const int b = f % kWfBufs, gsi = f & 1;  // wavefront buffer, gen stream
        WfState w = c->wf[b];
        w.list = dlist;
        w.begin = begin;
        w.stride = stride;
        w.n = count;
        w.nb = sched[f];
        w.ni = (int64_t)w.nb * count;
        w.cam_nb = cam_nb[b];
        cam_nb[b] = std::max(cam_nb[b], w.nb);
        w.bounces = c->counters;
        w.stall = reinterpret_cast<int*>(c->counters + 4);
        w.stall_ticks = c->stall_ticks;
        w.drop_k = c->drop_k;
        w.conc = two_gen ? 1 : 0;
        unsigned* queue = c->queue + b * 8 * 16;
        const unsigned iblocks = (unsigned)((w.ni + kBlock - 1) / kBlock);
        const unsigned cblocks = (unsigned)std::min<int64_t>(c->sc == 2 ? TPT_CONN_GRID_WALK : TPT_CONN_GRID,
                                                             (w.ni * 24 + kBlock - 1) / kBlock + 1);
        if (f >= kWfBufs) HIP_TRY(c, hipStreamWaitEvent(gs[gsi], c->ev_fold[b], 0));
        hipLaunchKernelGGL(gen_k, dim3(gblocks), dim3(kBlock), shmem, gs[gsi], c->ds, w, f, queue);
        size_t bytes = c->scan_bytes;
        HIP_TRY(c, rocprim::inclusive_scan(c->scan_tmp_g[gsi], bytes, w.np, w.incl, (size_t)w.ni,
                                           rocprim::plus<unsigned long long>(), gs[gsi]));
        bytes = c->scan_bytes;
        HIP_TRY(c, rocprim::inclusive_scan(c->scan_tmp_g[gsi], bytes, w.np2, w.incl2, (size_t)w.ni,
                                           rocprim::plus<unsigned long long>(), gs[gsi]));
        hipLaunchKernelGGL(tpt_bdpt_scatter_kernel, dim3(iblocks), dim3(kBlock), 0, gs[gsi], w, queue);
        HIP_TRY(c, hipEventRecord(c->ev_gen[b], gs[gsi]));
        HIP_TRY(c, hipStreamWaitEvent(s2, c->ev_gen[b], 0));
#if TPT_CONN_CLASS
        if (c->sc != 2) {  // s = 0 in its own launch (tpt_bdpt_conn_cls_kernel)
            float* sp = dsplat ? c->splat_part : nullptr;
            const dim3 g0((unsigned)std::min<int64_t>(TPT_CONN_GRID, (w.ni * 6 + kBlock - 1) / kBlock + 1));
            if (c->sc == 1) {
                hipLaunchKernelGGL((tpt_bdpt_conn_cls_kernel<1, -2>), dim3(cblocks), dim3(kBlock), shmem, s2, c->ds, w, sp);
                hipLaunchKernelGGL((tpt_bdpt_conn_cls_kernel<1, 0>), g0, dim3(kBlock), shmem, s2, c->ds, w, sp);
            } else {
                hipLaunchKernelGGL((tpt_bdpt_conn_cls_kernel<0, -2>), dim3(cblocks), dim3(kBlock), shmem, s2, c->ds, w, sp);
                hipLaunchKernelGGL((tpt_bdpt_conn_cls_kernel<0, 0>), g0, dim3(kBlock), shmem, s2, c->ds, w, sp);
            }
        } else
#endif
        {
            hipLaunchKernelGGL(conn_k, dim3(cblocks), dim3(kBlock), shmem, s2, c->ds, w, dsplat ? c->splat_part : nullptr);
        }
        if (w.nb == 1) {
            hipLaunchKernelGGL(tpt_bdpt_fold_kernel, dim3(pblocks), dim3(kBlock), 0, s2, w, inv);
        } else {
            hipLaunchKernelGGL(tpt_bdpt_isum_kernel, dim3(iblocks), dim3(kBlock), 0, s2, w);
            hipLaunchKernelGGL(tpt_bdpt_fold_items_kernel, dim3(pblocks), dim3(kBlock), 0, s2, w, inv);
        }
        if (dsplat && ((it0 + w.nb) / TPT_SPLAT_FOLD_SPP > it0 / TPT_SPLAT_FOLD_SPP || it0 + w.nb >= spp)) {
            const int64_t nf = (int64_t)c->hs.width * c->hs.height * 3;
            hipLaunchKernelGGL(tpt_splat_fold_kernel, dim3((unsigned)std::min<int64_t>(4096, (nf + 255) / 256)), dim3(256), 0,
                               s2, dsplat, c->splat_part, nf);
        }
        HIP_TRY(c, hipEventRecord(c->ev_fold[b], s2));
        if (it0 + w.nb >= spp) HIP_TRY(c, hipStreamWaitEvent(c->stream, c->ev_fold[b], 0));
    }
    WfState w = c->wf[0];
    w.list = dlist;
    w.begin = begin;
    w.stride = stride;
    w.n = count;
    hipLaunchKernelGGL(tpt_bdpt_out_kernel, dim3(pblocks), dim3(kBlock), 0, c->stream, w, drows, dlist ? 1 : 0);
    return TPT_OK;
}

// Launch the integration kernel for `count` pixels; rows/splat are device buffers.
int launch(tpt_ctx* c, int mode, int flags, int spp, int64_t begin, int64_t stride, int64_t count,
           const int64_t* dlist, float* drows, float* dsplat, tpt_stats* st) {
    const bool seeded = (flags & TPT_FLAG_SAMPLE_SEED) != 0;
    if (st) std::memset(st, 0, sizeof(*st));  // an empty shard or list reports zeros
    if (count <= 0) {  // nothing to trace; the caller's memsets still complete before returning
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        return TPT_OK;
    }
    HIP_TRY(c, hipMemsetAsync(c->counters, 0, sizeof(unsigned long long) * 32, c->stream));
    HIP_TRY(c, hipEventRecord(c->ev0, c->stream));
    const size_t shmem = (size_t)c->ds.lds_bytes;
    if (mode == TPT_MODE_PT) {
        const bool q16 = kQ < 16 && count <= TPT_PT_SMALL_PIXELS;
        const int qm = q16 ? 16 : kQ;
        // the grid's last TPT_PT_TAIL_WAVES x (resident waves) pixel streams run one
        // wave each (tpt_pt_kernel's second tier), at most a quarter of the pixels
        const int64_t resident = (int64_t)std::max(c->num_cu, 1) * 4 * TPT_PT_MINWAVES;
        const int64_t tail = seeded ? 0 : std::min<int64_t>(count / 4, (int64_t)TPT_PT_TAIL_WAVES * resident);
        const int64_t k_tail = count - tail;
        const int64_t b_tail = (k_tail * qm + kBlock - 1) / kBlock;
        const int64_t qblocks = b_tail + (tail * kQT + kBlock - 1) / kBlock;
        size_t pshmem = shmem + (size_t)kPixSlots * kBlock * sizeof(float);
        // The jump table only where the workgroup still fits 5 times (TPT_PT_MINWAVES) in a
        // CU's LDS.  Measured: 31,872 B per workgroup keeps 5 resident, 32,128 B does not
        // (46.4 vs 49.9 ms, Standard); consistent with 1,280-B allocation granules in 160 KB.
        const int use_jump = !seeded && TPT_PT_JUMP && pshmem + kJumpWords * 4 <= kLdsGranule * (160 * 1024 / kLdsGranule / TPT_PT_MINWAVES);
        if (use_jump) pshmem += kJumpWords * 4;
        auto pick = [&](auto q) {
            constexpr int Q = decltype(q)::value;
            return c->sc == 2   ? (seeded ? tpt_pt_kernel<2, true, Q> : tpt_pt_kernel<2, false, Q>)
                   : c->sc == 1 ? (seeded ? tpt_pt_kernel<1, true, Q> : tpt_pt_kernel<1, false, Q>)
                                : (seeded ? tpt_pt_kernel<0, true, Q> : tpt_pt_kernel<0, false, Q>);
        };
        auto k = q16 ? pick(std::integral_constant<int, 16>{}) : pick(std::integral_constant<int, kQ>{});
        hipLaunchKernelGGL(k, dim3((unsigned)qblocks), dim3(kBlock), pshmem, c->stream, c->ds, spp, begin, stride,
                           count, dlist, drows, use_jump, k_tail, b_tail);
    } else if (mode == TPT_MODE_PT_INDIRECT) {
        const int64_t lanes = count * (seeded ? kQ : 1);
        auto k = c->sc == 2   ? (seeded ? tpt_pti_kernel<2, true> : tpt_pti_kernel<2, false>)
                 : c->sc == 1 ? (seeded ? tpt_pti_kernel<1, true> : tpt_pti_kernel<1, false>)
                              : (seeded ? tpt_pti_kernel<0, true> : tpt_pti_kernel<0, false>);
        hipLaunchKernelGGL(k, dim3((unsigned)((lanes + kBlock - 1) / kBlock)), dim3(kBlock), shmem, c->stream, c->ds,
                           spp, begin, stride, count, dlist, drows, c->counters);
    } else {
#if TPT_DIAG_HOOKS
        const char* dk = std::getenv("TPT_DIAG_DROP_PUBLISH");
        const char* dt = std::getenv("TPT_DIAG_STALL_TICKS");
        c->drop_k = dk && *dk ? std::atoi(dk) : -1;
        c->stall_ticks = dt && *dt ? (unsigned)std::strtoul(dt, nullptr, 10) : kStallTicks;
#endif
        // Shards larger than kWfChunk pixel streams run as consecutive chunks.
        const int64_t chunk = std::min(count, kWfChunk), last = count - (count - 1) / kWfChunk * kWfChunk;
        if (dsplat) {
            const int rp = ensure_part(c);
            if (rp) return rp;
        }
        const int64_t want = std::max(chunk * wf_iters(chunk, spp), last * wf_iters(last, spp));
        // a size that failed before for this shard size is not retried (each failed
        // hipMalloc / hipFree pair synchronises the device): the fallback capacity stays
        const bool known_bad = c->wf_failed && c->wf_failed_count == count && want >= c->wf_failed;
        int rc = known_bad ? TPT_E_ALLOC : ensure_wf(c, want);
        if (rc) {
            // not enough device memory for multi-iteration wavefronts (~19 KB per item):
            // fall back to one iteration per wavefront (launch_bdpt_chunk caps nb at
            // wf_cap / count), which needs a shard's worth of items only
            (void)hipGetLastError();
            if (!known_bad) {
                c->wf_failed = want;
                c->wf_failed_count = count;
            }
            rc = ensure_wf(c, chunk);
            if (rc) return fail(c, TPT_E_ALLOC, "BDPT wavefront buffers: " + c->err);
        }
        for (int64_t c0 = 0; c0 < count; c0 += kWfChunk) {
            rc = launch_bdpt_chunk(c, spp, dlist ? 0 : begin + c0 * stride, stride, std::min(kWfChunk, count - c0),
                                   dlist ? dlist + c0 : nullptr, dlist ? drows + 3 * c0 : drows, dsplat);
            if (rc) return rc;
        }
    }
    HIP_TRY(c, hipGetLastError());
    HIP_TRY(c, hipEventRecord(c->ev1, c->stream));
    const int64_t npix = (int64_t)c->hs.width * c->hs.height;
    if (mode == TPT_MODE_BDPT && dsplat) {
        int64_t n = npix * 3;
        hipLaunchKernelGGL(tpt_scale_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream, dsplat, n,
                           (float)spp);
        HIP_TRY(c, hipGetLastError());
    }
    if (st) {  // non-finite pixels of the output: listed rows, or the whole frame buffer of a shard
        const int64_t rows = dlist ? count : npix;
        auto grid = [](int64_t r) { return (unsigned)std::min<int64_t>(2048, (r + kBlock - 1) / kBlock); };
        hipLaunchKernelGGL(tpt_count_nonfinite_kernel, dim3(grid(rows)), dim3(kBlock), 0, c->stream, drows, rows,
                           c->counters + 2);
        if (mode == TPT_MODE_BDPT && dsplat)
            hipLaunchKernelGGL(tpt_count_nonfinite_kernel, dim3(grid(npix)), dim3(kBlock), 0, c->stream, dsplat, npix,
                               c->counters + 3);
        HIP_TRY(c, hipGetLastError());
    }
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (mode == TPT_MODE_BDPT) {
        int stall = 0;
        HIP_TRY(c, hipMemcpy(&stall, c->counters + 4, sizeof(stall), hipMemcpyDeviceToHost));
        if (stall) return fail(c, TPT_E_DEVICE, "BDPT: a gen lane timed out waiting for the previous wavefront");
    }
    if (st) {
        float ms = 0.f;
        HIP_TRY(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
        st->kernel_ms = ms;
        st->pixels = count;
        st->samples = count * (int64_t)spp;
        unsigned long long cnt[4] = {0, 0, 0, 0};
        HIP_TRY(c, hipMemcpy(cnt, c->counters, sizeof(cnt), hipMemcpyDeviceToHost));
        st->bounces = (int64_t)cnt[0];
        st->nonfinite = (int64_t)cnt[2];
        st->nonfinite_splat = (int64_t)cnt[3];
    }
    return TPT_OK;
}

int check_render_args(tpt_ctx* c, int spp, int mode, int flags = 0) {
    if (!c) return TPT_E_INVALID;
    if (!c->has_scene) return fail(c, TPT_E_NOSCENE, "no scene uploaded");
    if (spp <= 0) return fail(c, TPT_E_INVALID, "spp must be positive");
    if (mode != TPT_MODE_PT && mode != TPT_MODE_BDPT && mode != TPT_MODE_PT_INDIRECT)
        return fail(c, TPT_E_INVALID, "unknown mode");
    if (flags & ~TPT_FLAG_SAMPLE_SEED) return fail(c, TPT_E_INVALID, "unknown flags");
    if ((flags & TPT_FLAG_SAMPLE_SEED) && mode == TPT_MODE_BDPT)
        return fail(c, TPT_E_UNSUPPORTED, "per-sample seeding (TPT_FLAG_SAMPLE_SEED) is for PT and PT-indirect");
    if (mode == TPT_MODE_BDPT && c->hs.emitters.empty())
        return fail(c, TPT_E_INVALID, "BDPT needs an emitter (BDPT.cpp:287 uses m_emissionObjects[0])");
    return TPT_OK;
}

}  // namespace

extern "C" {

int tpt_abi_version(void) { return TPT_ABI_VERSION; }
void tpt_hip_versions(int* compiled, int* runtime) {
    if (compiled) *compiled = HIP_VERSION;
    int v = -1;
    if (runtime && hipRuntimeGetVersion(&v) != hipSuccess) v = -1;
    if (runtime) *runtime = v;
}
#if TPT_GEN_STATS
// diagnostics build only: the gen kernels' per-wave statistics since the last reset
int tpt_diag_walkstats(unsigned long long* host, int reset) {
    if (hipDeviceSynchronize() != hipSuccess || hipMemcpyFromSymbol(host, HIP_SYMBOL(tpt_walkstat), 64) != hipSuccess) return -1;
    if (reset) {
        const unsigned long long z[8] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(tpt_walkstat), z, 64) != hipSuccess) return -1;
    }
    return 0;
}
int tpt_diag_genstats(unsigned long long* host, int64_t n, int reset) {
    unsigned cnt = 0;
    if (hipDeviceSynchronize() != hipSuccess || hipMemcpyFromSymbol(&cnt, HIP_SYMBOL(tpt_genstat_n), 4) != hipSuccess) return -1;
    cnt = std::min<unsigned>(cnt, (unsigned)kGenStatMax);
    const int64_t m = std::min<int64_t>(n, cnt);
    if (m > 0 && hipMemcpyFromSymbol(host, HIP_SYMBOL(tpt_genstats), (size_t)m * 5 * 8) != hipSuccess) return -1;
    if (reset) {
        const unsigned z = 0;
        if (hipMemcpyToSymbol(HIP_SYMBOL(tpt_genstat_n), &z, 4) != hipSuccess) return -1;
    }
    return (int)m;
}
#endif
#if TPT_PT_WAVETIME
// diagnostics build only: copy the PT kernel's per-wave (start, end, HW_ID) records
int tpt_diag_wavetime(unsigned long long* host, int64_t n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(tpt_wavetime), (size_t)std::min<int64_t>(n, 3 * kWaveTimeMax) * 8) == hipSuccess ? 0 : -1;
}
#endif
float tpt_camera_scale(double fov) { return camera_scale(fov); }
uint32_t tpt_sample_seed(int64_t pixel, int32_t sample) { return sample_seed(pixel, sample); }

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
        hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&c->stream3, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_start, hipEventDisableTiming) != hipSuccess ||
        hipMalloc(&c->counters, sizeof(unsigned long long) * 32) != hipSuccess ||
        hipMalloc(&c->queue, kQueueBytes) != hipSuccess ||
        hipDeviceGetAttribute(&c->num_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) {
        tpt_destroy(c);  // releases what was created
        return TPT_E_DEVICE;
    }
    for (int b = 0; b < kWfBufs; ++b) {
        if (hipEventCreateWithFlags(&c->ev_gen[b], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&c->ev_fold[b], hipEventDisableTiming) != hipSuccess) {
            tpt_destroy(c);
            return TPT_E_DEVICE;
        }
    }
    // Fail here, not in the first launch, when this device has no code object of
    // ours (the library is built for gfx950 only; there is no fallback).
    hipFuncAttributes fa;
    if (hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(tpt_scale_kernel)) != hipSuccess) {
        (void)hipGetLastError();
        tpt_destroy(c);
        return TPT_E_DEVICE;
    }
    *out = c;
    return TPT_OK;
}

void tpt_destroy(tpt_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (void* p : {(void*)c->blob, (void*)c->rgb, (void*)c->splat, (void*)c->splat_part, (void*)c->list, (void*)c->rows, (void*)c->counters,
                    (void*)c->queue, c->wf_mem, c->scan_tmp})
        if (p) (void)hipFree(p);
    if (c->stream2) (void)hipStreamSynchronize(c->stream2);
    if (c->stream3) (void)hipStreamSynchronize(c->stream3);
    for (int b = 0; b < kWfBufs; ++b)
        for (hipEvent_t e : {c->ev_gen[b], c->ev_fold[b]})
            if (e) (void)hipEventDestroy(e);
    if (c->ev_start) (void)hipEventDestroy(c->ev_start);
    if (c->stream2) (void)hipStreamDestroy(c->stream2);
    if (c->stream3) (void)hipStreamDestroy(c->stream3);
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
    if (hs.nodes.size() > (size_t)0x7fffffff) return fail(c, TPT_E_UNSUPPORTED, "too many BVH nodes");
    // LDS staging (stage_scene): every array the traversals read when it all fits in
    // 64 KB (the Cornell presets, ~6 KB: lds_full), else only the flat-query arrays --
    // materials, leaves, groups and the flat leaves' triangles (the bunny scene,
    // ~2 KB) -- with the trees read through L2.  leaves[j].b indexes the triangle
    // array flat queries read: tris itself (full) or ftris (flat-only).
    const size_t mats16 = (hs.mats.size() * sizeof(DMat) + 15) & ~(size_t)15;
    const size_t lg = (hs.leaves.size() + hs.groups.size()) * sizeof(DNode);
    const size_t full_b = hs.nodes.size() * sizeof(DNode) + hs.tris.size() * sizeof(DTri) + mats16 + lg;
    const size_t flat_b = mats16 + lg + hs.leaves.size() * sizeof(DTri);
    int lds_full = 0;
    size_t lds_b = 0;
    if (full_b <= 64 * 1024) {
        lds_full = 1;
        lds_b = full_b;
    } else if (hs.leaves.size() <= (size_t)kFlatMaxLeaves && flat_b <= 64 * 1024) {
        lds_b = flat_b;
    }
    hs.ftris.clear();
    for (size_t j = 0; j < hs.leaves.size(); ++j) {
        DNode& l = hs.leaves[j];
        const int prim = -1 - l.a;
        const bool tri = prim < (int)hs.tris.size();
        if (lds_full) {
            l.b = tri ? prim : 0;
        } else {
            l.b = (int)j;
            DTri t;
            std::memset(&t, 0, sizeof(t));
            hs.ftris.push_back(tri ? hs.tris[prim] : t);  // a sphere leaf's slot is unused
        }
    }
    std::vector<char> blob;
    size_t o_nodes = push_array(blob, hs.nodes), o_area = push_array(blob, hs.node_area),
           o_tris = push_array(blob, hs.tris), o_trix = push_array(blob, hs.trix), o_sph = push_array(blob, hs.sph),
           o_mats = push_array(blob, hs.mats), o_objs = push_array(blob, hs.objs),
           o_em = push_array(blob, hs.emitters), o_t = push_array(blob, hs.tnodes),
           o_lf = push_array(blob, hs.leaves), o_gr = push_array(blob, hs.groups), o_ft = push_array(blob, hs.ftris),
           o_q4 = push_array(blob, hs.qnodes);
    if (hs.grank.size() < hs.tris.size()) hs.grank.resize(hs.tris.size(), 0);
    const size_t o_rk = push_array(blob, hs.grank);
    if (c->blob) { (void)hipFree(c->blob); c->blob = nullptr; }
    HIP_TRY(c, hipMalloc(&c->blob, blob.size()));
    HIP_TRY(c, hipMemcpy(c->blob, blob.data(), blob.size(), hipMemcpyHostToDevice));
    char* b = (char*)c->blob;
    DScene ds;
    std::memset(&ds, 0, sizeof(ds));
    ds.nodes = (const DNode*)(b + o_nodes);
    ds.node_area = (const float*)(b + o_area);
    ds.tris = (const DTri*)(b + o_tris);
    ds.gtris = ds.tris;
    ds.trix = (const DTriX*)(b + o_trix);
    ds.sph = (const DSphere*)(b + o_sph);
    ds.mats = (const DMat*)(b + o_mats);
    ds.objs = (const DObj*)(b + o_objs);
    ds.emitters = (const int32_t*)(b + o_em);
    ds.tnodes = (const DNode*)(b + o_t);
    ds.leaves = (const DNode*)(b + o_lf);
    ds.nleaf = (int)hs.leaves.size();
    ds.groups = (const DNode*)(b + o_gr);
    ds.ngroup = (int)hs.groups.size();
    ds.ftris = lds_full ? ds.tris : (const DTri*)(b + o_ft);
    ds.qnodes = (const QNode4*)(b + o_q4);
    ds.grank = (const uint16_t*)(b + o_rk);
    ds.lds_full = lds_full;
    ds.nmats = (int)hs.mats.size();
    ds.n_emitters = (int)hs.emitters.size();
    // BVHAccel::Sample (1 draw) + Triangle::Sample (2) per mesh emitter, Sphere::Sample (2)
    ds.light_draws = 0;
    for (int e : hs.emitters) ds.light_draws += hs.objs[e].kind == TPT_OBJ_MESH ? 3 : 2;
    ds.ntri = (int)hs.tris.size();
    ds.nsph = (int)hs.sph.size();
    ds.nnodes = (int)hs.nodes.size();
    ds.nobj = (int)hs.objs.size();
    ds.width = hs.width;
    ds.height = hs.height;
    ds.scale = camera_scale(hs.fov);
    for (int k = 0; k < 6; ++k) ds.lbox[k] = hs.lbox[k];
    ds.cone_delta = hs.cone_delta;
    for (int k = 0; k < 3; ++k) { ds.eye[k] = hs.eye[k]; ds.bg[k] = hs.bg[k]; }
    ds.lds_bytes = (int)lds_b;
    // flat (all-leaves) queries for small scenes; TPT_FLAT overrides the bits: 0 walks
    // the threaded tree everywhere (the cross-check tests/test_gpu_parity.py runs)
    const char* fl = std::getenv("TPT_FLAT");
    ds.flat = fl ? std::atoi(fl) : TPT_FLAT_DEFAULT;
    if (ds.nleaf > kFlatMaxLeaves || ds.lds_bytes == 0) ds.flat = 0;
    ds.big = 0;
    for (const DNode& g : hs.groups) ds.big |= g.b < 0;
    c->sc = ds.lds_bytes == 0 ? 0 : ds.big ? 2 : 1;
    c->ds = ds;
    c->hs = std::move(hs);
    c->has_scene = true;
    return ensure_fb(c);
}

int tpt_render_device(tpt_ctx* c, const tpt_render_params* p, float* rgb_dev, float* splat_dev, tpt_stats* st) {
    if (!c || !p) return TPT_E_INVALID;
    int rc = check_render_args(c, p->spp, p->mode, p->flags);
    if (rc) return rc;
    if (p->pixel_begin < 0 || p->pixel_stride < 1) return fail(c, TPT_E_INVALID, "bad pixel shard");
    if (!rgb_dev || (p->mode == TPT_MODE_BDPT && !splat_dev)) return fail(c, TPT_E_INVALID, "null output buffer");
    HIP_TRY(c, hipSetDevice(c->device));
    auto t0 = std::chrono::steady_clock::now();
    const int64_t npix = (int64_t)c->hs.width * c->hs.height;
    HIP_TRY(c, hipMemsetAsync(rgb_dev, 0, npix * 3 * sizeof(float), c->stream));
    if (p->mode == TPT_MODE_BDPT) HIP_TRY(c, hipMemsetAsync(splat_dev, 0, npix * 3 * sizeof(float), c->stream));
    const int64_t count = shard_count(npix, p->pixel_begin, p->pixel_stride);
    rc = launch(c, p->mode, p->flags, p->spp, p->pixel_begin, p->pixel_stride, count, nullptr, rgb_dev,
                p->mode == TPT_MODE_BDPT ? splat_dev : nullptr, st);
    if (rc) return rc;
    if (st) st->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return TPT_OK;
}

int tpt_render(tpt_ctx* c, const tpt_render_params* p, float* rgb, float* splat, tpt_stats* st) {
    if (!c || !p || !rgb) return TPT_E_INVALID;
    int rc = check_render_args(c, p->spp, p->mode, p->flags);
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
    rc = launch(c, mode, 0, spp, 0, 1, n, c->list, c->rows, mode == TPT_MODE_BDPT ? c->splat : nullptr, st);
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
    if (!rc) {
        // primitive id (triangles first, then spheres) -> the scene's object-order
        // ordinal: each mesh's triangles in file order, a sphere in its Add position
        std::vector<int> ord(c->hs.tris.size() + c->hs.sph.size());
        int next = 0;
        for (size_t o = 0; o < c->hs.objs.size(); ++o) {
            const DObj& ob = c->hs.objs[o];
            if (ob.kind == TPT_OBJ_SPHERE) {
                ord[ob.sphere_prim] = next++;
            } else {
                for (size_t t = 0; t < c->hs.tri_object.size(); ++t)
                    if (c->hs.tri_object[t] == (int)o) ord[t] = next++;
            }
        }
        for (int64_t k = 0; k < n; ++k) {
            const int prim = (int)out[8 * k + 7];
            if (prim >= 0 && prim < (int)ord.size()) out[8 * k + 7] = (float)ord[prim];
        }
    }
    (void)hipFree(dr);
    (void)hipFree(dout);
    if (rc) c->err = "intersect kernel failed";
    return rc;
}

}  // extern "C"
#endif  // !TPT_TU_CONN2
