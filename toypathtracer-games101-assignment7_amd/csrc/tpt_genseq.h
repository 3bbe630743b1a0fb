// tpt_genseq.h -- the BDPT gen hand-off's per-pixel sequence words (WfState::rngseq),
// shared by the gen kernel (tpt_capi.hip) and the host-side protocol test
// (tests/native/genseq_check.cpp).
//
// A pixel stream's word is (wavefronts completed) << 32 | XorShift32 state.  gen(f)
// may start pixel k only once the word carries f; when it has run k's samples it
// publishes f + 1 with the new state in ONE 64-bit store, so a reader never sees the
// sequence number of one wavefront with the state of another.  A lane whose wait
// exceeds the watchdog gives the pixel up and publishes f + 1 with state 1 (a valid
// XorShift32 state), so later wavefronts do not wait on it too; the render is then
// reported as failed.
#pragma once

#include <cstdint>

#if defined(__HIPCC__)
#define TPT_GS_HD __host__ __device__ inline
#else
#define TPT_GS_HD inline
#endif

namespace tpt {
TPT_GS_HD bool seq_ready(unsigned long long word, int batch) { return (word >> 32) == (unsigned long long)batch; }
TPT_GS_HD uint32_t seq_state(unsigned long long word) { return (uint32_t)word; }
TPT_GS_HD unsigned long long seq_publish(int batch, uint32_t state) {
    return (unsigned long long)(batch + 1) << 32 | state;
}
TPT_GS_HD unsigned long long seq_give_up(int batch) { return seq_publish(batch, 1u); }
// The two-stream hand-off cannot deadlock while gen(f - 1) can always be scheduled:
// gen(f) spins on at most its own grid, so each gen grid may hold at most half of the
// workgroups resident at once (connect never waits and frees its slots as it ends).
TPT_GS_HD bool gen_grid_ok(long long grid, long long resident) { return 2 * grid <= resident; }
}  // namespace tpt
