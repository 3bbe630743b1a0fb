// Host-side test of the BDPT gen hand-off protocol (VERDICT r3 Next #8), with the
// device's own sequence-word functions (csrc/tpt_genseq.h).
//
// gen(f) is a "grid" of G workers taking pixel streams from a shared queue; a worker
// may start pixel k only once k's word carries f (seq_ready), runs the pixel's nb
// samples (here: XorShift32 steps, a pixel-dependent number of them) and publishes
// f + 1 with the new state (seq_publish).  Even wavefronts run on stream A, odd ones
// on stream B (each stream in order, the two concurrently), as launch_bdpt_chunk
// issues them.  A worker must hold one of R "resident slots" to run (a workgroup
// resident on the chip), and a connect-like kernel that never waits holds some slots
// for a while.  Checks:
//   1. every pixel's final state equals the serial application of all its samples, and
//      nothing deadlocks, when each gen grid holds <= R / 2 slots (gen_grid_ok);
//   2. a dropped publication (the diagnostics hook of TPT_DIAG_HOOKS) ends in the
//      watchdog: the waiting worker gives the pixel up (seq_give_up), the stall is
//      flagged, later wavefronts do not wait on it, and every other pixel is exact;
//   3. gen_grid_ok accepts exactly the grids of at most half the resident slots.
//   g++ -std=c++17 -O2 -pthread -I toypathtracer-games101-assignment7_amd/csrc tests/native/genseq_check.cpp
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <mutex>
#include <thread>
#include <vector>

#include "tpt_genseq.h"

using namespace tpt;
using Clock = std::chrono::steady_clock;

static uint32_t xs(uint32_t x) {
    x ^= x << 13;
    x ^= x >> 17;
    x ^= x << 5;
    return x;
}

struct Slots {  // counting semaphore of resident workgroup slots
    std::mutex m;
    std::condition_variable cv;
    int free;
    explicit Slots(int n) : free(n) {}
    void take() {
        std::unique_lock<std::mutex> l(m);
        cv.wait(l, [&] { return free > 0; });
        --free;
    }
    void give() {
        {
            std::lock_guard<std::mutex> l(m);
            ++free;
        }
        cv.notify_one();
    }
};

struct Run {
    int n, frames, nb, grid, resident, drop_k, drop_f;
    std::chrono::milliseconds watchdog;
    std::vector<std::atomic<unsigned long long>> seq;
    std::atomic<int> stall{0};
    Run(int n_, int frames_, int nb_, int grid_, int resident_, int drop_k_, int drop_f_, int wd_ms)
        : n(n_), frames(frames_), nb(nb_), grid(grid_), resident(resident_), drop_k(drop_k_), drop_f(drop_f_),
          watchdog(wd_ms), seq(n_) {}
    static int steps(int k) { return 3 + k % 7; }  // XorShift draws per sample (pixel-dependent)
};

static void gen(Run& r, Slots& slots, int f) {
    std::atomic<int> q{0};
    std::vector<std::thread> wg;
    for (int g = 0; g < r.grid; ++g)
        wg.emplace_back([&] {
            slots.take();  // resident from here until the worker's queue is drained
            for (;;) {
                const int k = q.fetch_add(1);
                if (k >= r.n) break;
                uint32_t st = 0;
                if (f == 0) {
                    st = (uint32_t)k + 1;  // ResetRandom(i + 1)
                } else {
                    const auto t0 = Clock::now();
                    bool ok = true;
                    for (;;) {
                        const unsigned long long v = r.seq[k].load(std::memory_order_acquire);
                        if (seq_ready(v, f)) {
                            st = seq_state(v);
                            break;
                        }
                        if (Clock::now() - t0 > r.watchdog) {  // give up: publish so later wavefronts go on
                            r.seq[k].store(seq_give_up(f), std::memory_order_release);
                            r.stall.store(1);
                            ok = false;
                            break;
                        }
                        std::this_thread::yield();
                    }
                    if (!ok) continue;
                }
                for (int b = 0; b < r.nb; ++b)
                    for (int d = 0; d < Run::steps(k); ++d) st = xs(st);
                if (k == r.drop_k && f == r.drop_f) continue;  // the diagnostics hook: never published
                r.seq[k].store(seq_publish(f, st), std::memory_order_release);
            }
            slots.give();
        });
    for (auto& t : wg) t.join();
}

// Streams A (even wavefronts) and B (odd ones), concurrent; a connect-like hog takes
// `hog` slots for a while at the start and never waits on anything.
static bool run(Run& r, int hog, double limit_s) {
    Slots slots(r.resident);
    std::atomic<bool> done{false};
    std::thread hogger([&] {
        for (int i = 0; i < hog; ++i) slots.take();
        std::this_thread::sleep_for(std::chrono::milliseconds(30));
        for (int i = 0; i < hog; ++i) slots.give();
    });
    std::thread a([&] { for (int f = 0; f < r.frames; f += 2) gen(r, slots, f); });
    std::thread b([&] {
        for (int f = 1; f < r.frames; f += 2) gen(r, slots, f);
    });
    const auto t0 = Clock::now();
    std::thread watch([&] {
        while (!done.load() && std::chrono::duration<double>(Clock::now() - t0).count() < limit_s)
            std::this_thread::sleep_for(std::chrono::milliseconds(5));
    });
    a.join();
    b.join();
    hogger.join();
    const bool in_time = std::chrono::duration<double>(Clock::now() - t0).count() < limit_s;
    done.store(true);
    watch.join();
    return in_time;
}

int main() {
    int fails = 0;
    auto expect = [&](bool c, const char* what) {
        std::printf("%s: %s\n", c ? "ok  " : "FAIL", what);
        fails += !c;
    };
    // 1. exactness and progress at the invariant's limit (grid = resident / 2), with a
    //    hog holding the rest of the slots at the start
    {
        Run r(4096, 8, 3, 4, 8, -1, -1, 2000);
        const bool t = run(r, 4, 20.0);
        bool exact = true;
        for (int k = 0; k < r.n; ++k) {
            uint32_t st = (uint32_t)k + 1;
            for (int f = 0; f < r.frames * r.nb; ++f)
                for (int d = 0; d < Run::steps(k); ++d) st = xs(st);
            exact &= r.seq[k].load() == seq_publish(r.frames - 1, st);
        }
        expect(t, "two gen streams at grid = resident / 2 finish (no deadlock)");
        expect(exact, "every pixel's final word = (frames, serial XorShift state)");
        expect(r.stall.load() == 0, "no watchdog in a good run");
    }
    // 2. a dropped publication: the watchdog takes over, the rest stays exact
    {
        Run r(512, 6, 2, 2, 4, 17, 1, 50);
        const bool t = run(r, 0, 20.0);
        bool others = true;
        for (int k = 0; k < r.n; ++k) {
            if (k == 17) continue;
            uint32_t st = (uint32_t)k + 1;
            for (int f = 0; f < r.frames * r.nb; ++f)
                for (int d = 0; d < Run::steps(k); ++d) st = xs(st);
            others &= r.seq[k].load() == seq_publish(r.frames - 1, st);
        }
        uint32_t st = 1;  // seq_give_up at wavefront 2, then wavefronts 3..5 run on
        for (int f = 3; f < r.frames; ++f)
            for (int b = 0; b < r.nb; ++b)
                for (int d = 0; d < Run::steps(17); ++d) st = xs(st);
        expect(t, "a dropped publication does not hang the pipeline");
        expect(r.stall.load() == 1, "the watchdog flags the stall");
        expect(r.seq[17].load() == seq_publish(r.frames - 1, st), "the given-up pixel continues from state 1");
        expect(others, "every other pixel is exact");
    }
    // 3. the invariant the library checks before a two-stream launch
    expect(gen_grid_ok(512, 1024) && !gen_grid_ok(513, 1024) && gen_grid_ok(0, 1), "gen_grid_ok = grid <= resident / 2");
    expect(seq_ready(seq_publish(4, 0xdeadbeefu), 5) && !seq_ready(seq_publish(4, 7u), 4) &&
               seq_state(seq_publish(9, 0xdeadbeefu)) == 0xdeadbeefu && seq_state(seq_give_up(3)) == 1u,
           "sequence words: f + 1 with the state, in one 64-bit word");
    std::printf("%s\n", fails ? "FAILED" : "ALL OK");
    return fails != 0;
}
