"""TPT_FLAG_SAMPLE_SEED, the per-sample-seeding throughput mode (SURVEY.md §8f rank 4;
include/tpt.h).  It is NOT the reference's replay: sample j of pixel i starts its own
XorShift32 stream at tpt_sample_seed(i, j) instead of continuing ResetRandom(i + 1)'s
stream (Renderer.cpp:42).  Pinned two ways: the GPU against the oracle's restatement of
the same seeding (bit-exact, tests/test_gpu_parity.py), and the seeded estimator against
the reference's replay (same expectation: sums over pixels agree within Monte-Carlo
noise; the bounds below hold with a 4x margin over the observed differences)."""
import numpy as np

import pytpt
from oracle_bind import Oracle


def test_seed_function_matches_the_oracle():
    o = Oracle("standard")
    L = pytpt.lib()
    rng = np.random.default_rng(3)
    cases = [(0, 0), (1, 0), (0, 1), (784 * 784 - 1, 4095), (2**31 - 2, 2**31 - 1)]
    cases += [(int(i), int(j)) for i, j in zip(rng.integers(0, 1 << 31, 200), rng.integers(0, 1 << 31, 200))]
    for i, j in cases:
        a = L.tpt_sample_seed(i, j)
        assert a == o.sample_seed(i, j) and a != 0, (i, j)
    # distinct seeds for the samples of one pixel and for neighbouring pixels
    seeds = {L.tpt_sample_seed(i, j) for i in range(64) for j in range(64)}
    assert len(seeds) == 64 * 64


def test_seeded_pt_estimates_the_reference_image():
    o = Oracle("standard")
    pix = np.sort(np.random.default_rng(1).choice(784 * 784, 64, replace=False))
    replay = o.trace_pixels(pytpt.MODE_PT, 512, pix)[0].astype(np.float64)
    seeded = o.trace_pixels_seeded(pytpt.MODE_PT, 512, pix, 1)[0].astype(np.float64)
    assert not np.array_equal(replay, seeded)  # different random numbers ...
    rel = np.abs(replay.sum(0) - seeded.sum(0)) / replay.sum(0)
    assert rel.max() < 0.01, rel  # ... same estimator (observed 0.21 %)


def test_seeded_pt_indirect_estimates_the_reference_image():
    o = Oracle("standard")
    pix = np.sort(np.random.default_rng(2).choice(784 * 784, 256, replace=False))
    replay = o.trace_pixels(pytpt.MODE_PT_INDIRECT, 256, pix)[0].astype(np.float64)
    seeded = o.trace_pixels_seeded(pytpt.MODE_PT_INDIRECT, 256, pix, 8)[0].astype(np.float64)
    rel = np.abs(replay.sum(0) - seeded.sum(0)) / replay.sum(0)
    assert rel.max() < 0.015, rel  # observed 0.38 %
