"""Pixel sharding across ranks + framebuffer reduce.

The reference splits pixels over CPU threads by interleaving (`for (i = off; i <
pixelCount; i += threadCount)`, Renderer.cpp:38) and merges the per-thread splat
buffers after the radiance (Renderer.cpp:98-114).  Across GPUs the same interleave
is used: rank r renders pixels i = r, r + N, r + 2N, ... into a full-size, zeroed
framebuffer (plus a splat buffer for BDPT), and the buffers are summed onto rank 0
with ONE collective (dist.reduce, RCCL over xGMI on MI355X; gloo in the CPU tests).
PT shards are disjoint, so the sum equals the 1-GPU frame bit for bit (x + 0 = x);
BDPT splats land anywhere and are a genuine sum.

The per-rank RNG streams are untouched (a pixel's stream starts at ResetRandom(i+1)
whichever rank renders it), which is why the frame does not depend on N.
"""


def shard(rank, world):
    """(pixel_begin, pixel_stride) of `rank` among `world` ranks (Renderer.cpp:38)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world: %r/%r" % (rank, world))
    return rank, world


def shard_pixels(npix, rank, world):
    begin, stride = shard(rank, world)
    return range(begin, npix, stride)


def reduce_frame(dist, fb, dst=0):
    """Sum the rank-local framebuffer(s) `fb` (one contiguous tensor: [2, H*W*3] rgb +
    splat for BDPT, the [1, H*W*3] rgb row for PT, which splats nothing) onto `dst`
    with a single collective."""
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        dist.reduce(fb, dst=dst)
    return fb


def shard_model(render, ns=(2, 4, 8), full=None):
    """One-GPU model of the N-way split.  `render(begin, stride)` renders one shard
    alone and returns (kernel_ms, wall_ms).  For each N every shard r = 0..N-1 is
    rendered in turn (the frame rank r of an N-GPU run would render); the model is

        T_N = max_r T(shard r of N),   eff_N = T_1 / (N * T_N)

    with T_1 the whole frame's time: eff_N = 1 when the split costs nothing (the work
    divides evenly and no per-launch cost fails to shrink).  Both the device time
    (HIP events around the kernels) and the wall time of the synchronous call are
    reported; the reduce is not part of the model.  `full`: the whole frame's (kernel_ms,
    wall_ms) when the caller has just measured it."""
    k1, w1 = full if full is not None else render(0, 1)
    out = {"full_kernel_ms": round(k1, 3), "full_wall_ms": round(w1, 3)}
    for n in ns:
        ks, ws = zip(*[render(r, n) for r in range(n)])
        out["n%d" % n] = {"kernel_ms": [round(k, 3) for k in ks], "wall_ms": [round(w, 3) for w in ws],
                          "slowest_rank": int(max(range(n), key=lambda r: ks[r])),
                          "eff_kernel": round(k1 / (n * max(ks)), 4), "eff_wall": round(w1 / (n * max(ws)), 4),
                          "imbalance": round(max(ks) / (sum(ks) / n), 4)}
    return out


def merge(rgb, splat):
    """Renderer.cpp:98-114: framebuffer[j] += splat[j] after the radiance."""
    return rgb + splat if splat is not None else rgb
