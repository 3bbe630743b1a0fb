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


def merge(rgb, splat):
    """Renderer.cpp:98-114: framebuffer[j] += splat[j] after the radiance."""
    return rgb + splat if splat is not None else rgb
