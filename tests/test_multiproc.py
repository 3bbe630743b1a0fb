"""World-size-2 rehearsal of the multi-GPU path on the CPU (gloo).

Each rank renders its interleaved pixel shard (sharding.shard, the reference's
`i = off; i += j` split, Renderer.cpp:38) -- here with the CPU restatement standing
in for the GPU kernel -- into a full-size zeroed framebuffer + splat buffer, and
rank 0 receives the sum through ONE dist.reduce, exactly the code path bench.py
runs over RCCL.  PT must equal the single-process frame bit for bit; BDPT splats
are a real sum (rounding-order tolerance)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import bits

W = H = 64  # small frame so the oracle finishes in seconds


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _render_shard(rank, world, mode, spp):
    import sharding
    from oracle_bind import Oracle
    o = Oracle("standard", W, H)
    pix = np.array(list(sharding.shard_pixels(W * H, rank, world)), np.int64)
    rows, splat, _ = o.trace_pixels(mode, spp, pix, want_splat=(mode == 1))
    rgb = np.zeros((W * H, 3), np.float32)
    rgb[pix] = rows
    sp = splat.reshape(-1, 3) if splat is not None else np.zeros_like(rgb)
    return np.stack([rgb.reshape(-1), sp.reshape(-1)])


def _worker(rank, world, port, mode, spp, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sharding
    fb = torch.from_numpy(_render_shard(rank, world, mode, spp))
    # as bench.py: PT splats nothing, so only the rgb row is summed; BDPT sums both
    sharding.reduce_frame(dist, fb if mode == 1 else fb[:1], dst=0)
    if rank == 0:
        np.save(out_path, fb.numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize("mode,spp", [(0, 4), (1, 1)])
def test_two_rank_shard_reduce(tmp_path, mode, spp):
    import sharding
    out = str(tmp_path / "fb.npy")
    mp.spawn(_worker, args=(2, _free_port(), mode, spp, out), nprocs=2, join=True)
    got = np.load(out)
    want = _render_shard(0, 1, mode, spp)
    if mode == 0:
        assert np.array_equal(bits(got), bits(want))
        assert not got[1].any()
    else:
        assert np.array_equal(bits(got[0]), bits(want[0]))  # radiance: disjoint shards
        img_g, img_w = sharding.merge(got[0], got[1]), sharding.merge(want[0], want[1])
        err = np.linalg.norm(img_g.astype(np.float64) - img_w) / np.linalg.norm(img_w.astype(np.float64))
        assert err < 1e-6


def test_shard_partition():
    import sharding
    for world in (1, 2, 3, 8):
        seen = np.zeros(1000, int)
        for r in range(world):
            for i in sharding.shard_pixels(1000, r, world):
                seen[i] += 1
        assert (seen == 1).all()
    with pytest.raises(ValueError):
        sharding.shard(2, 2)


def _bench(*args, timeout=240):
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    return subprocess.run([sys.executable, os.path.join(root, "bench.py")] + list(args), capture_output=True,
                          text=True, timeout=timeout, env=env)


def test_bench_spawns_ranks_without_a_launcher():
    """`python bench.py --gpus 2` with no WORLD_SIZE starts torch.distributed.run as a
    child (VERDICT r3 Next #1); --rehearse runs the ranks on gloo with a pattern in
    place of the renderer, and rank 0 checks the reduced frame and prints ONE line."""
    import json
    p = _bench("--gpus", "2", "--rehearse", "--steps", "2", "--warmup", "1")
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["reduce_check"] is True
    assert sorted(r["rank"] for r in line["ranks"]) == [0, 1]
    assert sum(r["pixels"] for r in line["ranks"]) == 64 * 64


def test_bench_refuses_more_gpus_than_visible():
    """On a box with fewer GPUs than --gpus the bench exits non-zero and names the
    visible-device count (here: a CPU container, 0 devices)."""
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("this box has 2+ GPUs")
    p = _bench("--gpus", "2", "--steps", "1", "--warmup", "0", timeout=120)
    assert p.returncode == 2
    assert "visible GPUs, this box has %d" % torch.cuda.device_count() in p.stderr
