"""Render one stride-N shard (or the full frame) for kernel-trace diagnostics.
    python scripts/diag/shard_run.py SCENE MODE SPP N [RANK] [REPEAT]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "toypathtracer-games101-assignment7_amd"))
import torch  # noqa: E402
import pytpt  # noqa: E402

scene, mode, spp, n = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
rank = int(sys.argv[5]) if len(sys.argv) > 5 else 0
rep = int(sys.argv[6]) if len(sys.argv) > 6 else 1
ctx = pytpt.Context(0)
ctx.upload(pytpt.Preset(scene))
fb = torch.zeros(2, 784 * 784 * 3, device="cuda")
m = {"pt": pytpt.MODE_PT, "bdpt": pytpt.MODE_BDPT}[mode]
for _ in range(rep):
    st = ctx.render_device(spp, m, fb[0].data_ptr(), fb[1].data_ptr(), rank, n)
    print("kernel_ms %.3f" % st.kernel_ms, flush=True)
