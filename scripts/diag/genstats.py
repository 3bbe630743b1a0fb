"""Per-wave gen loop statistics of one stride-N BDPT shard (a TPT_GEN_STATS build via TPT_LIB).
    TPT_LIB=variants/X/libtpt.so python scripts/diag/genstats.py SCENE SPP N"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "toypathtracer-games101-assignment7_amd"))
import torch  # noqa: E402
import pytpt  # noqa: E402

scene, spp, n = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
L = pytpt.lib()
L.tpt_diag_genstats.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int]
ctx = pytpt.Context(0)
ctx.upload(pytpt.Preset(scene))
fb = torch.zeros(2, 784 * 784 * 3, device="cuda")
for rep in range(2):
    buf = np.zeros((1 << 16, 5), np.uint64)
    L.tpt_diag_genstats(None, 0, 1)
    st = ctx.render_device(spp, pytpt.MODE_BDPT, fb[0].data_ptr(), fb[1].data_ptr(), 0, n)
    m = L.tpt_diag_genstats(buf.ctypes.data, buf.shape[0], 1)
    a = buf[:m].astype(np.float64)
    kind = (buf[:m, 0] & 255).astype(int)
    print("render %d: kernel %.2f ms, %d wave records" % (rep, st.kernel_ms, m))
    for kd in sorted(set(kind)):
        r = a[kind == kd]
        it, ls, idle, t = r[:, 1], r[:, 2], r[:, 3], r[:, 4] / 100.0  # us
        print("  kind %d: waves %d  step iters/wave %.0f  lanes/step %.1f  idle iters/wave %.0f  "
              "wave time %.0f us  us/step-iter %.2f  lane-steps total %.3g" % (
                  kd, len(r), it.mean(), ls.sum() / max(it.sum(), 1), idle.mean(), t.mean(),
                  t.sum() / max(it.sum() + idle.sum(), 1), ls.sum()))
