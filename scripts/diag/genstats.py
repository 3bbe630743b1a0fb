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
L.tpt_diag_walkstats.argtypes = [ctypes.c_void_p, ctypes.c_int]
for rep in range(2):
    buf = np.zeros((1 << 16, 5), np.uint64)
    ws = np.zeros(8, np.uint64)
    L.tpt_diag_genstats(None, 0, 1)
    L.tpt_diag_walkstats(ws.ctypes.data, 1)
    st = ctx.render_device(spp, pytpt.MODE_BDPT, fb[0].data_ptr(), fb[1].data_ptr(), 0, n)
    m = L.tpt_diag_genstats(buf.ctypes.data, buf.shape[0], 1)
    L.tpt_diag_walkstats(ws.ctypes.data, 1)
    print("  wave-steps %d, mean step %.2f us; walks %d (%.1f lanes each), mean walk %.2f us, walk share of step time %.2f" % (
        ws[4], ws[3] / max(ws[4], 1) / 100.0, ws[1], ws[2] / max(ws[1], 1), ws[0] / max(ws[1], 1) / 100.0,
        ws[0] / max(ws[3], 1)))
    print("  walk iterations per walking lane %.1f, per walk (wave max) %.1f" % (ws[5] / max(ws[2], 1), ws[6] / max(ws[1], 1)))
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
