"""PT per-wave timing (diagnostics build, -DTPT_PT_WAVETIME=1): render a full frame and a
1/8 shard, dump per-wave start / end, summarise the distribution of wave durations,
per-block spans and the kernel's tail.   TPT_LIB=variants/wt/libtpt.so python scripts/diag/pt_wavetime.py"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "toypathtracer-games101-assignment7_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import pytpt  # noqa: E402

L = pytpt.lib()
L.tpt_diag_wavetime.argtypes = [ctypes.c_void_p, ctypes.c_int64]
ctx = pytpt.Context(0)
ctx.upload(pytpt.Preset(sys.argv[1] if len(sys.argv) > 1 else "standard"))
fb = torch.zeros(2, 784 * 784 * 3, device="cuda")
out = {}
for n in (1, 8):
    ctx.render_device(1024, pytpt.MODE_PT, fb[0].data_ptr(), fb[1].data_ptr(), 0, n)  # warm
    st = ctx.render_device(1024, pytpt.MODE_PT, fb[0].data_ptr(), fb[1].data_ptr(), 0, n)
    count = (784 * 784 + n - 1) // n
    q = 16 if count <= 400000 else 8  # launch(): TPT_PT_SMALL_PIXELS
    nw = (count * q + 63) // 64
    buf = np.zeros(3 * (1 << 17), np.uint64)
    assert L.tpt_diag_wavetime(ctypes.c_void_p(buf.ctypes.data), buf.size) == 0
    r = buf.reshape(-1, 3)[:nw].astype(np.int64)
    t0 = r[:, 0].min()
    s, e = (r[:, 0] - t0) / 100.0, (r[:, 1] - t0) / 100.0  # us (100 MHz counter)
    d = e - s
    nb4 = len(d) // 4 * 4
    blk = d[:nb4].reshape(-1, 4)
    bspan = (e[:nb4].reshape(-1, 4).max(1) - s[:nb4].reshape(-1, 4).min(1))
    xcc = (r[:, 2] >> 32) & 15
    out["n%d" % n] = {"kernel_ms": st.kernel_ms, "waves": int(nw), "lanes_per_pixel": q, "span_us": float(e.max()),
                      "wave_us_mean": float(d.mean()), "wave_us_p50": float(np.median(d)),
                      "wave_us_p99": float(np.quantile(d, 0.99)), "wave_us_max": float(d.max()),
                      "block_span_mean": float(bspan.mean()), "block_span_max": float(bspan.max()),
                      "block_wave_imbalance": float((blk.max(1) / np.maximum(blk.mean(1), 1e-9)).mean()),
                      "last_start_us": float(s.max()), "end_p50_us": float(np.median(e)),
                      "xcc_busy_us": [float(d[xcc == x].sum()) for x in range(8)],
                      "busy_frac": float(d.sum() / (e.max() * 5120))}
    np.save(os.path.join(ROOT, "gpurun_out", "wavetime_n%d.npy" % n), r)
print(json.dumps(out, indent=1))
