"""Does the process keep a usable HIP context after the 2400x1800 BDPT render
(test_bdpt_wavefront_chunks)?  Prints each step's outcome."""
import os
import sys
import ctypes

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "toypathtracer-games101-assignment7_amd"))
import pytpt  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
def last():
    e = hip.hipGetLastError()
    hip.hipGetErrorString.restype = ctypes.c_char_p
    return e, hip.hipGetErrorString(e).decode()
def count():
    n = ctypes.c_int(-1)
    e = hip.hipGetDeviceCount(ctypes.byref(n))
    return e, n.value
print("start", count(), last(), flush=True)
big = len(sys.argv) > 1 and sys.argv[1] == "big"
c = pytpt.Context(0)
if big:
    c.upload(pytpt.Preset("standard", 2400, 1800))
    rgb, splat, st = c.render(1, pytpt.MODE_BDPT)
    print("big render", st.samples, count(), last(), flush=True)
else:
    c.upload(pytpt.Preset("standard"))
    rgb, splat, st = c.render(4, pytpt.MODE_BDPT)
    print("small render", st.samples, count(), last(), flush=True)
c.close()
print("closed", count(), last(), flush=True)
import torch
print("torch count", torch.cuda.device_count(), flush=True)
try:
    x = torch.zeros(4, device="cuda")
    print("torch ok", float(x.sum()), flush=True)
except Exception as e:
    print("torch fail", e, flush=True)
try:
    m = pytpt.Multi([0])
    print("multi ok", flush=True)
    m.close()
except Exception as e:
    print("multi fail", e, flush=True)
