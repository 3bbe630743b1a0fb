"""torch / RCCL initialisation in a process that holds an open libtpt context.
    python scripts/diag/torch_after_ctx.py MODE(pt|bdpt|none) [import_torch_first]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "toypathtracer-games101-assignment7_amd"))
if len(sys.argv) > 2:
    import torch  # noqa: F401
import pytpt  # noqa: E402

mode = sys.argv[1]
c = pytpt.Context(0)
c.upload(pytpt.Preset("standard"))
if mode != "none":
    c.render(2, pytpt.MODE_BDPT if mode == "bdpt" else pytpt.MODE_PT)
import torch  # noqa: E402
try:
    print(mode, "torch", float(torch.zeros(4, device="cuda").sum()), flush=True)
except Exception as e:
    print(mode, "torch FAIL", e, flush=True)
try:
    m = pytpt.Multi([0])
    m.close()
    print(mode, "multi ok", flush=True)
except Exception as e:
    print(mode, "multi FAIL", e, flush=True)
c.close()
