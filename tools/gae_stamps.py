"""Diagnostic: per-role cycle breakdown of the staged GAE scan (GS_STAMPS build, block 0).

    python tools/gae_stamps.py --build      # here: builds tools/libgsamd_stamps.so
    python tools/gae_stamps.py T N          # on the GPU box
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gymnasium-solver_amd")]
VARIANT = os.path.join(ROOT, "tools", "libgsamd_stamps.so")
if "--build" in sys.argv:
    import build_lib
    build_lib.build_variant(VARIANT, ["GS_STAMPS"])
    print("built", VARIANT)
    sys.exit(0)
os.environ["GSAMD_LIB"] = VARIANT
import numpy as np  # noqa: E402
import torch  # noqa: E402
from gsamd import _lib  # noqa: E402
from gsamd.rollout import compute_batched_gae_advantages_and_returns as gae  # noqa: E402

T, N = int(sys.argv[1]), int(sys.argv[2])
dev = torch.device("cuda:0")
v, r, b = (torch.randn(T, N, device=dev) for _ in range(3))
d = (torch.rand(T, N, device=dev) < 0.05).to(torch.uint8)
to = (d.bool() & (torch.rand(T, N, device=dev) < 0.3)).to(torch.uint8)
lv = torch.randn(N, device=dev)
f = _lib.lib.gs_debug_gae_stamps
f.argtypes = [ctypes.c_void_p]
a0 = np.zeros(12, np.uint64)
gae(v, r, d, to, lv, b, 0.99, 0.95)
torch.cuda.synchronize()
f(a0.ctypes.data)
reps = 10
for _ in range(reps):
    gae(v, r, d, to, lv, b, 0.99, 0.95)
torch.cuda.synchronize()
a1 = np.zeros(12, np.uint64)
f(a1.ctypes.data)
acc = ((a1 - a0).astype(np.float64) / reps).reshape(3, 4)
nC = (T + 63) // 64
for role, name in enumerate(("scanner", "loader", "helpers(w2,w3)")):
    print(f"{name:16s} work {acc[role, 0] / nC:8.0f}  barrier {acc[role, 1] / nC:8.0f}  vmcnt {acc[role, 2] / nC:8.0f}"
          f"  cycles per chunk ({nC} chunks)")
