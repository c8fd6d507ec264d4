#!/usr/bin/env python3
"""Time gs_gemm_f32 against torch.matmul (hipBLASLt/rocBLAS) on the NatureCNN GEMM shapes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "gymnasium-solver_amd")):
    sys.path.insert(0, p)
import torch  # noqa: E402

from gsamd._lib import check, lib  # noqa: E402

B = 1024
SHAPES = [  # name, ta, tb, M, N, K
    ("conv1 fwd", 0, 1, B * 400, 32, 256), ("conv2 fwd", 0, 1, B * 81, 64, 512), ("conv3 fwd", 0, 1, B * 49, 64, 576),
    ("fc fwd", 0, 1, B, 512, 3136), ("fc wgrad", 1, 0, 512, 3136, B), ("fc dgrad", 0, 0, B, 3136, 512),
    ("conv3 dgrad", 0, 0, B * 49, 576, 64), ("conv2 dgrad", 0, 0, B * 81, 512, 64),
    ("conv3 wgrad/32", 1, 0, 64, 576, B * 49 // 32), ("conv1 wgrad/32", 1, 0, 32, 256, B * 400 // 32),
]


def t_ms(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    for name, ta, tb, M, N, K in SHAPES:
        A = torch.randn((K, M) if ta else (M, K), device=dev)
        Bm = torch.randn((N, K) if tb else (K, N), device=dev)
        C = torch.empty(M, N, device=dev)
        opA = A.t() if ta else A
        opB = Bm.t() if tb else Bm
        mine = t_ms(lambda: check(lib.gs_gemm_f32(ta, tb, M, N, K, A.data_ptr(), A.shape[1], Bm.data_ptr(),
                                                  Bm.shape[1], C.data_ptr(), N, 0.0, None, 0, s), "gemm"))
        ref = t_ms(lambda: torch.matmul(opA, opB, out=C))
        fl = 2.0 * M * N * K
        print(f"{name:16s} M={M:7d} N={N:5d} K={K:6d}  gs {mine*1e3:8.1f} us ({fl/mine/1e9:6.1f} TF)   "
              f"torch {ref*1e3:8.1f} us ({fl/ref/1e9:6.1f} TF)", flush=True)


if __name__ == "__main__":
    main()
