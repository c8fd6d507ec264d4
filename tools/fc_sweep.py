"""Launch-shape sweep of the NatureCNN fc products (csrc/gs_fc.hip gs_debug_fc_variant, a
GS_FC_SWEEP diagnostic build) at the C4 / C5 shapes (B = 1024, HID = 512, F = 3136): every variant
checked against a float64 reference (the bar of tests/test_gpu_gemm.py::_fc_case), then timed over
50 back-to-back launches between HIP events.  Prints one JSON object per (op, precision, variant).

  GSAMD_LIB=sweeplibs/libgsamd_fcsweep.so python tools/fc_sweep.py"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gymnasium-solver_amd")]

import torch  # noqa: E402

from gsamd._lib import lib  # noqa: E402

NAMES = {0: "fwd", 1: "wgrad", 2: "dgrad"}


def main():
    fn = lib.gs_debug_fc_variant
    vp, i64 = ctypes.c_void_p, ctypes.c_int64
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, i64, i64, i64, vp, i64, vp, i64, vp, i64, vp, vp, vp]
    dev = torch.device("cuda:0")
    B, HID, F = 1024, 512, 3136
    g = torch.Generator(device="cpu").manual_seed(0)
    shapes = {0: (B, HID, F), 1: (HID, F, B), 2: (B, F, HID)}
    st = torch.cuda.current_stream()
    parts = torch.empty(16 * B * F, device=dev)
    for op in (0, 1, 2):
        M, N, K = shapes[op]
        if op == 0:
            A, Bm, aux = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g), torch.randn(N, generator=g)
            opA, opB = A, Bm.t()
        elif op == 1:
            A, Bm, aux = torch.randn(K, M, generator=g), torch.randn(K, N, generator=g), None
            opA, opB = A.t(), Bm
        else:
            A, Bm, aux = torch.randn(M, K, generator=g), torch.randn(K, N, generator=g), torch.randn(M, N, generator=g)
            opA, opB = A, Bm
        Ad, Bd = A.to(dev), Bm.to(dev)
        auxd = aux.to(dev) if aux is not None else None
        for bf16 in (0, 1):
            rd = (lambda t: t.to(torch.bfloat16).double()) if bf16 else (lambda t: t.double())
            ref = rd(opA) @ rd(opB)
            if op == 0:
                ref = (ref + aux.double()).clamp_min(0)
            elif op == 2:
                ref = torch.where(aux.double() > 0, ref, torch.zeros_like(ref))
            scale = (rd(opA).abs() @ rd(opB).abs()).max().item() + 1.0
            bar = 2e-6 * scale * max(1.0, K ** 0.5 / 8)
            for v in range(10):
                out = torch.full((M, N), float("nan"), device=dev)

                def run():
                    return fn(op, v, bf16, M, N, K, Ad.data_ptr(), Ad.shape[1], Bd.data_ptr(), Bd.shape[1],
                              out.data_ptr(), N, auxd.data_ptr() if auxd is not None else None, parts.data_ptr(),
                              st.cuda_stream)
                if run() != 0:
                    continue
                torch.cuda.synchronize()
                err = (out.cpu().double() - ref).abs().max().item()
                for _ in range(3):
                    run()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(50):
                    run()
                e1.record(st)
                e1.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / 50
                tf = 2.0 * M * N * K / (us * 1e-6) / 1e12
                print(json.dumps({"op": NAMES[op], "bf16": bf16, "variant": v, "us": round(us, 2),
                                  "TFLOPs": round(tf, 1), "frac": round(tf / (2500.0 if bf16 else 157.3), 3),
                                  "err_over_bar": round(err / bar, 3), "ok": bool(err <= bar)}), flush=True)


if __name__ == "__main__":
    main()
