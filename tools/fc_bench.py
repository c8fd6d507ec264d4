"""Timing of the NatureCNN fc layer's GEMMs (csrc/gs_fc.hip, gs_fc_gemm) at the C4/C5 shapes
(B = 1024, HID = 512, F = 3136), fp32 and bf16 operands: 50 back-to-back launches between HIP events on
the launch stream.  Prints us per launch, TFLOP/s and the MFMA
fraction (fp32 157.3 TF, bf16 2500 TF dense)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gymnasium-solver_amd")]

import torch  # noqa: E402

from gsamd._lib import check, lib  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    B, HID, F = 1024, 512, 3136
    a3 = torch.rand(B, F, device=dev) - 0.3
    Wf = torch.randn(HID, F, device=dev) * 0.02
    dh = torch.randn(B, HID, device=dev)
    bf = torch.randn(HID, device=dev)
    h = torch.empty(B, HID, device=dev)
    dW = torch.empty(HID, F, device=dev)
    da3 = torch.empty(B, F, device=dev)
    parts = torch.empty(2 * B * F, device=dev)     # the fp32 forward's split-K partials (as the update)
    cases = {"fwd": (0, B, HID, F, a3, F, Wf, F, h, HID, bf), "wgrad": (1, HID, F, B, dh, HID, a3, F, dW, F, None),
             "dgrad": (2, B, F, HID, dh, HID, Wf, F, da3, F, a3)}
    st = torch.cuda.current_stream()
    for bf16 in (0, 1):
        for name, (op, M, N, K, A, lda, Bm, ldb, C, ldc, aux) in cases.items():
            run = lambda: check(lib.gs_fc_gemm(op, bf16, M, N, K, A.data_ptr(), lda, Bm.data_ptr(), ldb,  # noqa: E731
                                               C.data_ptr(), ldc, aux.data_ptr() if aux is not None else None,
                                               parts.data_ptr(), st.cuda_stream), "gs_fc_gemm")
            for _ in range(3):
                run()
            torch.cuda.synchronize()
            # eager back-to-back launches on the stream (each launch takes far less host time than
            # the kernel runs, so the queue never drains)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(50):
                run()
            e1.record(st)
            e1.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / 50
            tf = 2.0 * M * N * K / (us * 1e-6) / 1e12
            peak = 2500.0 if bf16 else 157.3
            print(f"{'bf16' if bf16 else 'fp32'} {name:6s} {M}x{N}x{K}: {us:8.2f} us  {tf:7.1f} TF/s  "
                  f"{tf / peak:.3f} of peak", flush=True)


if __name__ == "__main__":
    main()
