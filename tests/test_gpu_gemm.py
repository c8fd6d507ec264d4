"""GPU: the hand-written fp32 MFMA GEMM (csrc/gs_gemm.hip) against torch fp32 matmul on the
same device (fp32 reference of the same op; tolerance 2e-5 relative to the row's |A||B| scale:
fp32 accumulation in a different order)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _check(cuda, ta, tb, M, N, K, beta=0.0, bias=False, relu=False, lda_pad=0, ldb_pad=0):
    from gsamd._lib import check, lib
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N * 3 + K)
    a_rows, a_cols = (K, M) if ta else (M, K)
    b_rows, b_cols = (N, K) if tb else (K, N)
    A = torch.randn(a_rows, a_cols + lda_pad, generator=g).to(cuda)
    Bm = torch.randn(b_rows, b_cols + ldb_pad, generator=g).to(cuda)
    C = torch.randn(M, N, generator=g).to(cuda)
    bv = torch.randn(N, generator=g).to(cuda) if bias else None
    opA = A[:, :a_cols].t() if ta else A[:, :a_cols]
    opB = Bm[:, :b_cols].t() if tb else Bm[:, :b_cols]
    ref = opA.double() @ opB.double() + beta * C.double()
    if bias:
        ref = ref + bv.double()
    if relu:
        ref = ref.clamp_min(0)
    out = C.clone()
    check(lib.gs_gemm_f32(int(ta), int(tb), M, N, K, A.data_ptr(), A.shape[1], Bm.data_ptr(), Bm.shape[1],
                          out.data_ptr(), N, float(beta), bv.data_ptr() if bias else None, int(relu),
                          torch.cuda.current_stream().cuda_stream), "gs_gemm_f32")
    torch.cuda.synchronize()
    scale = (opA.abs().double() @ opB.abs().double()).max().item() + 1.0
    err = (out.double() - ref).abs().max().item()
    assert err <= 2e-6 * scale * max(1.0, K ** 0.5 / 8), (ta, tb, M, N, K, err, scale)


@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("M,N,K", [(64, 64, 16), (130, 70, 37), (1, 1, 1), (1000, 32, 256), (257, 512, 64),
                                   (18, 512, 1024)])
def test_gemm_matches_fp64_reference(cuda, ta, tb, M, N, K):
    _check(cuda, ta, tb, M, N, K)


def test_gemm_epilogue_and_unaligned_ld(cuda):
    _check(cuda, False, True, 300, 64, 576, bias=True, relu=True)
    _check(cuda, True, False, 18, 512, 100, lda_pad=1)          # lda = 19 (the heads' dz rows)
    _check(cuda, False, False, 77, 45, 33, beta=1.0, ldb_pad=3)
