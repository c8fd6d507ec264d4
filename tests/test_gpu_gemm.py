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


def _fc_case(cuda, op, bf16, M, N, K, seed=0, split=False):
    """gs_fc_gemm (csrc/gs_fc.hip, the NatureCNN fc layer's kernels) against a float64 reference
    on the same operands (bf16: the operands rounded to bf16 first, as the kernel rounds them;
    fp32 accumulation either way).  Bar: 2e-6 x the |A||B| scale (x sqrt(K)/8 for long K)."""
    from gsamd._lib import check, lib
    g = torch.Generator(device="cpu").manual_seed(seed + 131 * op + 7 * M + N + K)
    if op == 0:
        A, B = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g)
        aux = torch.randn(N, generator=g)
        opA, opB = A, B.t()
    elif op == 1:
        A, B = torch.randn(K, M, generator=g), torch.randn(K, N, generator=g)
        aux, opA, opB = None, A.t(), B
    else:
        A, B = torch.randn(M, K, generator=g), torch.randn(K, N, generator=g)
        aux = torch.randn(M, N, generator=g)
        opA, opB = A, B
    rd = (lambda t: t.to(torch.bfloat16).double()) if bf16 else (lambda t: t.double())
    ref = rd(opA) @ rd(opB)
    if op == 0:
        ref = (ref + aux.double()).clamp_min(0)
    elif op == 2:
        ref = torch.where(aux.double() > 0, ref, torch.zeros_like(ref))
    out = torch.full((M, N), float("nan"), device=cuda)
    Ad, Bd = A.to(cuda), B.to(cuda)
    auxd = aux.to(cuda) if aux is not None else None
    parts = torch.full((2 * M * N,), float("nan"), device=cuda) if split else None
    check(lib.gs_fc_gemm(op, int(bf16), M, N, K, Ad.data_ptr(), Ad.shape[1], Bd.data_ptr(), Bd.shape[1],
                         out.data_ptr(), N, auxd.data_ptr() if auxd is not None else None,
                         parts.data_ptr() if split else None, torch.cuda.current_stream().cuda_stream), "gs_fc_gemm")
    torch.cuda.synchronize()
    scale = (rd(opA).abs() @ rd(opB).abs()).max().item() + 1.0
    err = (out.cpu().double() - ref).abs().max().item()
    assert err <= 2e-6 * scale * max(1.0, K ** 0.5 / 8), (op, bf16, M, N, K, err, scale)


@pytest.mark.parametrize("bf16", [False, True])
@pytest.mark.parametrize("op,M,N,K", [(0, 1024, 512, 3136), (1, 512, 3136, 1024), (2, 1024, 3136, 512),
                                      (0, 100, 72, 192), (1, 36, 100, 128), (2, 68, 92, 64), (0, 4, 4, 64)])
def test_fc_gemm_matches_fp64_reference(cuda, op, M, N, K, bf16):
    """The NatureCNN fc GEMMs at the C4/C5 shapes (B = 1024, HID = 512, F = 3136: forward with the
    bias + ReLU epilogue, weight gradient, input gradient with the relu' mask) and ragged M / N
    tiles, fp32 and bf16 operands."""
    _fc_case(cuda, op, bf16, M, N, K)


@pytest.mark.parametrize("M,N,K", [(1024, 512, 3136), (100, 72, 192), (4, 4, 64), (68, 92, 128)])
def test_fc_forward_split_form_matches_fp64_reference(cuda, M, N, K):
    """The fp32 fc forward's split-K form (what the update runs when it hands the fc kernels a
    partials buffer: 64 x 64 tiles over two K halves, summed in order, bias + ReLU after) against
    the same float64 reference and bar, ragged tiles included."""
    _fc_case(cuda, 0, False, M, N, K, split=True)


def test_fc_gemm_refuses_unsupported_shapes(cuda):
    from gsamd._lib import check, lib
    A = torch.zeros(64, 100, device=cuda)
    with pytest.raises(ValueError):     # K % 64 != 0
        check(lib.gs_fc_gemm(0, 0, 64, 64, 100, A.data_ptr(), 100, A.data_ptr(), 100, A.data_ptr(), 64, A.data_ptr(),
                             None, torch.cuda.current_stream().cuda_stream), "gs_fc_gemm")
