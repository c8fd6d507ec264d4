// gs_gemm.h — the fp32 MFMA GEMM engine of the NatureCNN path (gs_gemm.hip).
//
// One kernel template serves dense GEMMs and the convolutions as implicit GEMMs: the A and B
// tiles are produced by operand loaders, so the conv1 patches are read straight from the u8
// frame stacks of the rollout (through the minibatch index) and the conv2/conv3 patches from
// the NHWC activations — no im2col matrix ever exists in HBM.
#pragma once

#include "gs_common.h"

namespace gs {

// Convolution geometry: input R x H x W x C (NHWC, or NCHW u8 frames for conv1), kernel k,
// stride s, output R x OH x OW x Cout.
struct ConvGeom {
    int R, H, W, C, k, s, OH, OW, Cout;
    int64_t rows() const { return (int64_t)R * OH * OW; }
    int patch() const { return k * k * C; }
};

// u8 frame source of conv1: obs[(T*N) rows][C][H][W]; minibatch row r reads rollout row
// idx[r] (env-major sample index, rollout_buffer.py:11-13) or r itself when idx == nullptr.
struct FrameSrc {
    const uint8_t *obs;
    const int32_t *idx;
    int64_t T, N;
};

// Every NatureCNN product takes its operand precision as an argument (bf16: GS_HP_BF16, bf16
// MFMA operands with fp32 accumulation; false: the fp32 parity path).
//
// Dense row-major GEMM: C[M][N] = op(A) op(B) (+ beta C) (+ bias[n]) (ReLU), with
// op(A)[m][k] = TA ? A[k*lda + m] : A[m*lda + k], op(B)[k][n] = TB ? B[n*ldb + k] : B[k*ldb + n].
// splits > 1: K is cut into `splits` slices; slice z writes its partial product to
// C + z*sC (beta/bias/relu/mask must then be off) — the caller sums them in a fixed order.
// mask (leading dimension ldc): C[m][n] is kept only where mask[m][n] > 0 (relu' of the
// activation the product is the gradient of), zero elsewhere.
int gemm_f32(hipStream_t s, bool bf16, bool ta, bool tb, int64_t M, int64_t N, int64_t K, const float *A, int64_t lda,
             const float *B, int64_t ldb, float *C, int64_t ldc, float beta, const float *bias, bool relu,
             int splits = 1, int64_t sC = 0, const float *mask = nullptr);

// The NatureCNN fc layer's GEMMs on the hand-written MFMA kernels of gs_fc.hip (fp32, or bf16
// operands with fp32 accumulation): op 0 C = relu(A B^T + aux[n]) (A [M][K], B [N][K]); op 1
// C = A^T B (A [K][M], B [K][N]); op 2 C = (A B) * (aux > 0) (A [M][K], B [K][N], aux like C).
// fc_supported: the shapes they take (K % 64 == 0, 16-B rows, K-strided operands in 4-row blocks).
bool fc_supported(int op, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc);
// parts (optional, 2 M N floats): the fp32 forward's split-K partials (faster at the C4 shape).
// act16 (needs bf16): every operand but the bias is stored as bf16 — a3 (op 0's A, op 1's B, op
// 2's aux, gs_common.h act_bf16), dh (op 1's and op 2's A) and Wf (op 0's and op 2's B, the
// update's bf16 weight copy) — so the operand pointers are void
int fc_gemm(hipStream_t s, int op, bool bf16, int64_t M, int64_t N, int64_t K, const void *A, int64_t lda,
            const void *B, int64_t ldb, float *C, int64_t ldc, const void *aux, const int32_t *stop = nullptr,
            float *parts = nullptr, bool act16 = false, ActOut ao = ActOut{});
// ao (GS_HP_ACT_STATS): op 0's bias + ReLU epilogue records the activation statistics of the
// pre-activation outputs (neuron = column), in fc_fwd_act_slots(M, N) slots
int fc_fwd_act_slots(int64_t M, int64_t N);
// the fc forward product as split-K fp32 partials (no epilogue) for small row counts (the
// rollout): C + z M ldc = A[:, z K/splits ..] B[:, z K/splits ..]^T for z < splits;
// fc_fwd_splits picks the split (1 when the plain tiles already fill the chip)
int fc_fwd_splits(int64_t M, int64_t N, int64_t K);
int fc_fwd_partials(hipStream_t s, int splits, int64_t M, int64_t N, int64_t K, const float *A, int64_t lda,
                    const float *B, int64_t ldb, float *C, int64_t ldc);


// out[r,oy,ox,co] = relu(bias[co] + sum_{c,ky,kx} W[co][c][ky][kx] * frame[c][oy*s+ky][ox*s+kx] / 255)
// (relu = false: the pre-activation, for the activation statistics)
int conv_fwd_u8(hipStream_t s, bool bf16, const ConvGeom &g, const FrameSrc &f, const float *Wt, const float *bias, float *out,
                bool relu = true);
// out[r,oy,ox,co] = relu(bias[co] + sum_{ky,kx,c} W[co][ky][kx][c] * in[r, oy*s+ky, ox*s+kx, c])
int conv_fwd_nhwc(hipStream_t s, bool bf16, const ConvGeom &g, const float *in, const float *Wt, const float *bias, float *out,
                  bool relu = true);
// dW[co][patch] = sum over rows of dY[row][co] * patch(row): split over `splits` row slices
// into parts (splits * Cout * patch floats), then summed in slice order into dW.
int conv_wgrad_u8(hipStream_t s, bool bf16, const ConvGeom &g, const FrameSrc &f, const float *dY, float *parts, int splits,
                  float *dW);
// conv_wgrad_nhwc also produces db[co] (column sums of dY, summed from the A tiles in LDS
// by the n-block-0 workgroups); parts: splits * Cout * (patch + 1) floats
int conv_wgrad_nhwc(hipStream_t s, bool bf16, const ConvGeom &g, const float *in, const float *dY, float *parts, int splits,
                    float *dW, float *db);
// [dW | db] partials of a dense weight gradient: parts[z] (M x (N+1)) = [dY^T X | rowsum dY^T]
// over split z of K; then sum_parts_wb scatters column N of each row into db
int gemm_wgrad_bias(hipStream_t s, bool bf16, int64_t M, int64_t N, int64_t K, const float *dY, int64_t lddy, const float *X,
                    int64_t ldx, float *parts, int splits);
// out[i] = sum over p of parts[p pstride + i] (float4 loads; np >= 64, n and pstride multiples of 4,
// parts 16-B aligned)
int sum_parts4(hipStream_t s, const float *parts, int np, int64_t pstride, int64_t n, float *out);
// [dW | db] of 64-filter conv weight gradients from partials in MFMA tile order (k_conv_wgrad's
// layout, gs_conv.hip): the sums of sum_parts_wb, scattered to dW [64][ncols] and db [64]
int sum_parts_tiles(hipStream_t s, const float *parts, int np, int64_t pstride, int ncols, float *dW, float *db);
int sum_parts_wb(hipStream_t s, const float *parts, int np, int64_t pstride, int rows, int ncols, float *dW,
                 float *db);
// out[i] = (bias/relu epilogue of) sum_{p < np} parts[p*n + i], fixed order; C = row length
// for the bias index (i % C)
// (pstride: distance between consecutive partials, default n)
int sum_parts(hipStream_t s, const float *parts, int np, int64_t n, float *out, const float *bias = nullptr,
              int C = 1, bool relu = false, int64_t pstride = 0);
// heads: z[r][a] = h[r] . Wp[a] (a < A), z[r][A] = h[r] . Wv — row stride A+1, no bias
int heads_fwd(hipStream_t s, bool bf16, int64_t R, int HID, int A, const float *h, const float *Wp, const float *Wv, float *z,
              float *parts, int splits);

}  // namespace gs
