// gs_conv.h — LDS-resident NatureCNN conv1 kernels (gs_conv.hip) for 4 x 84 x 84 u8 stacks.
#pragma once

#include "gs_common.h"

namespace gs {

#ifndef GS_C1WGF_BUFS
#define GS_C1WGF_BUFS 1
#endif
constexpr int kConv1WgradF32Bufs = GS_C1WGF_BUFS;              // LDS tile buffers of the fp32 form
constexpr int kConv1WgradWG = kConv1WgradF32Bufs == 1 ? 512 : 256;   // its workgroups (= partials)
#ifndef GS_C1WG_BUFS
#define GS_C1WG_BUFS 1
#endif
constexpr int kConv1WgradBfBufs = GS_C1WG_BUFS;                // LDS tile buffers of the bf16 form
#ifndef GS_C1WG_WGS
#define GS_C1WG_WGS (GS_C1WG_BUFS == 1 ? 512 : 256)
#endif
constexpr int kConv1WgradBfWG = GS_C1WG_WGS;                   // its workgroups (= partials)
constexpr int kConvWgradWG = 256;      // workgroups (= partials) of the conv2 / conv3 weight gradients

bool conv1_lds_supported(int C, int H, int W);
// out[r][oy][ox][co] = relu(b1[co] + sum W1[co][c][ky][kx] * frame(r)[c][4 oy + ky][4 ox + kx] / 255)
// bf: bf16 MFMA operands (GS_HP_BF16), fp32 accumulation; false: the fp32 parity path.
// xh (needs bf): the activations a1 / a2 / a3 this file's kernels write and read are stored as
// bf16 (gs_common.h act_bf16: the operand bits the bf16 mode rounds to anyway) and the forward /
// input-gradient filters come from the update's bf16 weight copy, so those pointers are void:
// fp32 or bf16 elements by xh (biases stay fp32)
// ao (GS_HP_ACT_STATS, update batches only): the forward's epilogue records the activation statistics
int conv1_lds_fwd(hipStream_t s, bool bf, bool xh, int R, const uint8_t *obs, const int32_t *idx, int64_t T, int64_t N,
                  const void *W1, const float *b1, void *out, uint8_t *obs_copy = nullptr, ActOut ao = ActOut{});
// dW1 = sum_rows dA1^T . patches, db1 = column sums of dA1; parts: kConv1WgradWG x (32*256 + 32) floats
// np_out: only the partials (their count written there); the caller sums them
int conv1_lds_wgrad(hipStream_t s, bool bf, int R, const uint8_t *obs, const int32_t *idx, int64_t T, int64_t N,
                    const float *dA, float *parts, float *dW1, float *db1, int *np_out = nullptr);
int conv1_lds_wgrad_parts();
// conv2 (20x20x32 -> 9x9x64, k4 s2) / conv3 (9x9x64 -> 7x7x64, k3 s1) forward with bias + ReLU,
// NHWC, LDS-resident samples (layer = 2 or 3)
bool conv23_lds_supported(int layer, int H, int W, int C, int k, int st, int Cout);
int conv23_lds_fwd(hipStream_t s, bool bf, bool xh, int layer, int R, const void *in, const void *Wt,
                   const float *bias, void *out, ActOut ao = ActOut{});
// statistics slots (workgroup x 4 waves) of an update batch's stats-epilogue forward of layer 1 / 2 / 3
int conv_fwd_act_slots(int layer, int R, bool bf, bool xh);
// input gradient of conv2 / conv3 masked by ReLU'(act) (act = the layer's input activation):
// dX = (dY conv^T W) * (act > 0), NHWC fp32
int conv23_lds_dgrad(hipStream_t s, bool bf, bool xh, int layer, int R, const float *dY, const void *act,
                     const void *Wt, float *dX);
// dW (64 x patch) and db (64) of conv2 / conv3; parts: kConvWgradWG x 64 x (patch + 1) floats.
// sum = false: only the partials (the caller's fused tail sums them, k_sum_parts_tiles' order)
int conv23_lds_wgrad(hipStream_t s, bool bf, bool xh, int layer, int R, const void *in, const float *dY, float *parts,
                     float *dW, float *db, bool sum = true);

}  // namespace gs
