"""Timing-only experiments on the product kernels, as source substitutions applied to a copy of
csrc/ by tools/ab_build.py (never compiled into libgsamd.so).  Several give WRONG results on
purpose: they price one cost of the lagged forward by removing it."""

ADAM_DENOM = ("gs_mlp.hip",
              "    const float denom = __builtin_amdgcn_sqrtf(v) * inv_bc2s + aa.eps;\n"
              "    p = p + neg_step * (m * __builtin_amdgcn_rcpf(denom));",
              "    const float denom = v * inv_bc2s + aa.eps;\n"
              "    p = p + neg_step * (m * denom);")

def _zero_loss(call):
    """a loss_rows_lds call replaced by a constant dz fill of the same rows (wrong results)"""
    return ("gs_mlp.hip", call, "for (int u = threadIdx.x; u < 256 * 3; u += 256) dzs[u] = 1e-3f;")


EXPERIMENTS = {
    # role A / B / C without their loss rows (wrong results): what the redundant loss costs each role
    "no_loss_A": [_zero_loss("loss_rows_lds<S>(P, L, zpart, ff, la, B, kstep, 0, B, dzs, nullptr);")],
    "no_loss_B": [("gs_mlp.hip",
                   "            loss_rows_lds<S>(P, L, zpart, ff, la, B, kstep, b0, kRowsB, dzs, nullptr, kLd, 256 - kLd);",
                   "            for (int u = threadIdx.x; u < kRowsB * 3; u += 256) dzs[u] = 1e-3f;")],
    "no_loss_C": [("gs_mlp.hip",
                   "                loss_rows_lds<S>(P, L, zpart, ff, la, B, kstep, 0, Bp, dzs, ge > gs ? dscrC : nullptr, 0, 256,\n"
                   "                                 kTile * gs, kTile * ge);",
                   "                for (int u = threadIdx.x; u < Bp * 3; u += 256) dzs[u] = 1e-3f;")],
    # role B on 64-row slabs (4 dW1|db1 partials instead of 8; correct results, other rounding):
    # each wave takes one 16-row tile over the whole K = H2 instead of half of it
    "rows64": [("gs_common.h", "constexpr int kRowsB = 32;", "constexpr int kRowsB = 64;"),
               ("gs_mlp.hip", "        const int rt = wave >> 1, half = wave & 1;\n"
                              "        const int chb = half ? nchB / 2 : 0, che = half ? nchB : nchB / 2;",
                "        const int rt = wave;\n        const int chb = 0, che = nchB;"),
               ("gs_mlp.hip",
                "            const float g = kred[(2 * t) * 256 + rr * kTile + col] + kred[(2 * t + 1) * 256 + rr * kTile + col];",
                "            const float g = kred[t * 256 + rr * kTile + col];")],
    # the lagged forward without the W2 rows' Adam-state loads (m, v, g copied from p: wrong
    # results): the price of the 48 KB per workgroup
    "no_w2_state": [("gs_mlp.hip",
                     "            w2m[j] = ld4(af.Min, q);\n            w2v[j] = ld4(af.Vin, q);\n            w2g[j] = ld4(af.G, q);",
                     "            w2m[j] = w2r[j];\n            w2v[j] = w2r[j];\n            w2g[j] = w2r[j];")],
    # Adam without sqrt / rcp (wrong results): the transcendental cost of the lagged step
    "no_trans": [ADAM_DENOM],
    # new W2 / W1 set stored from three row blocks instead of one
    "split_stores": [("gs_mlp.hip",
                      "        const bool stW2[3] = {own2, own2, own2};\n"
                      "        const bool stW1[3] = {own1, own1, own1};",
                      "        const int gy = (int)gridDim.y, gx = (int)gridDim.x;\n"
                      "        const bool stW2[3] = {apply && rb == 0, apply && rb == 1 % gy, apply && rb == 2 % gy};\n"
                      "        const bool stW1[3] = {apply && rb == 3 % gy && cb == 0, apply && rb == 3 % gy && cb == 1 % gx,\n"
                      "                              apply && rb == 3 % gy && cb == 2 % gx};")],
    # the new set never stored (wrong results)
    "no_owner_stores": [("gs_mlp.hip",
                         "        const bool stW2[3] = {own2, own2, own2};\n"
                         "        const bool stW1[3] = {own1, own1, own1};",
                         "        const bool stW2[3] = {false, false, false};\n"
                         "        const bool stW1[3] = {false, false, false};")],
    # one of the 8 dW1|db1 row-block partials loaded (wrong results): the fold's price
    "one_partial": [("gs_mlp.hip",
                     "                t[j][b] = ld4(tsrc + (int64_t)b * tstride, nrm ? min(tid + 256 * j, nq1 - 1) : 0);",
                     "                t[j][b] = b == 0 ? ld4(tsrc, nrm ? min(tid + 256 * j, nq1 - 1) : 0) : z4;")],
    # x / h1 stores after the heads, as with 256 threads
    "late_x_h1": [("gs_mlp.hip", "    constexpr bool kEarly = NT == 512;", "    constexpr bool kEarly = false;")],
    # k_bwd grid padded to a multiple of 8 (the extra workgroups exit at once): every kernel of the
    # chain then has a grid that is a multiple of the XCD count
    "pad_bwd8": [("gs_mlp.hip",
                  "    const unsigned nblk = (unsigned)(sh0.nA + sh0.nB + sh0.nC);",
                  "    const unsigned nblk = (unsigned)((sh0.nA + sh0.nB + sh0.nC + 7) / 8 * 8);"),
                 ("gs_mlp.hip",
                  "    GS_SPAN_T0\n    if (stop && *stop) return;\n    // multi-GPU: every output value goes through bwd_exchange",
                  "    {\n        const BwdShape s0 = BwdShape::make(S::lay(Lrt), S::batch(Brt));\n"
                  "        if ((int)blockIdx.x >= s0.nA + s0.nB + s0.nC) return;\n    }\n"
                  "    GS_SPAN_T0\n    if (stop && *stop) return;\n    // multi-GPU: every output value goes through bwd_exchange")],
    # role A tile (n-block, k-group) by n-block fastest: the 8 workgroups of an n-block share an XCD
    # with the forward workgroups that read their dW2 rows (with pad_bwd8)
    "roleA_xcd": [("gs_mlp.hip",
                   "        const int nb = bid / nkg, kb = (bid - nb * nkg) * sh.ka;   // first of the ka k-blocks",
                   "        const int nb = bid % sh.ncb, kb = (bid / sh.ncb) * sh.ka;   // first of the ka k-blocks")],
    # every row block stores its share of the new set (row i of the column block by row block
    # i mod gridDim.y; W1|b1 chunks q by row block q mod gridDim.y of column block 0)
    "spread_stores": [("gs_mlp.hip",
                       "                if (stW1[0]) reinterpret_cast<float4 *>(af.Pout)[q] = p4;\n"
                       "                if (stW1[1]) reinterpret_cast<float4 *>(af.Mout)[q] = make_float4(m[0], m[1], m[2], m[3]);\n"
                       "                if (stW1[2]) reinterpret_cast<float4 *>(af.Vout)[q] = make_float4(v[0], v[1], v[2], v[3]);",
                       "                if (cb == 0 && q % (int)gridDim.y == rb) {\n"
                       "                    reinterpret_cast<float4 *>(af.Pout)[q] = p4;\n"
                       "                    reinterpret_cast<float4 *>(af.Mout)[q] = make_float4(m[0], m[1], m[2], m[3]);\n"
                       "                    reinterpret_cast<float4 *>(af.Vout)[q] = make_float4(v[0], v[1], v[2], v[3]);\n"
                       "                }"),
                      ("gs_mlp.hip",
                       "                if (stW2[0]) reinterpret_cast<float4 *>(af.Pout)[q] = w2r[j];\n"
                       "                if (stW2[1]) reinterpret_cast<float4 *>(af.Mout)[q] = make_float4(m[0], m[1], m[2], m[3]);\n"
                       "                if (stW2[2]) reinterpret_cast<float4 *>(af.Vout)[q] = make_float4(v[0], v[1], v[2], v[3]);",
                       "                if (i % (int)gridDim.y == rb) {\n"
                       "                    reinterpret_cast<float4 *>(af.Pout)[q] = w2r[j];\n"
                       "                    reinterpret_cast<float4 *>(af.Mout)[q] = make_float4(m[0], m[1], m[2], m[3]);\n"
                       "                    reinterpret_cast<float4 *>(af.Vout)[q] = make_float4(v[0], v[1], v[2], v[3]);\n"
                       "                }")],
}

# the lagged forward's h2 MFMA on all 8 waves (2 of the 16 K chunks each) instead of waves 0..3
# (4 each), the x / h1 stores of waves 4..7 after their chunks: timing only (the 8 partials are
# summed in another order than the 256-thread kernel's 4)
EXPERIMENTS["mfma8"] = [
    ("gs_mlp.hip", "               round4(kTile * L.D) + kTile * (L.H1 + 4) + 1024 + kTile * 17;",
                   "               round4(kTile * L.D) + kTile * (L.H1 + 4) + 2048 + kTile * 17;"),
    ("gs_mlp.hip", "    float *h2s = red + 1024;", "    float *h2s = red + 2048;"),
    ("gs_mlp.hip", "    if (kEarly && wave >= 4) store_x_h1(tid - 256, 256);\n", ""),
    ("gs_mlp.hip", "    if (wave < 4) {\n        const int i = lane & 15, q = lane >> 4;\n        const int nch = H1 / kTile;\n"
                   "        const int ch0 = (wave * nch) / 4, ch1 = ((wave + 1) * nch) / 4;",
                   "    {\n        const int i = lane & 15, q = lane >> 4;\n        const int nch = H1 / kTile;\n"
                   "        const int ch0 = (wave * nch) / (NT / 64), ch1 = ((wave + 1) * nch) / (NT / 64);"),
    ("gs_mlp.hip", "        for (int r = 0; r < 4; ++r) red[wave * 256 + (q * 4 + r) * kTile + i] = acc[r];\n    }\n    __syncthreads();\n    GS_STAMP(5)",
                   "        for (int r = 0; r < 4; ++r) red[wave * 256 + (q * 4 + r) * kTile + i] = acc[r];\n    }\n"
                   "    if (kEarly && wave >= 4) store_x_h1(tid - 256, 256);\n    __syncthreads();\n    GS_STAMP(5)"),
    ("gs_mlp.hip", "        const float s = ((red[tid] + red[256 + tid]) + red[512 + tid]) + red[768 + tid];",
                   "        float s = ((red[tid] + red[256 + tid]) + red[512 + tid]) + red[768 + tid];\n"
                   "        if (NT == 512) s = (((s + red[1024 + tid]) + red[1280 + tid]) + red[1536 + tid]) + red[1792 + tid];"),
]

# role C's n-blocks paired per XCD (n-blocks 2m, 2m+1 — one 128-B line of each h2 row — on XCD m):
# correct results, half the h2 column-tile fetch from memory
EXPERIMENTS["roleC_pair"] = [
    ("gs_mlp.hip", "        const int nb = bid;\n        const int n0 = nb * kTile;\n        const int Bp = (B + 15) / 16 * 16;",
                   "        const int nb = (sh.ncb == 16 && bid < 16) ? 2 * (bid & 7) + (bid >> 3) : bid;\n"
                   "        const int n0 = nb * kTile;\n        const int Bp = (B + 15) / 16 * 16;"),
]
