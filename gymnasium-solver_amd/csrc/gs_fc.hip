// gs_fc.hip — the NatureCNN fc layer's three GEMMs on hand-written CDNA4 MFMA kernels (no vendor
// library): utils/models.py:56-110, h = relu(a3 Wf^T + bf) (3136 -> 512) and its backward.
//
//   fwd   h[B][HID]   = relu(a3[B][F] . Wf[HID][F]^T + bf)     both operands K-contiguous
//   wgrad dWf[HID][F] = dh[B][HID]^T . a3[B][F]                  both operands K-strided (K = B)
//   dgrad da3[B][F]   = (dh[B][HID] . Wf[HID][F]) * (a3 > 0)     A K-contiguous, B K-strided
//
// k_fc<BM, BN, WGM, KS, BF, AK, BKC, EPI, PD, KT>: 256 threads = 4 waves arranged WGM x WGN x KS;
// a wave owns (BM/WGM) x (BN/WGN) of the output as 32 x 32 MFMA sub-tiles and, with KS > 1, every
// KS-th k-group of each K tile (the KS partial tiles are added in ks order through LDS at the end:
// deterministic).  Both operands are staged global -> registers -> LDS as [row][k] with k
// contiguous (a K-strided source is transposed in registers from 4 x 4 blocks on the way), so an
// MFMA operand is one ds_read_b128 per lane:
//   fp32 (v_mfma_f32_32x32x2_f32, exact fp32): lane (r, q) reads k0 + 4q .. k0 + 4q + 3 of its row
//        and MFMA j takes element j — the four MFMAs of a k-group cover k0 .. k0 + 7 once each, the
//        same k in both operands;
//   bf16 (GS_HP_BF16, v_mfma_f32_32x32x16_bf16): the tile is converted to bf16 (round to nearest
//        even) as it is staged; lane (r, q) reads 8 bf16 at k0 + 8q: one MFMA per 16-k group.
// A K tile is KT x 128 B of every row plus a 16-B pad, two LDS buffers, PD register sets of
// tiles in flight, one barrier per tile.  Launch shapes (same-box fc_bench sweeps):
// fwd 32 x 32 with the 4 waves splitting the k-groups (KS = 4: 512 workgroups, two per CU);
// wgrad 64 x 64 on 32x32x2 MFMAs and dgrad 64 x 64 on 16x16x4 blocks (k_fc16) in fp32 (392 / 784
// workgroups); fp32 tiles are 64 deep (KT = 2).
#include <mutex>
#include <type_traits>
#include <unordered_map>

#include "gs_gemm.h"

namespace gs {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

enum FcEpi { kEpiStore = 0, kEpiBiasRelu = 1, kEpiMask = 2 };

// One K tile holds KT 128-B chunks of every staged row (32 KT fp32 or 64 KT bf16 elements) plus a
// 16-B pad: a row stride of 4 (mod 64) dwords puts the 16 rows a ds_read_b128 lane group reads on
// distinct banks.
template <bool BF, int KT>
struct FcK {
    static constexpr int KE = (BF ? 64 : 32) * KT;   // K elements per tile
    static constexpr int GK = BF ? 16 : 8;           // K elements per k-group (one ds_read_b128 per lane)
    static constexpr int NG = KE / GK;               // k-groups per tile (4 KT)
    static constexpr int RB = 128 * KT + 16;         // LDS bytes per staged row
};

#ifndef FC_SWZ
#define FC_SWZ 1            // LDS chunk swizzle (0: plain chunk order, for A/B runs)
#endif
#ifndef FC_MI16
#define FC_MI16 1           // fp32 on v_mfma_f32_16x16x4_f32 (0: the 32 x 32 x 2 form, for A/B runs)
#endif
#ifndef FC_XCD
#define FC_XCD 1            // XCD-aware tile order (0: plain blockIdx order, for A/B runs)
#endif

// register prefetch depth (K tiles in flight) per launch shape and operand precision
#ifndef FC_PD_FWD32
#define FC_PD_FWD32 3
#endif
#ifndef FC_PD_FWD16
#define FC_PD_FWD16 4      // round 5, bf16 storage: 24.8 -> 22.4 us (6: 22.4; the wgrad / dgrad lose with 4)
#endif
#ifndef FC_PD_WG32
#define FC_PD_WG32 2
#endif
#ifndef FC_PD_WG16
#define FC_PD_WG16 2
#endif
#ifndef FC_PD_DG32
#define FC_PD_DG32 2
#endif
#ifndef FC_PD_DG16
#define FC_PD_DG16 2
#endif

// 4 fp32 -> 4 bf16 (8 bytes)
__device__ __forceinline__ uint2 pack_bf16x4(float4 v)
{
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    bf16x4 r;
    r[0] = (__bf16)v.x, r[1] = (__bf16)v.y, r[2] = (__bf16)v.z, r[3] = (__bf16)v.w;
    return *reinterpret_cast<uint2 *>(&r);
}

// LDS chunk swizzle: the 16-B chunk c of staged row r lives at chunk c ^ swz(r).  A K-strided
// staging store writes rows 4 apart from consecutive lanes (row stride 4 (mod 64) dwords, so 16
// (mod 64) every 4 rows: 4-way bank conflicts without it); XOR-ing the chunk with bits 4-5 of the
// row spreads those lanes over all banks, and the operand reads (16 consecutive rows, one swizzle
// value per 16-row group) stay conflict-free
__device__ __forceinline__ int swz(int row) { return FC_SWZ ? (row >> 4) & 3 : 0; }

__device__ __forceinline__ float f4at(const float4 &v, int c)
{
    return c == 0 ? v.x : c == 1 ? v.y : c == 2 ? v.z : v.w;
}

// staging of one operand's K tile: ROWS rows (m or n) x KE k.  KC: source element (row, k) at
// p[row * ld + k] (K-contiguous), else at p[k * ld + row].  Every thread moves the same number of
// units (no divergent branches, so the waitcnt counts stay exact); rows past n_rows load clamped
// and are zeroed at the store.  SH (bf16 operands only): the source holds bf16 (a bf16-stored
// activation / weight copy), 4 elements per 8-B load kept as raw bits until the store writes them
// (expanding them at the load made the compiler wait for each tile's loads as soon as they were
// issued: the fc forward ran 28 -> 36 us)
template <int ROWS, bool BF, bool KC, int KT, bool SH = false>
struct Stage {
    static_assert(!SH || BF, "bf16 source: bf16 staging");
    static constexpr int KE = FcK<BF, KT>::KE, RB = FcK<BF, KT>::RB;
    // K-contiguous: one float4 (4 k of one row) per unit; K-strided: a 4 x 4 block per unit
    static constexpr int UNITS = KC ? ROWS * KE / 4 : ROWS * KE / 16;
    static constexpr int PER = UNITS / 256;
    static_assert(UNITS % 256 == 0, "whole units per thread");
    static constexpr int NV = KC ? 1 : 4;
    using RT = typename std::conditional<SH, uint2, float4>::type;
    using ST = typename std::conditional<SH, uint16_t, float>::type;
    RT r[PER][NV];

    __device__ __forceinline__ void load(const ST *__restrict__ p, int64_t ld, int row0, int n_rows, int k0)
    {
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int u = (int)threadIdx.x + 256 * j;
            if constexpr (KC) {
                const int row = u / (KE / 4), k4 = u - row * (KE / 4);
                const int gr = min(row0 + row, n_rows - 1);
                r[j][0] = *reinterpret_cast<const RT *>(p + (int64_t)gr * ld + k0 + 4 * k4);
            } else {
                const int kb = u / (ROWS / 4), rb = u - kb * (ROWS / 4);
                const int gr = min(row0 + 4 * rb, n_rows - 4);     // n_rows % 4 == 0 (host check)
#pragma unroll
                for (int v = 0; v < 4; ++v)
                    r[j][v] = *reinterpret_cast<const RT *>(p + (int64_t)(k0 + 4 * kb + v) * ld + gr);
            }
        }
    }

    // bf16 bits of element c of a raw 4-element unit
    static __device__ __forceinline__ uint32_t h16(const uint2 &u, int c)
    {
        return ((c < 2 ? u.x : u.y) >> (16 * (c & 1))) & 0xffffu;
    }

    __device__ __forceinline__ void store(char *lds, int row0, int n_rows) const
    {
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int u = (int)threadIdx.x + 256 * j;
            if constexpr (KC) {
                const int row = u / (KE / 4), k4 = u - row * (KE / 4);
                const bool ok = row0 + row < n_rows;
                char *dst = lds + row * RB;
                if constexpr (SH) {
                    *reinterpret_cast<uint2 *>(dst + 16 * ((k4 >> 1) ^ swz(row)) + 8 * (k4 & 1)) =
                        ok ? r[j][0] : make_uint2(0u, 0u);
                } else {
                    const float4 v = ok ? r[j][0] : make_float4(0.f, 0.f, 0.f, 0.f);
                    if constexpr (BF)
                        *reinterpret_cast<uint2 *>(dst + 16 * ((k4 >> 1) ^ swz(row)) + 8 * (k4 & 1)) = pack_bf16x4(v);
                    else *reinterpret_cast<float4 *>(dst + 16 * (k4 ^ swz(row))) = v;
                }
            } else {
                const int kb = u / (ROWS / 4), rb = u - kb * (ROWS / 4);
                const bool ok = row0 + 4 * rb < n_rows;
                // r[j][v] = rows 4 rb .. 4 rb + 3 at k = 4 kb + v: column c is row 4 rb + c's 4 k
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    char *dst = lds + (4 * rb + c) * RB;
                    const int sr = swz(4 * rb + c);
                    if constexpr (SH) {
                        const uint2 w = ok ? make_uint2(h16(r[j][0], c) | (h16(r[j][1], c) << 16),
                                                        h16(r[j][2], c) | (h16(r[j][3], c) << 16))
                                           : make_uint2(0u, 0u);
                        *reinterpret_cast<uint2 *>(dst + 16 * ((kb >> 1) ^ sr) + 8 * (kb & 1)) = w;
                    } else {
                        const float4 v = ok ? make_float4(f4at(r[j][0], c), f4at(r[j][1], c), f4at(r[j][2], c),
                                                          f4at(r[j][3], c))
                                            : make_float4(0.f, 0.f, 0.f, 0.f);
                        if constexpr (BF)
                            *reinterpret_cast<uint2 *>(dst + 16 * ((kb >> 1) ^ sr) + 8 * (kb & 1)) = pack_bf16x4(v);
                        else *reinterpret_cast<float4 *>(dst + 16 * (kb ^ sr)) = v;
                    }
                }
            }
        }
    }
};

// f(integral_constant<I>) for I = B .. E-1 in order while it returns true (compile-time indices)
template <int I, int E, class F>
__device__ __forceinline__ void static_for(F &&f)
{
    if constexpr (I < E) {
        if (f(std::integral_constant<int, I>{})) static_for<I + 1, E>(f);
    }
}

// k_fc: 256 threads = 4 waves arranged WGM x WGN x KS; a wave owns (BM/WGM) x (BN/WGN) outputs as
// 32 x 32 sub-tiles and, with KS > 1, every KS-th k-group of each tile (the KS partial tiles are
// added in ks order through LDS at the end: deterministic).  Per tile a wave first issues every
// LDS operand read of its k-groups, then the MFMAs; the next tile's registers go to the other LDS
// buffer; one barrier per tile; tile kt + 1 + PD is loaded right after (tile j lives in register
// set j % PD, so its global latency hides under PD tiles of MFMAs).  Loads and stores are
// unconditional (the last tiles re-load a clamped tile) so the compiler's wait counts stay exact.
// H16 (bf16 updates): bit 1 — A, bit 2 — B, bit 4 — the mask operand aux are bf16-stored
// activations (gs_common.h act_bf16), 2 B per element
// AS (GS_HP_ACT_STATS, the bias + ReLU forward): the epilogue also records the activation statistics
// of the pre-activation outputs (gs_common.h ActOut; neuron = output column)
template <int BM, int BN, int WGM, int KS, bool BF, bool AK, bool BKC, int EPI, int PD, int KT, int H16 = 0,
          bool AS = false>
__global__ __launch_bounds__(256, 2) void k_fc(const void *__restrict__ Av, int64_t lda, const void *__restrict__ Bv,
                                               int64_t ldb, float *__restrict__ C, int64_t ldc, int M, int N, int K,
                                               const void *__restrict__ auxv, const int32_t *__restrict__ stop,
                                               int64_t sC, int gm, ActOut ao = ActOut{})
{
    static_assert(!AS || EPI == kEpiBiasRelu, "activation statistics: the bias + ReLU forward");
    static_assert(H16 == 0 || BF, "bf16 operand storage: bf16 MFMA operands only");
    static_assert(!(H16 & 4) || EPI == kEpiMask, "a bf16 aux is the mask operand");
    using AT = typename std::conditional<(H16 & 1) != 0, uint16_t, float>::type;
    using BT = typename std::conditional<(H16 & 2) != 0, uint16_t, float>::type;
    using XT = typename std::conditional<(H16 & 4) != 0, uint16_t, float>::type;
    const AT *A = static_cast<const AT *>(Av);
    const BT *Bm = static_cast<const BT *>(Bv);
    const XT *aux = static_cast<const XT *>(auxv);
    if (stop && *stop) return;      // KL early stop: the minibatch's product is never used
    // split-K (gridDim.z slices of K each, partial products at C + z sC; no epilogue)
    A += (AK ? 1 : lda) * (int64_t)blockIdx.z * K;
    Bm += (BKC ? 1 : ldb) * (int64_t)blockIdx.z * K;
    C += (int64_t)blockIdx.z * sC;
    constexpr int WGN = 4 / (WGM * KS);
    static_assert(WGM * WGN * KS == 4, "4 waves");
    constexpr int WM = BM / WGM, WN = BN / WGN, TM = WM / 32, TN = WN / 32;
    static_assert(TM >= 1 && TN >= 1 && WM % 32 == 0 && WN % 32 == 0, "32 x 32 sub-tiles");
    using K_ = FcK<BF, KT>;
    constexpr int KE = K_::KE, NG = K_::NG, RB = K_::RB, NGW = NG / KS;
    static_assert(NG % KS == 0, "k-groups split evenly over KS");
    static_assert(PD >= 1, "register prefetch depth");
    constexpr int TILE = (BM + BN) * RB;
    extern __shared__ __attribute__((aligned(16))) char lds[];     // 2 TILE bytes (launch_fc)

    // XCD-aware tile order: workgroup b runs on XCD b % 8 (round-robin dispatch), so XCD x is
    // given the contiguous run [x T/8, (x+1) T/8) of a grouped order (gm m-blocks per group, m
    // fastest within it): its L2 then holds a band of A rows and a band of B rows instead of
    // every XCD streaming all of A (T = tiles per split, a multiple of 8)
    int bx = blockIdx.x, by = blockIdx.y;
    {
        const int nbx = gridDim.x, nby = gridDim.y, T = nbx * nby;
        if (FC_XCD && T % 8 == 0 && gm > 0) {
            const int b = by * nbx + bx;
            const int t = (b & 7) * (T >> 3) + (b >> 3);
            const int gsize = gm * nbx, grp = t / gsize, first = grp * gm, gcnt = min(nby - first, gm);
            const int within = t - grp * gsize;
            by = first + within % gcnt;
            bx = within / gcnt;
        }
    }
    const int m0 = by * BM, n0 = bx * BN;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int ks = wave % KS, wmn = wave / KS;
    const int wm = (wmn / WGN) * WM, wn = (wmn % WGN) * WN;
    const int l32 = lane & 31, lh = lane >> 5;

    Stage<BM, BF, AK, KT, (H16 & 1) != 0> sa[PD];
    Stage<BN, BF, BKC, KT, (H16 & 2) != 0> sb[PD];
    // the bias + ReLU epilogue's bias, loaded before the K loop (at the epilogue it put a memory
    // latency in front of the stores)
    float bn[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int gn = min(n0 + wn + 32 * j + l32, N - 1);
        bn[j] = EPI == kEpiBiasRelu ? act_ld<(H16 & 4) != 0>(aux, gn) : 0.0f;
    }
    // the masked epilogue's relu' operands (the input gradient's activation), likewise
    float mk[EPI == kEpiMask ? TM : 1][EPI == kEpiMask ? TN : 1][EPI == kEpiMask ? 16 : 1];
    if constexpr (EPI == kEpiMask) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int gn = min(n0 + wn + 32 * j + l32, N - 1);
#pragma unroll
                for (int v = 0; v < 16; ++v) {
                    const int gm = min(m0 + wm + 32 * i + (v & 3) + 8 * (v >> 2) + 4 * lh, M - 1);
                    mk[i][j][v] = act_ld<(H16 & 4) != 0>(aux, (int64_t)gm * ldc + gn);
                }
            }
    }
    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;

    const int nk = K / KE;
    auto kof = [&](int t) { return min(t, nk - 1) * KE; };
#pragma unroll
    for (int u = 0; u < PD; ++u) {
        sa[u].load(A, lda, m0, M, kof(u));
        sb[u].load(Bm, ldb, n0, N, kof(u));
    }
    sa[0].store(lds, m0, M);
    sb[0].store(lds + BM * RB, n0, N);
    __syncthreads();
    sa[0].load(A, lda, m0, M, kof(PD));
    sb[0].load(Bm, ldb, n0, N, kof(PD));
    for (int kt0 = 0; kt0 < nk; kt0 += PD) {
        static_for<0, PD>([&](auto uc) -> bool {
            constexpr int u = decltype(uc)::value;
            const int kt = kt0 + u;
            if (kt >= nk) return false;
            const char *buf = lds + (kt & 1) * TILE;
            // every operand read of this wave's k-groups first, then the MFMAs
            float4 a[NGW][TM], b[NGW][TN];
#pragma unroll
            for (int q = 0; q < NGW; ++q) {
                const int g = ks + KS * q;
#pragma unroll
                for (int i = 0; i < TM; ++i)
                    a[q][i] = *reinterpret_cast<const float4 *>(buf + (wm + 32 * i + l32) * RB +
                                                                16 * ((2 * g + lh) ^ swz(wm + 32 * i + l32)));
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    b[q][j] = *reinterpret_cast<const float4 *>(buf + (BM + wn + 32 * j + l32) * RB +
                                                                16 * ((2 * g + lh) ^ swz(wn + 32 * j + l32)));
            }
#pragma unroll
            for (int q = 0; q < NGW; ++q) {
                if constexpr (BF) {
#pragma unroll
                    for (int i = 0; i < TM; ++i)
#pragma unroll
                        for (int j = 0; j < TN; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                                *reinterpret_cast<const bf16x8 *>(&a[q][i]), *reinterpret_cast<const bf16x8 *>(&b[q][j]),
                                acc[i][j], 0, 0, 0);
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
#pragma unroll
                        for (int i = 0; i < TM; ++i)
#pragma unroll
                            for (int j = 0; j < TN; ++j)
                                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(f4at(a[q][i], e), f4at(b[q][j], e),
                                                                                 acc[i][j], 0, 0, 0);
                }
            }
            constexpr int nv = (u + 1) % PD;     // the set holding tile kt + 1
            char *nb = lds + ((kt + 1) & 1) * TILE;
            sa[nv].store(nb, m0, M);             // (past the last tile: a clamped copy, never read)
            sb[nv].store(nb + BM * RB, n0, N);
            __syncthreads();
            sa[nv].load(A, lda, m0, M, kof(kt + 1 + PD));
            sb[nv].load(Bm, ldb, n0, N, kof(kt + 1 + PD));
            return true;
        });
    }
    if constexpr (KS > 1) {
        // the KS k-group partials of each wave tile, added in ks order (LDS is free after the loop)
        float *red = reinterpret_cast<float *>(lds);
        constexpr int PW = TM * TN * 16 * 64;      // floats per wave's partial tile
        static_assert(PW == WM * WN, "a wave's partial tile");     // launch_fc sizes the LDS for it
        __syncthreads();      // every wave's last operand reads of the K tiles are done
        if (ks > 0)
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
#pragma unroll
                    for (int v = 0; v < 16; ++v)
                        red[(((ks - 1) * (4 / KS) + wmn) * TM * TN + i * TN + j) * 16 * 64 + v * 64 + lane] = acc[i][j][v];
        __syncthreads();
        if (ks > 0) {
            if constexpr (AS)
                act_flush(ao, ((int64_t)blockIdx.x + gridDim.x * ((int64_t)blockIdx.y + gridDim.y * blockIdx.z)) * 4 +
                                  (threadIdx.x >> 6), 0.0f, 0.0f);
            return;
        }
        for (int q = 1; q < KS; ++q)
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
#pragma unroll
                    for (int v = 0; v < 16; ++v)
                        acc[i][j][v] += red[(((q - 1) * (4 / KS) + wmn) * TM * TN + i * TN + j) * 16 * 64 + v * 64 + lane];
    }
    float as_s = 0.0f, as_q = 0.0f;
    // epilogue: D col = lane & 31, row = (v & 3) + 8 (v >> 2) + 4 (lane >> 5) of each 32 x 32 sub-tile
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int gn = n0 + wn + 32 * j + l32;
            if (gn >= N) continue;
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                const int gm = m0 + wm + 32 * i + (v & 3) + 8 * (v >> 2) + 4 * lh;
                if (gm >= M) continue;
                float x = acc[i][j][v];
                if constexpr (EPI == kEpiBiasRelu) {
                    x += bn[j];
                    if constexpr (AS) act_acc(ao, x, gn, as_s, as_q);
                    x = x > 0.0f ? x : 0.0f;
                }
                if constexpr (EPI == kEpiMask) x = mk[i][j][v] > 0.0f ? x : 0.0f;
                C[(int64_t)gm * ldc + gn] = x;
            }
        }
    if constexpr (AS)
        act_flush(ao, ((int64_t)blockIdx.x + gridDim.x * ((int64_t)blockIdx.y + gridDim.y * blockIdx.z)) * 4 +
                          (threadIdx.x >> 6), as_s, as_q);
}

// k_fc16: the fp32 form on v_mfma_f32_16x16x4_f32 (exact fp32) — a wave's (BM/WGM) x (BN/WGN)
// outputs as 16 x 16 blocks (more independent accumulators per wave than the 32 x 32 form, the
// shape the vendor library picks for these GEMMs).  Same staging, buffers, tile order and KS split
// as k_fc; a 16-k chunk c of a tile: lane (r = lane & 15, q = lane >> 4) reads the 16 B at
// k = 16 c + 4 q .. + 3 of its row, and MFMA e takes element e — the four MFMAs of a chunk cover
// its 16 k once each, the same k in both operands.
template <int BM, int BN, int WGM, int KS, bool AK, bool BKC, int EPI, int PD, int KT>
__global__ __launch_bounds__(256, 2) void k_fc16(const float *__restrict__ A, int64_t lda, const float *__restrict__ Bm,
                                                 int64_t ldb, float *__restrict__ C, int64_t ldc, int M, int N, int K,
                                                 const float *__restrict__ aux, const int32_t *__restrict__ stop,
                                                 int64_t sC, int gm)
{
    if (stop && *stop) return;      // KL early stop: the minibatch's product is never used
    A += (AK ? 1 : lda) * (int64_t)blockIdx.z * K;
    Bm += (BKC ? 1 : ldb) * (int64_t)blockIdx.z * K;
    C += (int64_t)blockIdx.z * sC;
    constexpr int WGN = 4 / (WGM * KS);
    static_assert(WGM * WGN * KS == 4, "4 waves");
    constexpr int WM = BM / WGM, WN = BN / WGN, TM = WM / 16, TN = WN / 16;
    static_assert(TM >= 1 && TN >= 1 && WM % 16 == 0 && WN % 16 == 0, "16 x 16 blocks");
    using K_ = FcK<false, KT>;
    constexpr int KE = K_::KE, RB = K_::RB, NC = KE / 16, NCW = NC / KS;
    static_assert(NC % KS == 0, "16-k chunks split evenly over KS");
    constexpr int TILE = (BM + BN) * RB;
    extern __shared__ __attribute__((aligned(16))) char lds[];     // 2 TILE bytes (launch_fc)

    int bx = blockIdx.x, by = blockIdx.y;
    {
        const int nbx = gridDim.x, nby = gridDim.y, T = nbx * nby;
        if (FC_XCD && T % 8 == 0 && gm > 0) {
            const int b = by * nbx + bx;
            const int t = (b & 7) * (T >> 3) + (b >> 3);
            const int gsize = gm * nbx, grp = t / gsize, first = grp * gm, gcnt = min(nby - first, gm);
            const int within = t - grp * gsize;
            by = first + within % gcnt;
            bx = within / gcnt;
        }
    }
    const int m0 = by * BM, n0 = bx * BN;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int ks = wave % KS, wmn = wave / KS;
    const int wm = (wmn / WGN) * WM, wn = (wmn % WGN) * WN;
    const int r16 = lane & 15, q4 = lane >> 4;

    Stage<BM, false, AK, KT> sa[PD];
    Stage<BN, false, BKC, KT> sb[PD];
    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nk = K / KE;
    auto kof = [&](int t) { return min(t, nk - 1) * KE; };
#pragma unroll
    for (int u = 0; u < PD; ++u) {
        sa[u].load(A, lda, m0, M, kof(u));
        sb[u].load(Bm, ldb, n0, N, kof(u));
    }
    sa[0].store(lds, m0, M);
    sb[0].store(lds + BM * RB, n0, N);
    __syncthreads();
    sa[0].load(A, lda, m0, M, kof(PD));
    sb[0].load(Bm, ldb, n0, N, kof(PD));
    for (int kt0 = 0; kt0 < nk; kt0 += PD) {
        static_for<0, PD>([&](auto uc) -> bool {
            constexpr int u = decltype(uc)::value;
            const int kt = kt0 + u;
            if (kt >= nk) return false;
            const char *buf = lds + (kt & 1) * TILE;
            float4 a[NCW][TM], b[NCW][TN];
#pragma unroll
            for (int q = 0; q < NCW; ++q) {
                const int c = ks + KS * q;
#pragma unroll
                for (int i = 0; i < TM; ++i)
                    a[q][i] = *reinterpret_cast<const float4 *>(buf + (wm + 16 * i + r16) * RB +
                                                                16 * ((4 * c + q4) ^ swz(wm + 16 * i + r16)));
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    b[q][j] = *reinterpret_cast<const float4 *>(buf + (BM + wn + 16 * j + r16) * RB +
                                                                16 * ((4 * c + q4) ^ swz(wn + 16 * j + r16)));
            }
#pragma unroll
            for (int q = 0; q < NCW; ++q)
#pragma unroll
                for (int e = 0; e < 4; ++e)
#pragma unroll
                    for (int i = 0; i < TM; ++i)
#pragma unroll
                        for (int j = 0; j < TN; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(f4at(a[q][i], e), f4at(b[q][j], e),
                                                                             acc[i][j], 0, 0, 0);
            constexpr int nv = (u + 1) % PD;
            char *nb = lds + ((kt + 1) & 1) * TILE;
            sa[nv].store(nb, m0, M);
            sb[nv].store(nb + BM * RB, n0, N);
            __syncthreads();
            sa[nv].load(A, lda, m0, M, kof(kt + 1 + PD));
            sb[nv].load(Bm, ldb, n0, N, kof(kt + 1 + PD));
            return true;
        });
    }
    if constexpr (KS > 1) {
        float *red = reinterpret_cast<float *>(lds);
        constexpr int PW = TM * TN * 4 * 64;
        static_assert(PW == WM * WN, "a wave's partial tile");     // launch_fc sizes the LDS for it
        __syncthreads();
        if (ks > 0)
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
#pragma unroll
                    for (int v = 0; v < 4; ++v)
                        red[(((ks - 1) * (4 / KS) + wmn) * TM * TN + i * TN + j) * 4 * 64 + v * 64 + lane] = acc[i][j][v];
        __syncthreads();
        if (ks > 0) return;
        for (int q = 1; q < KS; ++q)
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
#pragma unroll
                    for (int v = 0; v < 4; ++v)
                        acc[i][j][v] += red[(((q - 1) * (4 / KS) + wmn) * TM * TN + i * TN + j) * 4 * 64 + v * 64 + lane];
    }
    // epilogue: D col = lane & 15, row = 4 (lane >> 4) + v of each 16 x 16 block
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int gn = n0 + wn + 16 * j + r16;
            if (gn >= N) continue;
            const float bn = EPI == kEpiBiasRelu ? aux[gn] : 0.0f;
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const int gmr = m0 + wm + 16 * i + 4 * q4 + v;
                if (gmr >= M) continue;
                float x = acc[i][j][v];
                if constexpr (EPI == kEpiBiasRelu) {
                    x += bn;
                    x = x > 0.0f ? x : 0.0f;
                }
                if constexpr (EPI == kEpiMask) x = aux[(int64_t)gmr * ldc + gn] > 0.0f ? x : 0.0f;
                C[(int64_t)gmr * ldc + gn] = x;
            }
        }
}

// a kernel's dynamic LDS above the 64 KB default: the attribute is set once per kernel (keyed on
// the kernel's own address: every k_fc instantiation has the same function type, so a flag keyed
// on the type would let the first one stand for all), before any capture (the first call of a
// shape is eager)
template <class KF>
void lds_attr(KF k, size_t bytes)
{
    if (bytes <= 65536) return;
    static std::mutex mu;
    static std::unordered_map<const void *, size_t> done;
    std::lock_guard<std::mutex> lk(mu);
    auto it = done.find((const void *)k);
    if (it != done.end() && it->second >= bytes) return;
    (void)hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    done[(const void *)k] = bytes;
}

// two staged K tiles, or the KS partial tiles of the in-workgroup k split if larger
template <int BM, int BN, int WGM, int KS, bool BF, int KT>
constexpr size_t fc_lds_bytes()
{
    const size_t tiles = 2 * (size_t)(BM + BN) * FcK<BF, KT>::RB;
    const size_t red = (size_t)(KS - 1) * (4 / KS) * (BM / WGM) * (BN / (4 / (WGM * KS))) * 4;
    return tiles > red ? tiles : red;
}

template <int BM, int BN, int WGM, int KS, bool AK, bool BKC, int EPI, int PD32, int PD16, int KT32, int KT16,
          bool MI16 = false, int H16 = 0>
int launch_fc(hipStream_t s, bool bf, const void *A, int64_t lda, const void *B, int64_t ldb, float *C, int64_t ldc,
              int64_t M, int64_t N, int64_t K, const void *aux, const int32_t *stop, int gm, int splits = 1,
              int64_t sC = 0, ActOut ao = ActOut{})
{
    const dim3 grid((unsigned)((N + BN - 1) / BN), (unsigned)((M + BM - 1) / BM), (unsigned)splits);
    GS_REQUIRE(H16 == 0 || (bf && splits == 1), "k_fc: bf16 operand storage needs bf16 operands, no K split");
    K /= splits;
    if constexpr (EPI == kEpiBiasRelu) {
        if (ao.cnt) {    // GS_HP_ACT_STATS: the statistics epilogue (slots: workgroups x 4 waves)
            GS_REQUIRE(splits == 1, "k_fc: activation statistics without a K split");
            if (bf) {
                constexpr size_t L = fc_lds_bytes<BM, BN, WGM, KS, true, KT16>();
                auto k = k_fc<BM, BN, WGM, KS, true, AK, BKC, EPI, PD16, KT16, H16, true>;
                lds_attr(k, L);
                hipLaunchKernelGGL(k, grid, dim3(256), L, s, A, lda, B, ldb, C, ldc, (int)M, (int)N, (int)K, aux, stop,
                                   sC, gm, ao);
            } else {
                constexpr size_t L = fc_lds_bytes<BM, BN, WGM, KS, false, KT32>();
                auto k = k_fc<BM, BN, WGM, KS, false, AK, BKC, EPI, PD32, KT32, 0, true>;
                lds_attr(k, L);
                hipLaunchKernelGGL(k, grid, dim3(256), L, s, A, lda, B, ldb, C, ldc, (int)M, (int)N, (int)K, aux, stop,
                                   sC, gm, ao);
            }
            GS_LAUNCH_CHECK("k_fc<stats>");
            return GS_OK;
        }
    }
    if (bf) {
        constexpr size_t L = fc_lds_bytes<BM, BN, WGM, KS, true, KT16>();
        auto k = k_fc<BM, BN, WGM, KS, true, AK, BKC, EPI, PD16, KT16, H16>;
        lds_attr(k, L);
        hipLaunchKernelGGL(k, grid, dim3(256), L, s, A, lda, B, ldb, C, ldc, (int)M, (int)N, (int)K, aux, stop, sC, gm,
                           ActOut{});
    } else if (MI16 && FC_MI16) {
        constexpr size_t L = fc_lds_bytes<BM, BN, WGM, KS, false, KT32>();
        auto k = k_fc16<BM, BN, WGM, KS, AK, BKC, EPI, PD32, KT32>;
        lds_attr(k, L);
        hipLaunchKernelGGL(k, grid, dim3(256), L, s, static_cast<const float *>(A), lda, static_cast<const float *>(B),
                           ldb, C, ldc, (int)M, (int)N, (int)K, static_cast<const float *>(aux), stop, sC, gm);
    } else {
        constexpr size_t L = fc_lds_bytes<BM, BN, WGM, KS, false, KT32>();
        auto k = k_fc<BM, BN, WGM, KS, false, AK, BKC, EPI, PD32, KT32>;
        lds_attr(k, L);
        hipLaunchKernelGGL(k, grid, dim3(256), L, s, A, lda, B, ldb, C, ldc, (int)M, (int)N, (int)K, aux, stop, sC, gm,
                           ActOut{});
    }
    GS_LAUNCH_CHECK("k_fc");
    return GS_OK;
}

// split-K partials [S][M][ldp] summed in slice order, then the product's epilogue (bias + ReLU of
// the forward, the relu' mask of the input gradient, none for the weight gradient); 4 columns per
// thread (N % 4 == 0)
template <int EPI>
__global__ __launch_bounds__(256) void k_fc_sum(const float *__restrict__ parts, int S, int64_t sP, int M, int N,
                                                int ldp, float *__restrict__ C, int64_t ldc,
                                                const float *__restrict__ aux, const int32_t *__restrict__ stop)
{
    if (stop && *stop) return;
    const int n4 = N / 4;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)M * n4) return;
    const int row = (int)(i / n4), c = 4 * (int)(i - (int64_t)row * n4);
    const float *p = parts + (int64_t)row * ldp + c;
    float4 acc = *reinterpret_cast<const float4 *>(p);
    for (int z = 1; z < S; ++z) {
        const float4 v = *reinterpret_cast<const float4 *>(p + z * sP);
        acc.x += v.x, acc.y += v.y, acc.z += v.z, acc.w += v.w;
    }
    float x[4] = {acc.x, acc.y, acc.z, acc.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        if constexpr (EPI == kEpiBiasRelu) {
            x[q] += aux[c + q];
            x[q] = x[q] > 0.0f ? x[q] : 0.0f;
        }
        if constexpr (EPI == kEpiMask) x[q] = aux[(int64_t)row * ldc + c + q] > 0.0f ? x[q] : 0.0f;
    }
    *reinterpret_cast<float4 *>(C + (int64_t)row * ldc + c) = make_float4(x[0], x[1], x[2], x[3]);
}

template <int EPI>
int fc_sum(hipStream_t s, const float *parts, int S, int64_t M, int64_t N, float *C, int64_t ldc, const float *aux,
           const int32_t *stop)
{
    const int64_t n = M * (N / 4);
    hipLaunchKernelGGL(k_fc_sum<EPI>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, parts, S, M * N, (int)M,
                       (int)N, (int)N, C, ldc, aux, stop);
    GS_LAUNCH_CHECK("k_fc_sum");
    return GS_OK;
}

bool aligned16(const void *p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

bool fc_supported(int op, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc)
{
    // K tiles of 64 (bf16) / 32 (fp32) with no tail; 16-B rows; K-strided operands in 4-row blocks
    if (M < 4 || N < 4 || K < 64 || K % 64 != 0 || lda % 4 || ldb % 4 || ldc < N) return false;
    if (M > (1 << 20) || N > (1 << 20) || K > (1 << 20)) return false;
    if (op == 1) return M % 4 == 0 && N % 4 == 0;     // wgrad: both operands K-strided
    if (op == 2) return N % 4 == 0;                   // dgrad: B K-strided
    return true;
}

int fc_fwd_splits(int64_t M, int64_t N, int64_t K)
{
    // the largest split of K into 64-multiples that keeps the 32 x 32 tiles x splits within 512
    // workgroups (at most 16 slices)
    const int64_t tiles = ((M + 31) / 32) * ((N + 31) / 32);
    int best = 1;
    for (int sp = 2; sp <= 16; ++sp)
        if (K % (64 * sp) == 0 && tiles * sp <= 512) best = sp;
    return best;
}

int fc_fwd_partials(hipStream_t s, int splits, int64_t M, int64_t N, int64_t K, const float *A, int64_t lda,
                    const float *B, int64_t ldb, float *C, int64_t ldc)
{
    GS_REQUIRE(splits >= 1 && K % (64 * splits) == 0 && fc_supported(0, M, N, K / splits, lda, ldb, ldc),
               "fc_fwd_partials: shape %lld x %lld x %lld / %d not supported", (long long)M, (long long)N,
               (long long)K, splits);
    GS_REQUIRE(aligned16(A) && aligned16(B), "fc_fwd_partials: 16-B aligned operands required");
    return launch_fc<32, 32, 1, 4, true, true, kEpiStore, FC_PD_FWD32, FC_PD_FWD16, 2, 1>(
        s, false, A, lda, B, ldb, C, ldc, M, N, K, nullptr, nullptr, 4, splits, M * ldc);
}

int fc_gemm(hipStream_t s, int op, bool bf16, int64_t M, int64_t N, int64_t K, const void *A, int64_t lda,
            const void *B, int64_t ldb, float *C, int64_t ldc, const void *aux, const int32_t *stop, float *parts,
            bool act16, ActOut ao)
{
    GS_REQUIRE(!ao.cnt || (op == 0 && !parts), "fc_gemm: activation statistics: the single-pass forward only");
    GS_REQUIRE(op >= 0 && op <= 2, "fc_gemm: op %d", op);
    GS_REQUIRE(fc_supported(op, M, N, K, lda, ldb, ldc), "fc_gemm: shape %lld x %lld x %lld (op %d) not supported",
               (long long)M, (long long)N, (long long)K, op);
    GS_REQUIRE(aligned16(A) && aligned16(B) && (op == 1 || aux), "fc_gemm: 16-B aligned operands (and the epilogue "
               "operand) required");
    GS_REQUIRE(!act16 || (bf16 && !parts), "fc_gemm: bf16 activation storage needs bf16 operands, no partials");
    if (op == 0) {   // fwd: C = relu(A B^T + bias), both K-contiguous
        // fp32 with a partials buffer: 64 x 64 tiles (waves 2 x 1 x KS 2, 32 x 64 each) over two K
        // halves, summed in slice order with the bias + ReLU epilogue (tools/fc_sweep.py, round 5:
        // 42.95 vs 47.16 us back to back at the C4 shape, but 43.6 + 5.0 vs 46.0 us inside the
        // update, which therefore passes no partials buffer); K/2 must be whole 32-deep tiles
        if (!bf16 && parts && K % 64 == 0 && N % 4 == 0 && ldc == N) {
            int rc = launch_fc<64, 64, 2, 2, true, true, kEpiStore, 2, 2, 1, 1>(s, false, A, lda, B, ldb, parts, N, M, N,
                                                                               K, nullptr, stop, 4, 2, M * N);
            if (rc) return rc;
            return fc_sum<kEpiBiasRelu>(s, static_cast<float *>(parts), 2, M, N, C, ldc,
                                        static_cast<const float *>(aux), stop);
        }
        if (act16)      // A = a3, B = Wf: bf16 storage
            return launch_fc<32, 32, 1, 4, true, true, kEpiBiasRelu, FC_PD_FWD32, FC_PD_FWD16, 2, 1, false, 3>(
                s, true, A, lda, B, ldb, C, ldc, M, N, K, aux, stop, 4, 1, 0, ao);
        return launch_fc<32, 32, 1, 4, true, true, kEpiBiasRelu, FC_PD_FWD32, FC_PD_FWD16, 2, 1>(
            s, bf16, A, lda, B, ldb, C, ldc, M, N, K, aux, stop, 4, 1, 0, ao);
    }
    if (op == 1) {   // wgrad: C = A^T B with A [K][M], B [K][N] (the round-5 sweep's 16x16x4 form: 46.2
                     // vs 47.9 us back to back, 46.9 vs 46.7 inside the update — kept on 32x32x2)
        if (act16)      // A = dh, B = a3: bf16 storage
            return launch_fc<64, 64, 2, 1, false, false, kEpiStore, FC_PD_WG32, FC_PD_WG16, 2, 1, false, 3>(
                s, true, A, lda, B, ldb, C, ldc, M, N, K, nullptr, stop, 8);
        return launch_fc<64, 64, 2, 1, false, false, kEpiStore, FC_PD_WG32, FC_PD_WG16, 2, 1>(s, bf16, A, lda, B, ldb, C,
                                                                                            ldc, M, N, K, nullptr, stop, 8);
    }
    // dgrad: C = (A B) * (aux > 0) with A [M][K], B [K][N]
    if (act16)          // A = dh, B = Wf, aux = a3: bf16 storage
        return launch_fc<64, 64, 2, 1, true, false, kEpiMask, FC_PD_DG32, FC_PD_DG16, 2, 1, true, 7>(
            s, true, A, lda, B, ldb, C, ldc, M, N, K, aux, stop, 16);
    return launch_fc<64, 64, 2, 1, true, false, kEpiMask, FC_PD_DG32, FC_PD_DG16, 2, 1, true>(s, bf16, A, lda, B, ldb, C,
                                                                                                ldc, M, N, K, aux, stop, 16);
}

}  // namespace gs

using namespace gs;

extern "C" int gs_fc_gemm(int op, int bf16, int64_t M, int64_t N, int64_t K, const float *A, int64_t lda,
                          const float *B, int64_t ldb, float *C, int64_t ldc, const float *aux, float *parts,
                          void *stream)
{
    GS_REQUIRE(A && B && C, "gs_fc_gemm: null operand");
    return fc_gemm((hipStream_t)stream, op, bf16 != 0, M, N, K, A, lda, B, ldb, C, ldc, aux, nullptr, parts, false,
                   ActOut{});
}

#ifdef GS_FC_SWEEP
// Launch-shape sweep of the fc products for tools/fc_sweep.py (diagnostic builds only,
// build_lib.build_variant with GS_FC_SWEEP): variant v of product op, fp32 / bf16 operands; split-K
// variants write partials to `parts` (splits x M x N floats) and sum them in slice order.
// Returns GS_E_INVALID for a variant this op does not have.
extern "C" int gs_debug_fc_variant(int op, int v, int bf16, int64_t M, int64_t N, int64_t K, const float *A,
                                   int64_t lda, const float *B, int64_t ldb, float *C, int64_t ldc, const float *aux,
                                   float *parts, void *stream)
{
    hipStream_t s = (hipStream_t)stream;
    const bool bf = bf16 != 0;
    auto split = [&](auto launch, int S, auto epi) -> int {
        constexpr int E = decltype(epi)::value;
        int rc = launch(S);
        if (rc) return rc;
        return fc_sum<E>(s, parts, S, M, N, C, ldc, aux, nullptr);
    };
    using EBR = std::integral_constant<int, kEpiBiasRelu>;
    using EST = std::integral_constant<int, kEpiStore>;
    if (op == 0) {
        switch (v) {
        case 0: return launch_fc<32, 32, 1, 4, true, true, kEpiBiasRelu, 3, 2, 2, 1>(s, bf, A, lda, B, ldb, C, ldc, M, N, K, aux, nullptr, 4);
        case 1: return launch_fc<64, 32, 1, 4, true, true, kEpiBiasRelu, 2, 2, 2, 1>(s, bf, A, lda, B, ldb, C, ldc, M, N, K, aux, nullptr, 4);
        case 2: return launch_fc<32, 64, 1, 4, true, true, kEpiBiasRelu, 2, 2, 2, 1>(s, bf, A, lda, B, ldb, C, ldc, M, N, K, aux, nullptr, 4);
        case 3: return launch_fc<64, 32, 1, 4, true, true, kEpiBiasRelu, 2, 2, 4, 2>(s, bf, A, lda, B, ldb, C, ldc, M, N, K, aux, nullptr, 4);
        case 4: return split([&](int S) { return launch_fc<128, 64, 2, 2, true, true, kEpiStore, 2, 2, 1, 1>(
                                 s, bf, A, lda, B, ldb, parts, N, M, N, K, nullptr, nullptr, 4, S, M * N); }, 7, EBR{});
        case 5: return split([&](int S) { return launch_fc<64, 64, 2, 2, true, true, kEpiStore, 2, 2, 1, 1>(
                                 s, bf, A, lda, B, ldb, parts, N, M, N, K, nullptr, nullptr, 4, S, M * N); }, 2, EBR{});
        case 6: return launch_fc<64, 32, 1, 4, true, true, kEpiBiasRelu, 3, 3, 2, 1>(s, bf, A, lda, B, ldb, C, ldc, M, N, K, aux, nullptr, 4);
        // round 6: 128 x 128 tiles (2 x 2 waves of 64 x 64, a quarter of the
        // L2 -> LDS bytes per MFMA of the 32 x 32 tiles) split over K so 224 / 256 workgroups fill the
        // chip, the bias + ReLU epilogue in the ordered sum
        case 7: return split([&](int S) { return launch_fc<128, 128, 2, 1, true, true, kEpiStore, 2, 2, 1, 1>(
                                 s, bf, A, lda, B, ldb, parts, N, M, N, K, nullptr, nullptr, 4, S, M * N); }, 7, EBR{});
        case 8: return split([&](int S) { return launch_fc<128, 64, 2, 1, true, true, kEpiStore, 2, 2, 1, 1>(
                                 s, bf, A, lda, B, ldb, parts, N, M, N, K, nullptr, nullptr, 4, S, M * N); }, 7, EBR{});
        default: break;
        }
    } else if (op == 1) {
        switch (v) {
        case 0: return launch_fc<64, 64, 2, 1, false, false, kEpiStore, 2, 2, 2, 1>(s, bf, A, lda, B, ldb, C, ldc, M, N, K, nullptr, nullptr, 8);
        case 1: return launch_fc<64, 64, 1, 4, false, false, kEpiStore, 2, 2, 2, 1>(s, bf, A, lda, B, ldb, C, ldc, M, N, K, nullptr, nullptr, 8);
        case 2: return launch_fc<128, 64, 2, 2, false, false, kEpiStore, 2, 2, 2, 1>(s, bf, A, lda, B, ldb, C, ldc, M, N, K, nullptr, nullptr, 4);
        case 3: return split([&](int S) { return launch_fc<128, 64, 2, 2, false, false, kEpiStore, 2, 2, 2, 1>(
                                 s, bf, A, lda, B, ldb, parts, N, M, N, K, nullptr, nullptr, 4, S, M * N); }, 2, EST{});
        case 4: return launch_fc<64, 64, 1, 4, false, false, kEpiStore, 2, 2, 4, 2>(s, bf, A, lda, B, ldb, C, ldc, M, N, K, nullptr, nullptr, 8);
        case 5: return launch_fc<64, 64, 2, 1, false, false, kEpiStore, 2, 2, 2, 1, true>(s, bf, A, lda, B, ldb, C, ldc, M, N, K, nullptr, nullptr, 8);
        case 6: return split([&](int S) { return launch_fc<128, 128, 2, 1, false, false, kEpiStore, 2, 2, 1, 1>(
                                 s, bf, A, lda, B, ldb, parts, N, M, N, K, nullptr, nullptr, 4, S, M * N); }, 2, EST{});
        case 7: return split([&](int S) { return launch_fc<128, 128, 2, 1, false, false, kEpiStore, 2, 2, 1, 1>(
                                 s, bf, A, lda, B, ldb, parts, N, M, N, K, nullptr, nullptr, 4, S, M * N); }, 4, EST{});
        default: break;
        }
    } else if (op == 2) {
        switch (v) {
        case 0: return launch_fc<64, 64, 2, 1, true, false, kEpiMask, 2, 2, 2, 1, true>(s, bf, A, lda, B, ldb, C, ldc, M, N, K, aux, nullptr, 16);
        case 1: return launch_fc<64, 64, 1, 4, true, false, kEpiMask, 2, 2, 2, 1>(s, bf, A, lda, B, ldb, C, ldc, M, N, K, aux, nullptr, 16);
        case 2: return launch_fc<128, 64, 2, 2, true, false, kEpiMask, 2, 2, 2, 1>(s, bf, A, lda, B, ldb, C, ldc, M, N, K, aux, nullptr, 8);
        case 3: return launch_fc<128, 64, 2, 2, true, false, kEpiMask, 2, 2, 2, 1, true>(s, bf, A, lda, B, ldb, C, ldc, M, N, K, aux, nullptr, 8);
        case 4: return launch_fc<64, 64, 1, 4, true, false, kEpiMask, 2, 2, 2, 1, true>(s, bf, A, lda, B, ldb, C, ldc, M, N, K, aux, nullptr, 16);
        case 5: return launch_fc<64, 64, 2, 1, true, false, kEpiMask, 2, 2, 2, 1>(s, bf, A, lda, B, ldb, C, ldc, M, N, K, aux, nullptr, 16);
        default: break;
        }
    }
    GS_REQUIRE(false, "gs_debug_fc_variant: op %d has no variant %d", op, v);
    return GS_E_INVALID;
}
#endif

namespace gs {
// statistics slots of the fc forward's stats epilogue (32 x 32 tiles, 4 waves each)
int fc_fwd_act_slots(int64_t M, int64_t N) { return (int)(4 * ((N + 31) / 32) * ((M + 31) / 32)); }
}  // namespace gs
