// MLP actor-critic forward / PPO loss / backward / clip + Adam kernels for gfx950.
//
// Reference ops replaced (SURVEY.md §2 native-work table rows 1, 3-6, 8):
//   MLPActorCritic.forward         utils/models.py:328-346 (+ build_mlp :20-53)
//   Categorical log_prob/entropy   utils/policy_ops.py:44-75 -> torch.distributions
//   PPOAgent.losses_for_batch      agents/ppo/ppo_agent.py:21-152
//   batch_normalize / KL metrics   utils/torch.py:97-119
//   manual_backward + clip_grad_norm_ + Adam.step   agents/base_agent.py:591-621
//   slice_trajectories (collate)   utils/rollout_collector.py:657-682
//
// All arithmetic is fp32 (the reference never leaves fp32).  The three
// B x H x H products of a minibatch step (forward h2, dW2, dh1) run on the exact-f32
// MFMA v_mfma_f32_16x16x4_f32 (64 FLOP/clk/SIMD, = the f32 vector peak); partial tiles
// are summed through LDS in a fixed order, so results are deterministic run to run.
// K = obs_dim and N = A+1 (heads) products are VALU dot products fused into the
// neighbouring kernels.
//
// At B = 256 every kernel is latency-bound, not throughput-bound: the design rule is
// that each kernel has at most two dependent global round trips.  Every operand a
// workgroup needs is fetched in ONE cooperative, vectorised phase into LDS (all loads
// in flight together), then the math runs out of LDS/registers.
//
// One minibatch step = 4 launches (the dependency chain has exactly 3 all-to-all seams:
// h2 -> logits, loss -> dh2/dh1, grads -> global norm):
//   k_fwd_hidden  : gather rows by sampler index (+ the step's act/logp/value/adv/ret
//                   fields), h1 = relu(x W1^T + b1) recomputed per workgroup, h2 tile on
//                   MFMA, per-tile partial head dot products
//   k_loss        : one workgroup: logits/value, log-softmax, ratio, clipped surrogate,
//                   clipped value loss, entropy, batch advantage normalisation, all
//                   metrics, and the analytic dLoss/dlogits, dLoss/dvalue
//   k_bwd         : dW2 tiles (MFMA, K = batch), dh1 slabs (MFMA, K = H2) + dW1/db1
//                   partials per 64 rows, head weight/bias grads; dh2 = relu'(h2) (dz Wh)
//                   is recomputed on the fly, never stored; per-tile sum of squares
//   k_clip_adam   : global grad norm from the per-tile sums (identical in every
//                   workgroup), clip coefficient, torch.optim.Adam update
#include <float.h>

#include <mutex>
#include <unordered_map>

#include "gs_common.h"
#include "gs_xgmi_dev.h"
#include "gs_synth_env.h"

namespace gs {

#ifdef GS_STAMPS
__device__ unsigned long long g_stamp_acc[8][16];
__device__ unsigned long long g_stamp_cnt[8];
#endif
#if defined(GS_STAMPS) || defined(GS_SPANS)
// chain timeline (diagnostic build): per minibatch k < kSpanK and workgroup, the start (thread 0)
// and each wave's end after its memory ops drained, low 32 bits of s_memrealtime (100 MHz, one
// clock for the whole device); plain per-workgroup stores (atomics on shared words would
// serialise and distort the timeline); kernel 0 = lagged forward, 1 = k_bwd
constexpr int kSpanK = 2048, kSpanWG = 288;
__device__ unsigned g_span[2][kSpanK][kSpanWG][9];   // start + up to 8 wave ends
__device__ __forceinline__ int span_wg() { return (int)(blockIdx.x + blockIdx.y * gridDim.x); }
__device__ __forceinline__ void span_start(int kern, int64_t k, unsigned long long t0)
{
    if (threadIdx.x == 0 && k >= 0 && k < kSpanK && span_wg() < kSpanWG) g_span[kern][k][span_wg()][0] = (unsigned)t0;
}
__device__ __forceinline__ void span_end(int kern, int64_t k)
{
    if ((threadIdx.x & 63) == 0 && k >= 0 && k < kSpanK && span_wg() < kSpanWG) {
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        g_span[kern][k][span_wg()][1 + (threadIdx.x >> 6)] = (unsigned)__builtin_amdgcn_s_memrealtime();
    }
}
#define GS_SPAN_T0 const unsigned long long _sp_t0 = __builtin_amdgcn_s_memrealtime();
#define GS_SPAN_START(slot, k) span_start(slot, k, _sp_t0);
#define GS_SPAN_END(slot, k) span_end(slot, k);
#else
#define GS_SPAN_T0
#define GS_SPAN_START(slot, k) ;
#define GS_SPAN_END(slot, k) ;
#endif

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c)
{
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// bf16 mode: two K-chunks of 16 (lane quarter q's k = 4q..4q+3 of each chunk, the fp32 chain's
// operand layout) as one v_mfma_f32_16x16x32_bf16 — elements 0..3 from chunk c, 4..7 from chunk
// c + 1, the same order in both operands, so the product sums all 32 k; fp32 accumulation
__device__ __forceinline__ f32x4 mfma_bf16_pair(float4 a0, float4 a1, float4 b0, float4 b1, f32x4 c)
{
    return mfma16_bf16(bf16_frag(a0, a1), bf16_frag(b0, b1), c);
}
__device__ __forceinline__ float4 f4(const float (&v)[4]) { return make_float4(v[0], v[1], v[2], v[3]); }

// env-major sample index (utils/rollout_buffer.py:11-13) -> time-major buffer row
__device__ __forceinline__ int sample_row(int s, int T, int N)
{
    const unsigned e = (unsigned)s / (unsigned)T;
    const unsigned t = (unsigned)s - e * (unsigned)T;
    return (int)(t * (unsigned)N + e);
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__host__ __device__ constexpr int round4(int n) { return (n + 3) & ~3; }

constexpr int kNumSums = 14;   // metric sums of one minibatch (loss_row)

// Sum NV per-thread values over the 256-thread block in a fixed order (deterministic),
// through LDS (two levels of 16) — __shfl would lower to ds_bpermute chains (~100+ cycles
// per step).  Every thread returns the totals.  scratch: NV*(256+16) elements of T.
// In a block wider than 256 threads only threads 0..255 contribute (the others only meet the
// barriers and read the totals), so the sum order is the 256-thread one.
template <int NV, typename T>
__device__ __forceinline__ void block_reduce(T (&v)[NV], T *scratch)
{
    const int tid = threadIdx.x;
    if (tid < 256)
#pragma unroll
        for (int k = 0; k < NV; ++k) scratch[k * 256 + tid] = v[k];
    __syncthreads();
    T *part = scratch + NV * 256;
    if (tid < NV * 16) {
        const int k = tid >> 4, j = tid & 15;
        T acc = 0;
#pragma unroll
        for (int m = 0; m < 16; ++m) acc += scratch[k * 256 + j * 16 + m];
        part[tid] = acc;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        T acc = 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) acc += part[k * 16 + j];
        v[k] = acc;
    }
    __syncthreads();
}

__device__ __forceinline__ void store_component_norms(double (&hq)[2], double total_sq, float gscale, float *rec,
                                                      double *scratch)
{
    block_reduce<2>(hq, scratch);
    if (threadIdx.x == 0 && rec) {
        rec[GS_M_GN_POLICY_HEAD] = (float)sqrt(hq[0]) * gscale;
        rec[GS_M_GN_VALUE_HEAD] = (float)sqrt(hq[1]) * gscale;
        rec[GS_M_GN_BACKBONE] = (float)sqrt(fmax(0.0, total_sq - hq[0] - hq[1])) * gscale;
        rec[GS_M_GN_MLP] = 0.0f;
    }
}

// block_reduce's sums for thread 0 only (the others keep their own inputs): the same order and
// the same two levels, without the broadcast level and its trailing barrier — for epilogues
// whose single reader is thread 0 and which touch the scratch no more.
template <int NV, typename T>
__device__ __forceinline__ void block_reduce_t0(T (&v)[NV], T *scratch)
{
    const int tid = threadIdx.x;
    if (tid < 256)
#pragma unroll
        for (int k = 0; k < NV; ++k) scratch[k * 256 + tid] = v[k];
    __syncthreads();
    T *part = scratch + NV * 256;
    if (tid < NV * 16) {
        const int k = tid >> 4, j = tid & 15;
        T acc = 0;
#pragma unroll
        for (int m = 0; m < 16; ++m) acc += scratch[k * 256 + j * 16 + m];
        part[tid] = acc;
    }
    __syncthreads();
    if (tid == 0)
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            T acc = 0;
#pragma unroll
            for (int j = 0; j < 16; ++j) acc += part[k * 16 + j];
            v[k] = acc;
        }
}

// copy n floats global -> LDS, vectorised when both sides are 16-B aligned
__device__ __forceinline__ void copy_to_lds(float *dst, const float *src, int n)
{
    const int tid = threadIdx.x;
    if ((((uintptr_t)src | (uintptr_t)dst) & 15) == 0) {
        const int n4 = n >> 2;
#pragma unroll 8
        for (int u = tid; u < n4; u += 256)
            reinterpret_cast<float4 *>(dst)[u] = reinterpret_cast<const float4 *>(src)[u];
        for (int u = (n4 << 2) + tid; u < n; u += 256) dst[u] = src[u];
    } else {
#pragma unroll 4
        for (int u = tid; u < n; u += 256) dst[u] = src[u];
    }
}

// clip_grad_norm_'s coefficient (max_norm <= 0: no clip; agents/base_agent.py:591-621)
__device__ __forceinline__ float clip_coef(float total, const AdamArgs &aa)
{
    float coef = 1.0f;
    if (aa.max_norm > 0.0f) {
        coef = aa.max_norm / (total + 1e-6f);
        coef = fminf(coef, 1.0f);
    }
    return coef;
}

// Per-component pre-clip gradient norms of one step (utils/models.py:196-230 compute_grad_norms,
// recorded at agents/base_agent.py:607-608): policy_head and value_head from their gradients in G,
// backbone as the rest of the step's squared total (every component of the MLP policy is one of
// the three).  hq: this thread's {policy, value} sums of squares; every thread of the block calls
// it (threads 0..255 contribute); scratch: 2 x (256 + 16) doubles; thread 0 writes the record.
__device__ __forceinline__ void store_component_norms(double (&hq)[2], double total_sq, float gscale, float *rec,
                                                      double *scratch);
// head gradient u of the flat head index space: u < A1*H2 the weight rows (policy rows 0..A-1, then
// the value row), past it the A1 biases; *value = whether it belongs to the value head
__host__ __device__ inline int64_t head_grad_offset(const Layout &L, int u, bool *value)
{
    const int nw = (L.A + 1) * L.H2;
    if (u < nw) {
        const int a = u / L.H2;
        *value = a == L.A;
        return L.head_row(a) + (u - a * L.H2);
    }
    *value = u - nw == L.A;
    return L.head_bias(u - nw);
}

// One parameter of torch.optim.Adam (single-tensor path, amsgrad off) on the clipped gradient;
// shared by k_clip_adam and the lagged step in k_fwd_hidden so both round identically.
// inv_bc2s = f32(1 / sqrt(1 - beta2^t)) (host, double), so the bias correction is a multiply.
__device__ __forceinline__ float adam_param(float graw, float coef, float &m, float &v, float &p,
                                            const AdamArgs &aa, float neg_step, float inv_bc2s)
{
    const float g = graw * coef;
    m = m + aa.one_minus_b1 * (g - m);            // exp_avg.lerp_(grad, 1 - beta1)
    v = v * aa.b2;                                // exp_avg_sq.mul_(beta2)
    v = v + (aa.one_minus_b2 * g) * g;            //   .addcmul_(grad, grad, 1 - beta2)
    // hardware sqrt and reciprocal (v_sqrt_f32, v_rcp_f32: ~1 ulp each) instead of torch's
    // correctly rounded divisions: IEEE division lowers to a v_div_scale / v_div_fmas /
    // v_div_fixup sequence serialised through VCC, ~10x the latency, and this runs 4-21 times
    // per thread on the minibatch chain's critical path
    const float denom = __builtin_amdgcn_sqrtf(v) * inv_bc2s + aa.eps;
    p = p + neg_step * (m * __builtin_amdgcn_rcpf(denom));
    return g;
}

// ------------------------------------------------------------------------------------
// k_fwd_hidden: grid (ceil(H2/16), ceil(rows/16)), 256 threads.
// LDS (floats): srcs[16] W1s[H1*D] b1s[H1] W2s[16][H1+4] b2s[16] whs[A1][16] xs[16][D]
//               h1s[16][H1+4] red[4][256] h2s[16][17]
// ------------------------------------------------------------------------------------
size_t fwd_lds_bytes(const Layout &L)
{
    const int A1 = L.A + 1;
    size_t n = 16 + round4(L.H1 * L.D) + round4(L.H1) + kTile * (L.H1 + 4) + 16 + round4(A1 * 16) +
               round4(kTile * L.D) + kTile * (L.H1 + 4) + 1024 + kTile * 17;
    return n * sizeof(float);
}

template <int AMAX, int AEX>
__device__ __forceinline__ void gather_head_row(const float *__restrict__ zpart, const float *__restrict__ P,
                                                const Layout &L, int64_t r, float (&z)[AMAX + 1]);
template <int AMAX>
__device__ __forceinline__ void loss_row(const float (&z)[AMAX + 1], int A, int act, float olp, float ov, float adv,
                                         float ret, const LossArgs &la, float invB, float *__restrict__ dzr,
                                         double (&acc)[14]);

// FUSED (gs_ppo_update path): x comes pre-gathered (FusedFwd::xg, one load instead of the
// index -> row -> obs chain).  The head combine stays in the next launch (k_loss_rows): an
// in-launch last-arriver combine costs a release + acquire fence pair (~1.7 us each on
// gfx950) on top of the skew wait, more than the ~1.45 us kernel boundary it would remove.
//
// ADAM (the lagged chain's forward) runs 512 threads (kFwdAdamThreads): two waves per SIMD share
// the Adam step on the workgroup's W1|b1 and W2 rows and the h1 rows, so the prologue's
// per-thread arithmetic halves; the global norm keeps the 256-thread grouping (threads 0..255,
// k_clip_adam's order) and the h2 MFMA stays on waves 0..3, so every value is bit-identical to
// the 256-thread kernel.
#ifndef GS_FWD_ADAM_NT
#define GS_FWD_ADAM_NT 512
#endif
constexpr int kFwdAdamThreads = GS_FWD_ADAM_NT;
static_assert(kFwdAdamThreads == 256 || kFwdAdamThreads == 512, "lagged forward: 256 or 512 threads");

// STATS (GS_HP_ACT_STATS, fused chain): the workgroup also records the activation statistics of its
// rows (FusedFwd::act, kActRec words): dead counts of the 16 h1 columns of chunk cb and of its 16 h2
// columns and the float sums of z and z^2 of both (the pre-activation values of the forward hooks on
// backbone.0 / backbone.2, utils/models.py:121-147), on the block's last wave after the h2 epilogue
template <class S, bool FUSED, bool ADAM = false, bool STATS = false>
__global__ __launch_bounds__(ADAM ? kFwdAdamThreads : 256) void k_fwd_hidden(
    const float *__restrict__ P, Layout Lrt, const float *__restrict__ obs, const int32_t *__restrict__ idx, int T,
    int N, int rows, float *__restrict__ x_out, float *__restrict__ h1_out, float *__restrict__ h2_out,
    float *__restrict__ zpart, float *__restrict__ obs_copy, const int32_t *__restrict__ stop, RowGather rg,
    FusedFwd ff, LossArgs la, uint16_t *__restrict__ h2mask, AdamFwd af = AdamFwd{})
{
    GS_STAMP_BEGIN(0)
    GS_SPAN_T0
    if (stop && *stop) return;
    extern __shared__ float lds[];
    const Layout L = S::lay(Lrt);
    const int D = L.D, H1 = L.H1, H2 = L.H2, A1 = L.A + 1;
    const int cb = blockIdx.x, rb = blockIdx.y;
    const int r0 = rb * kTile;
    const int c0 = cb * kTile;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int NT = ADAM ? kFwdAdamThreads : 256;     // threads per workgroup
    const int ldh = H1 + 4;
    int *srcs = reinterpret_cast<int *>(lds);
    float *W1s = lds + 16;
    float *b1s = W1s + round4(H1 * D);
    float *W2s = b1s + round4(H1);
    float *b2s = W2s + kTile * ldh;
    float *whs = b2s + 16;
    float *xs = whs + round4(A1 * 16);
    float *h1s = xs + round4(kTile * D);
    float *red = h1s + kTile * ldh;
    float *h2s = red + 1024;

    if (rg.step_base && idx) idx += *rg.step_base * rows;
    const int64_t kstep = FUSED ? ff.k_local + (ff.step_base ? *ff.step_base : 0) : 0;
    if constexpr (ADAM) GS_SPAN_START(0, kstep)
    // ---- phase 0: every operand of this workgroup, all loads in flight together.
    //      Threads 0..15 run the dependent idx -> row -> obs/fields chain while the rest
    //      of the block streams the weights into LDS.
    // compile-time shapes on the fused path: every phase-0 operand goes to registers first
    // (one memory round trip), then to LDS
    constexpr bool kStage0 = FUSED && S::H1c > 0 && (S::H1c * 4) % 4 == 0;
    constexpr int kW2v = S::H1c > 0 ? kTile * S::H1c / 4 / NT : 0;
    float4 w2r[kW2v > 0 ? kW2v : 1];
    static_assert(!ADAM || (kStage0 && kW2v > 0), "lagged Adam: compile-time fused shapes only");
    if constexpr (ADAM) {
        // ---- lagged optimizer step: minibatch k-1's clip + Adam (k_clip_adam<S, NRB, NQ>'s
        //      norm order and per-parameter arithmetic, so the result is bit-identical) on the
        //      parameters this workgroup reads: W1|b1, its 16 W2 rows, its b2 and head-weight
        //      slices, and in workgroup (0,0) the head biases.  Every load is issued in one burst
        //      with the forward's own; row block 0 writes the results into the other parameter
        //      set (the rest of the grid still reads this one).
        constexpr Layout Lc = S::lay(Layout{});
        constexpr int cD = Lc.D, cH1 = Lc.H1, cA1 = Lc.A + 1, n1 = cH1 * (cD + 1), k4n = cH1 / 4;
        constexpr int NQ = (n1 / 4 + 255) / 256, NRB = (S::Bc + S::RB - 1) / S::RB, NS = 2;
        static_assert(Lc.oW1 == 0 && Lc.oW2 == n1 && (cH1 * cD) % 4 == 0 && cH1 % 4 == 0, "W1|b1: one float4 region");
        static_assert(NRB >= 1 && NRB <= 8 && NQ <= 2 && n1 <= kTile * (cH1 + 4), "lagged-Adam register / LDS budget");
        const AdamArgs &aa = af.aa;
        // multi-GPU chain: the exchange has already folded dW1|db1 into G (parameter order) and
        // its per-workgroup sums of squares cover the whole gradient (k_clip_adam<S, 0, 0>'s order)
        const bool fold = af.part1 != nullptr;
        const int64_t kprev = kstep - 1 + af.force;
        const bool apply = kprev >= 0;
        const bool own1 = apply && cb == 0 && rb == 0, own2 = apply && rb == 0;
        const bool stW2[3] = {own2, own2, own2};
        const bool stW1[3] = {own1, own1, own1};
        const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
        // global-address-space float4 loads (the AdamFwd pointers would otherwise lower to flat,
        // and a predicated float4 select to four dword loads); the moment / gradient buffers are
        // valid memory at k = 0 too, so only the range conditions stay
        auto ld4 = [](const float *base, int64_t q) {
            const f32x4 v = *(const __attribute__((address_space(1))) f32x4 *)(base + 4 * q);
            return make_float4(v[0], v[1], v[2], v[3]);
        };
        auto ld1 = [](const float *base, int64_t o) { return *(const __attribute__((address_space(1))) float *)(base + o); };
        // Every vector load below is unconditional, at an index clamped into its array, and the
        // lanes past an array's end discard what they loaded: a predicated load (`ok ? load : 0`)
        // compiles to an exec-masked branch per load, and the register moves around those
        // branches force s_waitcnt vmcnt stalls in the middle of the burst (one memory round trip
        // per stall instead of one for the whole prologue)
        constexpr int nq1 = n1 / 4;
        // Adam: W1|b1 quad q = tid + NT*j; norm partials: threads 0..255, quad tid + 256*j (the
        // 256-thread grouping of k_clip_adam, wave-uniform branch for the wider block)
        constexpr int NQP = (nq1 + NT - 1) / NT;
        const bool nrm = NT == 256 || tid < 256;
        // The lanes that take no part in the norm (waves 4..7 of a 512-thread block) load quad 0,
        // and without the fold (G already holds dW1|db1) every partial slot re-reads G: no load
        // sits in a branch, and no loaded register is merged with a constant at a join — either
        // puts an s_waitcnt vmcnt(0) inside the burst, a memory round trip each.  The unused
        // values are dropped where they are consumed.
        // Issue order = the order the phases consume them (vmcnt counts in order): the norm's
        // slots and partials first, so the fold + norm start while the Adam operands are in flight.
        float sl[NS];     // slots past n_slots and the non-norm lanes are dropped in the norm
#pragma unroll
        for (int j = 0; j < NS; ++j) sl[j] = ld1(af.sumsq, nrm ? min(tid + 256 * j, aa.n_slots - 1) : 0);
        float4 w1p[NQP], w1m[NQP], w1v[NQP], t[NQ][NRB];  // W1|b1 (param order), dW1|db1 partials
        const float *tsrc = fold ? af.part1 : af.G;
        const int64_t tstride = fold ? (int64_t)n1 : 0;
        const int nrb_used = fold ? NRB : 1;
#pragma unroll
        for (int j = 0; j < NQ; ++j)
#pragma unroll
            for (int b = 0; b < NRB; ++b)
                t[j][b] = ld4(tsrc + (int64_t)b * tstride, nrm ? min(tid + 256 * j, nq1 - 1) : 0);
#pragma unroll
        for (int j = 0; j < NQP; ++j) {
            const int q = min(tid + NT * j, nq1 - 1);
            w1p[j] = ld4(P, q);
            w1m[j] = ld4(af.Min, q);
            w1v[j] = ld4(af.Vin, q);
        }
        float4 w2m[kW2v], w2v[kW2v], w2g[kW2v];           // this workgroup's 16 W2 rows
#pragma unroll
        for (int j = 0; j < kW2v; ++j) {
            const int u = tid + NT * j, i = u / k4n, k4 = u - i * k4n;
            const int64_t q = (Lc.oW2 + (int64_t)min(c0 + i, H2 - 1) * cH1) / 4 + k4;
            w2r[j] = ld4(P, q);
            w2m[j] = ld4(af.Min, q);
            w2v[j] = ld4(af.Vin, q);
            w2g[j] = ld4(af.G, q);
        }
        // scalar slices {p, m, v, g}: b2 (threads < 16), head weights (< 16*A1), head biases ((0,0), < A1)
        const int64_t ob = tid < kTile && c0 + tid < H2 ? Lc.ob2 + c0 + tid : -1;
        const int64_t ow = tid < cA1 * kTile && c0 + (tid & 15) < H2 ? Lc.head_row(tid >> 4) + c0 + (tid & 15) : -1;
        const int64_t oh = own1 && tid < cA1 ? Lc.head_bias(tid) : -1;
        float sb[4], sw[4], shb[4];
        auto load_slice = [&](float (&e)[4], int64_t o) {
            const int64_t oc = o < 0 ? 0 : o;
            e[0] = ld1(P, oc);
            e[1] = ld1(af.Min, oc);
            e[2] = ld1(af.Vin, oc);
            e[3] = ld1(af.G, oc);
        };
        load_slice(sb, ob);
        load_slice(sw, ow);
        load_slice(shb, oh);
        // then the loads behind the graph replay's step base: this minibatch's x rows (stored to
        // LDS after the Adam step, where nothing waits for them) and step k-1's schedule entries
        const bool okx = tid < kTile * cD && r0 + min(tid / cD, kTile - 1) < rows;
        const float xv = ff.xg[(kstep * rows + r0) * cD + (okx ? tid : 0)];
        const float neg_step = apply && aa.sched ? aa.sched[2 * kprev] : aa.neg_step_size;
        const float bc2s = apply && aa.sched ? aa.sched[2 * kprev + 1] : aa.inv_bc2_sqrt;
#ifdef GS_STAMPS
        __builtin_amdgcn_s_waitcnt(0);     // diagnostic build only: split "loads landed" from the norm
        __syncthreads();
#endif
        GS_STAMP(0)
        // global norm -> clip coefficient: the per-tile slots, then the folded dW1|db1 (k_clip_adam's order)
        float coef = 0.0f;
        float *w1g = h1s;      // dW1|db1: part1 order when folded here, else parameter order (h1s is unused until phase 1)
        if (apply) {
            double ss = 0.0;
#pragma unroll
            for (int j = 0; j < NS; ++j)
                if (nrm && tid + 256 * j < aa.n_slots) ss += (double)sl[j];
#pragma unroll
            for (int j = 0; j < NQ; ++j) {
                if (!nrm) break;
                float4 g = z4;
#pragma unroll
                for (int b = 0; b < NRB; ++b) {
                    if (b >= nrb_used) break;
                    g.x += t[j][b].x;
                    g.y += t[j][b].y;
                    g.z += t[j][b].z;
                    g.w += t[j][b].w;
                }
                if (4 * (tid + 256 * j) < n1) {
                    reinterpret_cast<float4 *>(w1g)[tid + 256 * j] = g;
                    if (fold) {
                        ss += (double)g.x * (double)g.x;
                        ss += (double)g.y * (double)g.y;
                        ss += (double)g.z * (double)g.z;
                        ss += (double)g.w * (double)g.w;
                    }
                }
            }
            double tt[1] = {ss};
            block_reduce<1>(tt, reinterpret_cast<double *>(red));   // its barriers also publish w1g
            const float total = (float)sqrt(tt[0]) * aa.grad_scale;
            coef = clip_coef(total, aa) * aa.grad_scale;
            if (own1 && tid == 0 && af.metrics) af.metrics[kprev * GS_NUM_METRICS + GS_M_GRAD_NORM] = total;
            if (own1 && tid == 0 && aa.normsq)
                aa.normsq[kprev] = tt[0] * (double)aa.grad_scale * (double)aa.grad_scale;
        }
        GS_STAMP(1)
        // Adam on the owned parameters: new values to LDS / registers, and from row block 0 to the other set
#pragma unroll
        for (int j = 0; j < NQP; ++j) {
            const int q = tid + NT * j;
            if (4 * q >= n1) continue;
            float4 p4 = w1p[j];
            if (apply) {
                float p[4] = {p4.x, p4.y, p4.z, p4.w};
                float m[4] = {w1m[j].x, w1m[j].y, w1m[j].z, w1m[j].w};
                float v[4] = {w1v[j].x, w1v[j].y, w1v[j].z, w1v[j].w};
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    adam_param(w1g[fold ? part1_index(Lc, 4 * q + e) : 4 * q + e], coef, m[e], v[e], p[e], aa,
                               neg_step, bc2s);
                p4 = make_float4(p[0], p[1], p[2], p[3]);
                // the new W1|b1 p / m / v are stored by three different workgroups of row block 3
                // (workgroup-uniform choice: one workgroup storing all three drained last)
                if (stW1[0]) reinterpret_cast<float4 *>(af.Pout)[q] = p4;
                if (stW1[1]) reinterpret_cast<float4 *>(af.Mout)[q] = make_float4(m[0], m[1], m[2], m[3]);
                if (stW1[2]) reinterpret_cast<float4 *>(af.Vout)[q] = make_float4(v[0], v[1], v[2], v[3]);
            }
            reinterpret_cast<float4 *>(W1s)[q] = p4;
        }
        if (apply) {
#pragma unroll
            for (int j = 0; j < kW2v; ++j) {
                const int u = tid + NT * j, i = u / k4n, k4 = u - i * k4n;
                if (c0 + i >= H2) continue;
                float p[4] = {w2r[j].x, w2r[j].y, w2r[j].z, w2r[j].w};
                float m[4] = {w2m[j].x, w2m[j].y, w2m[j].z, w2m[j].w};
                float v[4] = {w2v[j].x, w2v[j].y, w2v[j].z, w2v[j].w};
                const float g[4] = {w2g[j].x, w2g[j].y, w2g[j].z, w2g[j].w};
#pragma unroll
                for (int e = 0; e < 4; ++e) adam_param(g[e], coef, m[e], v[e], p[e], aa, neg_step, bc2s);
                w2r[j] = make_float4(p[0], p[1], p[2], p[3]);
                // this column block's 16 new W2 rows: p by row block 0, m by 1, v by 2 (16 KB each)
                const int64_t q = (Lc.oW2 + (int64_t)(c0 + i) * cH1) / 4 + k4;
                if (stW2[0]) reinterpret_cast<float4 *>(af.Pout)[q] = w2r[j];
                if (stW2[1]) reinterpret_cast<float4 *>(af.Mout)[q] = make_float4(m[0], m[1], m[2], m[3]);
                if (stW2[2]) reinterpret_cast<float4 *>(af.Vout)[q] = make_float4(v[0], v[1], v[2], v[3]);
            }
        }
        auto step_slice = [&](float (&e)[4], int64_t o, bool own) {
            if (o < 0 || !apply) return;
            adam_param(e[3], coef, e[1], e[2], e[0], aa, neg_step, bc2s);
            if (own) {
                af.Pout[o] = e[0];
                af.Mout[o] = e[1];
                af.Vout[o] = e[2];
            }
        };
        step_slice(sb, ob, own2);
        step_slice(sw, ow, own2);
        step_slice(shb, oh, own1);
        if (tid < kTile) b2s[tid] = ob < 0 ? 0.0f : sb[0];
        if (tid < cA1 * kTile) whs[tid] = ow < 0 ? 0.0f : sw[0];
        if (tid < kTile * cD) xs[tid] = okx ? xv : 0.0f;
        GS_STAMP(2)
    } else if constexpr (kStage0) {
        constexpr Layout Lc = S::lay(Layout{});
        constexpr int cD = Lc.D, cH1 = Lc.H1, cA1 = Lc.A + 1;
        static_assert((cH1 * cD) % 4 == 0 && cH1 % 4 == 0, "float4 staging");
        constexpr int NW1 = (cH1 * cD / 4 + 255) / 256, NB1 = (cH1 / 4 + 255) / 256;
        float4 w1v[NW1], b1v[NB1];
        float xv = 0.0f, b2v = 0.0f, whv = 0.0f;
        if (tid < kTile * cD) {
            const int i = tid / cD;
            xv = r0 + i < rows ? ff.xg[(kstep * rows + r0) * cD + tid] : 0.0f;
        }
#pragma unroll
        for (int j = 0; j < NW1; ++j) {
            const int u = tid + 256 * j;
            w1v[j] = u < cH1 * cD / 4 ? reinterpret_cast<const float4 *>(P + Lc.oW1)[u] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int j = 0; j < NB1; ++j) {
            const int u = tid + 256 * j;
            b1v[j] = u < cH1 / 4 ? reinterpret_cast<const float4 *>(P + Lc.ob1)[u] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        if (tid < kTile) b2v = c0 + tid < H2 ? P[Lc.ob2 + c0 + tid] : 0.0f;
        if (tid < cA1 * kTile) {
            const int a = tid >> 4, j = tid & 15;
            whv = c0 + j < H2 ? P[Lc.head_row(a) + c0 + j] : 0.0f;
        }
        if (tid < kTile * cD) xs[tid] = xv;
#pragma unroll
        for (int j = 0; j < NW1; ++j)
            if (tid + 256 * j < cH1 * cD / 4) reinterpret_cast<float4 *>(W1s)[tid + 256 * j] = w1v[j];
#pragma unroll
        for (int j = 0; j < NB1; ++j)
            if (tid + 256 * j < cH1 / 4) reinterpret_cast<float4 *>(b1s)[tid + 256 * j] = b1v[j];
        if (tid < kTile) b2s[tid] = b2v;
        if (tid < cA1 * kTile) whs[tid] = whv;
    } else if (FUSED) {
        if (tid < kTile * D) {
            const int i = tid / D;
            xs[tid] = r0 + i < rows ? ff.xg[(kstep * rows + r0) * D + tid] : 0.0f;
        }
    } else if (tid < kTile) {
        const int r = r0 + tid;
        // a negative index is another rank's row of a global minibatch (gs_ppo_update_global):
        // zero observation, action -1 (no loss, no gradient)
        const int si = r < rows ? (idx ? idx[r] : r) : -1;
        const int src = si >= 0 ? (idx ? sample_row(si, T, N) : si) : -1;
        srcs[tid] = src;
        for (int d = 0; d < D; ++d) xs[tid * D + d] = src >= 0 ? obs[(int64_t)src * D + d] : 0.0f;
        if (cb == 0 && rg.f_act && src >= 0) {
            rg.f_act[r] = (int32_t)rg.actions[src];
            rg.f_olp[r] = rg.logprobs[src];
            rg.f_ov[r] = rg.values[src];
            rg.f_adv[r] = rg.advantages[src];
            rg.f_ret[r] = rg.returns[src];
        } else if (cb == 0 && rg.f_act && r < rows) {
            rg.f_act[r] = -1;
            rg.f_olp[r] = rg.f_ov[r] = rg.f_adv[r] = rg.f_ret[r] = 0.0f;
        }
    }
    if constexpr (!kStage0) {
        copy_to_lds(W1s, P + L.oW1, H1 * D);
        copy_to_lds(b1s, P + L.ob1, H1);
        if (tid < kTile) b2s[tid] = c0 + tid < H2 ? P[L.ob2 + c0 + tid] : 0.0f;
        if (tid < A1 * kTile) {
            const int a = tid >> 4, j = tid & 15;
            whs[tid] = c0 + j < H2 ? P[L.head_row(a) + c0 + j] : 0.0f;
        }
    }
    // W2 tile: with compile-time shapes the loads go to registers AFTER the h1 operands, so the
    // barrier below waits only for those (in-order vmcnt) and h1 is computed while the 16 KB
    // tile is still in flight; it is written to LDS after h1.
    if constexpr (ADAM) {
        // w2r holds the updated tile: to LDS now, under the barrier below (the lagged forward forms
        // h1 in registers inside the MFMA loop, so there is no h1 phase to overlap it with)
        const int k4n = H1 >> 2;
#pragma unroll
        for (int j = 0; j < kW2v; ++j) {
            const int u = tid + NT * j, i = u / k4n, k4 = u - i * k4n;
            *reinterpret_cast<float4 *>(W2s + i * ldh + 4 * k4) = w2r[j];
        }
    } else if constexpr (kW2v > 0) {
        const int k4n = H1 >> 2;
#pragma unroll
        for (int j = 0; j < kW2v; ++j) {
            const int u = tid + NT * j, i = u / k4n, k4 = u - i * k4n;
            w2r[j] = c0 + i < H2 ? *reinterpret_cast<const float4 *>(P + L.oW2 + (int64_t)(c0 + i) * H1 + 4 * k4)
                                 : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    } else {
        const int k4n = H1 >> 2;
#pragma unroll 4
        for (int u = tid; u < kTile * k4n; u += 256) {
            const int i = u / k4n, k4 = u - i * k4n;
            float4 w = make_float4(0.f, 0.f, 0.f, 0.f);
            if (c0 + i < H2) w = *reinterpret_cast<const float4 *>(P + L.oW2 + (int64_t)(c0 + i) * H1 + 4 * k4);
            *reinterpret_cast<float4 *>(W2s + i * ldh + 4 * k4) = w;
        }
    }
    __syncthreads();
    GS_STAMP(3)
    // ---- phase 1: h1 = relu(x W1^T + b1) out of LDS; one hidden unit per thread, rows
    //      [i0, i0 + RPT) of the tile (all 16 with 256 threads, 8 with 512)
    constexpr int RPT = kTile * 256 / NT;
    const int i0 = (tid >> 8) * RPT;
    // the lagged forward (ADAM) has no h1 phase: h1 = relu(x W1^T + b1) is formed in registers,
    // as the h2 MFMA's A operand on waves 0..3 and for the h1 store share on waves 4..7, with this
    // loop's arithmetic and order (bit-identical values; no h1 tile, one barrier less)
    if constexpr (!ADAM)
    for (int k = tid & 255; k < H1; k += 256) {
        float w[8];
        const bool small = D <= 8;
#pragma unroll
        for (int d = 0; d < 8; ++d) w[d] = (small && d < D) ? W1s[k * D + d] : 0.0f;
        const float bk = b1s[k];
        if (small && D % 4 == 0) {
            // every x row first (float4 LDS reads; xs is 16-B aligned), then the 16 outputs: the
            // h1s stores may alias xs as far as the compiler knows, so reads interleaved with them
            // would each wait for the LDS round trip
            float4 xq[RPT][2];
#pragma unroll
            for (int i = 0; i < RPT; ++i)
#pragma unroll
                for (int d4 = 0; d4 < 2; ++d4)
                    xq[i][d4] = 4 * d4 < D ? reinterpret_cast<const float4 *>(xs + (i0 + i) * D)[d4]
                                           : make_float4(0.f, 0.f, 0.f, 0.f);
            float hv[RPT];
#pragma unroll
            for (int i = 0; i < RPT; ++i) {
                const float xr[8] = {xq[i][0].x, xq[i][0].y, xq[i][0].z, xq[i][0].w,
                                     xq[i][1].x, xq[i][1].y, xq[i][1].z, xq[i][1].w};
                float acc = 0.0f;
#pragma unroll
                for (int d = 0; d < 8; ++d)
                    if (d < D) acc = fmaf(xr[d], w[d], acc);
                acc += bk;
                hv[i] = acc > 0.0f ? acc : 0.0f;
            }
#pragma unroll
            for (int i = 0; i < RPT; ++i) h1s[(i0 + i) * ldh + k] = hv[i];
        } else if (small) {
#pragma unroll
            for (int i = i0; i < i0 + RPT; ++i) {
                float xr[8];
#pragma unroll
                for (int d = 0; d < 8; ++d) xr[d] = d < D ? xs[i * D + d] : 0.0f;
                float acc = 0.0f;
#pragma unroll
                for (int d = 0; d < 8; ++d)
                    if (d < D) acc = fmaf(xr[d], w[d], acc);
                acc += bk;
                h1s[i * ldh + k] = acc > 0.0f ? acc : 0.0f;
            }
        } else {
            for (int i = i0; i < i0 + RPT; ++i) {
                float acc = 0.0f;
                for (int d = 0; d < D; ++d) acc = fmaf(xs[i * D + d], W1s[k * D + d], acc);
                acc += bk;
                h1s[i * ldh + k] = acc > 0.0f ? acc : 0.0f;
            }
        }
    }
    if constexpr (kW2v > 0 && !ADAM) {
        const int k4n = H1 >> 2;
#pragma unroll
        for (int j = 0; j < kW2v; ++j) {
            const int u = tid + NT * j, i = u / k4n, k4 = u - i * k4n;
            *reinterpret_cast<float4 *>(W2s + i * ldh + 4 * k4) = w2r[j];
        }
    }
    if constexpr (!ADAM) __syncthreads();
    GS_STAMP(4)
    // h1[i][k..k+3] from the LDS x row and W1 / b1 (ADAM path): phase 1's fmaf order over d,
    // then + b1, then relu
    auto h1_quad = [&](int i, int k) {
        static_assert(!ADAM || (S::lay(Layout{}).D % 4 == 0 && S::lay(Layout{}).D <= 8), "h1 in registers: D = 4 or 8");
        constexpr int cD = ADAM ? S::lay(Layout{}).D : 4;
        float xr[8];
#pragma unroll
        for (int d4 = 0; d4 < 2; ++d4) {
            const float4 v = 4 * d4 < cD ? *reinterpret_cast<const float4 *>(xs + i * cD + 4 * d4)
                                         : make_float4(0.f, 0.f, 0.f, 0.f);
            xr[4 * d4] = v.x, xr[4 * d4 + 1] = v.y, xr[4 * d4 + 2] = v.z, xr[4 * d4 + 3] = v.w;
        }
        const float4 bq = *reinterpret_cast<const float4 *>(b1s + k);
        const float bk[4] = {bq.x, bq.y, bq.z, bq.w};
        float h[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float w[8];
#pragma unroll
            for (int d4 = 0; d4 < 2; ++d4) {
                const float4 v = 4 * d4 < cD ? *reinterpret_cast<const float4 *>(W1s + (k + j) * cD + 4 * d4)
                                             : make_float4(0.f, 0.f, 0.f, 0.f);
                w[4 * d4] = v.x, w[4 * d4 + 1] = v.y, w[4 * d4 + 2] = v.z, w[4 * d4 + 3] = v.w;
            }
            float acc = 0.0f;
#pragma unroll
            for (int d = 0; d < 8; ++d)
                if (d < cD) acc = fmaf(xr[d], w[d], acc);
            acc += bk[j];
            h[j] = acc > 0.0f ? acc : 0.0f;
        }
        return make_float4(h[0], h[1], h[2], h[3]);
    };
    // x rows and this workgroup's share of h1 to HBM (read only xs / h1s, final from here on):
    // in a 512-thread block waves 4..7 store them while waves 0..3 run the h2 MFMA
    const int nrow = min(kTile, rows - r0);
    auto store_x_h1 = [&](int t0, int stride) {
        if (cb == 0)
            for (int u = t0; u < nrow * D; u += stride) {
                if (x_out) x_out[(int64_t)r0 * D + u] = xs[u];
                if (obs_copy) obs_copy[(int64_t)r0 * D + u] = xs[u];
            }
        if (h1_out) {
            // every column-block workgroup of this row block holds all of h1: the store is split
            // between them (H1/16 units each) instead of falling on column block 0 alone
            const int k4n = H1 >> 2, ncbw = gridDim.x;
            const int kb0 = (cb * k4n) / ncbw, kb1 = ((cb + 1) * k4n) / ncbw, nk = kb1 - kb0;
            for (int u = t0; u < nrow * nk; u += stride) {
                const int i = u / nk, k4 = kb0 + (u - i * nk);
                *reinterpret_cast<float4 *>(h1_out + (int64_t)(r0 + i) * H1 + 4 * k4) =
                    ADAM ? h1_quad(i, 4 * k4) : *reinterpret_cast<const float4 *>(h1s + i * ldh + 4 * k4);
            }
        }
    };
    constexpr bool kEarly = NT == 512;
    if (kEarly && wave >= 4) store_x_h1(tid - 256, 256);
    // ---- phase 2: h2 tile = h1[16 x H1] . W2[c0:c0+16, :]^T, MFMA, K split over 4 waves
    //      (waves 0..3 of a wider block: the K ranges and their sum order stay those of 4 waves)
    if (wave < 4) {
        const int i = lane & 15, q = lane >> 4;
        const int nch = H1 / kTile;
        const int ch0 = (wave * nch) / 4, ch1 = ((wave + 1) * nch) / 4;
        f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
        if constexpr (S::BF) {
            const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 2
            for (int ch = ch0; ch < ch1; ch += 2) {
                const int k = ch * kTile + 4 * q;
                const bool two = ch + 1 < ch1;
                const float4 a0 = ADAM ? h1_quad(i, k) : *reinterpret_cast<const float4 *>(h1s + i * ldh + k);
                const float4 b0 = *reinterpret_cast<const float4 *>(W2s + i * ldh + k);
                const float4 a1 = !two ? z4 : ADAM ? h1_quad(i, k + kTile)
                                                   : *reinterpret_cast<const float4 *>(h1s + i * ldh + k + kTile);
                const float4 b1 = two ? *reinterpret_cast<const float4 *>(W2s + i * ldh + k + kTile) : z4;
                acc0 = mfma_bf16_pair(a0, a1, b0, b1, acc0);
            }
        } else {
#pragma unroll 4
        for (int ch = ch0; ch < ch1; ++ch) {
            const int k = ch * kTile + 4 * q;
            const float4 a = ADAM ? h1_quad(i, k) : *reinterpret_cast<const float4 *>(h1s + i * ldh + k);
            const float4 b = *reinterpret_cast<const float4 *>(W2s + i * ldh + k);
            acc0 = mfma4(a.x, b.x, acc0);
            acc1 = mfma4(a.y, b.y, acc1);
            acc0 = mfma4(a.z, b.z, acc0);
            acc1 = mfma4(a.w, b.w, acc1);
        }
        }
        const f32x4 acc = acc0 + acc1;
#pragma unroll
        for (int r = 0; r < 4; ++r) red[wave * 256 + (q * 4 + r) * kTile + i] = acc[r];
    }
    __syncthreads();
    GS_STAMP(5)
    if (tid < 256) {
        const int row = tid >> 4, col = tid & 15;
        const float s = ((red[tid] + red[256 + tid]) + red[512 + tid]) + red[768 + tid];
        float h = 0.0f;
        if (c0 + col < H2) {
            h = s + b2s[col];
            // the pre-activation z2 into this thread's own partial slot (read above, by it alone)
            if constexpr (STATS) red[tid] = h;
            h = h > 0.0f ? h : 0.0f;
            if (h2_out && r0 + row < rows) h2_out[(int64_t)(r0 + row) * H2 + c0 + col] = h;
        } else if constexpr (STATS) {
            red[tid] = 0.0f;
        }
        h2s[row * 17 + col] = h;
    }
    __syncthreads();
    if constexpr (STATS) {
        // lanes 0..15: h1 column cb*16 + c (z1 = x W1^T + b1 from the LDS operands, h1_quad's
        // order), lanes 16..31: h2 column c0 + c (red); 16 rows each (fused: B % 16 == 0)
        if (wave == NT / 64 - 1 && lane < 32) {
            const bool l2 = lane >= 16;
            const int c = lane & 15;
            const bool have = l2 ? c0 + c < H2 : cb * kTile + c < H1;
            const int k1 = min(cb * kTile + c, H1 - 1);
            float w1[8];
#pragma unroll
            for (int d = 0; d < 8; ++d) w1[d] = d < D ? W1s[k1 * D + d] : 0.0f;
            const float bk = b1s[k1];
            float sz = 0.0f, sq = 0.0f;
            unsigned dead = 0;
#pragma unroll 4
            for (int i = 0; i < kTile; ++i) {
                float z;
                if (l2) {
                    z = red[i * kTile + c];
                } else {
                    float acc = 0.0f;
#pragma unroll
                    for (int d = 0; d < 8; ++d)
                        if (d < D) acc = fmaf(xs[i * D + d], w1[d], acc);
                    z = acc + bk;
                }
                sz += z;
                sq += z * z;
                dead += fabsf(z) < 1e-6f ? 1u : 0u;
            }
            if (!have) sz = 0.0f, sq = 0.0f, dead = 0u;
#pragma unroll
            for (int o = 8; o > 0; o >>= 1) {
                sz += __shfl_xor(sz, o, 64);
                sq += __shfl_xor(sq, o, 64);
            }
            const unsigned word = dead | (__shfl_down(dead, 1, 64) << 8) | (__shfl_down(dead, 2, 64) << 16) |
                                  (__shfl_down(dead, 3, 64) << 24);
            uint32_t *out = ff.act + ((kstep * gridDim.y + rb) * gridDim.x + cb) * kActRec;
            if ((c & 3) == 0) out[(l2 ? 4 : 0) + (c >> 2)] = word;
            if (c == 0) {
                out[8 + (l2 ? 2 : 0)] = __float_as_uint(sz);
                out[9 + (l2 ? 2 : 0)] = __float_as_uint(sq);
            }
        }
    }
    // relu'(h2) bits of each row's 16 columns (a 512-thread block: on wave 4, beside the heads)
    const int hm = tid - (NT == 512 ? 256 : 0);
    if (h2mask && hm >= 0 && hm < kTile && r0 + hm < rows) {
        unsigned m = 0;
#pragma unroll
        for (int c = 0; c < kTile; ++c) m |= (h2s[hm * 17 + c] > 0.0f ? 1u : 0u) << c;
        h2mask[(int64_t)(r0 + hm) * gridDim.x + cb] = (uint16_t)m;
    }
    // ---- phase 3: partial head outputs over this tile's 16 hidden units
    const int ncbz = gridDim.x;
    for (int u = tid; u < kTile * A1; u += NT) {
        const int row = u / A1, a = u - row * A1;
        if (r0 + row >= rows) continue;
        float z = 0.0f;
#pragma unroll
        for (int c = 0; c < kTile; ++c) z = fmaf(h2s[row * 17 + c], whs[a * 16 + c], z);
        zpart[((int64_t)(r0 + row) * ncbz + cb) * A1 + a] = z;
    }
    if (!kEarly) store_x_h1(tid, NT);
    GS_STAMP_END(6)
    if constexpr (ADAM) GS_SPAN_END(0, kstep)
}

static int set_lds_limit(const void *fn, size_t bytes);
template <class F>
static int with_shape(const Layout &L, int64_t B, F &&f);

int launch_fwd_hidden(const float *params, const Layout &L, const float *obs, const int32_t *idx, int64_t T,
                      int64_t N, int64_t rows, float *x_out, float *h1_out, float *h2_out, float *zpart,
                      float *obs_copy, const int32_t *stop_flag, const RowGather *rg, hipStream_t s,
                      uint16_t *h2mask)
{
    const dim3 grid((unsigned)((L.H2 + kTile - 1) / kTile), (unsigned)((rows + kTile - 1) / kTile));
    RowGather g{};
    if (rg) g = *rg;
    return with_shape(L, 0, [&](auto sh) {
        using Sh = decltype(sh);
        int rc = set_lds_limit((const void *)k_fwd_hidden<Sh, false>, fwd_lds_bytes(L));
        if (rc) return rc;
        hipLaunchKernelGGL((k_fwd_hidden<Sh, false>), grid, dim3(256), fwd_lds_bytes(L), s, params, L, obs, idx,
                           (int)T, (int)N, (int)rows, x_out, h1_out, h2_out, zpart, obs_copy, stop_flag, g,
                           FusedFwd{}, LossArgs{}, h2_out ? h2mask : (uint16_t *)nullptr);
        GS_LAUNCH_CHECK("k_fwd_hidden");
        return GS_OK;
    });
}

// ------------------------------------------------------------------------------------
// per-row categorical head math shared by rollout and loss kernels
// ------------------------------------------------------------------------------------
struct HeadRow {
    float lse;    // logsumexp of raw logits
    float m2;     // max of normalised logits
    float S;      // sum exp(ln - m2)
};

// z: raw logits of one row held in registers (AMAX = compile-time bound on A).
template <int AMAX>
__device__ __forceinline__ HeadRow head_stats(const float (&z)[AMAX + 1], int A)
{
    float m = -INFINITY;
#pragma unroll
    for (int a = 0; a < AMAX; ++a)
        if (a < A) m = fmaxf(m, z[a]);
    float se = 0.0f;
#pragma unroll
    for (int a = 0; a < AMAX; ++a)
        if (a < A) se += expf(z[a] - m);
    HeadRow h;
    h.lse = m + logf(se);
    float m2 = -INFINITY;
#pragma unroll
    for (int a = 0; a < AMAX; ++a)
        if (a < A) m2 = fmaxf(m2, z[a] - h.lse);
    h.m2 = m2;
    float S = 0.0f;
#pragma unroll
    for (int a = 0; a < AMAX; ++a)
        if (a < A) S += expf((z[a] - h.lse) - m2);
    h.S = S;
    return h;
}

// logits/value of row r from the per-16-column partials (+ bias): the row's partials are
// contiguous ([row][col-block][A+1]) and are loaded as one burst before any add.
// AEX = exact action count when known at compile time (static register indexing), else 0.
template <int AMAX, int AEX>
__device__ __forceinline__ void gather_head_row(const float *__restrict__ zpart, const float *__restrict__ P,
                                                const Layout &L, int64_t r, float (&z)[AMAX + 1])
{
    const int ncb = (L.H2 + kTile - 1) / kTile;
#pragma unroll
    for (int a = 0; a < AMAX + 1; ++a) z[a] = 0.0f;
    if constexpr (AEX > 0) {
        constexpr int A1c = AEX + 1;
        const float *zp = zpart + r * ncb * A1c;
        if (ncb == 16 && (16 * A1c) % 4 == 0) {
            // the row's 16 x A1 partials as float4 loads (one burst), summed in column-block order
            // (zpart is 256-B aligned in the workspace and a row is 16 x A1 floats: 16-B aligned)
            constexpr int NV = 16 * A1c / 4;
            float buf[16 * A1c];
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                const float4 q = reinterpret_cast<const float4 *>(zp)[v];
                buf[4 * v + 0] = q.x;
                buf[4 * v + 1] = q.y;
                buf[4 * v + 2] = q.z;
                buf[4 * v + 3] = q.w;
            }
#pragma unroll
            for (int j = 0; j < 16; ++j)
#pragma unroll
                for (int a = 0; a < A1c; ++a) z[a] += buf[j * A1c + a];
        } else
        for (int cb0 = 0; cb0 < ncb; cb0 += 16) {
            float buf[16][A1c];
#pragma unroll
            for (int j = 0; j < 16; ++j)
#pragma unroll
                for (int a = 0; a < A1c; ++a) buf[j][a] = cb0 + j < ncb ? zp[(cb0 + j) * A1c + a] : 0.0f;
#pragma unroll
            for (int j = 0; j < 16; ++j)
#pragma unroll
                for (int a = 0; a < A1c; ++a) z[a] += buf[j][a];
        }
    } else {
        const int A1 = L.A + 1;
        const float *zp = zpart + r * ncb * A1;
        for (int cb = 0; cb < ncb; ++cb) {
#pragma unroll
            for (int a = 0; a < AMAX + 1; ++a)
                if (a < A1) z[a] += zp[cb * A1 + a];
        }
    }
    const int A1 = L.A + 1;
#pragma unroll
    for (int a = 0; a < AMAX + 1; ++a)
        if (a < A1) z[a] += P[L.head_bias(a)];
}

__device__ __forceinline__ uint64_t mix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// ------------------------------------------------------------------------------------
// k_heads_act: rollout head — logits/value from partials, action select, log_prob.
// one thread per env row.
// ------------------------------------------------------------------------------------
// value, action (sampled / argmax / replayed) and its log-prob of one env row from its raw
// logits | value z; ctr = the rollout step's counter of the counter-based uniform
template <int AMAX>
__device__ __forceinline__ void head_act_row(const float (&z)[AMAX + 1], int A, int mode, uint64_t seed, uint64_t ctr,
                                             int64_t r, int64_t *__restrict__ action, float *__restrict__ logp,
                                             float *__restrict__ value)
{
    float v = 0.0f;
#pragma unroll
    for (int a = 0; a < AMAX + 1; ++a)
        if (a == A) v = z[a];
    if (value) *value = v;
    if (!action) return;
    const HeadRow h = head_stats<AMAX>(z, A);
    int act = 0;
    if (mode == 2) {            // replay recorded actions
        act = (int)*action;
    } else if (mode == 1) {     // Categorical.mode = probs.argmax(-1), first max wins
        float best = -INFINITY;
#pragma unroll
        for (int a = 0; a < AMAX; ++a) {
            if (a < A) {
                const float p = expf((z[a] - h.lse) - h.m2) / h.S;
                if (p > best) { best = p; act = a; }
            }
        }
        *action = act;
    } else {                    // inverse-CDF sample with a counter-based uniform
        const uint64_t hh = mix64(mix64(mix64(seed) ^ ctr) ^ (uint64_t)r);
        const float u = (float)(hh >> 40) * (1.0f / 16777216.0f);
        float c = 0.0f;
        act = -1;
#pragma unroll
        for (int a = 0; a < AMAX; ++a) {
            if (a < A) {
                c += expf((z[a] - h.lse) - h.m2) / h.S;
                if (act < 0 && u < c) act = a;
            }
        }
        if (act < 0) act = A - 1;
        *action = act;
    }
    float za = 0.0f;
#pragma unroll
    for (int a = 0; a < AMAX; ++a)
        if (a == act) za = z[a];
    *logp = za - h.lse;
}

template <class S>
__global__ __launch_bounds__(256) void k_heads_act(const float *__restrict__ P, Layout Lrt,
                                                   const float *__restrict__ zpart, int64_t rows, int mode,
                                                   uint64_t seed, uint64_t counter, int64_t *__restrict__ actions,
                                                   float *__restrict__ logp, float *__restrict__ value,
                                                   const uint64_t *__restrict__ clock)
{
    constexpr int AMAX = S::AMAX, AEX = S::AEX;
    const Layout L = S::lay(Lrt);
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= rows) return;
    float z[AMAX + 1];
    gather_head_row<AMAX, AEX>(zpart, P, L, r, z);
    const uint64_t ctr = counter + (clock && mode == 0 ? clock[0] : 0ull);   // rollout clock (graph replay)
    head_act_row<AMAX>(z, L.A, mode, seed, ctr, r, actions ? actions + r : nullptr, logp ? logp + r : nullptr,
                       value ? value + r : nullptr);
}

// ------------------------------------------------------------------------------------
// k_rollout_synth: a whole rollout of the synthetic env in one launch (C3-sized MLPs, whose
// weights fit in LDS).  Workgroup = 16 envs (one MFMA row tile) for all T vector steps: the
// policy's act with gs_policy_act's arithmetic in its order (h1 fmaf chain + bias; each h2
// column block's 4 K-range MFMA partials summed in range order, as the 4 waves of
// k_fwd_hidden do; partial heads per column block summed in block order as k_heads_act), so the
// rows are bit-identical to the step-wise rollout; then the env step (gs_synth_env.h).  No
// launch and no HBM round trip per step: the envs' observations stay in LDS.
// LDS (floats): W1 [H1*D] b1 [H1] W2 [H2][H1+4] b2 [H2] Wh [A1][H2] bh [round4(A1)] x [16][D]
//               h1 [16][H1+4] h2 [ncb][16][17] zp [16][ncb][A1]
// ------------------------------------------------------------------------------------
size_t rollout_synth_lds_bytes(const Layout &L)
{
    const int A1 = L.A + 1, ncb = (L.H2 + kTile - 1) / kTile;
    const size_t n = round4(L.H1 * L.D) + round4(L.H1) + (size_t)L.H2 * (L.H1 + 4) + round4(L.H2) +
                     round4(A1 * L.H2) + round4(A1) + round4(kTile * L.D) + kTile * (L.H1 + 4) + (size_t)ncb * kTile * 17 +
                     round4(kTile * ncb * A1);
    return n * sizeof(float);
}

template <class S>
__global__ __launch_bounds__(256) void k_rollout_synth(const float *__restrict__ P, Layout Lrt, int64_t N, int T,
                                                       int mode, uint64_t rng_seed, uint64_t counter0, SynthEnvArgs ev,
                                                       RolloutRows rw)
{
    constexpr int AMAX = S::AMAX;
    const Layout L = S::lay(Lrt);
    const int D = L.D, H1 = L.H1, H2 = L.H2, A = L.A, A1 = A + 1;
    const int ncb = (H2 + kTile - 1) / kTile, nch = H1 / kTile, ldh = H1 + 4;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, li = lane & 15, lq = lane >> 4;
    const int64_t e0 = (int64_t)blockIdx.x * kTile;
    extern __shared__ float lds[];
    float *W1s = lds;
    float *b1s = W1s + round4(H1 * D);
    float *W2s = b1s + round4(H1);
    float *b2s = W2s + (size_t)H2 * ldh;
    float *whs = b2s + round4(H2);
    float *bhs = whs + round4(A1 * H2);
    float *xs = bhs + round4(A1);
    float *h1s = xs + round4(kTile * D);
    float *h2s = h1s + kTile * ldh;
    float *zps = h2s + ncb * kTile * 17;
    // ---- the policy into LDS, once
    for (int u = tid; u < H1 * D; u += 256) W1s[u] = P[L.oW1 + u];
    for (int u = tid; u < H1; u += 256) b1s[u] = P[L.ob1 + u];
    for (int u = tid; u < H2 * (H1 / 4); u += 256) {
        const int n = u / (H1 / 4), k4 = u - n * (H1 / 4);
        *reinterpret_cast<float4 *>(W2s + n * ldh + 4 * k4) =
            *reinterpret_cast<const float4 *>(P + L.oW2 + (int64_t)n * H1 + 4 * k4);
    }
    for (int u = tid; u < H2; u += 256) b2s[u] = P[L.ob2 + u];
    for (int u = tid; u < A1 * H2; u += 256) {
        const int a = u / H2, n = u - a * H2;
        whs[u] = P[L.head_row(a) + n];
    }
    if (tid < A1) bhs[tid] = P[L.head_bias(tid)];
    // ---- this workgroup's envs: state in registers of threads 0..15, observations in LDS
    const int64_t me = e0 + (tid < kTile ? tid : 0);
    const bool env_thread = tid < kTile && me < N;
    int32_t st[3] = {0, 0, 0};
    float er = 0.0f;
    if (env_thread) {
        st[0] = ev.state[4 * me + 0];
        st[1] = ev.state[4 * me + 1];
        st[2] = ev.state[4 * me + 2];
        er = ev.ep_ret[me];
    }
    for (int u = tid; u < kTile * D; u += 256) {
        const int i = u / D;
        xs[u] = e0 + i < N ? ev.obs[(e0 + i) * D + (u - i * D)] : 0.0f;
    }
    constexpr int kW1Reg = 16;
    const bool w1reg = H1 <= 256 && 256 % H1 == 0 && D <= kW1Reg;
    float w1r[kW1Reg];
    float b1r = 0.0f;
    if (w1reg) {
        const int k = tid % H1;
#pragma unroll
        for (int d = 0; d < kW1Reg; ++d) w1r[d] = d < D ? P[L.oW1 + (int64_t)k * D + d] : 0.0f;
        b1r = P[L.ob1 + k];
    }
    __syncthreads();
    for (int t = 0; t < T; ++t) {
        const int64_t row0 = (int64_t)t * N;
        // obs row t of the buffer (the observation the action is taken on)
        for (int u = tid; u < kTile * D; u += 256) {
            const int i = u / D;
            if (e0 + i < N) rw.obs[(row0 + e0 + i) * D + (u - i * D)] = xs[u];
        }
        // h1 = relu(x W1^T + b1): fmaf over d in order, then + b1 (k_fwd_hidden's order)
        if (w1reg) {       // this thread's hidden unit is fixed: its W1 row and bias in registers
            const int k = tid % H1;
            for (int i = tid / H1; i < kTile; i += 256 / H1) {
                float acc = 0.0f;
#pragma unroll
                for (int d = 0; d < kW1Reg; ++d)
                    if (d < D) acc = fmaf(xs[i * D + d], w1r[d], acc);
                acc += b1r;
                h1s[i * ldh + k] = acc > 0.0f ? acc : 0.0f;
            }
        } else {
            for (int u = tid; u < kTile * H1; u += 256) {
                const int i = u / H1, k = u - i * H1;
                float acc = 0.0f;
                for (int d = 0; d < D; ++d) acc = fmaf(xs[i * D + d], W1s[k * D + d], acc);
                acc += b1s[k];
                h1s[i * ldh + k] = acc > 0.0f ? acc : 0.0f;
            }
        }
        __syncthreads();
        // h2 column blocks, one wave each: the 4 K-range partials (k_fwd_hidden's 4 waves) summed
        // in range order, + b2, relu, into h2s[cb]
        for (int cb = wave; cb < ncb; cb += 4) {
            const int c0 = cb * kTile;
            // the 4 partials' MFMA chains interleaved (8 independent accumulators hide the MFMA
            // latency); each partial keeps its own chunk order, so the sums are unchanged
            f32x4 acc0[4], acc1[4], part[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) acc0[q] = acc1[q] = f32x4{0.f, 0.f, 0.f, 0.f};
            const int nmax = (nch + 3) / 4;
            for (int c = 0; c < nmax; ++c) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int ch = (q * nch) / 4 + c;
                    if (ch >= ((q + 1) * nch) / 4) continue;
                    const int k = ch * kTile + 4 * lq;
                    const float4 a = *reinterpret_cast<const float4 *>(h1s + li * ldh + k);
                    const float4 b = c0 + li < H2 ? *reinterpret_cast<const float4 *>(W2s + (c0 + li) * ldh + k)
                                                  : make_float4(0.f, 0.f, 0.f, 0.f);
                    acc0[q] = mfma4(a.x, b.x, acc0[q]);
                    acc1[q] = mfma4(a.y, b.y, acc1[q]);
                    acc0[q] = mfma4(a.z, b.z, acc0[q]);
                    acc1[q] = mfma4(a.w, b.w, acc1[q]);
                }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) part[q] = acc0[q] + acc1[q];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = lq * 4 + r;
                const float s = ((part[0][r] + part[1][r]) + part[2][r]) + part[3][r];
                float h = 0.0f;
                if (c0 + li < H2) {
                    h = s + b2s[c0 + li];
                    h = h > 0.0f ? h : 0.0f;
                }
                h2s[(cb * kTile + row) * 17 + li] = h;
            }
        }
        __syncthreads();
        // partial heads per column block (fmaf over its 16 hidden units in order)
        for (int u = tid; u < ncb * kTile * A1; u += 256) {
            const int cb = u / (kTile * A1), rem = u - cb * kTile * A1, row = rem / A1, a = rem - row * A1;
            float z = 0.0f;
#pragma unroll
            for (int c = 0; c < kTile; ++c) {
                const float w = cb * kTile + c < H2 ? whs[a * H2 + cb * kTile + c] : 0.0f;
                z = fmaf(h2s[(cb * kTile + row) * 17 + c], w, z);
            }
            zps[(row * ncb + cb) * A1 + a] = z;
        }
        __syncthreads();
        // heads + action (threads 0..15, one env each), then the env step
        if (env_thread) {
            float z[AMAX + 1];
#pragma unroll
            for (int a = 0; a < AMAX + 1; ++a) z[a] = 0.0f;
            if constexpr (S::AEX > 0) {     // gather_head_row's order: blocks of 16, zeros past ncb
                for (int cbb = 0; cbb < ncb; cbb += 16)
#pragma unroll
                    for (int j = 0; j < 16; ++j)
#pragma unroll
                        for (int a = 0; a < AMAX + 1; ++a)
                            if (a < A1) z[a] += cbb + j < ncb ? zps[(tid * ncb + cbb + j) * A1 + a] : 0.0f;
            } else {
                for (int cb = 0; cb < ncb; ++cb)
#pragma unroll
                    for (int a = 0; a < AMAX + 1; ++a)
                        if (a < A1) z[a] += zps[(tid * ncb + cb) * A1 + a];
            }
#pragma unroll
            for (int a = 0; a < AMAX + 1; ++a)
                if (a < A1) z[a] += bhs[a];
            const int64_t o = row0 + me;
            head_act_row<AMAX>(z, A, mode, rng_seed, counter0 + (uint64_t)t, me, rw.actions + o, rw.logp + o,
                               rw.value + o);
            const SynthStep so = synth_env_step(st, er, ev.L, ev.trunc_every, ev.reward,
                                                ev.ep_cnt ? ev.ep_cnt + me : nullptr,
                                                ev.ep_ret_sum ? ev.ep_ret_sum + me : nullptr,
                                                ev.ep_len_sum ? ev.ep_len_sum + me : nullptr);
            rw.reward[o] = so.reward;
            rw.done[o] = so.done ? 1 : 0;
            rw.timeout[o] = so.timeout ? 1 : 0;
        }
        // next observations (after step0 + t + 1 vector steps)
        for (int u = tid; u < kTile * D; u += 256) {
            const int i = u / D;
            if (e0 + i < N)
                xs[u] = synth_obs(ev.seed, (uint64_t)(ev.env_offset + e0 + i), ev.step0 + (uint64_t)t + 1,
                                  (uint64_t)(u - i * D));
        }
        __syncthreads();
    }
    // ---- the envs' state and observations back
    if (env_thread) {
        ev.state[4 * me + 0] = st[0];
        ev.state[4 * me + 1] = st[1];
        ev.state[4 * me + 2] = st[2];
        ev.ep_ret[me] = er;
    }
    for (int u = tid; u < kTile * D; u += 256) {
        const int i = u / D;
        if (e0 + i < N) ev.obs[(e0 + i) * D + (u - i * D)] = xs[u];
    }
}

bool rollout_synth_fits(const Layout &L)
{
    return L.H1 % kTile == 0 && L.H1 >= kTile && rollout_synth_lds_bytes(L) <= 160 * 1024;
}

int launch_rollout_synth(const float *P, const Layout &L, int64_t N, int T, int mode, uint64_t rng_seed,
                         uint64_t counter0, const SynthEnvArgs &ev, const RolloutRows &rw, hipStream_t s)
{
    GS_REQUIRE(rollout_synth_fits(L), "gs_rollout_synth: the policy does not fit in LDS");
    const size_t lds = rollout_synth_lds_bytes(L);
    const dim3 grid((unsigned)((N + kTile - 1) / kTile));
    return with_shape(L, 0, [&](auto sh) {
        int rc = set_lds_limit((const void *)k_rollout_synth<decltype(sh)>, lds);
        if (rc) return rc;
        hipLaunchKernelGGL(k_rollout_synth<decltype(sh)>, grid, dim3(256), lds, s, P, L, N, T, mode, rng_seed,
                           counter0, ev, rw);
        GS_LAUNCH_CHECK("k_rollout_synth");
        return GS_OK;
    });
}

// ------------------------------------------------------------------------------------
// One minibatch row of PPOAgent.losses_for_batch (agents/ppo/ppo_agent.py:21-152) with its
// analytic gradients: z = raw logits | value, adv already batch-normalised.  Writes
// dLoss/dlogits | dLoss/dvalue to dzr and adds the row's terms to the 14 metric sums.
// ------------------------------------------------------------------------------------
template <int AMAX>
__device__ __forceinline__ void loss_row(const float (&z)[AMAX + 1], int A, int act, float olp, float ov, float adv,
                                         float ret, const LossArgs &la, float invB, float *__restrict__ dzr,
                                         double (&acc)[kNumSums])
{
    float v = 0.0f;
#pragma unroll
    for (int a = 0; a < AMAX + 1; ++a)
        if (a == A) v = z[a];
    const HeadRow h = head_stats<AMAX>(z, A);
    const float invS = 1.0f / h.S;
    // ln = normalised logits, p = softmax(ln) (Categorical.probs), pe = exp(ln)
    float ln[AMAX], p[AMAX];
    float H = 0.0f, lp = 0.0f;
#pragma unroll
    for (int a = 0; a < AMAX; ++a) {
        ln[a] = z[a] - h.lse;
        p[a] = a < A ? expf(ln[a] - h.m2) * invS : 0.0f;
        if (a < A) {
            H += fmaxf(ln[a], -FLT_MAX) * p[a];   // entropy: -sum clamp(ln, f32min) * p
            if (a == act) lp = ln[a];
        }
    }
    H = -H;
    const float ratio = expf(lp - olp);
    const float rc = fminf(fmaxf(ratio, la.clip_lo), la.clip_hi);
    const float s1 = adv * ratio, s2 = adv * rc;
    const float mn = fminf(s1, s2);
    const float vdelta = v - ov;
    const float du = v - ret;
    const float vu = du * du;
    const float vcl = ov + fminf(fmaxf(vdelta, -la.clip_vf), la.clip_vf);
    const float dc = vcl - ret;
    const float vc = dc * dc;
    const float vmax = fmaxf(vu, vc);
    const float ldiff = fminf(fmaxf(lp - olp, -20.0f), 20.0f);
    const float r2 = expf(ldiff);
    const float akl = (r2 - 1.0f) - logf(r2);
    const float rv = ret - v;
    acc[0] += (double)mn;
    acc[1] += (double)vmax;
    acc[2] += (double)H;
    acc[3] += (ratio < la.clip_lo || ratio > la.clip_hi) ? 1.0 : 0.0;
    acc[4] += (vdelta < -la.clip_vf || vdelta > la.clip_vf) ? 1.0 : 0.0;
    acc[5] += (double)(olp - lp);
    acc[6] += (double)akl;
    acc[7] += (double)rv;
    acc[8] += (double)rv * (double)rv;
    acc[9] += (double)ret;
    acc[10] += (double)ret * (double)ret;
    acc[11] += (double)adv;
    acc[12] += (double)adv * (double)adv;
    // ---- analytic gradients (torch autograd tie rules: min/max ties split halves)
    const float ga = s1 < s2 ? 1.0f : (s1 == s2 ? 0.5f : 0.0f);
    const float gb = s2 < s1 ? 1.0f : (s1 == s2 ? 0.5f : 0.0f);
    const float inclip = (ratio >= la.clip_lo && ratio <= la.clip_hi) ? 1.0f : 0.0f;
    const float g_mn = -invB;
    const float dratio = adv * (g_mn * ga) + adv * (g_mn * gb) * inclip;
    const float dlp = dratio * ratio;
    const float dH = -la.ent_coef * invB;
#pragma unroll
    for (int a = 0; a < AMAX; ++a) {
        if (a < A) {
            const float pe = expf(ln[a]);   // softmax(z) as seen by logsumexp backward
            float g = dlp * ((a == act ? 1.0f : 0.0f) - pe);
            g += dH * (-p[a] * (ln[a] + H));
            dzr[a] = g;
        }
    }
    const float hu = vu > vc ? 1.0f : (vu == vc ? 0.5f : 0.0f);
    const float hc = vc > vu ? 1.0f : (vu == vc ? 0.5f : 0.0f);
    const float invc = (vdelta >= -la.clip_vf && vdelta <= la.clip_vf) ? 1.0f : 0.0f;
    const float gv = la.vf_coef * invB;
    dzr[A] = (gv * hu) * (2.0f * du) + (gv * hc) * (2.0f * dc) * invc;
}

// metrics record from the 14 sums (shared by k_loss and the fused path's k_metrics_all)
__device__ __forceinline__ void write_metrics(const double *t, double Bd, const LossArgs &la, float *metrics,
                                              bool adv_stats)
{
    const float pl = (float)(-t[0] / Bd);
    const float vl = (float)(t[1] / Bd);
    const float ent = (float)(t[2] / Bd);
    const float loss = pl + la.vf_coef * vl + la.ent_coef * (-ent);
    const double var_rv = (t[8] - t[7] * t[7] / Bd) / (Bd - 1.0);
    const double var_r = (t[10] - t[9] * t[9] / Bd) / (Bd - 1.0);
    const float approx_kl = (float)(t[6] / Bd);
    const bool kl_stop = la.target_kl > 0.0f && approx_kl > la.target_kl;
    metrics[GS_M_LOSS] = loss;
    metrics[GS_M_POLICY_LOSS] = pl;
    metrics[GS_M_VALUE_LOSS] = vl;
    metrics[GS_M_ENTROPY] = ent;
    metrics[GS_M_CLIP_FRAC] = (float)(t[3] / Bd);
    metrics[GS_M_CLIP_FRAC_VF] = (float)(t[4] / Bd);
    metrics[GS_M_EXPLAINED_VAR] = (float)(1.0 - var_rv / var_r);
    metrics[GS_M_KL] = (float)(t[5] / Bd);
    metrics[GS_M_APPROX_KL] = approx_kl;
    if (adv_stats) {
        const double amean = t[11] / Bd;
        const double astd = sqrt(fmax(0.0, (t[12] - t[11] * t[11] / Bd) / (Bd - 1.0)));
        metrics[GS_M_ADV_NORM_MEAN] = la.normalize ? (float)amean : 0.0f;
        metrics[GS_M_ADV_NORM_STD] = la.normalize ? (float)astd : 0.0f;
    }
    metrics[GS_M_KL_STOP] = kl_stop ? 1.0f : 0.0f;
    metrics[GS_M_SKIPPED] = kl_stop ? 1.0f : 0.0f;
    metrics[GS_M_UNEVALUATED] = 0.0f;
    metrics[GS_M_RES1] = 0.0f;
}

// ------------------------------------------------------------------------------------
// k_loss: single workgroup of 256 threads over the B <= 1024 minibatch rows.
// ------------------------------------------------------------------------------------


template <class S>
__global__ __launch_bounds__(256) void k_loss(const float *__restrict__ P, Layout Lrt, const float *__restrict__ zpart,
                                              int Brt, const int32_t *__restrict__ f_act,
                                              const float *__restrict__ f_olp, const float *__restrict__ f_ov,
                                              const float *__restrict__ f_adv, const float *__restrict__ f_ret,
                                              LossArgs la, float *__restrict__ dz, float *__restrict__ metrics,
                                              int32_t *__restrict__ stop)
{
    __shared__ double sred[kNumSums * (256 + 16)];
    constexpr int AMAX = S::AMAX, AEX = S::AEX;
    const Layout L = S::lay(Lrt);
    const int B = S::batch(Brt);
    const int tid = threadIdx.x;
    if (la.step_base) metrics += *la.step_base * GS_NUM_METRICS;
    GS_STAMP_BEGIN(1)
    if (stop && *stop) {
        if (tid == 0) {
            for (int k = 0; k < GS_NUM_METRICS; ++k) metrics[k] = 0.0f;
            metrics[GS_M_SKIPPED] = 1.0f;
            metrics[GS_M_KL_STOP] = 1.0f;
            metrics[GS_M_UNEVALUATED] = 1.0f;
        }
        return;
    }
    const int A = L.A, A1 = A + 1;
    const float invB = la.inv_batch;
    const int64_t kb = la.step_base ? *la.step_base : 0;

    // ---- batch advantage normalisation: (a - mean) / (std_unbiased + 1e-8)
    float meanf = 0.0f, stdf = 1.0f;
    if (la.normalize && la.adv_stats) {      // global mode: the whole minibatch's statistics
        meanf = la.adv_stats[2 * kb];
        stdf = la.adv_stats[2 * kb + 1];
    } else if (la.normalize) {
        double m1[1] = {0.0};
        for (int r = tid; r < B; r += 256) m1[0] += (double)f_adv[r];
        block_reduce<1>(m1, sred);
        const double mean = m1[0] / (double)B;
        double q[1] = {0.0};
        for (int r = tid; r < B; r += 256) {
            const double dv = (double)f_adv[r] - mean;
            q[0] += dv * dv;
        }
        block_reduce<1>(q, sred);
        meanf = (float)mean;
        stdf = (float)sqrt(q[0] / (double)(B - 1));
    }
    GS_STAMP(0)

    double acc[kNumSums];
#pragma unroll
    for (int k = 0; k < kNumSums; ++k) acc[k] = 0.0;
    for (int r = tid; r < B; r += 256) {
        // every input of the row first (one round trip), then the math
        float z[AMAX + 1];
        gather_head_row<AMAX, AEX>(zpart, P, L, r, z);
        const int act = f_act[r];
        float adv = f_adv[r];
        if (la.normalize) adv = (adv - meanf) / (stdf + 1e-8f);
        if (act < 0) {      // another rank's row of a global minibatch
            for (int a = 0; a < A1; ++a) dz[(int64_t)r * A1 + a] = 0.0f;
            continue;
        }
        loss_row<AMAX>(z, A, act, f_olp[r], f_ov[r], adv, f_ret[r], la, invB, dz + (int64_t)r * A1, acc);
    }
    GS_STAMP(1)
    block_reduce<kNumSums>(acc, sred);     // fixed order -> deterministic
    GS_STAMP(2)
    if (tid == 0) {
        const double rows = (double)la.batch_rows;
        write_metrics(acc, rows, la, metrics, true);
        metrics[GS_M_GRAD_NORM] = 0.0f;
        if (la.sums_out)
            for (int q = 0; q < kNumSums; ++q) la.sums_out[kb * kNumSums + q] = acc[q];
        if (la.kl_part) {           // global KL stop: decided after the exchange (k_kl_decide)
            la.kl_part[0] = (float)(acc[6] * (double)invB);
            metrics[GS_M_KL_STOP] = metrics[GS_M_SKIPPED] = 0.0f;
        } else {
            const float approx_kl = (float)(acc[6] / rows);
            if (la.target_kl > 0.0f && approx_kl > la.target_kl && stop) *stop = 1;
        }
    }
    GS_STAMP_END(3)
}

// ------------------------------------------------------------------------------------
// k_bwd: three roles by block range.
//   role A: dW2 tiles (n-block, ka k-blocks), K = batch -> grads
//   role B: dh1 slab (32 rows, k-block), K = H2        -> dW1/db1 partial per 32 rows
//   role C: head grads and db2 for an n-block, metric row groups; one extra block for the
//           head biases
// sum-of-squares slot map: [0, nA) dW2 tiles, [nA, nA+ncb) db2 blocks,
//                          [nA+ncb, nA+2ncb) head weight blocks, nA+2ncb head biases.
// ------------------------------------------------------------------------------------
__device__ __forceinline__ void block_sumsq_store(float v, float *slot, float *sbuf)
{
    float t[1] = {v};
    block_reduce_t0<1>(t, sbuf);      // sbuf: 272 floats
    if (threadIdx.x == 0) *slot = t[0];
}

// role C's sum-of-squares slot, and with a fused update's per-step head record (headsq != null)
// the {policy head, value head} split of the same values for the per-component gradient norms
// (utils/models.py:196-230; k_metrics_all turns them into the record).  The slot's sum is the
// first of the reduced values, so it is the same sum in the same order as block_sumsq_store's.
// after block_sumsq_store: thread 0 splits the head values the reduction's LDS levels still hold
// (v[a]: head row / bias a's share) into the step's {policy, value} record
__device__ __forceinline__ void store_head_split(const float *v, int A, float *headsq, int64_t o)
{
    if (threadIdx.x == 0 && headsq) {
        float p = 0.0f;
        for (int a = 0; a < A; ++a) p += v[a];
        headsq[o] = p;
        headsq[o + 1] = v[A];
    }
}

__device__ __forceinline__ void store_head_sums(float sq, float sqp, float sqv, float *slot, float *headsq,
                                                int64_t o, float *sbuf)
{
    if (!headsq) {
        block_sumsq_store(sq, slot, sbuf);
        return;
    }
    float t[3] = {sq, sqp, sqv};
    block_reduce_t0<3>(t, sbuf);      // sbuf: 3 x 272 floats
    if (threadIdx.x == 0) {
        *slot = t[0];
        headsq[o] = t[1];
        headsq[o + 1] = t[2];
    }
}

// The role-C workgroup that stores metric row group g (16 rows) of a minibatch of G groups: a
// contiguous range of groups per workgroup
__host__ __device__ inline int metric_owner(int g, int G, int nW) { return G <= nW ? g : (int)(((int64_t)g * nW) / G); }
__host__ __device__ inline int metric_groups_per_wg(int G, int nW) { return G <= nW ? 1 : (G + nW - 1) / nW; }

struct BwdShape {
    int ncb, nkb, nrbB, ka, nT, nA, nB, nC;
    __host__ __device__ static BwdShape make(const Layout &L, int B, int rb)
    {
        const int kRowsB = rb;
        BwdShape s;
        s.ncb = (L.H2 + kTile - 1) / kTile;
        s.nkb = (L.H1 + kTile - 1) / kTile;
        s.nrbB = (B + kRowsB - 1) / kRowsB;
        // role A: ka k-blocks of the same n-block per workgroup (the loss rows, the relu' mask
        // and dh2 are computed once for them); keeps the grid near one workgroup per CU
        s.ka = s.nkb % 2 == 0 ? 2 : 1;
        s.nT = s.ncb * s.nkb;                   // dW2 tiles (sum-of-squares slots)
        s.nA = s.ncb * (s.nkb / s.ka);
        s.nB = s.nrbB * s.nkb;
        s.nC = s.ncb + 1;   // + one block for the head-bias gradients
        return s;
    }
};

size_t bwd_lds_bytes(const Layout &L, int64_t B)
{
    const int kRowsB = rows_b(L, B);
    const int A1 = L.A + 1;
    const int64_t Bp64 = (B + 63) / 64 * 64, Bp16 = (B + 15) / 16 * 16;
    const int64_t H2p = (L.H2 + 63) / 64 * 64;
    const BwdShape shp = BwdShape::make(L, (int)B, kRowsB);
    // the fast paths (A1 <= 5) form dh2 in registers: role A has no dh2 tile (and its block
    // reduction reuses the h1 tile after the MFMA loop), role B only the dW1 partial scratch in
    // place of its dh2 slab — role A's 49 KB (+ 3 KB static) keep three workgroups per CU, so
    // ranks sharing a GPU find room for each other's grids
    const bool fastA = A1 <= 5, regsB = A1 <= 5 && L.H2 % 64 == 0;
    const int64_t roleA = round4((int)B * A1) + round4(A1 * 16) + ((fastA ? 0 : 1) + 2) * kTile * (Bp64 + 4) + 3072 +
                          Bp64 + (fastA ? 0 : 816);
    const int64_t roleB = (regsB ? (int64_t)round4(kRowsB / 16 * 16 * (L.D + 1)) : (int64_t)kRowsB * (H2p + 4)) +
                          kTile * (H2p + 4) + round4(A1 * L.H2) + round4(kRowsB * A1) +
                          kRowsB * 16 + round4(kRowsB * L.D) + kRowsB * 17 + 1024 +
                          (int64_t)kRowsB * n_col_blocks(L.H2);
    const int64_t roleC = Bp16 * 17 + round4((int)Bp16 * A1) + (A1 * 256 > 1024 ? A1 * 256 : 1024) + 2 +
                          (int64_t)metric_groups_per_wg((int)B / kTile, shp.nC) * kTile * kNumSums * 2;
    int64_t m = roleA;
    if (roleB > m) m = roleB;
    if (roleC > m) m = roleC;
    return (size_t)m * sizeof(float);
}

// Fused path: the loss rows a workgroup needs (dLoss/dlogits | dLoss/dvalue) are computed
// from the forward's partial heads straight into LDS, so the chain has no separate loss
// launch.  Threads [t0, t0 + nthr) take rows [r0, r0 + n); dscr != nullptr also keeps the 14
// metric sums of the rows in [d0, d1) ((d1 - d0) x 14 doubles of LDS) for store_metric_groups
// after a barrier.
template <class S>
__device__ __forceinline__ void loss_rows_lds(const float *__restrict__ P, const Layout &L,
                                              const float *__restrict__ zpart, const FusedFwd &ff,
                                              const LossArgs &la, int B, int64_t k, int r0, int n, float *dzs,
                                              double *dscr, int t0 = 0, int nthr = 256, int d0 = 0,
                                              int d1 = 1 << 30)
{
    constexpr int AMAX = S::AMAX, AEX = S::AEX;
    const int A1 = L.A + 1;
    const int me = (int)threadIdx.x - t0;
    if (me < 0 || me >= nthr) return;
    for (int i = me; i < n; i += nthr) {
        const int r = r0 + i;
        double acc[kNumSums];
#pragma unroll
        for (int q = 0; q < kNumSums; ++q) acc[q] = 0.0;
        // rows past B (padding) load row B-1 unconditionally and discard the result: a predicated
        // load burst would compile to branches with vmcnt stalls inside it
        const int rc = r < B ? r : B - 1;
        const int64_t o = k * B + rc;
        // the row's fields are loaded before the head partials: one memory round trip
        const int fa = ff.fa[o];
        const float folp = ff.folp[o], fov = ff.fov[o], fadv = ff.fadv[o], fret = ff.fret[o];
        float z[AMAX + 1];
        gather_head_row<AMAX, AEX>(zpart, P, L, rc, z);
        // action < 0: another rank's row of a global minibatch (gs_ppo_update_global)
        const bool live = r < B && fa >= 0;
        loss_row<AMAX>(z, L.A, fa, folp, fov, fadv, fret, la, la.inv_batch, dzs + i * A1, acc);
        if (!live) {
            for (int a = 0; a < A1; ++a) dzs[i * A1 + a] = 0.0f;
#pragma unroll
            for (int q = 0; q < kNumSums; ++q) acc[q] = 0.0;
        }
        if (dscr && r >= d0 && r < d1)      // rows of the metric window [d0, d1) only
#pragma unroll
            for (int q = 0; q < kNumSums; ++q) dscr[(r - d0) * kNumSums + q] = acc[q];
    }
}

// the 14 metric sums of every 16-row group of [r0, r0 + n) (after a barrier)
__device__ __forceinline__ void store_metric_groups(const double *dscr, int n, int r0, int B, int64_t k,
                                                    double *__restrict__ mp)
{
    const int ng = n / kTile;
    if ((int)threadIdx.x < ng * kNumSums) {
        const int g = threadIdx.x / kNumSums, q = threadIdx.x - g * kNumSums;
        double t = 0.0;
        for (int i = 0; i < kTile; ++i) t += dscr[(g * kTile + i) * kNumSums + q];
        mp[(k * (B / kTile) + r0 / kTile + g) * kNumSums + q] = t;
    }
}

template <class S, bool FUSED>
__global__ __launch_bounds__(256) void k_bwd(const float *__restrict__ P, Layout Lrt, int Brt,
                                             const float *__restrict__ x, const float *__restrict__ h1,
                                             const float *__restrict__ h2, const float *__restrict__ dz,
                                             float *__restrict__ G, float *__restrict__ part1,
                                             float *__restrict__ sumsq, const int32_t *__restrict__ stop,
                                             const float *__restrict__ zpart, FusedFwd ff, LossArgs la,
                                             const uint16_t *__restrict__ h2mask, BwdXchg bx)
{
    GS_SPAN_T0
    if (stop && *stop) return;
    // multi-GPU: every output value goes through bwd_exchange before it is stored (its
    // counter is read here, off the epilogue's critical path)
    const bool xchg = bx.world > 1;
    const uint32_t xseq = xchg ? bx.seq[blockIdx.x] + 1u : 0u;
    // this minibatch's index in the update (graph replay: + the chunk's device step base), read
    // once here: a later re-read (the metric-group stores come after LDS/global stores the
    // compiler cannot order it against) would be a dependent round trip in the middle of a phase
    const int64_t kstep = FUSED ? ff.k_local + (ff.step_base ? *ff.step_base : 0) : 0;
    if constexpr (FUSED) GS_SPAN_START(1, kstep)
    extern __shared__ float lds[];
    __shared__ float sbuf[FUSED ? 3 * 272 : 272];    // fused: role C's {slot, policy, value} sums
    const Layout L = S::lay(Lrt);
    const int B = S::batch(Brt);
    const int D = L.D, H1 = L.H1, H2 = L.H2, A = L.A, A1 = A + 1;
    constexpr int kRowsB = S::RB;      // this shape's role-B slab height (shadows the default)
    const BwdShape sh = BwdShape::make(L, B, kRowsB);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int li = lane & 15, lq = lane >> 4;
    // dispatch order: role B (the longest) first, then A, then C; bid keeps the A, B, C numbering
    int bid = (int)blockIdx.x;
    if (bid < sh.nB) bid += sh.nA;
    else if (bid < sh.nB + sh.nA) bid -= sh.nB;

    if (bid < sh.nA) {
        // ---------------- role A: dW2[n0:n0+16, k0:k0+16*ka] = sum_b dh2[b,n] h1[b,k]
        const int nkg = sh.nkb / sh.ka;
        const int nb = bid / nkg, kb = (bid - nb * nkg) * sh.ka;   // first of the ka k-blocks
        const int n0 = nb * kTile, k0 = kb * kTile, kw = kTile * sh.ka;
        GS_STAMP_BEGIN_IF(2, bid == 0)
        const int Bp = (B + 63) / 64 * 64;      // padded K (batch) for 4 waves x 16
        const int ld = Bp + 4;
        const bool fast = A1 <= 5;                   // dh2 in registers (no dh2 tile)
        float *dzs = lds;                            // [B][A1]
        float *whs = dzs + round4(B * A1);           // [A1][16]
        float *dh2T = whs + round4(A1 * 16);         // [16][Bp+4]  (n, b): h2 first, then dh2 (!fast)
        float *h1T = dh2T + (fast ? 0 : kTile * ld); // [16*ka][Bp+4]  (k, b)
        float *red = h1T + kw * ld;                  // [4][3][256]
        // relu'(h2) bits of this n-block (one word per row) and the h1 column tile (16 contiguous
        // floats per row = 4 float4, transposed into LDS); dh2T is filled by the dh2 pass
        int *mkA = reinterpret_cast<int *>(red + 3072);   // [Bp]
        if constexpr (S::H1c > 0 && S::Bc > 0) {
            // compile-time shapes: the tile loads are issued before the loss rows, which
            // then run while they are in flight; LDS writes follow
            constexpr Layout Lc = S::lay(Layout{});
            constexpr int cB = S::Bc, cBp = (cB + 63) / 64 * 64, cncb = (Lc.H2 + kTile - 1) / kTile;
            constexpr int cka = (Lc.H1 / kTile) % 2 == 0 ? 2 : 1, ckw = kTile * cka, cq = ckw / 4;
            constexpr int NMk = (cBp + 255) / 256, NH1 = (cBp * cq + 255) / 256;
            int mr[NMk];
            float4 hr[NH1];
            float wh = 0.0f;
            // unconditional loads at clamped indices, out-of-range lanes zeroed at the LDS stores
            // (predicated loads would put vmcnt stalls inside the burst)
#pragma unroll
            for (int j = 0; j < NMk; ++j) {
                const int b = tid + 256 * j;
                mr[j] = (int)h2mask[(int64_t)min(b, cB - 1) * cncb + nb];
            }
#pragma unroll
            for (int j = 0; j < NH1; ++j) {
                const int u = tid + 256 * j, b = u / cq, c4 = u % cq;
                hr[j] = *reinterpret_cast<const float4 *>(h1 + (int64_t)min(b, cB - 1) * Lc.H1 +
                                                          min(k0 + 4 * c4, Lc.H1 - 4));
            }
            {
                const int a = min(tid >> 4, A1 - 1), j = tid & 15;
                wh = P[L.head_row(a) + min(n0 + j, H2 - 1)];
            }
            if constexpr (FUSED)
                loss_rows_lds<S>(P, L, zpart, ff, la, B, kstep, 0, B, dzs, nullptr);
            else
                copy_to_lds(dzs, dz, B * A1);
            if (tid < A1 * kTile) whs[tid] = n0 + (tid & 15) < H2 ? wh : 0.0f;
#pragma unroll
            for (int j = 0; j < NMk; ++j)
                if (tid + 256 * j < cBp) mkA[tid + 256 * j] = tid + 256 * j < cB ? mr[j] : 0;
#pragma unroll
            for (int j = 0; j < NH1; ++j) {
                const int u = tid + 256 * j, b = u / cq, c4 = u % cq;
                if (u < cBp * cq) {
                    const bool ok = b < cB && k0 + 4 * c4 < Lc.H1;
                    h1T[(4 * c4 + 0) * ld + b] = ok ? hr[j].x : 0.0f;
                    h1T[(4 * c4 + 1) * ld + b] = ok ? hr[j].y : 0.0f;
                    h1T[(4 * c4 + 2) * ld + b] = ok ? hr[j].z : 0.0f;
                    h1T[(4 * c4 + 3) * ld + b] = ok ? hr[j].w : 0.0f;
                }
            }
        } else {
            if constexpr (FUSED)
                loss_rows_lds<S>(P, L, zpart, ff, la, B, kstep, 0, B, dzs, nullptr);
            else
                copy_to_lds(dzs, dz, B * A1);
            if (tid < A1 * kTile) {
                const int a = tid >> 4, j = tid & 15;
                whs[tid] = n0 + j < H2 ? P[L.head_row(a) + n0 + j] : 0.0f;
            }
            for (int b = tid; b < Bp; b += 256) mkA[b] = b < B ? (int)h2mask[(int64_t)b * sh.ncb + nb] : 0;
            const int q4 = kw / 4;
#pragma unroll 4
            for (int u = tid; u < Bp * q4; u += 256) {
                const int b = u / q4, c4 = u - b * q4;
                float4 gv = make_float4(0.f, 0.f, 0.f, 0.f);
                if (b < B && k0 + 4 * c4 < H1)
                    gv = *reinterpret_cast<const float4 *>(h1 + (int64_t)b * H1 + k0 + 4 * c4);
                h1T[(4 * c4 + 0) * ld + b] = gv.x;
                h1T[(4 * c4 + 1) * ld + b] = gv.y;
                h1T[(4 * c4 + 2) * ld + b] = gv.z;
                h1T[(4 * c4 + 3) * ld + b] = gv.w;
            }
        }
        __syncthreads();
        GS_STAMP(0)
        const int nch = Bp / kTile;
        const int ch0 = (wave * nch) / 4, ch1 = ((wave + 1) * nch) / 4;
        // the ka dW2 tiles; k-block-0 workgroups also form db2[n] = sum_b dh2[b, n]: from the A
        // operands they already hold (fast path), or as an MFMA against a ones operand (t == ka)
        const int nt = sh.ka + (!fast && kb == 0 ? 1 : 0);
        if (fast) {
            // dh2 = relu'(h2) * (dz . Wh) formed in registers as the MFMA's A operand (lane: hidden
            // unit n0 + li, rows b..b+3 of its K chunk), with the two-phase path's arithmetic and
            // order, so no dh2 tile goes through LDS and one barrier less; the chunk's operand
            // feeds every tile of the workgroup
            float w[5];
#pragma unroll
            for (int a = 0; a < 5; ++a) w[a] = a < A1 ? whs[a * 16 + li] : 0.0f;
            f32x4 acc[3][2];
#pragma unroll
            for (int t = 0; t < 3; ++t) acc[t][0] = acc[t][1] = f32x4{0.f, 0.f, 0.f, 0.f};
            float dsum = 0.0f;      // db2 partial of this lane's rows (k-block 0)
            // lane's dh2 operand of rows b..b+3
            auto dh2_rows = [&](int b, float (&av)[4]) {
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    float sacc = 0.0f;
#pragma unroll
                    for (int a = 0; a < 5; ++a) sacc = a < A1 ? fmaf(dzs[(b + c) * A1 + a], w[a], sacc) : sacc;
                    av[c] = (mkA[b + c] >> li) & 1 ? sacc : 0.0f;
                }
            };
            if constexpr (S::BF) {
                // bf16 mode: chunk pairs (the fast path only has the ka dW2 tiles, no ones tile)
                const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 2
                for (int ch = ch0; ch < ch1; ch += 2) {
                    const int b = ch * kTile + 4 * lq;
                    const bool two = ch + 1 < ch1;
                    float av0[4], av1[4] = {0.f, 0.f, 0.f, 0.f};
                    dh2_rows(b, av0);
                    if (two) dh2_rows(b + kTile, av1);
                    if (kb == 0) {
                        dsum = (((dsum + av0[0]) + av0[1]) + av0[2]) + av0[3];
                        dsum = (((dsum + av1[0]) + av1[1]) + av1[2]) + av1[3];
                    }
#pragma unroll
                    for (int t = 0; t < 2; ++t) {
                        if (t >= nt) break;
                        const float *hb = h1T + (t * kTile + li) * ld + b;
                        const float4 bb0 = *reinterpret_cast<const float4 *>(hb);
                        const float4 bb1 = two ? *reinterpret_cast<const float4 *>(hb + kTile) : z4;
                        acc[t][0] = mfma_bf16_pair(f4(av0), f4(av1), bb0, bb1, acc[t][0]);
                    }
                }
            } else {
#pragma unroll 2
            for (int ch = ch0; ch < ch1; ++ch) {
                const int b = ch * kTile + 4 * lq;
                float av[4];
                dh2_rows(b, av);
                if (kb == 0) dsum = (((dsum + av[0]) + av[1]) + av[2]) + av[3];
#pragma unroll
                for (int t = 0; t < 3; ++t) {
                    if (t >= nt) break;
                    const float4 bb = t == sh.ka ? make_float4(1.f, 1.f, 1.f, 1.f)
                                                 : *reinterpret_cast<const float4 *>(h1T + (t * kTile + li) * ld + b);
                    acc[t][0] = mfma4(av[0], bb.x, acc[t][0]);
                    acc[t][1] = mfma4(av[1], bb.y, acc[t][1]);
                    acc[t][0] = mfma4(av[2], bb.z, acc[t][0]);
                    acc[t][1] = mfma4(av[3], bb.w, acc[t][1]);
                }
            }
            }
            GS_STAMP(1)
#pragma unroll
            for (int t = 0; t < 3; ++t) {
                if (t >= nt) break;
                const f32x4 at = acc[t][0] + acc[t][1];
#pragma unroll
                for (int r = 0; r < 4; ++r) red[(wave * 3 + t) * 256 + (lq * 4 + r) * kTile + li] = at[r];
            }
            if (kb == 0) red[(wave * 3 + 2) * 256 + lq * kTile + li] = dsum;   // slab 2 is free (nt <= 2)
        } else {
            // dh2 = relu'(h2) * (dz . Wh), in place; lane owns hidden unit i, rows stride 16
            {
                const int i = tid & 15;
                float w[kMaxActions + 1];
#pragma unroll
                for (int a = 0; a < kMaxActions + 1; ++a) w[a] = a < A1 ? whs[a * 16 + i] : 0.0f;
                for (int b = tid >> 4; b < Bp; b += 16) {
                    const bool on = (mkA[b] >> i) & 1;
                    float s = 0.0f;
#pragma unroll
                    for (int a = 0; a < kMaxActions + 1; ++a) s = a < A1 ? fmaf(dzs[b * A1 + a], w[a], s) : s;
                    dh2T[i * ld + b] = on ? s : 0.0f;
                }
            }
            __syncthreads();
            GS_STAMP(1)
            for (int t = 0; t < nt; ++t) {
                f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
                const float *hb = h1T + t * kTile * ld;
                const bool ones = t == sh.ka;
#pragma unroll 4
                for (int ch = ch0; ch < ch1; ++ch) {
                    const int b = ch * kTile + 4 * lq;
                    const float4 a = *reinterpret_cast<const float4 *>(dh2T + li * ld + b);
                    const float4 bb = ones ? make_float4(1.f, 1.f, 1.f, 1.f)
                                           : *reinterpret_cast<const float4 *>(hb + li * ld + b);
                    acc0 = mfma4(a.x, bb.x, acc0);
                    acc1 = mfma4(a.y, bb.y, acc1);
                    acc0 = mfma4(a.z, bb.z, acc0);
                    acc1 = mfma4(a.w, bb.w, acc1);
                }
                const f32x4 acc = acc0 + acc1;
#pragma unroll
                for (int r = 0; r < 4; ++r) red[(wave * 3 + t) * 256 + (lq * 4 + r) * kTile + li] = acc[r];
            }
        }
        __syncthreads();
        GS_STAMP(2)
        {
            // one sum-of-squares slot per dW2 tile (tile index nb*nkb + kb + t), one for db2
            const int row = tid >> 4, col = tid & 15;
            float gv[3] = {0.0f, 0.0f, 0.0f};
            bool ok[3] = {false, false, false};
            for (int t = 0; t < nt; ++t) {
                const float g = ((red[(0 + t) * 256 + tid] + red[(3 + t) * 256 + tid]) + red[(6 + t) * 256 + tid]) +
                                red[(9 + t) * 256 + tid];
                const int j = t < sh.ka ? t : 2;
                gv[j] = g;
                ok[j] = t < sh.ka ? (n0 + row < H2 && k0 + t * kTile + col < H1) : (col == 0 && n0 + row < H2);
            }
            // db2 element of this thread: n0 + row (ones tile, col 0) or n0 + tid (fast path: the 16
            // (wave, lane group) partials of column tid, in order)
            int db2n = n0 + row;
            if (fast && kb == 0) {
                db2n = n0 + tid;
                float d = 0.0f;
                if (tid < kTile)
#pragma unroll
                    for (int q = 0; q < 16; ++q) d += red[((q >> 2) * 3 + 2) * 256 + (q & 3) * kTile + tid];
                gv[2] = d;
                ok[2] = tid < kTile && n0 + tid < H2;
            }
            if (xchg) bwd_exchange<3>(bx, xseq, gv, ok);
            float sqt[3] = {0.0f, 0.0f, 0.0f};
            for (int t = 0; t < sh.ka; ++t) {
                if (!ok[t]) continue;
                G[L.oW2 + (int64_t)(n0 + row) * H1 + k0 + t * kTile + col] = gv[t];
                sqt[t] = gv[t] * gv[t];
            }
            if (ok[2]) {
                G[L.ob2 + db2n] = gv[2];
                sqt[2] = gv[2] * gv[2];
            }
            // 3 x (256 + 16) floats: the h1 tile, dead after the barrier above (fast path)
            block_reduce_t0<3>(sqt, fast ? h1T : reinterpret_cast<float *>(mkA + Bp));
            if (tid == 0) {
                for (int t = 0; t < sh.ka; ++t) sumsq[nb * sh.nkb + kb + t] = sqt[t];
                if (kb == 0) sumsq[sh.nT + nb] = sqt[2];
            }
        }
        GS_STAMP_END(3)
        if constexpr (FUSED) GS_SPAN_END(1, kstep)
        return;
    }
    bid -= sh.nA;
    if (bid < sh.nB) {
        // ---------------- role B: dh1 slab rows b0..b0+64, cols k0..k0+16 (K = H2);
        //                  wave w owns rows b0+16w .. b0+16w+15 with the full K
        // XCD-aware order (blocks b and b + 8 share an XCD): with 16 k-blocks and 8 role-A k-block
        // pairs, the role-B workgroups of XCD x take k-blocks 2x, 2x+1 — the h1 columns the role-A
        // workgroups on that XCD read — so each XCD's L2 fetches one h1 column slab, not two
        int rb, kb;
        if (sh.nkb == 16 && sh.ka == 2 && sh.nB % 8 == 0) {
            const int x = bid & 7, i = bid >> 3;
            kb = 2 * x + (i & 1);
            rb = i >> 1;
        } else {
            rb = bid / sh.nkb;
            kb = bid - rb * sh.nkb;
        }
        const int b0 = rb * kRowsB, k0 = kb * kTile;
        GS_STAMP_BEGIN_IF(4, bid == 0)
        const int H2p = (H2 + 63) / 64 * 64;
        const int ld = H2p + 4;
        const bool dh2_regs = A1 <= 5 && H2 % 64 == 0;   // dh2 formed in registers, no dh2 slab
        float *dh2s = lds;                          // [32][H2p+4]  dh2 (!dh2_regs); dW1 partial scratch
        float *W2T = dh2s + (dh2_regs ? round4(kRowsB / 16 * 16 * (D + 1)) : kRowsB * ld);   // [16][H2p+4]
        float *whs = W2T + kTile * ld;              // [A1][H2]
        float *dzs = whs + round4(A1 * H2);         // [64][A1]
        float *h1m = dzs + round4(kRowsB * A1);     // [64][16]
        float *xs = h1m + kRowsB * 16;              // [64][D]
        float *tile = xs + round4(kRowsB * D);      // [32][17]
        float *kred = tile + kRowsB * 17;           // [4][256] K-half partial tiles
        // waves 0-2 stream the slab's operands into LDS while wave 3 computes its loss rows
        // (fused path): the loss math overlaps the loads instead of following them
        constexpr int kLd = FUSED ? 192 : 256;
        int *mkB = reinterpret_cast<int *>(kred + 1024);   // [32][ncb] relu'(h2) bits
        if constexpr (S::H1c > 0 && S::Bc > 0) {
            // compile-time shapes: every operand load of the slab is issued before the first
            // LDS write (one memory round trip instead of one per operand loop)
            constexpr Layout Lc = S::lay(Layout{});
            constexpr int cH1 = Lc.H1, cH2 = Lc.H2, cD = Lc.D, cA1 = Lc.A + 1, cB = S::Bc;
            constexpr int cncb = (cH2 + kTile - 1) / kTile, cH2p = (cH2 + 63) / 64 * 64;
            constexpr int NM = (kRowsB * cncb + kLd - 1) / kLd, NW = (cH2p * 4 + kLd - 1) / kLd;
            constexpr int NH = (cA1 * cH2 + kLd - 1) / kLd, N1 = (kRowsB * 16 + kLd - 1) / kLd;
            constexpr int NX = (kRowsB * cD + kLd - 1) / kLd;
            if (tid < kLd) {
                int mr[NM];
                float4 wr[NW];
                float hr[NH], h1r[N1], xr[NX];
                // unconditional loads at clamped indices; out-of-range lanes zeroed at the stores
#pragma unroll
                for (int j = 0; j < NM; ++j) {
                    const int u = min(tid + j * kLd, kRowsB * cncb - 1), i = u / cncb, c = u - i * cncb;
                    mr[j] = (int)h2mask[(int64_t)min(b0 + i, cB - 1) * cncb + c];
                }
#pragma unroll
                for (int j = 0; j < NW; ++j) {
                    const int u = tid + j * kLd, n = min(u >> 2, cH2 - 1), c4 = u & 3;
                    wr[j] = *reinterpret_cast<const float4 *>(P + Lc.oW2 + (int64_t)n * cH1 + min(k0 + 4 * c4, cH1 - 4));
                }
#pragma unroll
                for (int j = 0; j < NH; ++j) {
                    const int u = min(tid + j * kLd, cA1 * cH2 - 1), a = u / cH2, n = u - a * cH2;
                    hr[j] = P[Lc.head_row(a) + n];
                }
#pragma unroll
                for (int j = 0; j < N1; ++j) {
                    const int u = tid + j * kLd, i = min(u >> 4, kRowsB - 1), jj = u & 15;
                    h1r[j] = h1[(int64_t)min(b0 + i, cB - 1) * cH1 + min(k0 + jj, cH1 - 1)];
                }
#pragma unroll
                for (int j = 0; j < NX; ++j) {
                    const int u = tid + j * kLd;
                    xr[j] = x[min((int64_t)b0 * cD + u, (int64_t)cB * cD - 1)];
                }
#pragma unroll
                for (int j = 0; j < NM; ++j) {
                    const int u = tid + j * kLd, i = u / cncb;
                    if (u < kRowsB * cncb) mkB[u] = b0 + i < cB ? mr[j] : 0;
                }
#pragma unroll
                for (int j = 0; j < NW; ++j) {
                    const int u = tid + j * kLd, n = u >> 2, c4 = u & 3;
                    if (u < cH2p * 4) {
                        const bool ok = n < cH2 && k0 + 4 * c4 < cH1;
                        W2T[(4 * c4 + 0) * ld + n] = ok ? wr[j].x : 0.0f;
                        W2T[(4 * c4 + 1) * ld + n] = ok ? wr[j].y : 0.0f;
                        W2T[(4 * c4 + 2) * ld + n] = ok ? wr[j].z : 0.0f;
                        W2T[(4 * c4 + 3) * ld + n] = ok ? wr[j].w : 0.0f;
                    }
                }
#pragma unroll
                for (int j = 0; j < NH; ++j)
                    if (tid + j * kLd < cA1 * cH2) whs[tid + j * kLd] = hr[j];
#pragma unroll
                for (int j = 0; j < N1; ++j) {
                    const int u = tid + j * kLd, i = u >> 4, jj = u & 15;
                    if (u < kRowsB * 16) h1m[u] = (b0 + i < cB && k0 + jj < cH1) ? h1r[j] : 0.0f;
                }
#pragma unroll
                for (int j = 0; j < NX; ++j) {
                    const int u = tid + j * kLd;
                    if (u < kRowsB * cD) xs[u] = b0 * cD + u < cB * cD ? xr[j] : 0.0f;
                }
            }
        } else if (!FUSED || tid < kLd) {
            for (int u = tid; u < kRowsB * sh.ncb; u += kLd) {
                const int i = u / sh.ncb, c = u - i * sh.ncb;
                mkB[u] = b0 + i < B ? (int)h2mask[(int64_t)(b0 + i) * sh.ncb + c] : 0;
            }
#pragma unroll 4
            for (int u = tid; u < H2p * 4; u += kLd) {
                const int n = u >> 2, c4 = u & 3;
                float4 w = make_float4(0.f, 0.f, 0.f, 0.f);
                if (n < H2 && k0 + 4 * c4 < H1)
                    w = *reinterpret_cast<const float4 *>(P + L.oW2 + (int64_t)n * H1 + k0 + 4 * c4);
                W2T[(4 * c4 + 0) * ld + n] = w.x;
                W2T[(4 * c4 + 1) * ld + n] = w.y;
                W2T[(4 * c4 + 2) * ld + n] = w.z;
                W2T[(4 * c4 + 3) * ld + n] = w.w;
            }
            for (int u = tid; u < A1 * H2; u += kLd) {
                const int a = u / H2, n = u - a * H2;
                whs[u] = P[L.head_row(a) + n];
            }
            for (int u = tid; u < kRowsB * 16; u += kLd) {
                const int i = u >> 4, j = u & 15;
                h1m[u] = (b0 + i < B && k0 + j < H1) ? h1[(int64_t)(b0 + i) * H1 + k0 + j] : 0.0f;
            }
            for (int u = tid; u < kRowsB * D; u += kLd) xs[u] = b0 * D + u < B * D ? x[(int64_t)b0 * D + u] : 0.0f;
        }
#ifdef GS_STAMPS
        const unsigned long long t_rb0 = __builtin_amdgcn_s_memtime();
        if (bid == 0 && tid == 0) {   // loader waves: issue + land of the slab operands
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            atomicAdd(&g_stamp_acc[6][0], __builtin_amdgcn_s_memtime() - t_rb0);
            atomicAdd(&g_stamp_cnt[6], 1ull);
        }
#endif
        if constexpr (FUSED)      // the kb == 0 slab also keeps its rows' metric sums
            loss_rows_lds<S>(P, L, zpart, ff, la, B, kstep, b0, kRowsB, dzs, nullptr, kLd, 256 - kLd);
#ifdef GS_STAMPS
        if (bid == 0 && tid == 192) {   // loss wave: its rows' loss + gradient
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            atomicAdd(&g_stamp_acc[7][0], __builtin_amdgcn_s_memtime() - t_rb0);
            atomicAdd(&g_stamp_cnt[7], 1ull);
        }
#endif
        else
            for (int u = tid; u < kRowsB * A1; u += 256)
                dzs[u] = b0 * A1 + u < B * A1 ? dz[(int64_t)b0 * A1 + u] : 0.0f;
        __syncthreads();
        GS_STAMP(0)
        // 32 rows = 2 row tiles; waves (0,1) / (2,3) split K = H2 of tile 0 / 1 in halves; 64 rows =
        // 4 row tiles, one per wave over the whole K
        static_assert(kRowsB == 32 || kRowsB == 64, "role-B slabs of 32 or 64 rows");
        const int nchB = H2p / kTile;
        const int rt = kRowsB == 64 ? wave : wave >> 1, half = kRowsB == 64 ? 0 : wave & 1;
        const int chb = half ? nchB / 2 : 0, che = (half || kRowsB == 64) ? nchB : nchB / 2;
        f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
        if (dh2_regs) {
            // dh2 = relu'(h2) * (dz . Wh) formed in registers as the MFMA's A operand (lane: slab
            // row rt*16 + li, hidden units n..n+3 of its K chunk), with the two-phase path's
            // arithmetic and order: no dh2 slab through LDS, one barrier less
            const int row = rt * 16 + li;
            float dzr[5];
#pragma unroll
            for (int a = 0; a < 5; ++a) dzr[a] = a < A1 ? dzs[row * A1 + a] : 0.0f;
            const float *brow = W2T + li * ld;
            // the lane's dh2 operand of hidden units n..n+3 (chunk ch)
            auto dh2_cols = [&](int ch, float (&av)[4]) {
                const int n = ch * kTile + 4 * lq;
                const unsigned m = (unsigned)(mkB[row * sh.ncb + ch] >> (4 * lq));
                float4 wh[5];
#pragma unroll
                for (int a = 0; a < 5; ++a)
                    wh[a] = a < A1 ? *reinterpret_cast<const float4 *>(whs + a * H2 + n) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    float sacc = 0.0f;
#pragma unroll
                    for (int a = 0; a < 5; ++a) {
                        const float wv = j == 0 ? wh[a].x : j == 1 ? wh[a].y : j == 2 ? wh[a].z : wh[a].w;
                        sacc = a < A1 ? fmaf(dzr[a], wv, sacc) : sacc;
                    }
                    av[j] = ((m >> j) & 1u) ? sacc : 0.0f;
                }
            };
            if constexpr (S::BF) {
                const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 2
                for (int ch = chb; ch < che; ch += 2) {
                    const int n = ch * kTile + 4 * lq;
                    const bool two = ch + 1 < che;
                    float av0[4], av1[4] = {0.f, 0.f, 0.f, 0.f};
                    dh2_cols(ch, av0);
                    if (two) dh2_cols(ch + 1, av1);
                    const float4 w0 = *reinterpret_cast<const float4 *>(brow + n);
                    const float4 w1 = two ? *reinterpret_cast<const float4 *>(brow + n + kTile) : z4;
                    acc0 = mfma_bf16_pair(f4(av0), f4(av1), w0, w1, acc0);
                }
            } else {
#pragma unroll 2
            for (int ch = chb; ch < che; ++ch) {
                const int n = ch * kTile + 4 * lq;
                float av[4];
                dh2_cols(ch, av);
                const float4 w = *reinterpret_cast<const float4 *>(brow + n);
                acc0 = mfma4(av[0], w.x, acc0);
                acc1 = mfma4(av[1], w.y, acc1);
                acc0 = mfma4(av[2], w.z, acc0);
                acc1 = mfma4(av[3], w.w, acc1);
            }
            }
            GS_STAMP(1)
        } else {
        // dh2 = relu'(h2) * (dz . Wh), in place
        if (A1 <= 5 && H2 <= 1024 && 1024 % H2 == 0) {
            // thread owns 4 consecutive hidden units (4 mask bits of one word, one float4 store)
            // and every (256/(H2/4))-th row; threads of one row read the same dz (broadcast)
            const int nt = H2 >> 2, rstep = 256 / nt;
            const int n0 = 4 * (tid % nt), nb = n0 >> 4, sh4 = n0 & 15;
            float w[5][4];
#pragma unroll
            for (int a = 0; a < 5; ++a)
#pragma unroll
                for (int j = 0; j < 4; ++j) w[a][j] = a < A1 ? whs[a * H2 + n0 + j] : 0.0f;
            // 8 rows at a time, all their LDS reads before their stores (the dh2s stores may
            // alias mkB / dzs as far as the compiler knows)
            for (int i0 = tid / nt; i0 < kRowsB; i0 += 8 * rstep) {
                unsigned mm[8];
                float dzr[8][5];
#pragma unroll
                for (int c = 0; c < 8; ++c) {
                    const int i = min(i0 + c * rstep, kRowsB - 1);
                    mm[c] = (unsigned)(mkB[i * sh.ncb + nb] >> sh4);
#pragma unroll
                    for (int a = 0; a < 5; ++a) dzr[c][a] = a < A1 ? dzs[i * A1 + a] : 0.0f;
                }
#pragma unroll
                for (int c = 0; c < 8; ++c) {
                    const int i = i0 + c * rstep;
                    float o[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        float sacc = 0.0f;
#pragma unroll
                        for (int a = 0; a < 5; ++a) sacc = a < A1 ? fmaf(dzr[c][a], w[a][j], sacc) : sacc;
                        o[j] = ((mm[c] >> j) & 1u) ? sacc : 0.0f;
                    }
                    if (i < kRowsB)
                        *reinterpret_cast<float4 *>(dh2s + i * ld + n0) = make_float4(o[0], o[1], o[2], o[3]);
                }
            }
        } else
        // thread owns hidden unit n, loops the rows
        for (int n = tid; n < H2; n += 256) {
            float w[kMaxActions + 1];
#pragma unroll
            for (int a = 0; a < kMaxActions + 1; ++a) w[a] = a < A1 ? whs[a * H2 + n] : 0.0f;
            const int nb = n >> 4, nbit = n & 15;
            if (A1 <= 5) {
#pragma unroll 8
                for (int i = 0; i < kRowsB; ++i) {
                    const bool on = (mkB[i * sh.ncb + nb] >> nbit) & 1;
                    float s = 0.0f;
#pragma unroll
                    for (int a = 0; a < 5; ++a) s = a < A1 ? fmaf(dzs[i * A1 + a], w[a], s) : s;
                    dh2s[i * ld + n] = on ? s : 0.0f;
                }
            } else {
                for (int i = 0; i < kRowsB; ++i) {
                    const bool on = (mkB[i * sh.ncb + nb] >> nbit) & 1;
                    float s = 0.0f;
#pragma unroll
                    for (int a = 0; a < kMaxActions + 1; ++a) s = a < A1 ? fmaf(dzs[i * A1 + a], w[a], s) : s;
                    dh2s[i * ld + n] = on ? s : 0.0f;
                }
            }
        }
        for (int u = tid; u < kRowsB * (H2p - H2); u += 256) {      // K padding (runtime shapes)
            const int i = u / (H2p - H2), n = H2 + (u - i * (H2p - H2));
            dh2s[i * ld + n] = 0.0f;
        }
        __syncthreads();
        GS_STAMP(1)
        {
            const float *arow = dh2s + (rt * 16 + li) * ld;
            const float *brow = W2T + li * ld;
#pragma unroll 4
            for (int ch = chb; ch < che; ++ch) {
                const int n = ch * kTile + 4 * lq;
                const float4 a = *reinterpret_cast<const float4 *>(arow + n);
                const float4 w = *reinterpret_cast<const float4 *>(brow + n);
                acc0 = mfma4(a.x, w.x, acc0);
                acc1 = mfma4(a.y, w.y, acc1);
                acc0 = mfma4(a.z, w.z, acc0);
                acc1 = mfma4(a.w, w.w, acc1);
            }
        }
        }
        {
            const f32x4 acc = acc0 + acc1;
#pragma unroll
            for (int r = 0; r < 4; ++r) kred[wave * 256 + (lq * 4 + r) * kTile + li] = acc[r];
        }
        __syncthreads();
        for (int u = tid; u < kRowsB * kTile; u += 256) {
            const int row = u >> 4, col = u & 15;
            const int t = row >> 4, rr = row & 15;
            const float g = kRowsB == 64 ? kred[t * 256 + rr * kTile + col]
                                         : kred[(2 * t) * 256 + rr * kTile + col] + kred[(2 * t + 1) * 256 + rr * kTile + col];
            tile[row * 17 + col] = h1m[row * 16 + col] > 0.0f ? g : 0.0f;   // relu'(h1)
        }
        __syncthreads();
        GS_STAMP(2)
        // dW1 / db1 partials over this slab's rows: row groups of 16, then combine in order
        {
            constexpr int ng = kRowsB / 16;
            float *pr = dh2s;                       // reuse: [ng][16*(D+1)]
            const int nout = kTile * (D + 1);
            for (int u = tid; u < ng * nout; u += 256) {
                const int g = u / nout, o = u - g * nout;
                const int col = o / (D + 1), d = o - col * (D + 1);
                float s = 0.0f;
#pragma unroll 4
                for (int row = g * 16; row < g * 16 + 16; ++row) {
                    const float xv = d < D ? xs[row * D + d] : 1.0f;
                    s = fmaf(tile[row * 17 + col], xv, s);
                }
                pr[u] = s;
            }
            __syncthreads();
            if (xchg) {      // nout <= 4 * 256 (bwd_xchg_fits)
                float pv[4];
                bool ok[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int o = tid + 256 * j, col = o / (D + 1);
                    ok[j] = o < nout && k0 + col < H1;
                    float t = 0.0f;
                    if (o < nout)
#pragma unroll
                        for (int g = 0; g < ng; ++g) t += pr[g * nout + o];
                    pv[j] = t;
                }
                bwd_exchange<4>(bx, xseq, pv, ok);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int o = tid + 256 * j, col = o / (D + 1), d = o - col * (D + 1);
                    if (ok[j]) part1[((int64_t)rb * H1 + k0 + col) * (D + 1) + d] = pv[j];
                }
            } else
            for (int o = tid; o < nout; o += 256) {
                const int col = o / (D + 1), d = o - col * (D + 1);
                float t = 0.0f;
#pragma unroll
                for (int g = 0; g < ng; ++g) t += pr[g * nout + o];
                if (k0 + col < H1) part1[((int64_t)rb * H1 + k0 + col) * (D + 1) + d] = t;
            }
        }
        GS_STAMP_END(3)
        if constexpr (FUSED) GS_SPAN_END(1, kstep)
        return;
    }
    bid -= sh.nB;
    {
        // ---------------- role C: head grads for hidden block nb (block ncb: head biases)
        // with 16 n-blocks the n-blocks 2m, 2m+1 (one 128-B line of every h2 row) go to workgroups m,
        // m + 8 — one XCD (the grid before role C is a multiple of 8), so each h2 line is fetched once
        const int nb = (sh.ncb == 16 && bid < 16) ? 2 * (bid & 7) + (bid >> 3) : bid;
        const int n0 = nb * kTile;
        const int Bp = (B + 15) / 16 * 16;
        GS_STAMP_BEGIN_IF(5, bid == 0)
        float *hs = lds;                    // [Bp][17]
        float *dzs = hs + Bp * 17;          // [Bp][A1]
        // metric row groups this workgroup stores (fused path): rows [16 gs, 16 ge), their 14 sums
        // each in dscrC (after partC)
        int gs = 0, ge = 0;
        if constexpr (FUSED) {
            const int G = B / kTile;
            gs = G;
            for (int g = 0; g < G; ++g)
                if (metric_owner(g, G, sh.nC) == nb) {
                    gs = min(gs, g);
                    ge = g + 1;
                }
            if (ge == 0) gs = 0;
        }
        double *dscrC = reinterpret_cast<double *>(
            (reinterpret_cast<uintptr_t>(dzs + Bp * A1 + (A1 * 256 > 1024 ? A1 * 256 : 1024)) + 7) & ~(uintptr_t)7);
        auto loss_in = [&]() {
            if constexpr (FUSED)
                loss_rows_lds<S>(P, L, zpart, ff, la, B, kstep, 0, Bp, dzs, ge > gs ? dscrC : nullptr, 0, 256,
                                 kTile * gs, kTile * ge);
            else
                for (int u = tid; u < Bp * A1; u += 256) dzs[u] = u < B * A1 ? dz[u] : 0.0f;
        };
        if constexpr (S::H1c > 0 && S::Bc > 0) {
            // compile-time shapes: the h2 column tile is in flight while the loss rows run
            constexpr Layout Lc = S::lay(Layout{});
            constexpr int cB = S::Bc, cBp = (cB + 15) / 16 * 16, NH = (cBp * 4 + 255) / 256;
            float4 hr[NH];
#pragma unroll
            for (int j = 0; j < NH; ++j) {      // clamped, unconditional; zeroed at the stores
                const int u = tid + 256 * j, b = u >> 2, c4 = u & 3;
                hr[j] = *reinterpret_cast<const float4 *>(h2 + (int64_t)min(b, cB - 1) * Lc.H2 +
                                                          min(n0 + 4 * c4, Lc.H2 - 4));
            }
            loss_in();
#pragma unroll
            for (int j = 0; j < NH; ++j) {
                const int u = tid + 256 * j, b = u >> 2, c4 = u & 3;
                if (u < cBp * 4) {
                    const bool ok = b < cB && n0 + 4 * c4 < Lc.H2;
                    hs[b * 17 + 4 * c4 + 0] = ok ? hr[j].x : 0.0f;
                    hs[b * 17 + 4 * c4 + 1] = ok ? hr[j].y : 0.0f;
                    hs[b * 17 + 4 * c4 + 2] = ok ? hr[j].z : 0.0f;
                    hs[b * 17 + 4 * c4 + 3] = ok ? hr[j].w : 0.0f;
                }
            }
        } else {
#pragma unroll 4
            for (int u = tid; u < Bp * 4; u += 256) {
                const int b = u >> 2, c4 = u & 3;
                float4 hv = make_float4(0.f, 0.f, 0.f, 0.f);
                if (b < B && n0 + 4 * c4 < H2)
                    hv = *reinterpret_cast<const float4 *>(h2 + (int64_t)b * H2 + n0 + 4 * c4);
                hs[b * 17 + 4 * c4 + 0] = hv.x;
                hs[b * 17 + 4 * c4 + 1] = hv.y;
                hs[b * 17 + 4 * c4 + 2] = hv.z;
                hs[b * 17 + 4 * c4 + 3] = hv.w;
            }
            loss_in();
        }
        __syncthreads();
        GS_STAMP(0)
        if constexpr (FUSED)      // this workgroup's metric row groups (rows' sums from the loss pass)
            for (int g = gs; g < ge; ++g)
                store_metric_groups(dscrC + (int64_t)(g - gs) * kTile * kNumSums, kTile, g * kTile, B, kstep,
                                    ff.mpart);
        float *partC = dzs + Bp * A1;           // [A1*16][16]
        if (nb < sh.ncb) {
            const int nout = kTile * A1;
            float sq = 0.0f, sqp = 0.0f, sqv = 0.0f;     // all head weights / policy rows / value row
            if (A1 <= kTile) {
                // dWh[a, n0+j] = sum_b dz[b, a] h2[b, n0+j] as one 16x16 MFMA tile (rows = actions,
                // padded) with K = the batch split over the 4 waves; the wave partials are summed
                // in wave order through LDS
                const int li = lane & 15, lq = lane >> 4;
                const int nch = Bp / kTile;
                const int ch0 = (wave * nch) / 4, ch1 = ((wave + 1) * nch) / 4;
                f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
                auto chunk = [&](int b, float (&av)[4], float (&bv)[4]) {
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        av[c] = li < A1 ? dzs[(b + c) * A1 + li] : 0.0f;
                        bv[c] = hs[(b + c) * 17 + li];
                    }
                };
                if constexpr (S::BF) {
#pragma unroll 2
                    for (int ch = ch0; ch < ch1; ch += 2) {
                        const int b = ch * kTile + 4 * lq;
                        float av0[4], bv0[4], av1[4] = {0.f, 0.f, 0.f, 0.f}, bv1[4] = {0.f, 0.f, 0.f, 0.f};
                        chunk(b, av0, bv0);
                        if (ch + 1 < ch1) chunk(b + kTile, av1, bv1);
                        acc0 = mfma_bf16_pair(f4(av0), f4(av1), f4(bv0), f4(bv1), acc0);
                    }
                } else {
    #pragma unroll 2
                for (int ch = ch0; ch < ch1; ++ch) {
                    const int b = ch * kTile + 4 * lq;
                    float av[4], bv[4];
                    chunk(b, av, bv);
                    acc0 = mfma4(av[0], bv[0], acc0);
                    acc1 = mfma4(av[1], bv[1], acc1);
                    acc0 = mfma4(av[2], bv[2], acc0);
                    acc1 = mfma4(av[3], bv[3], acc1);
                }
                }
                const f32x4 acc = acc0 + acc1;
#pragma unroll
                for (int r = 0; r < 4; ++r) partC[wave * 256 + (lq * 4 + r) * kTile + li] = acc[r];
                __syncthreads();
                const int a = tid >> 4, i = tid & 15;
                float hv[1] = {tid < nout ? ((partC[tid] + partC[256 + tid]) + partC[512 + tid]) + partC[768 + tid]
                                          : 0.0f};
                bool ok[1] = {tid < nout && n0 + i < H2};
                if (xchg) bwd_exchange<1>(bx, xseq, hv, ok);
                if (ok[0]) {
                    G[L.head_row(a) + n0 + i] = hv[0];
                    sq = hv[0] * hv[0];
                }
            } else {
                // outputs (a, i): A1*16 of them; each summed over b by 16 threads into LDS partials
                for (int u = tid; u < nout * 16; u += 256) {
                    const int o = u >> 4, j = u & 15;
                    const int a = o >> 4, i = o & 15;
                    float s = 0.0f;
                    for (int b = j; b < Bp; b += 16) s = fmaf(dzs[b * A1 + a], hs[b * 17 + i], s);
                    partC[u] = s;
                }
                __syncthreads();
                // nout = A1 * 16 <= 4 * 256 (kMaxActions)
                float hv[4];
                bool ok[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int o = tid + 256 * j;
                    float s = 0.0f;
                    if (o < nout)
#pragma unroll
                        for (int m = 0; m < 16; ++m) s += partC[o * 16 + m];
                    hv[j] = s;
                    ok[j] = o < nout && n0 + (o & 15) < H2;
                }
                if (xchg) bwd_exchange<4>(bx, xseq, hv, ok);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int o = tid + 256 * j, a = o >> 4, i = o & 15;
                    if (ok[j]) {
                        G[L.head_row(a) + n0 + i] = hv[j];
                        sq += hv[j] * hv[j];
                        if (a == A) sqv += hv[j] * hv[j];
                        else sqp += hv[j] * hv[j];
                    }
                }
            }
            if (A1 <= kTile) {
                // the reduction's first level leaves the sum of each 16-thread group = head row a
                block_sumsq_store(sq, sumsq + sh.nT + sh.ncb + nb, sbuf);
                if constexpr (FUSED) store_head_split(sbuf + 256, A, ff.headsq, (kstep * (sh.ncb + 1) + nb) * 2);
            } else {
                store_head_sums(sq, sqp, sqv, sumsq + sh.nT + sh.ncb + nb, FUSED ? ff.headsq : nullptr,
                                (kstep * (sh.ncb + 1) + nb) * 2, sbuf);
            }
        } else {
            // the extra block: head-bias gradients (sum of dz over the batch)
            for (int u = tid; u < A1 * 16; u += 256) {
                const int a = u >> 4, j = u & 15;
                float s = 0.0f;
                for (int b = j; b < Bp; b += 16) s += dzs[b * A1 + a];
                partC[u] = s;
            }
            __syncthreads();
            float sqb = 0.0f;
            float bv[1] = {0.0f};
            bool ok[1] = {tid < A1};
            if (tid < A1)
#pragma unroll
                for (int m = 0; m < 16; ++m) bv[0] += partC[tid * 16 + m];
            if (xchg) bwd_exchange<1>(bx, xseq, bv, ok);
            if (ok[0]) {
                G[L.head_bias(tid)] = bv[0];
                sqb = bv[0] * bv[0];
            }
            block_sumsq_store(sqb, sumsq + sh.nT + 2 * sh.ncb, sbuf);
            // the reduction's input level: thread a's square = head bias a
            if constexpr (FUSED) store_head_split(sbuf, A, ff.headsq, (kstep * (sh.ncb + 1) + sh.ncb) * 2);
        }
        GS_STAMP_END(1)
        if constexpr (FUSED) GS_SPAN_END(1, kstep)
    }
}

// ------------------------------------------------------------------------------------
// k_clip_adam: grid ceil(P / 1024), 256 threads, 4 params per thread (strided).
// ------------------------------------------------------------------------------------

// Vectorised variant for the C2 shapes (NRB > 0: NRB row blocks of dW1|db1 partials; NQ =
// ceil(H1*(D+1)/1024) float4 partial columns per thread; oW2, H1*(D+1) multiples of 4 and
// 16-B aligned buffers, checked by the launcher): each thread owns 4 consecutive parameters
// (float4 loads / stores of p, g, m, v), the partials go straight to registers as float4
// with every load in flight at once, are folded there in row-block order, and only the folded
// values pass through LDS.  The generic variant (NRB == 0) stages the partials in LDS.
template <class S, int NRB, int NQ>
__global__ __launch_bounds__(256) void k_clip_adam(float *__restrict__ Pm, Layout Lrt, float *__restrict__ G,
                                                   float *__restrict__ M, float *__restrict__ V,
                                                   const float *__restrict__ part1, const float *__restrict__ sumsq,
                                                   AdamArgs aa, float *__restrict__ metrics,
                                                   const int32_t *__restrict__ stop)
{
    if (stop && *stop) {
        // a job-wide stop (the exchange ORs the ranks' stop bits): this minibatch takes no step on
        // any rank, also on one whose own approx_kl stayed under target_kl — its record says so
        if (metrics && blockIdx.x == 0 && threadIdx.x == 0) {
            float *m = metrics + (aa.step_base ? *aa.step_base : 0) * GS_NUM_METRICS;
            m[GS_M_SKIPPED] = 1.0f;
            m[GS_M_KL_STOP] = 1.0f;
        }
        return;
    }
    GS_STAMP_BEGIN(3)
    const int64_t kb = aa.step_base ? *aa.step_base : 0;
    if (metrics) metrics += kb * GS_NUM_METRICS;
    __shared__ double sred[2 * 272];
    __shared__ float s_coef;
    const Layout L = S::lay(Lrt);
    const int tid = threadIdx.x;
    const int64_t n1 = (int64_t)L.H1 * (L.D + 1);
    const int64_t base = (int64_t)blockIdx.x * 1024;
    extern __shared__ float stage[];
    double ss = 0.0;
    float gv[4], mv[4], vv[4], pv[4];
    // this thread's parameters: p0 + i (vectorised) or base + i*256 + tid (generic)
    const int64_t p0 = base + 4 * tid;
    auto pidx = [&](int i) -> int64_t { return NRB > 0 ? p0 + i : base + i * 256 + tid; };
    if constexpr (NRB > 0) {
        const bool full = p0 + 3 < L.P;
        if (full) {
            const float4 g4 = p0 >= L.oW2 ? *reinterpret_cast<const float4 *>(G + p0) : make_float4(0.f, 0.f, 0.f, 0.f);
            const float4 m4 = *reinterpret_cast<const float4 *>(M + p0);
            const float4 v4 = *reinterpret_cast<const float4 *>(V + p0);
            const float4 q4 = *reinterpret_cast<const float4 *>(Pm + p0);
            gv[0] = g4.x, gv[1] = g4.y, gv[2] = g4.z, gv[3] = g4.w;
            mv[0] = m4.x, mv[1] = m4.y, mv[2] = m4.z, mv[3] = m4.w;
            vv[0] = v4.x, vv[1] = v4.y, vv[2] = v4.z, vv[3] = v4.w;
            pv[0] = q4.x, pv[1] = q4.y, pv[2] = q4.z, pv[3] = q4.w;
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int64_t p = p0 + i;
                const bool ok = p < L.P;
                gv[i] = ok && p >= L.oW2 ? G[p] : 0.0f;
                mv[i] = ok ? M[p] : 0.0f;
                vv[i] = ok ? V[p] : 0.0f;
                pv[i] = ok ? Pm[p] : 0.0f;
            }
        }
        // every load before the first LDS write: one memory round trip
        constexpr int NS = 2;   // sum-of-squares slots per thread (launcher: n_slots <= 512)
        float sl[NS];
#pragma unroll
        for (int j = 0; j < NS; ++j) sl[j] = tid + 256 * j < aa.n_slots ? sumsq[tid + 256 * j] : 0.0f;
        float4 t[NQ][NRB];
#pragma unroll
        for (int j = 0; j < NQ; ++j) {
            const int64_t q = tid + 256 * j;
#pragma unroll
            for (int rb = 0; rb < NRB; ++rb)
                t[j][rb] = 4 * q < n1 ? *reinterpret_cast<const float4 *>(part1 + (int64_t)rb * n1 + 4 * q)
                                      : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int j = 0; j < NS; ++j)
            if (tid + 256 * j < aa.n_slots) stage[tid + 256 * j] = sl[j];
        float *w1s = stage + round4(aa.n_slots);
        float4 gsum[NQ];
#pragma unroll
        for (int j = 0; j < NQ; ++j) {
            const int64_t q = tid + 256 * j;
            float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int rb = 0; rb < NRB; ++rb) {
                g.x += t[j][rb].x;
                g.y += t[j][rb].y;
                g.z += t[j][rb].z;
                g.w += t[j][rb].w;
            }
            gsum[j] = g;
            if (4 * q < n1) *reinterpret_cast<float4 *>(w1s + 4 * q) = g;
        }
        __syncthreads();
        GS_STAMP(0)
        if (p0 < L.oW2) {
#pragma unroll
            for (int i = 0; i < 4; ++i) gv[i] = w1s[part1_index(L, p0 + i)];
        }
        for (int s0 = tid; s0 < aa.n_slots; s0 += 256) ss += (double)stage[s0];
#pragma unroll
        for (int j = 0; j < NQ; ++j)
            if (4 * (tid + 256 * j) < n1) {
                const float4 g = gsum[j];
                ss += (double)g.x * (double)g.x;
                ss += (double)g.y * (double)g.y;
                ss += (double)g.z * (double)g.z;
                ss += (double)g.w * (double)g.w;
            }
    } else {
        // W1|b1 gradients come from the dW1|db1 partials: summed after they are staged in
        // LDS (below) when staging is on, instead of 4 x nrb dependent global loads here
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t p = pidx(j);
            const bool ok = p < L.P;
            float g = 0.0f;
            if (ok) {
                if (aa.nrb > 0 && p < L.oW2) {
                    if (!aa.stage_lds) {
                        const int64_t u = part1_index(L, p);
#pragma unroll 4
                        for (int rb = 0; rb < aa.nrb; ++rb) g += part1[(int64_t)rb * n1 + u];
                    }
                } else {
                    g = G[p];
                }
            }
            gv[j] = g;
            mv[j] = ok ? M[p] : 0.0f;
            vv[j] = ok ? V[p] : 0.0f;
            pv[j] = ok ? Pm[p] : 0.0f;
        }
        // global squared norm (same order in every workgroup -> identical coef); the
        // per-tile sums and dW1/db1 partials are staged into LDS in one burst first
        const int64_t npart = (int64_t)aa.nrb * n1;
        if (aa.stage_lds) {
            copy_to_lds(stage, sumsq, aa.n_slots);
            const int off = round4(aa.n_slots);
            if (npart > 0) copy_to_lds(stage + off, part1, (int)npart);
            __syncthreads();
            GS_STAMP(0)
            if (aa.nrb > 0 && base < L.oW2) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int64_t p = pidx(j);
                    if (p < L.oW2) {
                        const int64_t u = part1_index(L, p);
                        float g = 0.0f;
                        for (int rb = 0; rb < aa.nrb; ++rb) g += stage[off + rb * n1 + u];
                        gv[j] = g;
                    }
                }
            }
            for (int s0 = tid; s0 < aa.n_slots; s0 += 256) ss += (double)stage[s0];
            for (int64_t u = tid; u < n1 && aa.nrb > 0; u += 256) {
                float g = 0.0f;
                for (int rb = 0; rb < aa.nrb; ++rb) g += stage[off + rb * n1 + u];
                ss += (double)g * (double)g;
            }
        } else {
            GS_STAMP(0)
            for (int s0 = tid; s0 < aa.n_slots; s0 += 256) ss += (double)sumsq[s0];
            for (int64_t u = tid; u < n1 && aa.nrb > 0; u += 256) {
                float g = 0.0f;
                for (int rb = 0; rb < aa.nrb; ++rb) g += part1[(int64_t)rb * n1 + u];
                ss += (double)g * (double)g;
            }
        }
    }
    GS_STAMP(1)
    double tt[1] = {ss};
    block_reduce<1>(tt, sred);
    GS_STAMP(2)
    if (tid == 0) {
        const double tot = tt[0];
        const float total = (float)sqrt(tot) * aa.grad_scale;
        s_coef = clip_coef(total, aa);
        if (blockIdx.x == 0 && metrics) metrics[GS_M_GRAD_NORM] = total;
        if (blockIdx.x == 0 && aa.normsq) aa.normsq[kb] = tot * (double)aa.grad_scale * (double)aa.grad_scale;
    }
    __syncthreads();
    const float coef = s_coef * aa.grad_scale;
    const float neg_step = aa.sched ? aa.sched[2 * (aa.sched_idx + kb)] : aa.neg_step_size;
    const float bc2s = aa.sched ? aa.sched[2 * (aa.sched_idx + kb) + 1] : aa.inv_bc2_sqrt;
    float go[4], mo[4], vo[4], po[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        float m = mv[j], v = vv[j], p = pv[j];
        go[j] = adam_param(gv[j], coef, m, v, p, aa, neg_step, bc2s);
        mo[j] = m;
        vo[j] = v;
        po[j] = p;
    }
    if (NRB > 0 && p0 + 3 < L.P) {
        *reinterpret_cast<float4 *>(G + p0) = make_float4(go[0], go[1], go[2], go[3]);
        *reinterpret_cast<float4 *>(Pm + p0) = make_float4(po[0], po[1], po[2], po[3]);
        *reinterpret_cast<float4 *>(M + p0) = make_float4(mo[0], mo[1], mo[2], mo[3]);
        *reinterpret_cast<float4 *>(V + p0) = make_float4(vo[0], vo[1], vo[2], vo[3]);
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t p = pidx(j);
            if (p >= L.P) break;
            G[p] = go[j];
            Pm[p] = po[j];
            M[p] = mo[j];
            V[p] = vo[j];
        }
    }
    GS_STAMP_END(3)
}

// sum of squares over a flat range (multi-GPU path: norm after the all-reduce)
__global__ __launch_bounds__(256) void k_sumsq_flat(const float *__restrict__ G, int64_t n, float *__restrict__ out)
{
    __shared__ float sbuf[272];
    float s = 0.0f;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) s += G[i] * G[i];
    block_sumsq_store(s, out + blockIdx.x, sbuf);
}

// reduce dW1/db1 partials into the flat gradient (multi-GPU path, before the all-reduce)
__global__ __launch_bounds__(256) void k_reduce_part1(const float *__restrict__ part1, Layout L, int nrb,
                                                      float *__restrict__ G, const int32_t *__restrict__ stop)
{
    if (stop && *stop) return;
    const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= L.oW2) return;
    const int64_t n1 = (int64_t)L.H1 * (L.D + 1);
    const int64_t u = part1_index(L, p);
    float g = 0.0f;
    for (int rb = 0; rb < nrb; ++rb) g += part1[(int64_t)rb * n1 + u];
    G[p] = g;
}

// ------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------
// Call f(shape_policy) with the compile-time instantiation matching (L, B), else the
// runtime fallback.  B <= 0: the minibatch size is not part of the instantiation.
template <class F>
static int with_shape(const Layout &L, int64_t B, F &&f)
{
    if (L.D == 4 && L.H1 == 256 && L.H2 == 256 && L.A == 2) {        // CartPole-v1:ppo (mlp_medium)
        if (B == 256) return f(ShapeC<4, 256, 256, 2, 256>{});          // 32-row role-B slabs (64-row slabs: 14.48 vs 14.38 us)
        return f(ShapeC<4, 256, 256, 2, 0>{});
    }
    if (L.D == 8 && L.H1 == 128 && L.H2 == 128 && L.A == 4) {        // LunarLander-v3:ppo (mlp_small)
        if (B == 64) return f(ShapeC<8, 128, 128, 4, 64>{});
        return f(ShapeC<8, 128, 128, 4, 0>{});
    }
    if (L.A <= 4) return f(ShapeR<4>{});
    return f(ShapeR<kMaxActions>{});
}

int rows_b(const Layout &L, int64_t B)
{
    int rb = kRowsB;
    with_shape(L, B, [&](auto sh) {
        rb = decltype(sh)::RB;
        return GS_OK;
    });
    return rb;
}

// Raise a kernel's dynamic-LDS limit once (never inside a stream capture: the first
// eager launch or prepare_kernels() does it before any graph is recorded).
static int set_lds_limit(const void *fn, size_t bytes)
{
    static std::mutex mu;
    static std::unordered_map<const void *, size_t> done;
    if (bytes <= 65536) return GS_OK;
    std::lock_guard<std::mutex> lk(mu);
    auto it = done.find(fn);
    if (it != done.end() && it->second >= bytes) return GS_OK;
    GS_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
    done[fn] = bytes;
    return GS_OK;
}

// the bf16 mode's instantiations: compile-time shapes whose backward forms dh2 in registers
// (the fast role-A / role-B paths carry the bf16 operand pairs)
template <class Sh>
constexpr bool bf16_shape()
{
    if constexpr (Sh::AEX == 0 || Sh::H1c == 0 || Sh::Bc == 0) {
        return false;
    } else {
        constexpr Layout Lc = Sh::lay(Layout{});
        return Lc.A + 1 <= 5 && Lc.H2 % 64 == 0;
    }
}

bool has_bf16_chain(const Layout &L, int64_t B)
{
    bool ok = false;
    with_shape(L, B, [&](auto sh) {
        ok = bf16_shape<decltype(sh)>();
        return GS_OK;
    });
    return ok && has_fused(L, B);
}

int prepare_kernels(const Layout &L, int64_t B)
{
    if (has_bf16_chain(L, B)) {
        const int rc = with_shape(L, B, [&](auto sh) {
            using Sh = decltype(sh);
            if constexpr (bf16_shape<Sh>())
                return set_lds_limit((const void *)k_bwd<Bf16Shape<Sh>, true>, bwd_lds_bytes(L, B));
            return GS_OK;
        });
        if (rc) return rc;
    }
    int rc = with_shape(L, B, [&](auto sh) {
        return set_lds_limit((const void *)k_bwd<decltype(sh), false>, bwd_lds_bytes(L, B));
    });
    if (rc) return rc;
    if (has_fused(L, B)) {
        rc = with_shape(L, B, [&](auto sh) {
            return set_lds_limit((const void *)k_bwd<decltype(sh), true>, bwd_lds_bytes(L, B));
        });
        if (rc) return rc;
    }
    rc = with_shape(L, 0, [&](auto sh) {
        return set_lds_limit((const void *)k_fwd_hidden<decltype(sh), false>, fwd_lds_bytes(L));
    });
    if (rc) return rc;
    if (!has_fused(L, B)) return GS_OK;
    return with_shape(L, B, [&](auto sh) {
        return set_lds_limit((const void *)k_fwd_hidden<decltype(sh), true>, fwd_lds_bytes(L));
    });
}

int launch_heads_act(const float *P, const Layout &L, const float *zpart, int64_t rows, int mode, uint64_t seed,
                     uint64_t counter, int64_t *actions, float *logp, float *value, hipStream_t s,
                     const uint64_t *clock)
{
    const dim3 grid((unsigned)((rows + 255) / 256));
    return with_shape(L, 0, [&](auto sh) {
        hipLaunchKernelGGL(k_heads_act<decltype(sh)>, grid, dim3(256), 0, s, P, L, zpart, rows, mode, seed, counter,
                           actions, logp, value, clock);
        GS_LAUNCH_CHECK("k_heads_act");
        return GS_OK;
    });
}

int launch_loss(const float *P, const Layout &L, int64_t B, const Workspace &ws, const LossArgs &la, float *metrics,
                int32_t *stop, hipStream_t s)
{
    return with_shape(L, B, [&](auto sh) {
        hipLaunchKernelGGL(k_loss<decltype(sh)>, dim3(1), dim3(256), 0, s, P, L, ws.zpart, (int)B, ws.f_act,
                           ws.f_olp, ws.f_ov, ws.f_adv, ws.f_ret, la, ws.dz, metrics, stop);
        GS_LAUNCH_CHECK("k_loss");
        return GS_OK;
    });
}

bool bwd_xchg_coresident(int64_t nblk, size_t lds_bytes, int colocated);

bool bwd_xchg_fits(const Layout &L, int64_t B, int colocated)
{
    const BwdShape sh = BwdShape::make(L, (int)B, rows_b(L, B));
    const int64_t nblk = sh.nA + sh.nB + sh.nC;
    return nblk <= kBwdXMaxWG && kTile * (L.D + 1) <= kBwdXSlot && (L.A + 1) * kTile <= kBwdXSlot &&
           bwd_xchg_coresident(nblk, bwd_lds_bytes(L, B), colocated);
}

// Progress of the exchange inside k_bwd: workgroup w of a rank waits only for workgroup w of its
// peers, and each rank's resident workgroups are a prefix of its grid (in-order dispatch), so
// the exchange completes unless one rank has no resident workgroup while the others fill the GPU.
// One rank per GPU never starves; c ranks on one GPU need (c - 1) grids to leave a free slot.
bool bwd_xchg_coresident(int64_t nblk, size_t lds_bytes, int colocated)
{
    if (colocated <= 1) return true;
    int dev = 0, ncu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return false;
    int64_t per_cu = (int64_t)(160 * 1024) / (int64_t)(lds_bytes > 0 ? lds_bytes : 1);
    if (per_cu > 4) per_cu = 4;       // 16 waves per CU at k_bwd's register use
    return (int64_t)(colocated - 1) * nblk < (int64_t)ncu * per_cu;
}

int launch_bwd(const float *P, const Layout &L, int64_t B, const Workspace &ws, float *G, const int32_t *stop,
               hipStream_t s, const FusedFwd *ff, const LossArgs *la, const BwdXchg *bxp)
{
    const BwdShape sh0 = BwdShape::make(L, (int)B, rows_b(L, B));
    const unsigned nblk = (unsigned)(sh0.nA + sh0.nB + sh0.nC);
    const size_t lds = bwd_lds_bytes(L, B);
    BwdXchg bx{};
    if (bxp && bxp->world > 1) {
        GS_REQUIRE(bwd_xchg_fits(L, B), "k_bwd exchange: %u workgroups or their output slots exceed the limits",
                   nblk);
        bx = *bxp;
    }
    return with_shape(L, B, [&](auto sh) {
        using Sh = decltype(sh);
        if (ff && la && la->bf16) {      // the bf16 mode (GS_HP_BF16)
            if constexpr (bf16_shape<Sh>()) {
                int rc = set_lds_limit((const void *)k_bwd<Bf16Shape<Sh>, true>, lds);
                if (rc) return rc;
                hipLaunchKernelGGL((k_bwd<Bf16Shape<Sh>, true>), dim3(nblk), dim3(256), lds, s, P, L, (int)B, ws.x,
                                   ws.h1, ws.h2, ws.dz, G, ws.part1, ws.sumsq, stop, ws.zpart, *ff, *la, ws.h2mask, bx);
                GS_LAUNCH_CHECK("k_bwd<bf16>");
                return GS_OK;
            } else {
                GS_REQUIRE(false, "precision bf16: no bf16 instantiation of the MLP chain for this shape");
            }
        }
        if (ff) {
            int rc = set_lds_limit((const void *)k_bwd<Sh, true>, lds);
            if (rc) return rc;
            hipLaunchKernelGGL((k_bwd<Sh, true>), dim3(nblk), dim3(256), lds, s, P, L, (int)B, ws.x, ws.h1, ws.h2,
                               ws.dz, G, ws.part1, ws.sumsq, stop, ws.zpart, *ff, *la, ws.h2mask, bx);
        } else {
            int rc = set_lds_limit((const void *)k_bwd<Sh, false>, lds);
            if (rc) return rc;
            hipLaunchKernelGGL((k_bwd<Sh, false>), dim3(nblk), dim3(256), lds, s, P, L, (int)B, ws.x, ws.h1, ws.h2,
                               ws.dz, G, ws.part1, ws.sumsq, stop, (const float *)nullptr, FusedFwd{}, LossArgs{},
                               ws.h2mask, bx);
        }
        GS_LAUNCH_CHECK("k_bwd");
        return GS_OK;
    });
}

// Per-component pre-clip gradient norms of the step k_clip_adam is about to take (utils/models.py:
// 196-230).  Its own kernel: k_clip_adam's workgroups overwrite G with the clipped gradients, so a
// workgroup of it cannot read the raw head gradients of another one race-free.  Total squared norm
// from the same slots + dW1|db1 partials k_clip_adam folds (double sums; order-only differences).
__global__ __launch_bounds__(256) void k_component_norms(Layout L, const float *__restrict__ G,
                                                         const float *__restrict__ part1,
                                                         const float *__restrict__ sumsq, int n_slots, int nrb,
                                                         float gscale, const int64_t *__restrict__ step_base,
                                                         float *__restrict__ metrics,
                                                         const int32_t *__restrict__ stop)
{
    if (stop && *stop) return;
    __shared__ double sred[2 * 272];
    const int tid = threadIdx.x;
    const int64_t n1 = (int64_t)L.H1 * (L.D + 1);
    double tt[1] = {0.0};
    for (int s0 = tid; s0 < n_slots; s0 += 256) tt[0] += (double)sumsq[s0];
    for (int64_t u = tid; u < n1 && nrb > 0; u += 256) {
        float g = 0.0f;
        for (int rb = 0; rb < nrb; ++rb) g += part1[(int64_t)rb * n1 + u];
        tt[0] += (double)g * (double)g;
    }
    block_reduce<1>(tt, sred);
    double hq[2] = {0.0, 0.0};
    const int nhg = (L.A + 1) * (L.H2 + 1);
    for (int u = tid; u < nhg; u += 256) {
        bool val;
        const double g = (double)G[head_grad_offset(L, u, &val)];
        hq[val ? 1 : 0] += g * g;
    }
    store_component_norms(hq, tt[0], gscale, metrics + (step_base ? *step_base : 0) * GS_NUM_METRICS, sred);
}

int launch_clip_adam(float *P, const Layout &L, float *G, float *M, float *V, const float *part1,
                     const float *sumsq, const AdamArgs &aa_in, float *metrics, const int32_t *stop, hipStream_t s,
                     bool comp_norms)
{
    AdamArgs aa = aa_in;
    if (metrics && comp_norms) {
        hipLaunchKernelGGL(k_component_norms, dim3(1), dim3(256), 0, s, L, G, part1, sumsq, aa.n_slots, aa.nrb,
                           aa.grad_scale, aa.step_base, metrics, stop);
        GS_LAUNCH_CHECK("k_component_norms");
    }
    const size_t stage = sizeof(float) * (round4(aa.n_slots) + (size_t)aa.nrb * L.H1 * (L.D + 1));
    aa.stage_lds = stage <= 65536 ? 1 : 0;
    const unsigned nblk = (unsigned)((L.P + 1023) / 1024);
    return with_shape(L, 0, [&](auto sh) {
        const int64_t n1 = (int64_t)L.H1 * (L.D + 1);
        const bool al = (((uintptr_t)P | (uintptr_t)G | (uintptr_t)M | (uintptr_t)V | (uintptr_t)part1) & 15) == 0;
        const int nq = (int)((n1 / 4 + 255) / 256);
        const bool vec = aa.stage_lds && n1 % 4 == 0 && L.oW2 % 4 == 0 && al && aa.n_slots <= 512 && nq <= 2;
        using Sh = decltype(sh);
        const void *fn = nullptr;   // the fused shapes: C2 (B 256 -> 8 row blocks), C3 (B 64 -> 2)
        if (vec && aa.nrb == 8) fn = nq == 2 ? (const void *)k_clip_adam<Sh, 8, 2> : (const void *)k_clip_adam<Sh, 8, 1>;
        if (vec && aa.nrb == 4) fn = nq == 2 ? (const void *)k_clip_adam<Sh, 4, 2> : (const void *)k_clip_adam<Sh, 4, 1>;
        if (vec && aa.nrb == 2) fn = nq == 2 ? (const void *)k_clip_adam<Sh, 2, 2> : (const void *)k_clip_adam<Sh, 2, 1>;
        if (fn) {
            void *args[] = {&P, (void *)&L, &G, &M, &V, &part1, &sumsq, &aa, &metrics, &stop};
            GS_HIP(hipLaunchKernel(fn, dim3(nblk), dim3(256), args, stage, s));
        } else {
            hipLaunchKernelGGL((k_clip_adam<Sh, 0, 0>), dim3(nblk), dim3(256), aa.stage_lds ? stage : 0, s, P, L, G,
                               M, V, part1, sumsq, aa, metrics, stop);
        }
        GS_LAUNCH_CHECK("k_clip_adam");
        return GS_OK;
    });
}

// ------------------------------------------------------------------------------------
// fused update path: per-update gather, per-update metrics
// ------------------------------------------------------------------------------------
// One workgroup per minibatch k: gather its B rows through the sampler indices, batch
// advantage normalisation (utils/torch.py:97-99, same double arithmetic as k_loss), and
// the ADV_NORM metrics of the normalised advantages.
template <class S>
__global__ __launch_bounds__(256) void k_gather_all(const int32_t *__restrict__ idx, int Brt, const float *__restrict__ obs,
                                                    const int64_t *__restrict__ actions,
                                                    const float *__restrict__ logprobs, const float *__restrict__ values,
                                                    const float *__restrict__ advantages,
                                                    const float *__restrict__ returns, int T, int N, int D,
                                                    int normalize, FusedFwd ff, float *__restrict__ metrics,
                                                    const float *__restrict__ adv_stats)
{
    __shared__ double sred[2 * (256 + 16)];
    const int B = S::batch(Brt);
    const int64_t k = blockIdx.x;
    const int tid = threadIdx.x;
    constexpr int kMaxRows = 4;     // B <= 1024
    float adv[kMaxRows];
    bool mine[kMaxRows];
    double m1[1] = {0.0};
#pragma unroll
    for (int j = 0; j < kMaxRows; ++j) {
        const int r = tid + 256 * j;
        adv[j] = 0.0f;
        mine[j] = false;
        if (r < B) {
            const int si = idx[k * B + r];
            const int64_t o = k * B + r;
            if (si < 0) {      // another rank's row of a global minibatch: no loss, no gradient
                for (int d = 0; d < D; ++d) const_cast<float *>(ff.xg)[o * D + d] = 0.0f;
                const_cast<int32_t *>(ff.fa)[o] = -1;
                const_cast<float *>(ff.folp)[o] = 0.0f;
                const_cast<float *>(ff.fov)[o] = 0.0f;
                const_cast<float *>(ff.fret)[o] = 0.0f;
                continue;
            }
            const int src = sample_row(si, T, N);
            for (int d = 0; d < D; ++d) const_cast<float *>(ff.xg)[o * D + d] = obs[(int64_t)src * D + d];
            const_cast<int32_t *>(ff.fa)[o] = (int32_t)actions[src];
            const_cast<float *>(ff.folp)[o] = logprobs[src];
            const_cast<float *>(ff.fov)[o] = values[src];
            const_cast<float *>(ff.fret)[o] = returns[src];
            adv[j] = advantages[src];
            mine[j] = true;
            m1[0] += (double)adv[j];
        }
    }
    if (normalize && adv_stats) {    // global mode: the whole minibatch's statistics (all ranks)
        const float meanf = adv_stats[2 * k], stdf = adv_stats[2 * k + 1];
#pragma unroll
        for (int j = 0; j < kMaxRows; ++j)
            if (tid + 256 * j < B)
                const_cast<float *>(ff.fadv)[k * B + tid + 256 * j] = mine[j] ? (adv[j] - meanf) / (stdf + 1e-8f) : 0.0f;
        return;     // ADV_NORM metrics: from the combined loss sums (host)
    }
    if (!normalize) {
#pragma unroll
        for (int j = 0; j < kMaxRows; ++j)
            if (tid + 256 * j < B) const_cast<float *>(ff.fadv)[k * B + tid + 256 * j] = adv[j];
        if (tid == 0) {
            metrics[k * GS_NUM_METRICS + GS_M_ADV_NORM_MEAN] = 0.0f;
            metrics[k * GS_NUM_METRICS + GS_M_ADV_NORM_STD] = 0.0f;
        }
        return;
    }
    block_reduce<1>(m1, sred);
    const double mean = m1[0] / (double)B;
    double q[1] = {0.0};
#pragma unroll
    for (int j = 0; j < kMaxRows; ++j)
        if (tid + 256 * j < B) {
            const double dv = (double)adv[j] - mean;
            q[0] += dv * dv;
        }
    block_reduce<1>(q, sred);
    const float meanf = (float)mean;
    const float stdf = (float)sqrt(q[0] / (double)(B - 1));
    double st[2] = {0.0, 0.0};
#pragma unroll
    for (int j = 0; j < kMaxRows; ++j)
        if (tid + 256 * j < B) {
            const float a = (adv[j] - meanf) / (stdf + 1e-8f);
            const_cast<float *>(ff.fadv)[k * B + tid + 256 * j] = a;
            st[0] += (double)a;
            st[1] += (double)a * (double)a;
        }
    block_reduce<2>(st, sred);
    if (tid == 0) {
        const double Bd = (double)B;
        metrics[k * GS_NUM_METRICS + GS_M_ADV_NORM_MEAN] = (float)(st[0] / Bd);
        metrics[k * GS_NUM_METRICS + GS_M_ADV_NORM_STD] =
            (float)sqrt(fmax(0.0, (st[1] - st[0] * st[0] / Bd) / (Bd - 1.0)));
    }
}

// ---- global-minibatch mode (gs_ppo_global_adv_stats / gs_ppo_global_records): everything the
// mode adds around the update stays on the device — the per-minibatch advantage sums of this
// rank's rows (k_global_adv_sums) and, after the communicator's f64 sum over ranks, the whole
// minibatch's mean / unbiased std (k_global_adv_stats, utils/torch.py:97-99; the one-pass double
// form of k_gather_all's two-pass statistics); after the update, the ranks' summed loss sums
// turned into every evaluated minibatch's record (k_global_records: write_metrics, the
// arithmetic of k_metrics_all over the whole global minibatch).
__global__ __launch_bounds__(256) void k_global_adv_sums(const int32_t *__restrict__ idx, int B,
                                                         const float *__restrict__ advantages, int T, int N,
                                                         double *__restrict__ sums)
{
    __shared__ double sred[2 * (256 + 16)];
    const int64_t k = blockIdx.x;
    double st[2] = {0.0, 0.0};
    for (int r = threadIdx.x; r < B; r += 256) {
        const int si = idx[k * B + r];
        if (si < 0) continue;       // another rank's row
        const double a = (double)advantages[sample_row(si, T, N)];
        st[0] += a;
        st[1] += a * a;
    }
    block_reduce<2>(st, sred);
    if (threadIdx.x == 0) {
        sums[2 * k] = st[0];
        sums[2 * k + 1] = st[1];
    }
}

__global__ __launch_bounds__(256) void k_global_adv_stats(const double *__restrict__ sums, int64_t n, int Bg,
                                                          float *__restrict__ stats)
{
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= n) return;
    const double Bd = (double)Bg, s1 = sums[2 * k], s2 = sums[2 * k + 1];
    const double mean = s1 / Bd;
    stats[2 * k] = (float)mean;
    stats[2 * k + 1] = (float)sqrt(fmax(0.0, (s2 - s1 * mean) / (Bd - 1.0)));
}

__global__ __launch_bounds__(256) void k_global_records(const double *__restrict__ sums, int64_t n, LossArgs la,
                                                        float *__restrict__ metrics)
{
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= n) return;
    float *rec = metrics + k * GS_NUM_METRICS;
    if (rec[GS_M_UNEVALUATED] != 0.0f) return;     // after the KL stop: never evaluated
    float tmp[GS_NUM_METRICS];
    write_metrics(sums + k * kNumSums, (double)la.batch_rows, la, tmp, true);
    const int cols[] = {GS_M_LOSS, GS_M_POLICY_LOSS, GS_M_VALUE_LOSS, GS_M_ENTROPY, GS_M_CLIP_FRAC,
                        GS_M_CLIP_FRAC_VF, GS_M_EXPLAINED_VAR, GS_M_KL, GS_M_APPROX_KL, GS_M_ADV_NORM_MEAN,
                        GS_M_ADV_NORM_STD};
#pragma unroll
    for (int c : cols) rec[c] = tmp[c];
}

int launch_global_adv_sums(const int32_t *idx, int64_t n, int64_t B, const float *adv, int64_t T, int64_t N,
                           double *sums, hipStream_t s)
{
    hipLaunchKernelGGL(k_global_adv_sums, dim3((unsigned)n), dim3(256), 0, s, idx, (int)B, adv, (int)T, (int)N, sums);
    GS_LAUNCH_CHECK("k_global_adv_sums");
    return GS_OK;
}

int launch_global_adv_stats(const double *sums, int64_t n, int64_t Bg, float *stats, hipStream_t s)
{
    hipLaunchKernelGGL(k_global_adv_stats, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, sums, n, (int)Bg, stats);
    GS_LAUNCH_CHECK("k_global_adv_stats");
    return GS_OK;
}

int launch_global_records(const double *sums, int64_t n, const LossArgs &la, float *metrics, hipStream_t s)
{
    hipLaunchKernelGGL(k_global_records, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, sums, n, la, metrics);
    GS_LAUNCH_CHECK("k_global_records");
    return GS_OK;
}

// thread per minibatch: the row-block sums (fixed order) -> the metrics record
__global__ __launch_bounds__(256) void k_metrics_all(const double *__restrict__ mpart, int nrb, int64_t n, int B,
                                                     LossArgs la, float *__restrict__ metrics,
                                                     const float *__restrict__ headsq, int nhw,
                                                     const double *__restrict__ normsq)
{
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= n) return;
    double t[kNumSums];
#pragma unroll
    for (int q = 0; q < kNumSums; ++q) t[q] = 0.0;
    for (int rb = 0; rb < nrb; ++rb)
#pragma unroll
        for (int q = 0; q < kNumSums; ++q) t[q] += mpart[(k * nrb + rb) * kNumSums + q];
    float *rec = metrics + k * GS_NUM_METRICS;
    write_metrics(t, (double)la.batch_rows, la, rec, la.sums_out != nullptr);
    if (la.sums_out)
#pragma unroll
        for (int q = 0; q < kNumSums; ++q) la.sums_out[k * kNumSums + q] = t[q];
    (void)B;
    if (headsq) {
        // per-component pre-clip norms (utils/models.py:196-230): the heads from role C's per-step
        // sums (the exchanged, scaled gradient's), the backbone as the rest of the recorded total
        double hq[2] = {0.0, 0.0};
        for (int w = 0; w < nhw; ++w) {
            hq[0] += (double)headsq[(k * nhw + w) * 2];
            hq[1] += (double)headsq[(k * nhw + w) * 2 + 1];
        }
        rec[GS_M_GN_POLICY_HEAD] = (float)sqrt(hq[0]);
        rec[GS_M_GN_VALUE_HEAD] = (float)sqrt(hq[1]);
        rec[GS_M_GN_BACKBONE] = (float)sqrt(fmax(0.0, normsq[k] - hq[0] - hq[1]));
        rec[GS_M_GN_MLP] = 0.0f;
    }
}

// ---- activation statistics of the backbone's Linear outputs (utils/models.py:120-145: forward
// hooks on backbone.0 and backbone.2, i.e. the pre-activation values z1 = W1 x + b1 and
// z2 = W2 relu(z1) + b2; recorded by BaseAgent.training_step, base_agent.py:336-347) for rows
// idx[0..R) of the rollout (idx null: rows 0..R).  One workgroup per 16 rows writes its part:
// per layer {sum z, sum z^2} (double) and per neuron the count of |z| < 1e-6; the host adds the
// parts (gsamd.metrics.activation_stats).  Diagnostics, off the minibatch chain: the agent
// calls it once per epoch on the epoch's first minibatch with the parameters that minibatch uses.
constexpr int kActRows = 16;
__host__ __device__ inline int act_part_stride(const Layout &L) { return 2 * (2 + (L.H1 > L.H2 ? L.H1 : L.H2)); }

__global__ __launch_bounds__(256) void k_mlp_act_stats(const float *__restrict__ P, Layout L,
                                                       const float *__restrict__ obs, const int32_t *__restrict__ idx,
                                                       int T, int N, int R, double *__restrict__ part,
                                                       const int64_t *__restrict__ step_base)
{
    extern __shared__ float lds[];
    if (step_base && idx) idx += *step_base * R;      // graph chunk replay: this step's rows
    __shared__ double sred[2 * 272];
    const int tid = threadIdx.x, D = L.D, H1 = L.H1, H2 = L.H2;
    const int r0 = blockIdx.x * kActRows, nr = min(kActRows, R - r0);
    float *xs = lds;                      // [16][D]
    float *h1s = xs + kActRows * D;       // [16][H1]
    for (int u = tid; u < kActRows * D; u += 256) {
        const int r = u / D, d = u - r * D;
        const int src = r < nr ? (idx ? sample_row(idx[r0 + r], T, N) : r0 + r) : -1;
        xs[u] = src >= 0 ? obs[(int64_t)src * D + d] : 0.0f;
    }
    __syncthreads();
    double* out = part + (int64_t)blockIdx.x * act_part_stride(L);
    const int HM = H1 > H2 ? H1 : H2;
    double st[2] = {0.0, 0.0};
    for (int n = tid; n < H1; n += 256) {
        int cnt = 0;
        for (int r = 0; r < nr; ++r) {
            float z = P[L.ob1 + n];
            for (int d = 0; d < D; ++d) z = fmaf(P[L.oW1 + (int64_t)n * D + d], xs[r * D + d], z);
            st[0] += (double)z;
            st[1] += (double)z * (double)z;
            cnt += fabsf(z) < 1e-6f ? 1 : 0;
            h1s[r * H1 + n] = z > 0.0f ? z : 0.0f;
        }
        out[2 + n] = (double)cnt;
    }
    block_reduce<2>(st, sred);       // its barriers also publish h1s
    if (tid == 0) out[0] = st[0], out[1] = st[1];
    double st2[2] = {0.0, 0.0};
    for (int n = tid; n < H2; n += 256) {
        float z[kActRows];
        const float b = P[L.ob2 + n];
#pragma unroll
        for (int r = 0; r < kActRows; ++r) z[r] = b;
        for (int k = 0; k < H1; ++k) {
            const float w = P[L.oW2 + (int64_t)n * H1 + k];
#pragma unroll
            for (int r = 0; r < kActRows; ++r) z[r] = fmaf(w, h1s[r * H1 + k], z[r]);
        }
        int cnt = 0;
#pragma unroll
        for (int r = 0; r < kActRows; ++r)
            if (r < nr) {
                st2[0] += (double)z[r];
                st2[1] += (double)z[r] * (double)z[r];
                cnt += fabsf(z[r]) < 1e-6f ? 1 : 0;
            }
        out[2 + HM + 2 + n] = (double)cnt;
    }
    block_reduce<2>(st2, sred);
    if (tid == 0) out[2 + HM] = st2[0], out[2 + HM + 1] = st2[1];
}

int launch_act_stats(const float *P, const Layout &L, const float *obs, const int32_t *idx, int64_t T, int64_t N,
                     int64_t R, double *part, hipStream_t s, const int64_t *step_base)
{
    const size_t lds = sizeof(float) * (size_t)kActRows * (L.D + L.H1);
    GS_REQUIRE(lds <= 64 * 1024, "activation stats: obs_dim + hidden1 too large");
    const unsigned nb = (unsigned)((R + kActRows - 1) / kActRows);
    hipLaunchKernelGGL(k_mlp_act_stats, dim3(nb), dim3(256), lds, s, P, L, obs, idx, (int)T, (int)N, (int)R, part,
                       step_base);
    GS_LAUNCH_CHECK("k_mlp_act_stats");
    return GS_OK;
}

// GS_HP_ACT_STATS on the unfused chain: one step's k_mlp_act_stats parts -> its record's GS_M_ACT
// slots (the arithmetic of k_act_stats_fused over the parts' double sums and counts).  A minibatch
// after a KL stop is never evaluated: the record stays as the loss kernel leaves it.
__global__ __launch_bounds__(256) void k_act_parts_record(const double *__restrict__ part, int nparts, int H1, int H2,
                                                          int R, const int32_t *__restrict__ stop,
                                                          float *__restrict__ metrics,
                                                          const int64_t *__restrict__ step_base)
{
    __shared__ double sred[4 * (256 + 16)];
    __shared__ unsigned smax[2];
    if (stop && *stop) return;
    const int tid = threadIdx.x, HM = H1 > H2 ? H1 : H2, stride = 2 * (2 + HM);
    if (tid < 2) smax[tid] = 0u;
    __syncthreads();
    double dsum[2] = {0.0, 0.0};
#pragma unroll
    for (int l = 0; l < 2; ++l) {
        const int H = l == 0 ? H1 : H2, off = l * (2 + HM) + 2;
        unsigned mx = 0u;
        for (int j = tid; j < H; j += 256) {
            double cnt = 0.0;
            for (int p = 0; p < nparts; ++p) cnt += part[(int64_t)p * stride + off + j];
            dsum[l] += cnt;
            mx = (unsigned)cnt > mx ? (unsigned)cnt : mx;
        }
        atomicMax(&smax[l], mx);
    }
    double zs[4] = {0.0, 0.0, 0.0, 0.0};
    for (int p = tid; p < nparts; p += 256)
#pragma unroll
        for (int q = 0; q < 4; ++q) zs[q] += part[(int64_t)p * stride + (q >> 1) * (2 + HM) + (q & 1)];
    block_reduce<2>(dsum, sred);
    block_reduce<4>(zs, sred);
    if (tid == 0) {
        float *rec = metrics + (step_base ? *step_base : 0) * GS_NUM_METRICS + GS_M_ACT;
#pragma unroll
        for (int l = 0; l < 2; ++l) {
            const double n = (double)R * (double)(l == 0 ? H1 : H2);
            const double s1 = zs[2 * l], s2 = zs[2 * l + 1];
            const double var = (s2 - s1 * s1 / n) / (n - 1.0);
            rec[4 * l + 0] = (float)(s1 / n);
            rec[4 * l + 1] = (float)sqrt(var > 0.0 ? var : 0.0);
            rec[4 * l + 2] = (float)(dsum[l] / n);
            rec[4 * l + 3] = (float)((double)smax[l] / (double)R);
        }
    }
}

int launch_act_parts_record(const Layout &L, int64_t R, const double *part, const int32_t *stop, float *metrics,
                            const int64_t *step_base, hipStream_t s)
{
    hipLaunchKernelGGL(k_act_parts_record, dim3(1), dim3(256), 0, s, part, (int)((R + kActRows - 1) / kActRows), L.H1,
                       L.H2, (int)R, stop, metrics, step_base);
    GS_LAUNCH_CHECK("k_act_parts_record");
    return GS_OK;
}

// After an exchange launched behind k_bwd (RCCL, or the xGMI kernel): step k's head record from
// the exchanged gradient in G (role C's sums were of this rank's own gradient), x scale (1/world)
__global__ __launch_bounds__(256) void k_head_sq(Layout L, const float *__restrict__ G, float scale,
                                                 const int64_t *__restrict__ step_base, int64_t k_local,
                                                 float *__restrict__ headsq)
{
    __shared__ double sred[2 * 272];
    const int tid = threadIdx.x;
    double hq[2] = {0.0, 0.0};
    const int nhg = (L.A + 1) * (L.H2 + 1);
    for (int u = tid; u < nhg; u += 256) {
        bool val;
        const double g = (double)G[head_grad_offset(L, u, &val)] * (double)scale;
        hq[val ? 1 : 0] += g * g;
    }
    block_reduce<2>(hq, sred);
    if (tid == 0) {
        const int nhw = (L.H2 + kTile - 1) / kTile + 1;
        float *o = headsq + (k_local + (step_base ? *step_base : 0)) * nhw * 2;
        o[0] = (float)hq[0];
        o[1] = (float)hq[1];
        for (int w = 1; w < nhw; ++w) o[2 * w] = o[2 * w + 1] = 0.0f;
    }
}

int launch_head_sq(const Layout &L, const float *G, float scale, const FusedFwd &ff, hipStream_t s)
{
    hipLaunchKernelGGL(k_head_sq, dim3(1), dim3(256), 0, s, L, G, scale, ff.step_base, (int64_t)ff.k_local, ff.headsq);
    GS_LAUNCH_CHECK("k_head_sq");
    return GS_OK;
}

// global mode, unfused chain: the KL early stop on the exchanged approx_kl of the whole minibatch
// (sticky, agents/base_agent.py:330-366): the tripping minibatch keeps its loss record with
// KL_STOP = SKIPPED = 1 and takes no optimizer step on any rank
__global__ void k_kl_decide(const float *__restrict__ kl, float target_kl, int32_t *__restrict__ stop,
                            float *__restrict__ metrics, const int64_t *__restrict__ step_base)
{
    if (threadIdx.x != 0 || (stop && *stop)) return;
    float *m = metrics + (step_base ? *step_base : 0) * GS_NUM_METRICS;
    m[GS_M_APPROX_KL] = kl[0];
    if (target_kl > 0.0f && kl[0] > target_kl) {
        if (stop) *stop = 1;
        m[GS_M_KL_STOP] = 1.0f;
        m[GS_M_SKIPPED] = 1.0f;
    }
}

int launch_kl_decide(const float *kl, float target_kl, int32_t *stop, float *metrics, const int64_t *step_base,
                     hipStream_t s)
{
    hipLaunchKernelGGL(k_kl_decide, dim3(1), dim3(64), 0, s, kl, target_kl, stop, metrics, step_base);
    GS_LAUNCH_CHECK("k_kl_decide");
    return GS_OK;
}

bool has_fused(const Layout &L, int64_t B)
{
    bool ok = false;
    with_shape(L, B, [&](auto sh) {
        using Sh = decltype(sh);
        ok = Sh::AEX > 0 && Sh::batch(0) > 0 && B % kTile == 0 && B <= 1024;
        return GS_OK;
    });
    return ok;
}

// the lagged optimizer step needs the compile-time W1|b1 / W2-tile register layout
template <class Sh>
constexpr bool lagged_shape()
{
    if constexpr (Sh::AEX == 0 || Sh::H1c == 0 || Sh::Bc == 0) {
        return false;
    } else {
        constexpr Layout Lc = Sh::lay(Layout{});
        constexpr int n1 = Lc.H1 * (Lc.D + 1);
        return (kTile * Lc.H1 / 4) % kFwdAdamThreads == 0 && Lc.H1 % 4 == 0 && (Lc.H1 * Lc.D) % 4 == 0 &&
               (Sh::Bc + Sh::RB - 1) / Sh::RB <= 8 && (n1 / 4 + 255) / 256 <= 2 && n1 <= kTile * (Lc.H1 + 4);
    }
}

bool has_lagged(const Layout &L, int64_t B)
{
    bool ok = false;
    with_shape(L, B, [&](auto sh) {
        ok = lagged_shape<decltype(sh)>() && n_sumsq_slots(L) <= 512;
        return GS_OK;
    });
    return ok && has_fused(L, B);
}

int launch_fwd_fused(const float *params, const Layout &L, int64_t B, const FusedFwd &ff, const LossArgs &la,
                     const Workspace &ws, const int32_t *stop, hipStream_t s, const AdamFwd *af)
{
    const dim3 grid((unsigned)((L.H2 + kTile - 1) / kTile), (unsigned)((B + kTile - 1) / kTile));
    // GS_HP_ACT_STATS (ff.act): the STATS instantiations, whose epilogue records the activation
    // statistics (compile-time shapes with D <= 8 and at most one h1 chunk per column block)
    GS_REQUIRE(!ff.act || (L.D <= 8 && L.H1 <= L.H2), "activation statistics in the fused forward: D <= 8, H1 <= H2");
    return with_shape(L, B, [&](auto sh) {
        using Sh = decltype(sh);
        auto go = [&](auto stats) -> int {
            constexpr bool ST = decltype(stats)::value && (Sh::H1c > 0);
            const float *no_obs = nullptr;
            const int32_t *no_idx = nullptr;
            float *no_copy = nullptr;
            if (la.bf16) {      // the bf16 mode (GS_HP_BF16)
                if constexpr (bf16_shape<Sh>() && lagged_shape<Sh>()) {
                    using Sb = Bf16Shape<Sh>;
                    if (af) {
                        GS_REQUIRE((af->part1 ? af->aa.nrb > 0 : af->aa.nrb == 0) && af->aa.n_slots <= 512,
                                   "lagged Adam: bad slot / partial counts");
                        hipLaunchKernelGGL((k_fwd_hidden<Sb, true, true, ST>), grid, dim3(kFwdAdamThreads),
                                           fwd_lds_bytes(L), s, params, L, no_obs, no_idx, 0, 0, (int)B, ws.x, ws.h1,
                                           ws.h2, ws.zpart, no_copy, stop, RowGather{}, ff, la, ws.h2mask, *af);
                    } else {
                        hipLaunchKernelGGL((k_fwd_hidden<Sb, true, false, ST>), grid, dim3(256), fwd_lds_bytes(L), s,
                                           params, L, no_obs, no_idx, 0, 0, (int)B, ws.x, ws.h1, ws.h2, ws.zpart,
                                           no_copy, stop, RowGather{}, ff, la, ws.h2mask, AdamFwd{});
                    }
                    GS_LAUNCH_CHECK("k_fwd_hidden<fused, bf16>");
                    return GS_OK;
                } else {
                    GS_REQUIRE(false, "precision bf16: no bf16 instantiation of the MLP chain for this shape");
                }
            }
            if (af) {   // forward carrying the previous minibatch's clip + Adam (dW1|db1 partials)
                if constexpr (lagged_shape<Sh>()) {
                    GS_REQUIRE((af->part1 ? af->aa.nrb > 0 : af->aa.nrb == 0) && af->aa.n_slots <= 512,
                               "lagged Adam: bad slot / partial counts");
                    hipLaunchKernelGGL((k_fwd_hidden<Sh, true, true, ST>), grid, dim3(kFwdAdamThreads),
                                       fwd_lds_bytes(L), s, params, L, no_obs, no_idx, 0, 0, (int)B, ws.x, ws.h1,
                                       ws.h2, ws.zpart, no_copy, stop, RowGather{}, ff, la, ws.h2mask, *af);
                    GS_LAUNCH_CHECK("k_fwd_hidden<fused, adam>");
                    return GS_OK;
                } else {
                    GS_REQUIRE(false, "lagged Adam: no compile-time instantiation for this shape");
                }
            }
            hipLaunchKernelGGL((k_fwd_hidden<Sh, true, false, ST>), grid, dim3(256), fwd_lds_bytes(L), s, params, L,
                               no_obs, no_idx, 0, 0, (int)B, ws.x, ws.h1, ws.h2, ws.zpart, no_copy, stop, RowGather{},
                               ff, la, ws.h2mask, AdamFwd{});
            GS_LAUNCH_CHECK("k_fwd_hidden<fused>");
            return GS_OK;
        };
        return ff.act ? go(std::true_type{}) : go(std::false_type{});
    });
}

// ---- GS_HP_ACT_STATS on the fused chain: one workgroup per minibatch step turns its forward
// workgroups' records (FusedFwd::act) into the record's GS_M_ACT slots: per layer the per-neuron
// dead counts summed over the row blocks (fraction of the B rows; dead_pct their mean, dead_max
// their max), and mean / unbiased std of z over B x H from the float partial sums (double).
__global__ __launch_bounds__(256) void k_act_stats_fused(const uint32_t *__restrict__ act, int nrb, int ncb, int H1,
                                                         int H2, int B, float *__restrict__ metrics)
{
    __shared__ double sred[4 * (256 + 16)];
    __shared__ unsigned smax[2];
    const int64_t k = blockIdx.x;
    const int tid = threadIdx.x;
    const uint32_t *a = act + k * (int64_t)nrb * ncb * kActRec;
    if (tid < 2) smax[tid] = 0u;
    __syncthreads();
    double dsum[2] = {0.0, 0.0};            // per layer: the neurons' dead counts summed
#pragma unroll
    for (int l = 0; l < 2; ++l) {
        const int H = l == 0 ? H1 : H2;
        unsigned mx = 0u;
        for (int j = tid; j < H; j += 256) {
            const int cb = j / kTile, c = j % kTile;
            unsigned cnt = 0u;
            for (int rb = 0; rb < nrb; ++rb)
                cnt += (a[(rb * ncb + cb) * kActRec + 4 * l + (c >> 2)] >> (8 * (c & 3))) & 0xffu;
            dsum[l] += (double)cnt;
            mx = cnt > mx ? cnt : mx;
        }
        atomicMax(&smax[l], mx);
    }
    double zs[4] = {0.0, 0.0, 0.0, 0.0};
    for (int w = tid; w < nrb * ncb; w += 256)
#pragma unroll
        for (int q = 0; q < 4; ++q) zs[q] += (double)__uint_as_float(a[w * kActRec + 8 + q]);
    block_reduce<2>(dsum, sred);
    block_reduce<4>(zs, sred);
    if (tid == 0) {
        float *rec = metrics + k * GS_NUM_METRICS + GS_M_ACT;
#pragma unroll
        for (int l = 0; l < 2; ++l) {
            const double H = l == 0 ? H1 : H2, n = (double)B * H;
            const double s1 = zs[2 * l], s2 = zs[2 * l + 1];
            const double var = (s2 - s1 * s1 / n) / (n - 1.0);
            rec[4 * l + 0] = (float)(s1 / n);
            rec[4 * l + 1] = (float)sqrt(var > 0.0 ? var : 0.0);
            rec[4 * l + 2] = (float)(dsum[l] / n);
            rec[4 * l + 3] = (float)((double)smax[l] / (double)B);
        }
    }
}

int launch_act_stats_fused(const Layout &L, int64_t B, int64_t n, const uint32_t *act, float *metrics, hipStream_t s)
{
    const int nrb = (int)(B / kTile), ncb = (L.H2 + kTile - 1) / kTile;
    hipLaunchKernelGGL(k_act_stats_fused, dim3((unsigned)n), dim3(256), 0, s, act, nrb, ncb, L.H1, L.H2, (int)B,
                       metrics);
    GS_LAUNCH_CHECK("k_act_stats_fused");
    return GS_OK;
}

int launch_gather_all(const Layout &L, int64_t B, int64_t n, const int32_t *idx, const float *obs,
                      const int64_t *actions, const float *logprobs, const float *values, const float *advantages,
                      const float *returns, int64_t T, int64_t N, int normalize, const FusedFwd &ff, float *metrics,
                      hipStream_t s, const float *adv_stats)
{
    return with_shape(L, B, [&](auto sh) {
        hipLaunchKernelGGL(k_gather_all<decltype(sh)>, dim3((unsigned)n), dim3(256), 0, s, idx, (int)B, obs, actions,
                           logprobs, values, advantages, returns, (int)T, (int)N, L.D, normalize, ff, metrics,
                           adv_stats);
        GS_LAUNCH_CHECK("k_gather_all");
        return GS_OK;
    });
}

int launch_metrics_all(const Layout &L, int64_t B, int64_t n, const FusedFwd &ff, const LossArgs &la, float *metrics,
                       hipStream_t s)
{
    hipLaunchKernelGGL(k_metrics_all, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, ff.mpart,
                       (int)(B / kTile), n, (int)B, la, metrics, ff.normsq ? ff.headsq : nullptr,
                       (L.H2 + kTile - 1) / kTile + 1, ff.normsq);
    GS_LAUNCH_CHECK("k_metrics_all");
    return GS_OK;
}

int launch_reduce_part1(const float *part1, const Layout &L, int nrb, float *G, const int32_t *stop, hipStream_t s)
{
    hipLaunchKernelGGL(k_reduce_part1, dim3((unsigned)((L.oW2 + 255) / 256)), dim3(256), 0, s, part1, L, nrb, G,
                       stop);
    GS_LAUNCH_CHECK("k_reduce_part1");
    return GS_OK;
}

int launch_sumsq_flat(const float *G, int64_t n, float *out, int nblocks, hipStream_t s)
{
    hipLaunchKernelGGL(k_sumsq_flat, dim3((unsigned)nblocks), dim3(256), 0, s, G, n, out);
    GS_LAUNCH_CHECK("k_sumsq_flat");
    return GS_OK;
}

#ifdef GS_STAMPS
extern "C" int gs_debug_stamps(unsigned long long *acc_out, unsigned long long *cnt_out)
{
    GS_HIP(hipMemcpyFromSymbol(acc_out, HIP_SYMBOL(g_stamp_acc), sizeof(unsigned long long) * 128));
    GS_HIP(hipMemcpyFromSymbol(cnt_out, HIP_SYMBOL(g_stamp_cnt), sizeof(unsigned long long) * 8));
    return GS_OK;
}

#endif

#if defined(GS_STAMPS) || defined(GS_SPANS)
// chain timeline: zero / read the 2 x kSpanK x kSpanWG x 9 words
extern "C" int gs_debug_span_reset()
{
    void *p = nullptr;
    GS_HIP(hipGetSymbolAddress(&p, HIP_SYMBOL(g_span)));
    GS_HIP(hipMemset(p, 0, sizeof(unsigned) * 2 * kSpanK * kSpanWG * 9));
    GS_HIP(hipDeviceSynchronize());
    return GS_OK;
}
extern "C" int gs_debug_span_read(unsigned *out)
{
    GS_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_span), sizeof(unsigned) * 2 * kSpanK * kSpanWG * 9));
    return GS_OK;
}
#endif

}  // namespace gs
