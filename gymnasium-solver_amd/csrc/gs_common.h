// Shared declarations for the libgsamd kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string>
#include <type_traits>

#include "../../include/gsamd.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

namespace gs {

// ---- diagnostic phase stamps (only in a -DGS_STAMPS build; never in the product library)
#ifdef GS_STAMPS
extern __device__ unsigned long long g_stamp_acc[8][16];
extern __device__ unsigned long long g_stamp_cnt[8];
// timestamps stay in registers; the global atomics happen once, at GS_STAMP_END, so the
// stamps never add a memory wait to a phase they measure
#define GS_STAMP_BEGIN_IF(k, cond)                                                 \
    unsigned long long _st_t[17];                                                  \
    int _st_n = 0;                                                                 \
    const bool _st_on = (cond) && threadIdx.x == 0;                                \
    const int _st_k = (k);                                                         \
    if (_st_on) _st_t[0] = __builtin_amdgcn_s_memtime();
#define GS_STAMP_BEGIN(k) GS_STAMP_BEGIN_IF(k, blockIdx.x == 0 && blockIdx.y == 0)
#define GS_STAMP(i)                                                                \
    if (_st_on) _st_t[(i) + 1] = __builtin_amdgcn_s_memtime();                     \
    _st_n = (i) + 1;
#define GS_STAMP_END(i)                                                            \
    GS_STAMP(i)                                                                    \
    if (_st_on) {                                                                  \
        for (int _j = 0; _j < _st_n; ++_j)                                         \
            atomicAdd(&g_stamp_acc[_st_k][_j], _st_t[_j + 1] - _st_t[_j]);         \
        atomicAdd(&g_stamp_cnt[_st_k], 1ull);                                      \
    }
#else
#define GS_STAMP_BEGIN(k)
#define GS_STAMP_BEGIN_IF(k, cond)
#define GS_STAMP(i)
#define GS_STAMP_END(i)
#endif

// ---- error plumbing (thread-local last error, like cudaGetLastError but with text)
void set_error(const char *fmt, ...);
int hip_fail(hipError_t e, const char *what, const char *file, int line);

#define GS_HIP(call)                                                         \
    do {                                                                     \
        hipError_t _e = (call);                                              \
        if (_e != hipSuccess) return gs::hip_fail(_e, #call, __FILE__, __LINE__); \
    } while (0)

#define GS_REQUIRE(cond, ...)                    \
    do {                                         \
        if (!(cond)) {                           \
            gs::set_error(__VA_ARGS__);          \
            return GS_E_INVALID;                 \
        }                                        \
    } while (0)

#define GS_LAUNCH_CHECK(name)                                                        \
    do {                                                                             \
        hipError_t _e = hipGetLastError();                                           \
        if (_e != hipSuccess) return gs::hip_fail(_e, "launch " name, __FILE__, __LINE__); \
    } while (0)

// ---- flat parameter layout, reference state_dict order (utils/models.py:285-326)
struct Layout {
    int D, H1, H2, A;
    int64_t oW1, ob1, oW2, ob2, oWp, obp, oWv, obv, P;
    __host__ __device__ static constexpr Layout make(int D, int H1, int H2, int A) {
        Layout L{};
        L.D = D; L.H1 = H1; L.H2 = H2; L.A = A;
        L.oW1 = 0;
        L.ob1 = L.oW1 + (int64_t)H1 * D;
        L.oW2 = L.ob1 + H1;
        L.ob2 = L.oW2 + (int64_t)H2 * H1;
        L.oWp = L.ob2 + H2;
        L.obp = L.oWp + (int64_t)A * H2;
        L.oWv = L.obp + A;
        L.obv = L.oWv + H2;
        L.P = L.obv + 1;
        return L;
    }
    // head row a in [0, A]: a < A -> policy_head.weight[a], a == A -> value_head.weight
    __host__ __device__ constexpr int64_t head_row(int a) const { return a < A ? oWp + (int64_t)a * H2 : oWv; }
    __host__ __device__ constexpr int64_t head_bias(int a) const { return a < A ? obp + a : obv; }
};

// W1/b1 gradient partials (part1[rb][H1][D+1], one slab per 32-row block of the minibatch)
// -> index of flat parameter p < oW2 inside one slab
__host__ __device__ __forceinline__ int64_t part1_index(const Layout &L, int64_t p)
{
    const int D1 = L.D + 1;
    if (p < L.ob1) {
        const int64_t k = p / L.D, d = p - k * L.D;
        return k * D1 + d;
    }
    return (p - L.ob1) * D1 + L.D;
}

// Kernel shape policies.  ShapeC bakes the MLP dims (and optionally the minibatch size)
// into the kernel, so every loop bound and parameter offset is a compile-time constant
// (fully unrolled, no integer division, no guard chains); the benchmarked / reference
// configs are instantiated this way.  ShapeR keeps them runtime (any other MLP shape).
template <int D_, int H1_, int H2_, int A_, int B_, int RB_ = 32>
struct ShapeC {
    static constexpr int AMAX = A_, AEX = A_, H1c = H1_, Bc = B_;
    static constexpr int RB = RB_;        // rows of a k_bwd role-B slab (one dW1|db1 partial each)
    static constexpr bool BF = false;     // bf16 MFMA operands (Bf16Shape)
    __host__ __device__ static constexpr Layout lay(const Layout &) { return Layout::make(D_, H1_, H2_, A_); }
    __host__ __device__ static constexpr int batch(int b) { return B_ > 0 ? B_ : b; }
};
template <int AMAX_>
struct ShapeR {
    static constexpr int AMAX = AMAX_, AEX = 0, H1c = 0, Bc = 0;
    static constexpr int RB = 32;
    static constexpr bool BF = false;
    __host__ __device__ static Layout lay(const Layout &L) { return L; }
    __host__ __device__ static int batch(int b) { return b; }
};

// The MLP update chain's bf16 mode (GS_HP_BF16, precision: bf16): the same compile-time shape with
// bf16 MFMA operands in the fused forward / backward (fp32 accumulation, parameters, moments,
// loss, clip and Adam)
template <class S>
struct Bf16Shape : S {
    static constexpr bool BF = true;
};

constexpr int kTile = 16;        // MFMA 16x16x4 f32 output tile

constexpr int kMaxObsDim = 64;
constexpr int kMaxHidden = 1024;
constexpr int kMaxActions = 32;

// Workspace carve-up for one minibatch step (bytes, 256-aligned), see gs_ppo.hip.
struct Workspace {
    float *x;        // (B, D)     gathered observations
    float *h1;       // (B, H1)    post-ReLU
    float *h2;       // (B, H2)    post-ReLU
    uint16_t *h2mask;  // (B, H2/16) relu'(h2) bits per 16-column block (what k_bwd reads instead of h2)
    float *zpart;    // (H2/16, B, A+1) partial head outputs
    float *dz;       // (B, A+1)   dLoss/dlogits | dLoss/dvalue
    float *part1;    // (ceil(B/64), H1, D+1) dW1|db1 partials per 64-row block
    float *sumsq;    // (n_slots)  per-tile sum of squared gradients
    float *kl4;      // (4)        global mode: the step's approx_kl share, exchanged in place
    double *act_parts;  // GS_HP_ACT_STATS on the unfused chain: k_mlp_act_stats parts of the step
    int32_t *f_act;  // (B)        gathered minibatch fields (written by k_fwd_hidden)
    float *f_olp, *f_ov, *f_adv, *f_ret;
    int n_slots;
    size_t bytes;
};
// rows per dh1 workgroup in k_bwd (2 row tiles x 2 K halves over 4 waves).  64 rows (one tile per
// wave over the whole K) halve the dW1|db1 partials the next forward folds: C2 0.08 us faster per
// minibatch, but C3 (B = 64: 8 role-B workgroups instead of 16) 9 % slower — kept at 32
// (profiles/r03_ab_chain.txt)
constexpr int kRowsB = 32;
// the role-B slab height of a shape (its S::RB; 32 for the runtime shapes): the dW1|db1 partial count
// is ceil(B / rows_b)
int rows_b(const Layout &L, int64_t B);

// Minibatch field gather done by the forward kernel (utils/rollout_collector.py:657-682).
struct RowGather {
    const int64_t *actions;
    const float *logprobs, *values, *advantages, *returns;
    int32_t *f_act;
    float *f_olp, *f_ov, *f_adv, *f_ret;
    const int64_t *step_base;   // graph chunk replay: minibatch offset read on device (null: 0)
};
Workspace carve_workspace(void *base, const Layout &L, int64_t B);

// Fused update path (gs_ppo_update): per-update gathered minibatch fields and the in-kernel
// head combine + row loss of k_fwd_hidden<S, true>.  Arrays are [k][B] over the update's
// minibatches; k = k_local + *step_base (graph chunk replay) or k_local (eager).
struct FusedFwd {
    const float *xg;           // (n, B, D) gathered observations
    const int32_t *fa;         // (n, B) actions
    const float *folp, *fov, *fadv, *fret;   // (n, B) old logp, old value, normalised adv, return
    double *mpart;             // (n, B/16, 14) per-row-block metric sums
    float *headsq;             // (n, H2/16 + 1, 2) per role-C workgroup {policy, value} head-gradient
                               // sums of squares (k_metrics_all: per-component gradient norms)
    double *normsq;            // (n) the steps' squared total norms (AdamArgs::normsq)
    float *dz;                 // (B, A+1) dLoss/dlogits | dLoss/dvalue of the current step
    const int64_t *step_base;
    int k_local;
    // GS_HP_ACT_STATS: (n, B/16, H2/16, 12) u32 per forward workgroup — the dead counts of its 16
    // h1 columns and its 16 h2 columns (one byte per column, 4 per word), then the float bits of
    // {sum z1, sum z1^2, sum z2, sum z2^2}; null = the forward computes no statistics
    uint32_t *act;
};
constexpr int kActRec = 12;    // u32 words of one forward workgroup's activation-statistics record

struct LossArgs {
    float clip_lo, clip_hi;     // f32(1 - clip), f32(1 + clip) (torch clamp casts scalars to f32)
    float clip_vf;              // f32(clip_range_vf)
    float vf_coef, ent_coef;
    float target_kl;            // <= 0: None
    const int64_t *step_base;   // graph chunk replay: metrics record offset (null: 0)
    int normalize;
    float inv_batch;            // f32(1 / batch_rows): the gradient of the loss's mean
    int batch_rows;             // rows of the minibatch the loss averages over (global mode: all ranks')
    // global mode (gs_ppo_update_global): rows whose action is < 0 are another rank's (padding:
    // no loss, no gradient); the step's advantage statistics come from all ranks; this rank's raw
    // loss sums are exported for the host to combine; the KL stop is decided on the global value
    const float *adv_stats;     // per minibatch {mean, std} (f32) of the global minibatch's advantages
    double *sums_out;           // per minibatch kNumSums raw loss sums of this rank's rows
    float *kl_part;             // unfused chain: this rank's share of approx_kl (the exchange sums it)
    int bf16;                   // GS_HP_BF16: the fused MLP chain's MFMA operands in bf16
};

struct AdamArgs {
    float max_norm;         // <= 0: no clip
    float one_minus_b1;     // lerp weight f32(1 - beta1)
    float b2;               // f32(beta2)
    float one_minus_b2;     // f32(1 - beta2)
    float neg_step_size;    // f32(-lr / (1 - beta1^t))
    float bc2_sqrt;         // f32(sqrt(1 - beta2^t))
    float inv_bc2_sqrt;     // f32(1 / sqrt(1 - beta2^t)) (MLP chain: a multiply instead of a division)
    float eps;
    float grad_scale;       // 1/world for all-reduced sums, else 1
    int n_slots;
    int nrb;                // dW1/db1 partial row blocks (0: grads already final in G)
    const float *sched;     // optional device table {neg_step_size, inv_bc2_sqrt} per step (graph replay)
    int sched_idx;
    const int64_t *step_base;   // graph chunk replay: added to sched_idx and the metrics record
    int stage_lds;          // set by the launcher: stage slots + partials through LDS
    // fused update: the step's squared pre-clip norm x grad_scale^2 in double, for k_metrics_all's
    // per-component norms.  Lagged forward: the update's array (indexed by the applied step);
    // k_clip_adam: offset to its step like its metrics record (+ *step_base in a replay)
    double *normsq;
};

// Lagged optimizer step of the single-GPU fused chain (gs_ppo_update): the forward of
// minibatch k first applies minibatch k-1's clip + Adam step to the parameters it reads
// (k_fwd_hidden<S, true, true>); the row-block-0 workgroups write the results into the other
// parameter set, which the backward of k then reads.
struct AdamFwd {
    const float *Min, *Vin;            // moments of the set the kernel's P belongs to
    const float *G, *part1, *sumsq;    // step k-1's head/W2 grads, dW1|db1 partials, per-tile sums
    float *Pout, *Mout, *Vout;         // the other set
    float *metrics;                    // the update's records (GS_M_GRAD_NORM of step k-1)
    AdamArgs aa;                       // step k-1's schedule: aa.sched[2(k-1)] when set, else the scalars
    int force;                         // apply at k = 0 too (gs_ppo_stage timing)
};

// Gradient exchange inside k_bwd (multi-GPU MLP chain over xGMI, gs_xgmi_dev.h): every
// backward workgroup pushes its output values into its peers' exchange regions, waits for theirs
// and keeps the rank-ordered mean, so the update's gradient leaves the backward already
// exchanged (no exchange launch).  world <= 1: no exchange (the single-GPU kernel).
constexpr int kBwdXMaxRanks = 8;       // one node
constexpr int kBwdXMaxWG = 1024;       // backward workgroups with a flag / data slot
constexpr int kBwdXSlot = 1024;        // floats per workgroup slot (4 per thread)
struct BwdXchg {
    char *peer[kBwdXMaxRanks];         // exchange region base per rank (peer[rank]: own)
    uint32_t off_flags1, off_flags2;   // [src][kBwdXMaxWG] u32 flag words (seq << 1)
    uint32_t off_data, off_res;        // data[parity][src][wg][slot], res[parity][wg][slot]
    int world, rank, rsag, region_bytes;
    float scale;                       // 1 / world
    uint64_t timeout;                  // spin limit, s_memrealtime ticks
    uint32_t *seq;                     // [kBwdXMaxWG] exchanges completed per workgroup (local)
    uint32_t *err;                     // sticky error word of the own region
};

// One-launch rollout of the synthetic env (gs_mlp.hip k_rollout_synth)
struct SynthEnvArgs {
    int32_t *state;                  // [N][4] {k, episode, len, -}
    float *ep_ret, *obs;             // [N], [N][D]: running return, current observation
    int32_t *ep_cnt;                 // [N] finished-episode counters (may be null)
    float *ep_ret_sum, *ep_len_sum;
    int L, trunc_every;
    float reward;
    uint64_t seed, step0;            // env seed, vector steps taken before this rollout
    int64_t env_offset;
};
struct RolloutRows {                 // time-major (T, N) rows of the rollout buffer
    float *obs;                      // (T, N, D)
    int64_t *actions;                // replayed from (mode 2) or written
    float *logp, *value, *reward;
    uint8_t *done, *timeout;
};

bool rollout_synth_fits(const Layout &L);
int launch_rollout_synth(const float *P, const Layout &L, int64_t N, int T, int mode, uint64_t rng_seed,
                         uint64_t counter0, const SynthEnvArgs &ev, const RolloutRows &rw, hipStream_t s);

inline int n_col_blocks(int H) { return (H + kTile - 1) / kTile; }
inline int n_sumsq_slots(const Layout &L) { return n_col_blocks(L.H2) * n_col_blocks(L.H1) + 2 * n_col_blocks(L.H2) + 1; }

// kernels' launch helpers (gs_mlp.hip)
int launch_fwd_fused(const float *params, const Layout &L, int64_t B, const FusedFwd &ff, const LossArgs &la,
                     const Workspace &ws, const int32_t *stop, hipStream_t s, const AdamFwd *af = nullptr);
bool has_lagged(const Layout &L, int64_t B);
int launch_gather_all(const Layout &L, int64_t B, int64_t n, const int32_t *idx, const float *obs,
                      const int64_t *actions, const float *logprobs, const float *values, const float *advantages,
                      const float *returns, int64_t T, int64_t N, int normalize, const FusedFwd &ff, float *metrics,
                      hipStream_t s, const float *adv_stats = nullptr);
int launch_kl_decide(const float *kl, float target_kl, int32_t *stop, float *metrics, const int64_t *step_base,
                     hipStream_t s);
int launch_metrics_all(const Layout &L, int64_t B, int64_t n, const FusedFwd &ff, const LossArgs &la, float *metrics,
                       hipStream_t s);
bool has_fused(const Layout &L, int64_t B);
bool has_bf16_chain(const Layout &L, int64_t B);     // the fused chain's bf16 instantiation exists
int launch_fwd_hidden(const float *params, const Layout &L, const float *obs, const int32_t *idx,
                      int64_t T, int64_t N, int64_t rows, float *x_out, float *h1_out, float *h2_out,
                      float *zpart, float *obs_copy, const int32_t *stop_flag, const RowGather *rg, hipStream_t s, uint16_t *h2mask = nullptr);
size_t fwd_lds_bytes(const Layout &L);
int launch_heads_act(const float *P, const Layout &L, const float *zpart, int64_t rows, int mode, uint64_t seed,
                     uint64_t counter, int64_t *actions, float *logp, float *value, hipStream_t s,
                     const uint64_t *clock = nullptr);
int launch_loss(const float *P, const Layout &L, int64_t B, const Workspace &ws, const LossArgs &la, float *metrics,
                int32_t *stop, hipStream_t s);
size_t bwd_lds_bytes(const Layout &L, int64_t B);
int prepare_kernels(const Layout &L, int64_t B);
int launch_bwd(const float *P, const Layout &L, int64_t B, const Workspace &ws, float *G, const int32_t *stop,
               hipStream_t s, const FusedFwd *ff = nullptr, const LossArgs *la = nullptr,
               const BwdXchg *bx = nullptr);
// whether k_bwd's in-kernel exchange covers this shape (grid and per-workgroup slot limits, and
// co-residency with `colocated` ranks sharing the GPU)
bool bwd_xchg_fits(const Layout &L, int64_t B, int colocated = 1);
// comp_norms: also record the step's per-component gradient norms (k_component_norms); the fused
// update leaves them to k_metrics_all (role C's per-step head sums)
int launch_clip_adam(float *P, const Layout &L, float *G, float *M, float *V, const float *part1,
                     const float *sumsq, const AdamArgs &aa, float *metrics, const int32_t *stop, hipStream_t s,
                     bool comp_norms = true);
// activation statistics parts of the MLP backbone (k_mlp_act_stats): ceil(R/16) x
// 2 * (2 + max(H1, H2)) doubles
int launch_act_stats(const float *P, const Layout &L, const float *obs, const int32_t *idx, int64_t T, int64_t N,
                     int64_t R, double *part, hipStream_t s, const int64_t *step_base = nullptr);
// GS_HP_ACT_STATS: one step's parts -> its record's GS_M_ACT slots (unfused chain; skipped after a
// KL stop), and the fused chain's per-workgroup records of n steps -> their records
int launch_act_parts_record(const Layout &L, int64_t R, const double *part, const int32_t *stop, float *metrics,
                            const int64_t *step_base, hipStream_t s);
int launch_act_stats_fused(const Layout &L, int64_t B, int64_t n, const uint32_t *act, float *metrics, hipStream_t s);
// fused update, exchange launched behind k_bwd: step ff.k_local's head record from the exchanged G
int launch_head_sq(const Layout &L, const float *G, float scale, const FusedFwd &ff, hipStream_t s);
int launch_reduce_part1(const float *part1, const Layout &L, int nrb, float *G, const int32_t *stop, hipStream_t s);
// global-minibatch mode around the update (gs_ppo_global_adv_stats / gs_ppo_global_records)
int launch_global_adv_sums(const int32_t *idx, int64_t n, int64_t B, const float *adv, int64_t T, int64_t N,
                           double *sums, hipStream_t s);
int launch_global_adv_stats(const double *sums, int64_t n, int64_t Bg, float *stats, hipStream_t s);
int launch_global_records(const double *sums, int64_t n, const LossArgs &la, float *metrics, hipStream_t s);
int launch_sumsq_flat(const float *G, int64_t n, float *out, int nblocks, hipStream_t s);

// ---- bf16 MFMA operands of the NatureCNN path (GS_HP_BF16 performance mode) ----------------
// 8 fp32 values -> one bf16 fragment of v_mfma_f32_16x16x32_bf16 / 32x32x16_bf16 (round to
// nearest even: v_cvt_pk_bf16_f32); accumulation stays fp32
__device__ __forceinline__ bf16x8 bf16_frag(float4 lo, float4 hi)
{
    bf16x8 r;
    r[0] = (__bf16)lo.x, r[1] = (__bf16)lo.y, r[2] = (__bf16)lo.z, r[3] = (__bf16)lo.w;
    r[4] = (__bf16)hi.x, r[5] = (__bf16)hi.y, r[6] = (__bf16)hi.z, r[7] = (__bf16)hi.w;
    return r;
}
__device__ __forceinline__ bf16x8 bf16_frag(const float (&v)[8])
{
    bf16x8 r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (__bf16)v[j];
    return r;
}
// 16x16 tile, K = 32: lane l holds A[l & 15][8 (l >> 4) + j] and B[8 (l >> 4) + j][l & 15];
// C/D as the fp32 16x16x4 form (col = l & 15, row = 4 (l >> 4) + reg)
__device__ __forceinline__ f32x4 mfma16_bf16(bf16x8 a, bf16x8 b, f32x4 c)
{
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// ---- bf16 activation storage (GS_HP_BF16 updates on the NatureCNN trunk's LDS kernels) -------
// The trunk's ReLU outputs a1 / a2 / a3 are only ever read as bf16 MFMA operands (rounded to
// nearest even at every read) and as ReLU masks (their sign), so in the bf16 mode the forward
// stores them rounded once: the same operand bits at half the bytes.  A positive value whose
// rounding would be zero (below 2^-134) is stored as the smallest subnormal so the mask keeps
// its sign.
__device__ __forceinline__ uint16_t act_bf16(float v)
{
    const uint16_t u = __builtin_bit_cast(uint16_t, (__bf16)v);
    return (v > 0.f && u == 0) ? (uint16_t)1 : u;
}
__device__ __forceinline__ float bf16_f32(uint16_t u) { return __uint_as_float((uint32_t)u << 16); }
// 4 stored bf16 (8 bytes, element 0 in the low half) -> 4 fp32, exactly
__device__ __forceinline__ float4 bf16x4_f32(uint2 u)
{
    return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                       __uint_as_float(u.y & 0xffff0000u));
}
// the activation type of a trunk kernel: fp32, or bf16 storage (XH)
template <bool XH>
using act_t = typename std::conditional<XH, uint16_t, float>::type;
template <bool XH>
__device__ __forceinline__ float act_ld(const act_t<XH> *p, int64_t i)
{
    if constexpr (XH) return bf16_f32(p[i]);
    else return p[i];
}
template <bool XH>
__device__ __forceinline__ float4 act_ld4(const act_t<XH> *p, int64_t i)
{
    if constexpr (XH) return bf16x4_f32(*reinterpret_cast<const uint2 *>(p + i));
    else return *reinterpret_cast<const float4 *>(p + i);
}
template <bool XH>
__device__ __forceinline__ void act_st(act_t<XH> *p, int64_t i, float v)
{
    if constexpr (XH) p[i] = act_bf16(v);
    else p[i] = v;
}

// GS_HP_ACT_STATS in the NatureCNN forward epilogues (the reference's forward hooks on cnn.0 / cnn.2
// / cnn.4 / mlp.0, utils/models.py:121-147): per neuron of the layer (a sample's output index) the
// count of pre-activation values |z| < 1e-6 — integer atomics, so the counts do not depend on the
// order — and per wave {sum z, sum z^2} (float) in slot [workgroup * 4 + wave], added in slot
// order by the step's reducer (k_cnn_act_record), which also zeroes the counts it read.
struct ActOut {
    uint32_t *cnt;
    float *part;
};
__device__ __forceinline__ void act_acc(const ActOut &ao, float z, int64_t neuron, float &s, float &q)
{
    s += z;
    q += z * z;
    if (fabsf(z) < 1e-6f) atomicAdd(ao.cnt + neuron, 1u);
}
// every lane of the wave calls it (the xor tree needs the whole wave); lane 0 writes the slot
__device__ __forceinline__ void act_flush(const ActOut &ao, int64_t slot, float s, float q)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        s += __shfl_xor(s, o, 64);
        q += __shfl_xor(q, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        ao.part[2 * slot] = s;
        ao.part[2 * slot + 1] = q;
    }
}

}  // namespace gs
