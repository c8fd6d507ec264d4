// Host orchestration of the device PPO path: policy act (rollout step), minibatch
// step (4 launches), the per-rollout update loop and its hipGraph.
//
// Replaces the host loop of the reference:
//   for batch in DataLoader(IndexDataset, sampler=MultiPassRandomSampler, collate):   dataloaders.py:63-77
//       BaseAgent.training_step -> losses_for_batch -> _backpropagate_and_step      base_agent.py:330-366,591-621
// Here the whole loop is enqueued from C++ on one stream (no per-minibatch host sync,
// no .item() calls: metrics stay on device, one record per minibatch).
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "gs_comm_internal.h"

namespace gs {

static size_t align256(size_t b) { return (b + 255) & ~size_t(255); }

Workspace carve_workspace(void *base, const Layout &L, int64_t B)
{
    Workspace w{};
    char *p = (char *)base;
    size_t off = 0;
    auto take = [&](size_t nfloats) {
        float *r = p ? (float *)(p + off) : nullptr;
        off += align256(nfloats * sizeof(float));
        return r;
    };
    const int A1 = L.A + 1;
    const int64_t nrb = (B + rows_b(L, B) - 1) / rows_b(L, B);
    w.x = take((size_t)B * L.D);
    w.h1 = take((size_t)B * L.H1);
    w.h2 = take((size_t)B * L.H2);
    w.h2mask = (uint16_t *)take(((size_t)B * n_col_blocks(L.H2) + 1) / 2);
    w.zpart = take((size_t)n_col_blocks(L.H2) * B * A1);
    w.dz = take((size_t)B * A1);
    w.part1 = take((size_t)nrb * L.H1 * (L.D + 1));
    w.f_act = (int32_t *)take((size_t)B);
    w.f_olp = take((size_t)B);
    w.f_ov = take((size_t)B);
    w.f_adv = take((size_t)B);
    w.f_ret = take((size_t)B);
    w.n_slots = n_sumsq_slots(L);
    const int comm_slots = kXgmiMaxWG;   // the xGMI exchange writes one partial per workgroup
    w.sumsq = take((size_t)(w.n_slots > comm_slots ? w.n_slots : comm_slots));
    w.kl4 = take(4);
    // k_mlp_act_stats parts of one step: ceil(B/16) x 2 (2 + max(H1, H2)) doubles
    w.act_parts = (double *)take((size_t)((B + kTile - 1) / kTile) * 4 * (2 + (L.H1 > L.H2 ? L.H1 : L.H2)));
    w.bytes = off;
    return w;
}

static int check_dims(const gs_mlp_dims &d)
{
    GS_REQUIRE(d.obs_dim > 0 && d.obs_dim <= kMaxObsDim, "obs_dim %d outside [1, %d]", d.obs_dim, kMaxObsDim);
    GS_REQUIRE(d.hidden1 > 0 && d.hidden1 % kTile == 0 && d.hidden1 <= kMaxHidden,
               "hidden1 %d must be a positive multiple of 16 <= %d", d.hidden1, kMaxHidden);
    GS_REQUIRE(d.hidden2 > 0 && d.hidden2 % kTile == 0 && d.hidden2 <= kMaxHidden,
               "hidden2 %d must be a positive multiple of 16 <= %d", d.hidden2, kMaxHidden);
    GS_REQUIRE(d.n_actions > 0 && d.n_actions <= kMaxActions, "n_actions %d outside [1, %d]", d.n_actions,
               kMaxActions);
    return GS_OK;
}

static Layout layout_of(const gs_mlp_dims &d) { return Layout::make(d.obs_dim, d.hidden1, d.hidden2, d.n_actions); }

static RowGather gather_of(const gs_rollout_view &ro, const Workspace &ws)
{
    RowGather g{};
    g.actions = ro.actions;
    g.logprobs = ro.logprobs;
    g.values = ro.values;
    g.advantages = ro.advantages;
    g.returns = ro.returns;
    g.f_act = ws.f_act;
    g.f_olp = ws.f_olp;
    g.f_ov = ws.f_ov;
    g.f_adv = ws.f_adv;
    g.f_ret = ws.f_ret;
    return g;
}

}  // namespace gs

using namespace gs;

extern "C" int64_t gs_mlp_param_count(gs_mlp_dims dims) { return layout_of(dims).P; }

extern "C" size_t gs_policy_scratch_bytes(gs_mlp_dims dims, int64_t N)
{
    const Layout L = layout_of(dims);
    return align256((size_t)n_col_blocks(L.H2) * N * (L.A + 1) * sizeof(float));
}

extern "C" int gs_policy_act(const float *params, gs_mlp_dims dims, const float *obs, int64_t N, int mode,
                             uint64_t rng_seed, uint64_t rng_counter, int64_t *actions, float *logp, float *value,
                             float *obs_store, void *scratch, const uint64_t *clock, void *stream)
{
    int rc = check_dims(dims);
    if (rc) return rc;
    GS_REQUIRE(N > 0, "gs_policy_act: N must be > 0");
    GS_REQUIRE(mode >= 0 && mode <= 2, "gs_policy_act: mode %d not in {0,1,2}", mode);
    GS_REQUIRE(params && obs && actions && logp && value && scratch, "gs_policy_act: null buffer");
    GS_REQUIRE(((uintptr_t)scratch & 15) == 0, "gs_policy_act: scratch must be 16-byte aligned");
    const Layout L = layout_of(dims);
    hipStream_t s = (hipStream_t)stream;
    float *zpart = (float *)scratch;
    rc = launch_fwd_hidden(params, L, obs, nullptr, 1, N, N, nullptr, nullptr, nullptr, zpart, obs_store, nullptr,
                           nullptr, s);
    if (rc) return rc;
    return launch_heads_act(params, L, zpart, N, mode, rng_seed, rng_counter, actions, logp, value, s, clock);
}

extern "C" int gs_rollout_synth_supported(gs_mlp_dims dims, int *supported)
{
    GS_REQUIRE(supported, "gs_rollout_synth_supported: null output");
    int rc = check_dims(dims);
    if (rc) return rc;
    *supported = rollout_synth_fits(layout_of(dims)) ? 1 : 0;
    return GS_OK;
}

extern "C" int gs_rollout_synth(const float *params, gs_mlp_dims dims, int64_t N, int64_t T, int mode,
                                uint64_t rng_seed, uint64_t rng_counter0, int32_t *env_state, float *env_ep_ret,
                                float *env_obs, int32_t episode_len, int32_t truncate_every, float reward,
                                uint64_t env_seed, int64_t env_offset, uint64_t env_step0, int32_t *ep_done_count,
                                float *ep_ret_sum, float *ep_len_sum, float *obs_rows, int64_t *action_rows,
                                float *logp_rows, float *value_rows, float *reward_rows, uint8_t *done_rows,
                                uint8_t *timeout_rows, void *stream)
{
    int rc = check_dims(dims);
    if (rc) return rc;
    GS_REQUIRE(N > 0 && T >= 0 && T < (int64_t)1 << 31, "gs_rollout_synth: bad N / T");
    GS_REQUIRE(mode >= 0 && mode <= 2, "gs_rollout_synth: mode %d not in {0,1,2}", mode);
    GS_REQUIRE(episode_len > 0, "gs_rollout_synth: episode_len must be > 0");
    GS_REQUIRE(params && env_state && env_ep_ret && env_obs && obs_rows && action_rows && logp_rows && value_rows &&
                   reward_rows && done_rows && timeout_rows,
               "gs_rollout_synth: null buffer");
    if (T == 0) return GS_OK;
    SynthEnvArgs ev{env_state, env_ep_ret, env_obs, ep_done_count, ep_ret_sum, ep_len_sum, episode_len,
                    truncate_every, reward, env_seed, env_step0, env_offset};
    RolloutRows rw{obs_rows, action_rows, logp_rows, value_rows, reward_rows, done_rows, timeout_rows};
    return launch_rollout_synth(params, layout_of(dims), N, (int)T, mode, rng_seed, rng_counter0, ev, rw,
                                (hipStream_t)stream);
}

extern "C" int gs_policy_value(const float *params, gs_mlp_dims dims, const float *obs, int64_t N, float *value,
                               void *scratch, void *stream)
{
    int rc = check_dims(dims);
    if (rc) return rc;
    GS_REQUIRE(N > 0 && params && obs && value && scratch, "gs_policy_value: bad argument");
    GS_REQUIRE(((uintptr_t)scratch & 15) == 0, "gs_policy_value: scratch must be 16-byte aligned");
    const Layout L = layout_of(dims);
    hipStream_t s = (hipStream_t)stream;
    float *zpart = (float *)scratch;
    rc = launch_fwd_hidden(params, L, obs, nullptr, 1, N, N, nullptr, nullptr, nullptr, zpart, nullptr, nullptr,
                           nullptr, s);
    if (rc) return rc;
    return launch_heads_act(params, L, zpart, N, 0, 0, 0, nullptr, nullptr, value, s);
}

extern "C" size_t gs_ppo_workspace_bytes(gs_mlp_dims dims, int64_t batch)
{
    return carve_workspace(nullptr, layout_of(dims), batch).bytes;
}

namespace {

constexpr int64_t kChunk = 512;    // minibatch steps per captured graph (chunked replay)
// Updates of up to this many minibatch steps are captured whole, every kernel with its absolute
// step index as an argument: no kernel of the chain then starts with a dependent load of the
// replay's step base (a scalar memory round trip ahead of every operand load of k_bwd).
constexpr int64_t kWholeCapture = 16384;
constexpr int64_t kNumSumsHost = 14;   // raw loss sums per minibatch (gs_mlp.hip kNumSums)

// The fused update path's per-update arrays, after the step workspace.
struct FusedWs {
    float *xg, *folp, *fov, *fadv, *fret;
    int32_t *fa;
    double *mpart;
    float *headsq;          // (n, H2/16 + 1, 2) role C's {policy, value} head sums of squares
    double *normsq;         // (n) squared total norm per step
    float *p1, *m1, *v1;    // the lagged chain's second parameter set (params | adam_m | adam_v)
    uint32_t *act;          // GS_HP_ACT_STATS: (n, B/16, H2/16, kActRec) forward-workgroup records
    size_t bytes;       // whole update workspace (step + fused)
};

FusedWs carve_fused(void *base, const Layout &L, int64_t B, int64_t n)
{
    const size_t step = carve_workspace(nullptr, L, B).bytes;
    char *p = (char *)base;
    size_t off = step;
    auto take = [&](size_t bytes) {
        void *q = p ? (void *)(p + off) : nullptr;
        off += align256(bytes);
        return q;
    };
    FusedWs f{};
    f.xg = (float *)take(sizeof(float) * (size_t)(n * B * L.D));
    f.fa = (int32_t *)take(sizeof(int32_t) * (size_t)(n * B));
    f.folp = (float *)take(sizeof(float) * (size_t)(n * B));
    f.fov = (float *)take(sizeof(float) * (size_t)(n * B));
    f.fadv = (float *)take(sizeof(float) * (size_t)(n * B));
    f.fret = (float *)take(sizeof(float) * (size_t)(n * B));
    f.mpart = (double *)take(sizeof(double) * (size_t)(n * (B / kTile) * 14));
    f.headsq = (float *)take(sizeof(float) * (size_t)(n * ((L.H2 + kTile - 1) / kTile + 1) * 2));
    f.normsq = (double *)take(sizeof(double) * (size_t)n);
    f.p1 = (float *)take(sizeof(float) * (size_t)L.P);
    f.m1 = (float *)take(sizeof(float) * (size_t)L.P);
    f.v1 = (float *)take(sizeof(float) * (size_t)L.P);
    f.act = (uint32_t *)take(sizeof(uint32_t) * (size_t)n * (size_t)(B / kTile) * (size_t)n_col_blocks(L.H2) * kActRec);
    f.bytes = off;
    return f;
}

}  // namespace

extern "C" size_t gs_ppo_update_workspace_bytes(gs_mlp_dims dims, int64_t batch, int64_t n_minibatches)
{
    if (check_dims(dims) || batch < 1 || n_minibatches < 0) return 0;
    const Layout L = layout_of(dims);
    if (!has_fused(L, batch)) return carve_workspace(nullptr, L, batch).bytes;
    return carve_fused(nullptr, L, batch, n_minibatches).bytes;
}

namespace {

struct StepArgs {
    LossArgs la;
    AdamArgs aa;
    bool sum_exchange;      // global mode: every rank's gradient is its share of the global mean (sum, no 1/world)
    bool act_stats;         // GS_HP_ACT_STATS (not in global mode): activation statistics into the records
};

// glob != nullptr: gs_ppo_update_global's global-minibatch mode (include/gsamd.h)
StepArgs make_step_args(const gs_ppo_hparams &hp, const Layout &L, int64_t B, int64_t t,
                        const gs_ppo_global *glob = nullptr)
{
    StepArgs a{};
    a.la.batch_rows = (int)(glob ? glob->batch_global : B);
    a.la.inv_batch = 1.0f / (float)a.la.batch_rows;
    if (glob) {
        a.la.adv_stats = glob->adv_stats;
        a.la.sums_out = glob->metric_sums;
        a.sum_exchange = true;
    }
    a.la.clip_lo = (float)(1.0 - (double)hp.clip_range);
    a.la.clip_hi = (float)(1.0 + (double)hp.clip_range);
    a.la.clip_vf = hp.clip_range_vf;
    a.la.vf_coef = hp.vf_coef;
    a.la.ent_coef = hp.ent_coef;
    a.la.target_kl = hp.target_kl;
    a.la.normalize = hp.normalize_adv;
    a.la.bf16 = (hp.flags & GS_HP_BF16) ? 1 : 0;
    a.act_stats = (hp.flags & GS_HP_ACT_STATS) && !glob;
    const double b1 = hp.adam_beta1, b2 = hp.adam_beta2;
    a.aa.max_norm = hp.max_grad_norm;
    a.aa.one_minus_b1 = (float)(1.0 - b1);
    a.aa.b2 = (float)b2;
    a.aa.one_minus_b2 = (float)(1.0 - b2);
    const double bc1 = 1.0 - pow(b1, (double)t);
    const double bc2 = 1.0 - pow(b2, (double)t);
    a.aa.neg_step_size = (float)(-(double)hp.lr / bc1);
    a.aa.bc2_sqrt = (float)sqrt(bc2);
    a.aa.inv_bc2_sqrt = (float)(1.0 / sqrt(bc2));
    a.aa.eps = hp.adam_eps;
    a.aa.grad_scale = 1.0f;
    a.aa.n_slots = n_sumsq_slots(L);
    a.aa.nrb = (int)((B + rows_b(L, B) - 1) / rows_b(L, B));
    return a;
}

// multi-GPU tail of a minibatch step: fold the W1 partials into the flat gradient, sum it
// over ranks (one xGMI exchange kernel, or reduce_part1 + RCCL + sumsq), then clip/Adam on
// the mean (grad_scale 1/world) with the exchange's sum-of-squares partials.
int exchange_and_adam(float *P, float *G, float *M, float *V, const Layout &L, const StepArgs &sa, float *metrics,
                      int32_t *stop, const Workspace &ws, gs_comm *comm, hipStream_t s, const FusedFwd *ff = nullptr)
{
    int world = 1, n_slots = 0;
    int rc = comm_grad_exchange(comm, G, L.P, Part1Fold{ws.part1, sa.aa.nrb, L}, ws.sumsq, &n_slots, stop, s,
                                &world);
    if (rc) return rc;
    AdamArgs aa = sa.aa;
    aa.n_slots = n_slots;
    aa.nrb = 0;
    aa.grad_scale = sa.sum_exchange ? 1.0f : 1.0f / (float)world;
    if (ff && (rc = launch_head_sq(L, G, aa.grad_scale, *ff, s))) return rc;
    return launch_clip_adam(P, L, G, M, V, nullptr, ws.sumsq, aa, metrics, stop, s, ff == nullptr);
}

int enqueue_step(float *P, float *G, float *M, float *V, const Layout &L, const StepArgs &sa,
                 const gs_rollout_view &ro, const int32_t *idx, int64_t B, float *metrics, int32_t *stop,
                 const Workspace &ws, gs_comm *comm, hipStream_t s)
{
    RowGather rg = gather_of(ro, ws);
    rg.step_base = sa.la.step_base;
    int rc = launch_fwd_hidden(P, L, ro.obs, idx, ro.T, ro.N, B, ws.x, ws.h1, ws.h2, ws.zpart, nullptr, stop, &rg, s,
                               ws.h2mask);
    if (rc) return rc;
    // the step's activation statistics under the parameters its loss uses, before the loss kernel
    // (which may set the KL stop: the tripping minibatch is evaluated, so it keeps its statistics)
    if (sa.act_stats && ((rc = launch_act_stats(P, L, ro.obs, idx, ro.T, ro.N, B, ws.act_parts, s, sa.la.step_base)) ||
                         (rc = launch_act_parts_record(L, B, ws.act_parts, stop, metrics, sa.la.step_base, s))))
        return rc;
    rc = launch_loss(P, L, B, ws, sa.la, metrics, stop, s);
    if (rc) return rc;
    if (sa.la.kl_part) {    // global mode's KL stop: this rank's approx_kl share summed over ranks first
        int world = 1;
        if (comm && (rc = comm_allreduce_sum(comm, sa.la.kl_part, 1, s, &world))) return rc;
        rc = launch_kl_decide(sa.la.kl_part, sa.la.target_kl, stop, metrics, sa.la.step_base, s);
        if (rc) return rc;
    }
    rc = launch_bwd(P, L, B, ws, G, stop, s);
    if (rc) return rc;
    if (!comm) return launch_clip_adam(P, L, G, M, V, ws.part1, ws.sumsq, sa.aa, metrics, stop, s);
    return exchange_and_adam(P, G, M, V, L, sa, metrics, stop, ws, comm, s);
}

// The fused chains' exchange inside k_bwd (xGMI transport, shapes within its limits): the
// gradient, the W1 partials and the per-tile sums of squares leave the backward as the mean
// over ranks, and the rest of the step is the single-GPU one.  False: exchange after k_bwd.
bool bwd_exchange_of(gs_comm *comm, const Layout &L, int64_t B, BwdXchg *bx, bool sum_exchange = false)
{
    if (!(comm && xgmi_bwd_args(comm, bx) && bwd_xchg_fits(L, B, comm->colocated))) return false;
    if (sum_exchange) bx->scale = 1.0f;     // global mode: the ranks' shares add up to the mean
    return true;
}

// One minibatch step of the fused chain: k_fwd_hidden<fused> (pre-gathered x), k_bwd<fused>
// (each workgroup computes the loss rows it needs from the partial heads: no loss launch,
// no block reduction; metric sums per 16 rows), then the same clip/Adam tail as enqueue_step.
int enqueue_step_fused(float *P, float *G, float *M, float *V, const Layout &L, const StepArgs &sa, int64_t B,
                       const FusedFwd &ff, float *metrics, int32_t *stop, const Workspace &ws, gs_comm *comm,
                       hipStream_t s)
{
    BwdXchg bx;
    const bool inbwd = bwd_exchange_of(comm, L, B, &bx, sa.sum_exchange);
    int rc = launch_fwd_fused(P, L, B, ff, sa.la, ws, stop, s);
    if (rc) return rc;
    rc = launch_bwd(P, L, B, ws, G, stop, s, &ff, &sa.la, inbwd ? &bx : nullptr);
    if (rc) return rc;
    if (!comm || inbwd) return launch_clip_adam(P, L, G, M, V, ws.part1, ws.sumsq, sa.aa, metrics, stop, s, false);
    return exchange_and_adam(P, G, M, V, L, sa, metrics, stop, ws, comm, s, &ff);
}

// GS_LAGGED_ADAM=0 in the environment keeps a separate clip/Adam launch per minibatch (the
// lagged chain is bit-identical and 4 % faster on MI355X)
bool lagged_enabled()
{
    const char *e = getenv("GS_LAGGED_ADAM");
    return !(e && e[0] == '0');
}

// The lagged chain's two parameter sets: [0] the caller's params / adam_m / adam_v, [1] a
// workspace copy.
struct ParamSet {
    float *P, *M, *V;
};

// The clip + Adam arguments of a step whose gradient went through the exchange: the gradient
// is final in G (W1 partials folded), the norm comes from the exchange's partial sums, and the
// sum over ranks is scaled by 1/world inside the norm and the update.
AdamArgs exchanged_adam_args(const AdamArgs &aa_in, const gs_comm *comm, bool sum_exchange = false)
{
    AdamArgs aa = aa_in;
    aa.n_slots = comm_sumsq_slots(comm);
    aa.nrb = 0;
    aa.grad_scale = sum_exchange ? 1.0f : 1.0f / (float)comm->nranks;
    return aa;
}

// Minibatch step k with the optimizer step lagged into the next forward (bit-identical to
// enqueue_step_fused): k_fwd_hidden<fused, adam> applies step k-1 (reads set (k+1)&1, its
// row-block-0 workgroups write set k&1; nothing at k = 0), then k_bwd<fused> on set k&1.
// With an xGMI communicator k_bwd exchanges its outputs itself (bwd_exchange_of) and the chain
// is the single-GPU one; with RCCL it is fwd(+Adam of k-1) -> bwd -> exchange of k.  The update's last optimizer step is one k_clip_adam
// after the loop.
int enqueue_step_lagged(const ParamSet (&ps)[2], float *G, const Layout &L, const StepArgs &sa_prev, int64_t B,
                        const FusedFwd &ff, int64_t k, float *metrics, int32_t *stop, const Workspace &ws,
                        gs_comm *comm, hipStream_t s)
{
    const ParamSet &cur = ps[k & 1], &prev = ps[(k & 1) ^ 1];
    BwdXchg bx;
    const bool inbwd = bwd_exchange_of(comm, L, B, &bx, sa_prev.sum_exchange);
    const bool after = comm && !inbwd;     // exchange launch after the backward
    AdamFwd af{};
    af.Min = prev.M, af.Vin = prev.V, af.G = G, af.part1 = after ? nullptr : ws.part1, af.sumsq = ws.sumsq;
    af.Pout = cur.P, af.Mout = cur.M, af.Vout = cur.V;
    af.metrics = metrics;
    af.aa = after ? exchanged_adam_args(sa_prev.aa, comm, sa_prev.sum_exchange) : sa_prev.aa;
    int rc = launch_fwd_fused(prev.P, L, B, ff, sa_prev.la, ws, stop, s, &af);
    if (rc) return rc;
    rc = launch_bwd(cur.P, L, B, ws, G, stop, s, &ff, &sa_prev.la, inbwd ? &bx : nullptr);
    if (rc || !after) return rc;
    int world = 1, n_slots = 0;
    rc = comm_grad_exchange(comm, G, L.P, Part1Fold{ws.part1, sa_prev.aa.nrb, L}, ws.sumsq, &n_slots, stop, s, &world);
    if (rc) return rc;
    return launch_head_sq(L, G, exchanged_adam_args(sa_prev.aa, comm, sa_prev.sum_exchange).grad_scale, ff, s);
}

int validate_update(const gs_mlp_dims &dims, const gs_rollout_view &ro, int64_t batch, const void *ws)
{
    int rc = check_dims(dims);
    if (rc) return rc;
    GS_REQUIRE(batch >= 2 && batch <= 1024, "batch %lld outside [2, 1024]", (long long)batch);
    GS_REQUIRE(ro.T > 0 && ro.N > 0, "empty rollout");
    GS_REQUIRE(ro.obs && ro.actions && ro.logprobs && ro.values && ro.advantages && ro.returns,
               "rollout view has a null buffer");
    GS_REQUIRE(ws, "null workspace");
    const Layout L = layout_of(dims);
    GS_REQUIRE(bwd_lds_bytes(L, batch) <= 160 * 1024, "batch %lld too large for the LDS budget", (long long)batch);
    GS_REQUIRE(fwd_lds_bytes(L) <= 160 * 1024, "obs_dim x hidden1 too large for the LDS budget");
    GS_REQUIRE(ro.T * ro.N < (int64_t)1 << 31, "rollout larger than 2^31 samples");
    return GS_OK;
}

}  // namespace

extern "C" int gs_ppo_minibatch_step(float *params, float *grads, float *adam_m, float *adam_v, gs_mlp_dims dims,
                                     gs_ppo_hparams hp, gs_rollout_view ro, const int32_t *idx, int64_t batch,
                                     int64_t adam_step, float *metrics, int32_t *stop_flag, void *workspace,
                                     gs_comm *comm, void *stream)
{
    int rc = validate_update(dims, ro, batch, workspace);
    if (rc) return rc;
    GS_REQUIRE(adam_step >= 1, "adam_step is 1-based");
    GS_REQUIRE(params && grads && adam_m && adam_v && idx && metrics, "gs_ppo_minibatch_step: null buffer");
    GS_REQUIRE(!(hp.flags & GS_HP_BF16), "gs_ppo_minibatch_step: precision bf16 is a mode of the fused chain "
                                         "(gs_ppo_update) only; the single-step entries are fp32");
    const Layout L = layout_of(dims);
    const Workspace ws = carve_workspace(workspace, L, batch);
    const StepArgs sa = make_step_args(hp, L, batch, adam_step);
    return enqueue_step(params, grads, adam_m, adam_v, L, sa, ro, idx, batch, metrics, stop_flag, ws, comm,
                        (hipStream_t)stream);
}

extern "C" int gs_mlp_activation_stats(const float *params, gs_mlp_dims dims, gs_rollout_view ro, const int32_t *idx,
                                       int64_t rows, double *part, void *stream)
{
    int rc = check_dims(dims);
    if (rc) return rc;
    GS_REQUIRE(params && ro.obs && part && rows >= 1, "gs_mlp_activation_stats: null buffer or no rows");
    GS_REQUIRE(idx || rows <= ro.T * ro.N, "gs_mlp_activation_stats: more rows than the rollout holds");
    return launch_act_stats(params, layout_of(dims), ro.obs, idx, ro.T, ro.N, rows, part, (hipStream_t)stream);
}

extern "C" int gs_ppo_loss(const float *params, gs_mlp_dims dims, gs_ppo_hparams hp, gs_rollout_view ro,
                           const int32_t *idx, int64_t batch, float *metrics, void *workspace, void *stream)
{
    int rc = validate_update(dims, ro, batch, workspace);
    if (rc) return rc;
    GS_REQUIRE(params && idx && metrics, "gs_ppo_loss: null buffer");
    GS_REQUIRE(!(hp.flags & GS_HP_BF16), "gs_ppo_loss: precision bf16 is a mode of the fused chain "
                                         "(gs_ppo_update) only; the single-step entries are fp32");
    const Layout L = layout_of(dims);
    const Workspace ws = carve_workspace(workspace, L, batch);
    const StepArgs sa = make_step_args(hp, L, batch, 1);
    hipStream_t s = (hipStream_t)stream;
    const RowGather rg = gather_of(ro, ws);
    rc = launch_fwd_hidden(params, L, ro.obs, idx, ro.T, ro.N, batch, ws.x, ws.h1, ws.h2, ws.zpart, nullptr,
                           nullptr, &rg, s, ws.h2mask);
    if (rc) return rc;
    return launch_loss(params, L, batch, ws, sa.la, metrics, nullptr, s);
}

extern "C" int gs_ppo_stage(int stage, float *params, float *grads, float *adam_m, float *adam_v, gs_mlp_dims dims,
                            gs_ppo_hparams hp, gs_rollout_view ro, const int32_t *idx, int64_t batch,
                            int64_t adam_step, float *metrics, void *workspace, void *stream)
{
    int rc = validate_update(dims, ro, batch, workspace);
    if (rc) return rc;
    GS_REQUIRE(stage >= 0 && stage <= 7, "gs_ppo_stage: stage %d not in [0, 7]", stage);
    const Layout L0 = layout_of(dims);
    // bf16 is a mode of the fused chain: its stages (4..7) run the chain's bf16 kernels where the
    // shape has them; the unfused stages are fp32 and refuse it instead of running fp32 silently
    GS_REQUIRE(!(hp.flags & GS_HP_BF16) || (stage >= 4 && has_bf16_chain(L0, batch)),
               "gs_ppo_stage: precision bf16 runs only on the fused chain's stages (4..7) of a shape with a bf16 "
               "instantiation; stage %d is fp32", stage);
    const Layout L = layout_of(dims);
    const Workspace ws = carve_workspace(workspace, L, batch);
    const StepArgs sa = make_step_args(hp, L, batch, adam_step < 1 ? 1 : adam_step);
    hipStream_t s = (hipStream_t)stream;
    if (stage >= 4) {     // the fused chain's kernels on minibatch 0 of a one-minibatch update
        GS_REQUIRE(has_fused(L, batch), "gs_ppo_stage: no fused instantiation for this shape");
        const FusedWs fw = carve_fused(workspace, L, batch, 1);
        FusedFwd ff{};
        ff.xg = fw.xg, ff.fa = fw.fa, ff.folp = fw.folp, ff.fov = fw.fov, ff.fadv = fw.fadv, ff.fret = fw.fret;
        ff.mpart = fw.mpart;
        ff.headsq = fw.headsq;
        ff.dz = ws.dz;
        if (stage == 6)
            return launch_gather_all(L, batch, 1, idx, ro.obs, ro.actions, ro.logprobs, ro.values, ro.advantages,
                                     ro.returns, ro.T, ro.N, hp.normalize_adv, ff, metrics, s);
        if (stage == 4) return launch_fwd_fused(params, L, batch, ff, sa.la, ws, nullptr, s);
        if (stage == 7) {   // the lagged forward: minibatch 0 with a clip + Adam step applied first
            // (the single-GPU form: dW1|db1 folded from the partials; the multi-GPU form reads the
            // same bytes less the partials, so this is the upper of the two)
            GS_REQUIRE(lagged_enabled() && has_lagged(L, batch), "gs_ppo_stage: no lagged optimizer step here");
            AdamFwd af{};
            af.Min = adam_m, af.Vin = adam_v, af.G = grads, af.part1 = ws.part1, af.sumsq = ws.sumsq;
            af.Pout = fw.p1, af.Mout = fw.m1, af.Vout = fw.v1;
            af.metrics = metrics;
            af.aa = sa.aa;
            af.force = 1;
            return launch_fwd_fused(params, L, batch, ff, sa.la, ws, nullptr, s, &af);
        }
        return launch_bwd(params, L, batch, ws, grads, nullptr, s, &ff, &sa.la);
    }
    switch (stage) {
    case 0: {
        const RowGather rg = gather_of(ro, ws);
        return launch_fwd_hidden(params, L, ro.obs, idx, ro.T, ro.N, batch, ws.x, ws.h1, ws.h2, ws.zpart, nullptr,
                                 nullptr, &rg, s, ws.h2mask);
    }
    case 1:
        return launch_loss(params, L, batch, ws, sa.la, metrics, nullptr, s);
    case 2:
        return launch_bwd(params, L, batch, ws, grads, nullptr, s);
    default:
        return launch_clip_adam(params, L, grads, adam_m, adam_v, ws.part1, ws.sumsq, sa.aa, metrics, nullptr, s);
    }
}

namespace {

// A captured update phase: keyed by every pointer/shape baked into its nodes.
struct GraphKey {
    const void *p[14];
    int64_t n[6];
    bool operator==(const GraphKey &o) const
    {
        for (int i = 0; i < 14; ++i)
            if (p[i] != o.p[i]) return false;
        for (int i = 0; i < 6; ++i)
            if (n[i] != o.n[i]) return false;
        return true;
    }
};
struct GraphKeyHash {
    size_t operator()(const GraphKey &k) const
    {
        size_t h = 1469598103934665603ull;
        for (int i = 0; i < 14; ++i) h = (h ^ (size_t)k.p[i]) * 1099511628211ull;
        for (int i = 0; i < 6; ++i) h = (h ^ (size_t)k.n[i]) * 1099511628211ull;
        return h;
    }
};
struct GraphEntry {
    hipGraphExec_t exec;
    float *sched;      // per-step {neg_step_size, inv_bc2_sqrt}, n_minibatches entries
    int64_t *base;     // first minibatch of the replayed chunk (device scalar)
    int64_t *hbase;    // pinned host table r * chunk, the source of each replay's base copy
    float *hsched;     // pinned staging for the schedule table
    hipEvent_t sched_copied;   // the last copy out of hsched (hsched is rewritten after it)
    uint32_t hbits[12];        // the hyper-parameters baked into exec's kernel arguments (lr excluded)
};
std::mutex g_graph_mu;
std::unordered_map<GraphKey, GraphEntry, GraphKeyHash> g_graphs;
int64_t g_graph_captures = 0;

// The hyper-parameter bits a capture bakes in.  lr is left out: the graph reads the step size
// only from the per-step schedule table, which every call refreshes, so an lr schedule replays
// the same graph.  A change of any other field (a scheduled clip_range, ent_coef, ...)
// re-captures into the same entry (the old exec is destroyed: no growth over a long run).
void baked_hparam_bits(const gs_ppo_hparams &hp, uint32_t (&out)[12])
{
    gs_ppo_hparams h = hp;
    h.lr = 0.0f;
    memcpy(out, &h, sizeof(out));
}

}  // namespace

static int ppo_update(float *params, float *grads, float *adam_m, float *adam_v, gs_mlp_dims dims,
                      gs_ppo_hparams hp, gs_rollout_view ro, const int32_t *idx, int64_t batch,
                      int64_t n_minibatches, int64_t adam_step0, float *metrics, int32_t *stop_flag,
                      void *workspace, size_t workspace_bytes, gs_comm *comm, int use_graph, void *stream,
                      const gs_ppo_global *glob)
{
    int rc = validate_update(dims, ro, batch, workspace);
    if (rc) return rc;
    GS_REQUIRE(n_minibatches >= 0 && adam_step0 >= 0, "bad n_minibatches/adam_step0");
    GS_REQUIRE(params && grads && adam_m && adam_v && idx && metrics, "gs_ppo_update: null buffer");
    if (n_minibatches == 0) return GS_OK;
    const Layout L = layout_of(dims);
    const Workspace ws = carve_workspace(workspace, L, batch);
    // every StepArgs of this update (glob: the global-minibatch mode)
    auto make_step_args = [&](const gs_ppo_hparams &h, const Layout &Lx, int64_t Bx, int64_t t) {
        StepArgs a = ::make_step_args(h, Lx, Bx, t, glob);
        if (glob && h.target_kl > 0.0f) a.la.kl_part = ws.kl4;
        return a;
    };
    // the unfused chain's per-step loss reads / writes minibatch k's rows of the global-mode
    // arrays (plus *step_base on device inside a replayed chunk, like its metrics record)
    auto at_step = [](StepArgs a, int64_t k) {
        if (a.la.adv_stats) a.la.adv_stats += 2 * k;
        if (a.la.sums_out) a.la.sums_out += kNumSumsHost * k;
        return a;
    };
    hipStream_t s = (hipStream_t)stream;
    // fused chain when this shape has a compile-time instantiation, no KL early stop is
    // configured (its per-minibatch decision needs the full loss before the backward) and the
    // caller's workspace holds the per-update arrays
    const bool fused = has_fused(L, batch) && !(hp.target_kl > 0.0f) &&
                       workspace_bytes >= carve_fused(nullptr, L, batch, n_minibatches).bytes &&
                       (((uintptr_t)params | (uintptr_t)grads | (uintptr_t)adam_m | (uintptr_t)adam_v) & 15) == 0;
    // precision bf16 (GS_HP_BF16) is a mode of the fused chain only (its kernels carry the bf16
    // operand pairs): no silent fp32 fallback for a configuration the chain does not run
    GS_REQUIRE(!(hp.flags & GS_HP_BF16) || (fused && has_bf16_chain(L, batch)),
               "precision bf16: the MLP update's bf16 mode runs on the fused chain of the compile-time shapes "
               "(CartPole 4-256-256-2 / LunarLander 8-128-128-4, B %% 16 == 0, no target_kl)");
    // the fused chain has no KL early stop (target_kl unset): its kernels get no stop flag, so
    // none of them starts with a dependent load of it
    if (fused) stop_flag = nullptr;
    FusedWs fw{};
    FusedFwd ff0{};
    if (fused) {
        fw = carve_fused(workspace, L, batch, n_minibatches);
        ff0.xg = fw.xg, ff0.fa = fw.fa, ff0.folp = fw.folp, ff0.fov = fw.fov, ff0.fadv = fw.fadv, ff0.fret = fw.fret;
        ff0.mpart = fw.mpart;
        ff0.headsq = fw.headsq;
        ff0.normsq = fw.normsq;
        ff0.dz = ws.dz;
        if ((hp.flags & GS_HP_ACT_STATS) && !glob) ff0.act = fw.act;
        rc = launch_gather_all(L, batch, n_minibatches, idx, ro.obs, ro.actions, ro.logprobs, ro.values,
                               ro.advantages, ro.returns, ro.T, ro.N, hp.normalize_adv, ff0, metrics, s,
                               glob ? glob->adv_stats : nullptr);
        if (rc) return rc;
    }
    // minibatch k's clip + Adam runs inside the forward of k+1 (enqueue_step_lagged), with or
    // without a communicator; step 0's forward reads set 1, which starts as a copy of the
    // caller's parameters
    const bool lagged = fused && lagged_enabled() && has_lagged(L, batch);
    const ParamSet ps[2] = {{params, adam_m, adam_v}, {fw.p1, fw.m1, fw.v1}};
    if (lagged) GS_HIP(hipMemcpyAsync(fw.p1, params, sizeof(float) * (size_t)L.P, hipMemcpyDeviceToDevice, s));
    auto step_ff = [&](int64_t k_local, int64_t slot, const int64_t *base) {
        FusedFwd f = ff0;
        f.k_local = (int)k_local;
        f.step_base = base;
        (void)slot;
        return f;
    };
    auto lag_step = [&](int64_t k, const int64_t *base, const float *sched, hipStream_t st) {
        StepArgs sp = make_step_args(hp, L, batch, adam_step0 + k > 0 ? adam_step0 + k : 1);   // step k-1's
        sp.aa.sched = sched;
        sp.aa.normsq = fw.normsq;      // the lagged forward indexes it by the applied step
        return enqueue_step_lagged(ps, grads, L, sp, batch, step_ff(k, k, base), k, metrics, stop_flag, ws, comm, st);
    };
    // the fused (non-lagged) chain's k_clip_adam of step k: its squared norm beside its record
    auto with_norm = [&](StepArgs a, int64_t k) {
        a.aa.normsq = fw.normsq ? fw.normsq + k : nullptr;
        return a;
    };
    auto finish = [&]() -> int {
        if (!fused) return GS_OK;
        if (lagged) {   // the update's last optimizer step, and its result back into the caller's set
            const int64_t k = n_minibatches - 1;
            const ParamSet &q = ps[k & 1];
            StepArgs sl = make_step_args(hp, L, batch, adam_step0 + k + 1);
            sl.aa.normsq = fw.normsq + k;
            BwdXchg bx;
            const bool after = comm && !bwd_exchange_of(comm, L, batch, &bx, sl.sum_exchange);
            int rc2 = after ? launch_clip_adam(q.P, L, grads, q.M, q.V, nullptr, ws.sumsq,
                                              exchanged_adam_args(sl.aa, comm, sl.sum_exchange),
                                              metrics + k * GS_NUM_METRICS,
                                              stop_flag, s, false)
                           : launch_clip_adam(q.P, L, grads, q.M, q.V, ws.part1, ws.sumsq, sl.aa,
                                              metrics + k * GS_NUM_METRICS, stop_flag, s, false);
            if (rc2) return rc2;
            if (k & 1) {
                const size_t nb = sizeof(float) * (size_t)L.P;
                GS_HIP(hipMemcpyAsync(params, q.P, nb, hipMemcpyDeviceToDevice, s));
                GS_HIP(hipMemcpyAsync(adam_m, q.M, nb, hipMemcpyDeviceToDevice, s));
                GS_HIP(hipMemcpyAsync(adam_v, q.V, nb, hipMemcpyDeviceToDevice, s));
            }
        }
        StepArgs sa = make_step_args(hp, L, batch, 1);
        const int rc3 = launch_metrics_all(L, batch, n_minibatches, ff0, sa.la, metrics, s);
        if (rc3 || !ff0.act) return rc3;
        return launch_act_stats_fused(L, batch, n_minibatches, ff0.act, metrics, s);
    };
    // Adam's bias corrections (computed in double on the host, exactly as
    // torch.optim.Adam's single-tensor path does) change every step; eager launches pass
    // them as kernel arguments, the graph reads them from a per-step device table that
    // is refreshed before each replay, so one capture serves every rollout.
    if (!use_graph) {
        for (int64_t k = 0; k < n_minibatches; ++k) {
            const StepArgs sa = make_step_args(hp, L, batch, adam_step0 + k + 1);
            rc = lagged  ? lag_step(k, nullptr, nullptr, s)
                 : fused ? enqueue_step_fused(params, grads, adam_m, adam_v, L, with_norm(sa, k), batch,
                                              step_ff(k, k, nullptr), metrics + k * GS_NUM_METRICS, stop_flag, ws,
                                              comm, s)
                         : enqueue_step(params, grads, adam_m, adam_v, L, at_step(sa, k), ro, idx + k * batch, batch,
                                        metrics + k * GS_NUM_METRICS, stop_flag, ws, comm, s);
            if (rc) return rc;
        }
        return finish();
    }
    // One graph holds a chunk of kChunk minibatch steps; it is replayed n / kChunk times
    // with the chunk's first minibatch index in a device scalar (step_base) that the
    // kernels add to their index-stream, metrics and Adam-schedule offsets.  The tail
    // (n % kChunk steps) runs eagerly.  Graph size stays bounded for C3's 327 680 steps.
    const int64_t chunk = n_minibatches <= kWholeCapture ? n_minibatches : kChunk;
    const int64_t n_full = n_minibatches / chunk;
    const bool whole = chunk == n_minibatches;      // absolute step indices, no device step base
    GraphKey key{};
    const void *ptrs[14] = {params, grads, adam_m, adam_v, ro.obs, ro.actions, ro.logprobs, ro.values,
                            ro.advantages, ro.returns, idx, metrics, glob ? glob->adv_stats : nullptr,
                            glob ? glob->metric_sums : nullptr};
    for (int i = 0; i < 14; ++i) key.p[i] = ptrs[i];
    key.n[0] = batch;
    key.n[1] = n_minibatches;
    key.n[2] = ((int64_t)dims.obs_dim << 48) ^ ((int64_t)dims.hidden1 << 32) ^ ((int64_t)dims.hidden2 << 16) ^ dims.n_actions;
    key.n[3] = (int64_t)(intptr_t)workspace;
    // the communicator's exchange placement is baked into the capture (gs_comm_xgmi_set_bwd_exchange)
    BwdXchg bx_key;
    const bool in_bwd = comm && bwd_exchange_of(comm, L, batch, &bx_key);
    key.n[4] = (int64_t)(intptr_t)stop_flag ^ ((int64_t)(intptr_t)comm << 1) ^ (fused ? 1 : 0) ^
               ((int64_t)lagged << 62) ^ ((int64_t)in_bwd << 61);
    key.n[5] = ro.T * 1000003 + ro.N + (glob ? glob->batch_global << 40 : 0);
    uint32_t hbits[12];
    baked_hparam_bits(hp, hbits);
    std::lock_guard<std::mutex> lk(g_graph_mu);
    auto it = g_graphs.find(key);
    const bool fresh = it == g_graphs.end();
    if (!fresh && memcmp(it->second.hbits, hbits, sizeof(hbits)) != 0) {
        // same buffers, new baked hyper-parameters: drop the old exec, re-capture below
        GS_HIP(hipEventSynchronize(it->second.sched_copied));
        GS_HIP(hipStreamSynchronize(s));    // the old exec may still be running on the caller's stream
        GS_HIP(hipGraphExecDestroy(it->second.exec));
        it->second.exec = nullptr;
    }
    if (fresh || it->second.exec == nullptr) {
        rc = prepare_kernels(L, batch);   // function attributes may not change inside a capture
        if (rc) return rc;
        GraphEntry ent{};
        if (fresh) {
            GS_HIP(hipMalloc(&ent.sched, sizeof(float) * 2 * (size_t)n_minibatches + 64));
            ent.base = (int64_t *)((char *)ent.sched + sizeof(float) * 2 * (size_t)n_minibatches);
            // pinned and never rewritten: an async copy may read it whenever it executes
            GS_HIP(hipHostMalloc((void **)&ent.hbase, sizeof(int64_t) * (size_t)(n_full + 1), hipHostMallocDefault));
            for (int64_t r = 0; r <= n_full; ++r) ent.hbase[r] = r * chunk;
            GS_HIP(hipHostMalloc((void **)&ent.hsched, sizeof(float) * 2 * (size_t)n_minibatches,
                                 hipHostMallocDefault));
            GS_HIP(hipEventCreateWithFlags(&ent.sched_copied, hipEventDisableTiming));
        } else {
            ent = it->second;
        }
        memcpy(ent.hbits, hbits, sizeof(hbits));
        // capture on a private stream (the caller's may be the legacy NULL stream, which
        // cannot capture); the instantiated graph is then launched on the caller's stream
        hipStream_t cs;
        GS_HIP(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
        hipGraph_t g;
        GS_HIP(hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal));
        const int64_t *base = whole ? nullptr : ent.base;
        for (int64_t k = 0; k < chunk; ++k) {
            StepArgs sa = make_step_args(hp, L, batch, 1);
            sa.aa.sched = ent.sched;
            sa.aa.sched_idx = (int)k;
            sa.aa.step_base = base;
            sa.la.step_base = base;
            if (lagged) {
                rc = lag_step(k, base, ent.sched, cs);
            } else if (fused) {
                LossArgs la_f = sa.la;
                la_f.step_base = nullptr;      // the fused fwd takes its base from FusedFwd
                StepArgs saf = sa;
                saf.la = la_f;
                rc = enqueue_step_fused(params, grads, adam_m, adam_v, L, with_norm(saf, k), batch,
                                        step_ff(k, k, base),
                                        metrics + k * GS_NUM_METRICS, stop_flag, ws, comm, cs);
            } else {
                rc = enqueue_step(params, grads, adam_m, adam_v, L, at_step(sa, k), ro, idx + k * batch, batch,
                                  metrics + k * GS_NUM_METRICS, stop_flag, ws, comm, cs);
            }
            if (rc) {
                hipGraph_t dummy;
                (void)hipStreamEndCapture(cs, &dummy);
                (void)hipStreamDestroy(cs);
                if (!fresh) g_graphs.erase(it);
                (void)hipFree(ent.sched);
                (void)hipHostFree(ent.hbase);
                (void)hipHostFree(ent.hsched);
                (void)hipEventDestroy(ent.sched_copied);
                return rc;
            }
        }
        GS_HIP(hipStreamEndCapture(cs, &g));
        GS_HIP(hipStreamDestroy(cs));
        GS_HIP(hipGraphInstantiate(&ent.exec, g, nullptr, nullptr, 0));
        GS_HIP(hipGraphDestroy(g));
        ++g_graph_captures;
        if (fresh)
            it = g_graphs.emplace(key, ent).first;
        else
            it->second = ent;
    }
    GraphEntry &e = it->second;
    GS_HIP(hipEventSynchronize(e.sched_copied));   // the previous call's copy has read hsched
    for (int64_t k = 0; k < n_minibatches; ++k) {
        const StepArgs sa = make_step_args(hp, L, batch, adam_step0 + k + 1);
        e.hsched[2 * k] = sa.aa.neg_step_size;
        e.hsched[2 * k + 1] = sa.aa.inv_bc2_sqrt;
    }
    GS_HIP(hipMemcpyAsync(e.sched, e.hsched, sizeof(float) * 2 * (size_t)n_minibatches, hipMemcpyHostToDevice, s));
    GS_HIP(hipEventRecord(e.sched_copied, s));
    for (int64_t r = 0; r < n_full; ++r) {
        GS_HIP(hipMemcpyAsync(it->second.base, it->second.hbase + r, sizeof(int64_t), hipMemcpyHostToDevice, s));
        GS_HIP(hipGraphLaunch(it->second.exec, s));
    }
    for (int64_t k = n_full * chunk; k < n_minibatches; ++k) {
        const StepArgs sa = make_step_args(hp, L, batch, adam_step0 + k + 1);
        rc = lagged  ? lag_step(k, nullptr, nullptr, s)
             : fused ? enqueue_step_fused(params, grads, adam_m, adam_v, L, with_norm(sa, k), batch,
                                          step_ff(k, k, nullptr), metrics + k * GS_NUM_METRICS, stop_flag, ws, comm,
                                          s)
                     : enqueue_step(params, grads, adam_m, adam_v, L, at_step(sa, k), ro, idx + k * batch, batch,
                                  metrics + k * GS_NUM_METRICS, stop_flag, ws, comm, s);
        if (rc) return rc;
    }
    return finish();
}

extern "C" int gs_ppo_update(float *params, float *grads, float *adam_m, float *adam_v, gs_mlp_dims dims,
                             gs_ppo_hparams hp, gs_rollout_view ro, const int32_t *idx, int64_t batch,
                             int64_t n_minibatches, int64_t adam_step0, float *metrics, int32_t *stop_flag,
                             void *workspace, size_t workspace_bytes, gs_comm *comm, int use_graph, void *stream)
{
    return ppo_update(params, grads, adam_m, adam_v, dims, hp, ro, idx, batch, n_minibatches, adam_step0, metrics,
                      stop_flag, workspace, workspace_bytes, comm, use_graph, stream, nullptr);
}

extern "C" int gs_ppo_update_global(float *params, float *grads, float *adam_m, float *adam_v, gs_mlp_dims dims,
                                    gs_ppo_hparams hp, gs_rollout_view ro, const int32_t *idx, int64_t batch,
                                    int64_t n_minibatches, int64_t adam_step0, float *metrics, int32_t *stop_flag,
                                    void *workspace, size_t workspace_bytes, gs_comm *comm, int use_graph,
                                    const gs_ppo_global *glob, void *stream)
{
    GS_REQUIRE(glob && glob->batch_global >= 2 && glob->metric_sums, "gs_ppo_update_global: bad global arguments");
    GS_REQUIRE(!hp.normalize_adv || glob->adv_stats, "gs_ppo_update_global: normalize_adv needs adv_stats");
    GS_REQUIRE(glob->batch_global >= batch || !comm, "gs_ppo_update_global: batch_global < local rows");
    return ppo_update(params, grads, adam_m, adam_v, dims, hp, ro, idx, batch, n_minibatches, adam_step0, metrics,
                      stop_flag, workspace, workspace_bytes, comm, use_graph, stream, glob);
}

extern "C" int gs_ppo_global_adv_stats(const int32_t *idx, int64_t n_minibatches, int64_t batch, int64_t batch_global,
                                       const float *advantages, int64_t T, int64_t N, gs_comm *comm, double *sums,
                                       float *adv_stats, void *stream)
{
    GS_REQUIRE(idx && advantages && sums && adv_stats, "gs_ppo_global_adv_stats: null buffer");
    GS_REQUIRE(n_minibatches >= 0 && batch >= 1 && batch <= 1 << 20 && batch_global >= 2 && T > 0 && N > 0,
               "gs_ppo_global_adv_stats: bad sizes");
    if (n_minibatches == 0) return GS_OK;
    hipStream_t s = (hipStream_t)stream;
    int rc = launch_global_adv_sums(idx, n_minibatches, batch, advantages, T, N, sums, s);
    if (rc) return rc;
    if (comm && (rc = gs_comm_allreduce_sum_f64(comm, sums, 2 * n_minibatches, stream))) return rc;
    return launch_global_adv_stats(sums, n_minibatches, batch_global, adv_stats, s);
}

extern "C" int gs_ppo_global_records(const gs_ppo_hparams *hp, int64_t n_minibatches, int64_t batch_global,
                                     gs_comm *comm, double *metric_sums, float *metrics, void *stream)
{
    GS_REQUIRE(hp && metric_sums && metrics && n_minibatches >= 0 && batch_global >= 2,
               "gs_ppo_global_records: bad argument");
    if (n_minibatches == 0) return GS_OK;
    int rc;
    if (comm && (rc = gs_comm_allreduce_sum_f64(comm, metric_sums, kNumSumsHost * n_minibatches, stream))) return rc;
    gs_ppo_global g{batch_global, nullptr, metric_sums};
    const StepArgs sa = make_step_args(*hp, Layout{}, batch_global, 1, &g);
    return launch_global_records(metric_sums, n_minibatches, sa.la, metrics, (hipStream_t)stream);
}

extern "C" int gs_ppo_graph_cache_info(int64_t *n_entries, int64_t *n_captures)
{
    std::lock_guard<std::mutex> lk(g_graph_mu);
    if (n_entries) *n_entries = (int64_t)g_graphs.size();
    if (n_captures) *n_captures = g_graph_captures;
    return GS_OK;
}

extern "C" int gs_ppo_exchange_inside_bwd(gs_comm *comm, gs_mlp_dims dims, int64_t batch, int *inside)
{
    GS_REQUIRE(comm && inside, "gs_ppo_exchange_inside_bwd: null argument");
    int rc = check_dims(dims);
    if (rc) return rc;
    GS_REQUIRE(batch >= 2 && batch <= 1024, "batch %lld outside [2, 1024]", (long long)batch);
    const Layout L = layout_of(dims);
    BwdXchg bx;
    *inside = has_fused(L, batch) && bwd_exchange_of(comm, L, batch, &bx) ? 1 : 0;
    return GS_OK;
}
