/*
 * gsamd.h — C-ABI of the MI355X-native rollout + GAE + PPO-update path
 * (libgsamd.so, built from gymnasium-solver_amd/csrc/ for gfx950).
 *
 * Conventions (SURVEY.md §8b "What the C-ABI must export"):
 *   - every pointer argument named *_dev is a caller-owned device (HBM) pointer;
 *     *_host pointers are caller-owned host memory;
 *   - kernels are enqueued on the caller's `stream` (a hipStream_t passed as void*;
 *     NULL = legacy default stream) and return without synchronising;
 *   - no hidden device allocation: scratch comes from a caller buffer sized by
 *     gs_ppo_workspace_bytes();
 *   - every function returns GS_OK (0) or a negative GS_E* code; the message of the
 *     last failure on the calling thread is returned by gs_last_error().
 *
 * Data layout in HBM:
 *   rollout buffers are time-major SoA: x[t * n_envs + env]; observations
 *   obs[(t * n_envs + env) * obs_dim + d]; the reference's env-major sample index
 *   i = env * T + t (utils/rollout_buffer.py:11-13) is mapped inside the kernels.
 *   Policy parameters are ONE flat fp32 vector in the reference's state_dict order
 *   (backbone.0.weight[H1][D], backbone.0.bias, backbone.2.weight[H2][H1],
 *   backbone.2.bias, policy_head.weight[A][H2], policy_head.bias,
 *   value_head.weight[1][H2], value_head.bias) — utils/models.py:285-326.
 *   Gradients and Adam moments use the same layout.
 */
#ifndef GSAMD_H
#define GSAMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GS_OK 0
#define GS_E_INVALID (-1)   /* bad argument / unsupported shape: like the reference's ValueError */
#define GS_E_HIP (-2)       /* HIP runtime error */
#define GS_E_COMM (-3)      /* RCCL error */

/* ---------------------------------------------------------------- misc
 * gs_abi_version() returns GS_ABI_VERSION of the header the library was built with; a binding
 * must refuse a library whose version differs (argument lists change between versions:
 * version 2 added the rollout clock argument of gs_policy_act / gs_cnn_policy_act /
 * gs_env_step / gs_atari_env_step and gs_comm_error_record; version 3 widened the metric record
 * to 24 floats and added gs_ppo_update_global; version 4 added gs_comm_xgmi_set_bwd_exchange, gs_comm_allreduce_sum_f64,
 * gs_ppo_global_adv_stats, gs_ppo_global_records, gs_cnn_ppo_update_global, gs_fc_gemm and
 * gs_episode_window; version 5 added the obs_store argument of gs_cnn_policy_act; version 6 added
 * gs_normalize_advantages(_scratch_bytes), gs_cnn_activation_stats, gs_build_source_hash,
 * gs_comm_xgmi_reset, gs_cnn_workspace_hidden_offset / _act_offset and the parts argument of
 * gs_fc_gemm; version 7 widened the metric record to 40 floats (the GS_M_ACT activation-statistics
 * slots of GS_HP_ACT_STATS updates). */
#define GS_ABI_VERSION 7
int gs_abi_version(void);
const char *gs_last_error(void);
/* sha256 prefix (16 hex digits) of the kernel sources this library was compiled from: path "mlp"
 * (the MLP chain + GAE), "cnn" (the NatureCNN update) or "" (every csrc/ file) — the key under
 * which measured PMC traffic (profiles/) is attributed to a build; NULL for an unknown path. */
const char *gs_build_source_hash(const char *path);

/* ---------------------------------------------------------------- GAE
 * Replaces utils/returns_advantages.py:115-155
 * (compute_batched_gae_advantages_and_returns), called from
 * utils/rollout_collector.py:372-384.  Bit-exact with the reference's float32 numpy
 * loop.  values/rewards/adv/ret are (T, N) f32, dones/timeouts (T, N) u8 (0/1),
 * bootstrap (T, N) f32 or NULL (= bootstrapped_next_values None), last_values (N).
 */
int gs_gae_f32(const float *values_dev, const float *rewards_dev, const uint8_t *dones_dev,
               const uint8_t *timeouts_dev, const float *bootstrap_dev, const float *last_values_dev,
               int64_t T, int64_t N, double gamma, double gae_lambda, float *adv_dev, float *ret_dev,
               void *stream);
/* Rollout-level advantage normalisation, in place over all n elements: replaces
 * utils/returns_advantages.py:61-64 (_normalize_advantages: (a - mean) / (std + eps), std biased),
 * applied by utils/rollout_collector.py:441-442 when normalize_advantages == "rollout".  Bit-exact
 * with numpy on the float32 array: the mean's and std's sums are numpy's float32 pairwise sums over
 * its 8192-element buffer chunks, the statistics and the elementwise pass float32.  scratch_dev:
 * gs_normalize_advantages_scratch_bytes(n) bytes; mean_std_out_dev (2 floats: the mean and std
 * applied) may be NULL.  1 <= n < 2^31. */
size_t gs_normalize_advantages_scratch_bytes(int64_t n);
int gs_normalize_advantages(float *adv_dev, int64_t n, float eps, float *scratch_dev, float *mean_std_out_dev,
                            void *stream);

/* ---------------------------------------------------------------- sampler (host)
 * Replaces utils/samplers.py:25-34 (MultiPassRandomSampler.set_epoch + __iter__):
 * seeds torch's CPU MT19937 with `seed` (= base_seed + epoch), draws
 * rand((num_passes, data_len)) and writes the unstable argsort of each row
 * (torch's introsort tie order) to out_host (num_passes * data_len int32).
 * Host-side by construction (a sequential generator + introsort); n_threads > 1
 * sorts passes in parallel.  The stream is then uploaded once per rollout.
 */
int gs_sampler_stream_i32(int64_t data_len, int64_t num_passes, uint64_t seed, int32_t *out_host,
                          int n_threads);

/* ---------------------------------------------------------------- MLP actor-critic
 * dims: obs_dim D, hidden H1, H2 (two ReLU layers, the reference's mlp_small/medium/
 * large presets; utils/model_registry.py:21-36), n_actions A.
 */
typedef struct gs_mlp_dims {
    int32_t obs_dim;
    int32_t hidden1;
    int32_t hidden2;
    int32_t n_actions;
} gs_mlp_dims;

int64_t gs_mlp_param_count(gs_mlp_dims dims);

/* Rollout clock (clock_dev, optional, 2 x uint64 in HBM): {rng counter base, env step base}.
 * When non-NULL the kernels add clock_dev[0] to rng_counter and clock_dev[1] to step_count, so
 * a captured T-step rollout graph replays with the next rollout's counters written into the
 * clock (one 16-byte copy) instead of re-capturing; NULL = the counters as passed. */

/* Policy forward for a rollout step — replaces utils/policy_ops.py:14-34 (policy_act)
 * on MLPActorCritic.forward (utils/models.py:328-346) + Categorical sample / mode /
 * log_prob.  obs_dev (N, D) f32.  mode: 0 = sample (counter-based RNG, key
 * (rng_seed, rng_counter, env)), 1 = deterministic (argmax, first max wins),
 * 2 = replay: actions_dev is an INPUT (recorded actions).  Writes actions (int64),
 * logp, value (N) and, when obs_store_dev != NULL, copies obs into it (the rollout
 * buffer slot of this step).  scratch_dev: gs_policy_scratch_bytes(dims, N) bytes, 16-byte aligned.
 */
size_t gs_policy_scratch_bytes(gs_mlp_dims dims, int64_t N);
int gs_policy_act(const float *params_dev, gs_mlp_dims dims, const float *obs_dev, int64_t N, int mode,
                  uint64_t rng_seed, uint64_t rng_counter, int64_t *actions_dev, float *logp_dev,
                  float *value_dev, float *obs_store_dev, void *scratch_dev, const uint64_t *clock_dev,
                  void *stream);

/* A whole rollout of the synthetic env (gs_env_*) in ONE launch, for MLP policies whose weights
 * fit in LDS (gs_rollout_synth_supported; the C3 shapes do, C2's 256x256 W2 does not): per
 * workgroup 16 envs for all T vector steps, the policy act with gs_policy_act's arithmetic in its
 * order and the env step with gs_env_step's, so every row equals the step-wise rollout bit for
 * bit (actions of mode 2 are read from action_rows).  Rows are time-major (T, N); the env state,
 * running returns and observations are left after the last step, as T gs_env_step calls leave
 * them; the rng counter of step t is rng_counter0 + t, the env step count env_step0 + t + 1.
 * Replaces (with gs_env_step) the loop of utils/rollout_collector.py:459-567. */
int gs_rollout_synth_supported(gs_mlp_dims dims, int *supported_host);
int gs_rollout_synth(const float *params_dev, gs_mlp_dims dims, int64_t N, int64_t T, int mode, uint64_t rng_seed,
                     uint64_t rng_counter0, int32_t *env_state_dev, float *env_ep_ret_dev, float *env_obs_dev,
                     int32_t episode_len, int32_t truncate_every, float reward, uint64_t env_seed, int64_t env_offset,
                     uint64_t env_step0, int32_t *ep_done_count_dev, float *ep_ret_sum_dev, float *ep_len_sum_dev,
                     float *obs_rows_dev, int64_t *action_rows_dev, float *logp_rows_dev, float *value_rows_dev,
                     float *reward_rows_dev, uint8_t *done_rows_dev, uint8_t *timeout_rows_dev, void *stream);

/* Value-only forward (utils/policy_ops.py:37-42 policy_predict_values), e.g. the
 * bootstrap value of the last observation (utils/rollout_collector.py:373). */
int gs_policy_value(const float *params_dev, gs_mlp_dims dims, const float *obs_dev, int64_t N,
                    float *value_dev, void *scratch_dev, void *stream);

/* ---------------------------------------------------------------- synthetic env
 * Device twin of gsamd/synthetic_env.py.  state_dev: 4 int32 per env
 * (k, episode_idx, ep_len, pad) + ep_ret f32 (N); writes next obs into obs_dev (N, D),
 * reward/done/timeout rows of step t into the (T, N) rollout buffers, and per-env
 * completed-episode stats (ep_done_count, ep_ret_sum, ep_len_sum: N each, accumulated).
 */
int gs_env_reset(int32_t *state_dev, float *ep_ret_dev, float *obs_dev, int64_t N, int32_t obs_dim,
                 int32_t episode_len, uint64_t seed, int64_t env_offset, void *stream);
int gs_env_step(int32_t *state_dev, float *ep_ret_dev, float *obs_dev, int64_t N, int32_t obs_dim,
                int32_t episode_len, int32_t truncate_every, float reward, uint64_t seed,
                int64_t env_offset, uint64_t step_count, float *rewards_row_dev, uint8_t *dones_row_dev,
                uint8_t *timeouts_row_dev, int32_t *ep_done_count_dev, float *ep_ret_sum_dev,
                float *ep_len_sum_dev, const uint64_t *clock_dev, void *stream);

/* Completed-episode records of a (T, N) rollout, for the collector's episode statistics
 * (utils/rollout_collector.py:210-294 _process_done_infos, :686-760 get_metrics): per env the
 * running return (f32, the rewards summed in step order) and length carry across rollouts in
 * run_ret_dev / run_len_dev (N each, zero after a reset); ep_ret_dev / ep_len_dev (T, N) receive
 * the finished episode's return and length where dones_dev is set, 0 elsewhere. */
int gs_episode_stats(const float *rewards_dev, const uint8_t *dones_dev, int64_t T, int64_t N, float *run_ret_dev,
                     int32_t *run_len_dev, float *ep_ret_dev, int32_t *ep_len_dev, void *stream);
/* The reference's rolling window of the last W finished episodes (rollout_collector.py:242-294,
 * 753-758; track_stats=False keeps it on the device): this rollout's episodes in (step, env) order
 * — dones (T, N) time-major and gs_episode_stats' ep_ret / ep_len rows — appended behind the
 * previous window (2 x W doubles: returns, then lengths; the oldest first), meta[0] += their count,
 * meta[1] = max(meta[1], their best return), *total_out = their count (may be NULL).  One launch,
 * no host round trip. */
int gs_episode_window(const uint8_t *dones_dev, const float *ep_ret_dev, const int32_t *ep_len_dev, int64_t T,
                      int64_t N, int64_t W, double *window_dev, double *meta_dev, int64_t *total_out_dev,
                      void *stream);

/* ---------------------------------------------------------------- PPO update
 * Replaces the minibatch loop: DataLoader(MultiPassRandomSampler) + collate
 * (utils/dataloaders.py:20-77, rollout_collector.py:657-682) + PPOAgent.losses_for_batch
 * (agents/ppo/ppo_agent.py:21-152) + BaseAgent._backpropagate_and_step
 * (agents/base_agent.py:591-621: backward, clip_grad_norm_, Adam.step).
 */
typedef struct gs_ppo_hparams {
    float clip_range;
    float clip_range_vf;
    float vf_coef;
    float ent_coef;
    float max_grad_norm;      /* <= 0: no clipping */
    float lr;
    float adam_beta1;
    float adam_beta2;
    float adam_eps;
    float target_kl;          /* <= 0: None */
    int32_t normalize_adv;    /* 1 = "batch" (utils/torch.py:97-99), 0 = off */
    int32_t flags;            /* GS_HP_* bits; 0 = the fp32 parity path */
} gs_ppo_hparams;
/* bf16 MFMA operands (fp32 accumulation, fp32 parameters / Adam / loss) — a performance mode
 * beside the fp32 one (SURVEY.md Appendix A "Precision modes"): the NatureCNN update's
 * convolutions and GEMMs, and the MLP update's fused chain (gs_ppo_update: the h2 product, the
 * dW2 / dh1 products and the head-weight gradient; compile-time shapes only, GS_E_INVALID
 * elsewhere).  The single-step MLP entries (gs_ppo_minibatch_step, gs_ppo_loss, gs_ppo_stage)
 * stay fp32. */
#define GS_HP_BF16 1
/* Activation statistics per minibatch (the reference's forward hooks, utils/models.py:121-147,
 * recorded by every BaseAgent.training_step, agents/base_agent.py:335-347): the update also writes,
 * into the record of every minibatch whose loss it evaluates, {mean, unbiased std, dead_pct,
 * dead_max} of each hooked layer's pre-activation output z over the minibatch's rows, under the
 * parameters that minibatch's loss used (dead: |z| < 1e-6; dead_pct / dead_max the mean / max over
 * neurons of the fraction of rows) — GS_M_ACT + 4 l + {0, 1, 2, 3} for layer l (MLP: backbone.0,
 * backbone.2; NatureCNN: cnn.0, cnn.2, cnn.4, mlp.0).  gs_ppo_update / gs_ppo_minibatch_step /
 * gs_cnn_ppo_update; not the global-minibatch entries.  Off: those slots stay 0. */
#define GS_HP_ACT_STATS 2

/* Per-minibatch metric record written by the loss kernel (floats, GS_NUM_METRICS each).
 * KL early stop (agents/base_agent.py:330-366, sticky): the minibatch whose approx_kl exceeds
 * target_kl keeps its loss metrics with KL_STOP = SKIPPED = 1 (no optimizer step); every later
 * one is zeros with SKIPPED = KL_STOP = UNEVALUATED = 1 (its loss was never computed). */
#define GS_NUM_METRICS 40
enum gs_metric_slot {
    GS_M_LOSS = 0, GS_M_POLICY_LOSS, GS_M_VALUE_LOSS, GS_M_ENTROPY, GS_M_CLIP_FRAC,
    GS_M_CLIP_FRAC_VF, GS_M_EXPLAINED_VAR, GS_M_KL, GS_M_APPROX_KL, GS_M_ADV_NORM_MEAN,
    GS_M_ADV_NORM_STD, GS_M_KL_STOP, GS_M_GRAD_NORM, GS_M_SKIPPED, GS_M_UNEVALUATED, GS_M_RES1,
    /* pre-clip gradient norms per component (utils/models.py:196-230 compute_grad_norms, recorded
     * at agents/base_agent.py:607-608): MLP backbone | NatureCNN cnn trunk, policy_head,
     * value_head, and the NatureCNN mlp (fc) trunk (0 for the MLP policy) */
    GS_M_GN_BACKBONE, GS_M_GN_POLICY_HEAD, GS_M_GN_VALUE_HEAD, GS_M_GN_MLP,
    GS_M_RES20, GS_M_RES21, GS_M_RES22, GS_M_RES23,
    /* GS_HP_ACT_STATS: 4 layers x {mean, std, dead_pct, dead_max} of the pre-activation outputs */
    GS_M_ACT = 24
};

size_t gs_ppo_workspace_bytes(gs_mlp_dims dims, int64_t batch);

/* Rollout buffers the update reads (time-major (T, N), see header comment). */
typedef struct gs_rollout_view {
    const float *obs;        /* (T, N, D) */
    const int64_t *actions;  /* (T, N) */
    const float *logprobs;   /* (T, N) */
    const float *values;     /* (T, N) */
    const float *advantages; /* (T, N) */
    const float *returns;    /* (T, N) */
    int64_t T;
    int64_t N;
} gs_rollout_view;

/* One fused PPO minibatch step on rows idx_dev[0:batch) (env-major sample indices into
 * the rollout, int32): forward, loss, backward, grad-norm clip and Adam update of
 * params/adam_m/adam_v in place.  adam_step is the 1-based optimizer step count.
 * metrics_dev receives GS_NUM_METRICS floats; stop_flag_dev is the sticky KL early-stop
 * flag (int32, agents/base_agent.py:331-355).  comm may be NULL (single GPU) or a
 * gs_comm handle: gradients are then all-reduced (mean) across ranks before clipping. */
struct gs_comm;
int gs_ppo_minibatch_step(float *params_dev, float *grads_dev, float *adam_m_dev, float *adam_v_dev,
                          gs_mlp_dims dims, gs_ppo_hparams hp, gs_rollout_view rollout,
                          const int32_t *idx_dev, int64_t batch, int64_t adam_step,
                          float *metrics_dev, int32_t *stop_flag_dev, void *workspace_dev,
                          struct gs_comm *comm, void *stream);

/* Forward + loss only (PPOAgent.losses_for_batch without the optimizer step): writes the
 * GS_NUM_METRICS record (loss, policy/value/entropy terms, clip fractions, KL ...). */
int gs_ppo_loss(const float *params_dev, gs_mlp_dims dims, gs_ppo_hparams hp, gs_rollout_view rollout,
                const int32_t *idx_dev, int64_t batch, float *metrics_dev, void *workspace_dev, void *stream);

/* Activation statistics of the MLP backbone (utils/models.py:120-145: hooks on backbone.0 and
 * backbone.2, i.e. the pre-activation outputs of the two Linear layers; recorded per
 * training_step, base_agent.py:336-347) over rows idx_dev[0..rows) of the rollout (idx_dev null:
 * rows 0..rows).  Writes ceil(rows/16) parts of 2 * (2 + max(hidden1, hidden2)) doubles: per layer
 * {sum z, sum z^2, then per neuron the count of |z| < 1e-6}; the caller adds the parts
 * (mean, unbiased std, dead_pct = mean over neurons of count / rows, dead_max = max). */
int gs_mlp_activation_stats(const float *params_dev, gs_mlp_dims dims, gs_rollout_view rollout,
                            const int32_t *idx_dev, int64_t rows, double *parts_dev, void *stream);

/* Enqueue ONE stage of a minibatch step on the current workspace.  Unfused chain:
 * 0 = k_fwd_hidden, 1 = k_loss, 2 = k_bwd, 3 = k_clip_adam.  Fused chain (the one
 * gs_ppo_update runs for the compile-time shapes): 6 = k_gather_all for a one-minibatch
 * update (run once first), 4 = k_fwd_hidden<fused>, 5 = k_bwd<fused> (loss rows inside),
 * then 3; 7 = k_fwd_hidden<fused> carrying the previous minibatch's clip + Adam step (the
 * lagged chain gs_ppo_update runs on one GPU; writes the update workspace's second parameter set, so the
 * workspace must be gs_ppo_update_workspace_bytes(dims, batch, n >= 1) large).  Used by bench.py
 * to time each kernel with events on the stream it is launched on (roofline measurement). */
int gs_ppo_stage(int stage, float *params_dev, float *grads_dev, float *adam_m_dev, float *adam_v_dev,
                 gs_mlp_dims dims, gs_ppo_hparams hp, gs_rollout_view rollout, const int32_t *idx_dev,
                 int64_t batch, int64_t adam_step, float *metrics_dev, void *workspace_dev, void *stream);

/* The whole update phase of one rollout: n_minibatches consecutive steps over
 * idx_dev (n_minibatches * batch indices), metrics_dev gets n_minibatches records.
 * adam_step0 is the optimizer step count BEFORE the first of these steps.
 * use_graph != 0 replays chunks of 512 steps from a captured hipGraph.  stop_flag_dev is the
 * KL early stop of hp.target_kl > 0 (sticky: set when a minibatch's approx_kl exceeds it, every
 * later step skipped); with target_kl unset the update never reads or writes it (the fused
 * chain's kernels then start without that dependent load). */
int gs_ppo_update(float *params_dev, float *grads_dev, float *adam_m_dev, float *adam_v_dev,
                  gs_mlp_dims dims, gs_ppo_hparams hp, gs_rollout_view rollout, const int32_t *idx_dev,
                  int64_t batch, int64_t n_minibatches, int64_t adam_step0, float *metrics_dev,
                  int32_t *stop_flag_dev, void *workspace_dev, size_t workspace_bytes, struct gs_comm *comm,
                  int use_graph, void *stream);

/* Global-minibatch mode of a data-parallel update (SURVEY.md §8e "exact global" option): the
 * reference's single-GPU math on G ranks.  Every rank runs the SAME n_minibatches global
 * minibatches of batch_global rows, drawn from the reference's permutation of ALL ranks' samples
 * (utils/samplers.py:25-34 over the global env-major index); idx_dev holds, per minibatch, this
 * rank's rows (local env-major indices) padded to `batch` entries with -1 (another rank's row: no
 * loss, no gradient).  The loss and its gradient are means over batch_global rows, so each rank's
 * gradient is its share of the global one and the exchange SUMS them (no 1/G); the advantage
 * normalisation uses the whole minibatch's statistics adv_stats (utils/torch.py:97-99, computed by
 * the caller from all ranks' rows); with target_kl the KL early stop is decided on approx_kl summed
 * over ranks (agents/ppo/ppo_agent.py:126-129), so every rank stops at the same minibatch.  This
 * rank's raw loss sums per minibatch (14 doubles: sum of min-surrogate, clipped value loss,
 * entropy, clip counts, kl, approx_kl, ret - v and its square, ret and its square, normalised adv
 * and its square, one unused slot) go to metric_sums; the caller adds them over ranks and forms the records
 * (gsamd.metrics.records_from_sums). */
typedef struct gs_ppo_global {
    int64_t batch_global;       /* rows of a global minibatch (all ranks) */
    const float *adv_stats;     /* (n_minibatches, 2) f32 {mean, std} of each global minibatch's advantages */
    double *metric_sums;        /* (n_minibatches, 14) out: this rank's raw loss sums */
} gs_ppo_global;
int gs_ppo_update_global(float *params_dev, float *grads_dev, float *adam_m_dev, float *adam_v_dev,
                         gs_mlp_dims dims, gs_ppo_hparams hp, gs_rollout_view rollout, const int32_t *idx_dev,
                         int64_t batch, int64_t n_minibatches, int64_t adam_step0, float *metrics_dev,
                         int32_t *stop_flag_dev, void *workspace_dev, size_t workspace_bytes, struct gs_comm *comm,
                         int use_graph, const gs_ppo_global *glob, void *stream);

/* Workspace for gs_ppo_update over n_minibatches steps.  When the shape has a compiled
 * fused chain (the BASELINE configs' MLP shapes) this includes the per-update gathered
 * minibatch fields and normalised advantages, so the per-step chain reads x in one load and
 * the loss runs row-parallel with metrics reduced once after the update; a smaller workspace
 * (>= gs_ppo_workspace_bytes) selects the index-chasing chain with bit-identical parameters.
 * The fused chain also needs params/grads/adam_m/adam_v 16-byte aligned (every torch
 * allocation is); unaligned buffers take the index-chasing chain.  The workspace also holds a
 * second params | adam_m | adam_v set for the lagged chain (single GPU: each minibatch's clip +
 * Adam runs inside the next forward kernel; bit-identical results; GS_LAGGED_ADAM=0 in the
 * environment selects a separate clip/Adam launch instead). */
size_t gs_ppo_update_workspace_bytes(gs_mlp_dims dims, int64_t batch, int64_t n_minibatches);

/* The update graphs gs_ppo_update keeps (one per distinct set of buffers and shapes) and the
 * number of captures made so far.  lr never causes a re-capture (the graph reads the step size
 * from a per-call table); a change of another hyper-parameter re-captures in place. */
int gs_ppo_graph_cache_info(int64_t *n_entries_host, int64_t *n_captures_host);
/* Where the fused MLP update (gs_ppo_update without target_kl) exchanges gradients over
 * `comm`: *inside_host = 1 when k_bwd exchanges its own outputs (xGMI transport, the shape
 * within the in-kernel exchange's limits and co-residency, include the one-rank case where the
 * exchange is empty), 0 when a separate exchange launch follows the backward (RCCL, or
 * GS_XGMI_BWD=0).  Host query (reads device attributes, launches nothing). */
int gs_ppo_exchange_inside_bwd(struct gs_comm *comm, gs_mlp_dims dims, int64_t batch, int *inside_host);
/* Global-minibatch mode, the device half around gs_ppo_update_global (no host round trip):
 * gs_ppo_global_adv_stats: Sum adv and Sum adv^2 (double) of this rank's rows (idx >= 0) of every
 * global minibatch, summed over ranks through `comm` (gs_comm_allreduce_sum_f64; comm NULL: one
 * rank), then the whole minibatch's mean and unbiased std into adv_stats[k][2] (f32) for
 * gs_ppo_global.adv_stats — utils/torch.py:97-99 over all G ranks' rows.  sums: 2 x n doubles of
 * workspace (16-B aligned).  gs_ppo_global_records: after the update, the ranks' raw loss sums
 * (gs_ppo_global.metric_sums, 14 doubles per minibatch) summed over ranks in place and every
 * evaluated minibatch's record rewritten from them (loss, policy / value loss, entropy, clip
 * fractions, explained variance, kl, approx_kl, normalised-advantage mean / std) — identical on
 * every rank.  Both are stream-ordered and graph-capturable. */
int gs_ppo_global_adv_stats(const int32_t *idx_dev, int64_t n_minibatches, int64_t batch, int64_t batch_global,
                            const float *advantages_dev, int64_t T, int64_t N, struct gs_comm *comm, double *sums_dev,
                            float *adv_stats_dev, void *stream);
int gs_ppo_global_records(const gs_ppo_hparams *hp, int64_t n_minibatches, int64_t batch_global, struct gs_comm *comm,
                          double *metric_sums_dev, float *metrics_dev, void *stream);

/* ---------------------------------------------------------------- NatureCNN actor-critic (C4/C5)
 * Replaces CNNActorCritic (utils/models.py:347-455; conv 8x8s4 -> 4x4s2 -> 3x3s1 with 32/64/64
 * channels, ReLU, Linear F->hidden ReLU, policy/value heads), action masking
 * (utils/policy_ops.py:44-75 + MaskedCategorical utils/distributions.py:8-82) and the same PPO
 * minibatch step as gs_ppo_update for image observations.  Observations are the u8 frame
 * stacks (T, N, in_c, in_h, in_w) exactly as the reference stores them; the model divides by
 * 255.  Flat parameter layout: the reference's tensor order (cnn.0, cnn.2, cnn.4, mlp.0,
 * policy_head, value_head; weight then bias) with conv2/conv3 weights stored (out, ky, kx, in)
 * and the fc weight (hidden, y, x, c) — gsamd.cnn converts state_dicts both ways. */
typedef struct gs_cnn_dims {
    int32_t in_c, in_h, in_w;  /* frame stack (4, 84, 84) */
    int32_t n_actions;         /* full action space (18 for ALE) */
    int32_t hidden;            /* fc width (512) */
    uint32_t valid_mask;       /* bit a set = action a valid; 0 = unmasked Categorical */
} gs_cnn_dims;

typedef struct gs_rollout_view_u8 {
    const uint8_t *obs;      /* (T, N, in_c, in_h, in_w) */
    const int64_t *actions;  /* (T, N) */
    const float *logprobs;   /* (T, N) */
    const float *values;     /* (T, N) */
    const float *advantages; /* (T, N) */
    const float *returns;    /* (T, N) */
    int64_t T;
    int64_t N;
} gs_rollout_view_u8;

int64_t gs_cnn_param_count(gs_cnn_dims dims);
/* scratch for `rows` rows (the minibatch B for updates, N envs for gs_cnn_policy_act); the workspace
 * base must be 16-byte aligned (every torch allocation is): the update places its internal buffers,
 * the bf16 parameter copy included, relative to it and refuses (GS_E_INVALID) an unaligned base */
size_t gs_cnn_workspace_bytes(gs_cnn_dims dims, int64_t rows);
/* Byte offset, inside a workspace of that many rows, of the fc layer's output h [rows][HID] fp32
 * (after relu): after gs_cnn_ppo_update / _global it holds the last minibatch step's values (the
 * device's fc ReLU decisions, which a teacher-forced comparison takes over); -1 on a bad shape. */
int64_t gs_cnn_workspace_hidden_offset(gs_cnn_dims dims, int64_t rows);
/* The same for the convolution activations: layer 1, 2, 3 -> a1, a2, a3 (NHWC, fp32 in the fp32
 * update: the device's conv ReLU decisions of the last minibatch step), 4 -> the fc output as
 * above; -1 on a bad shape or layer. */
int64_t gs_cnn_workspace_act_offset(gs_cnn_dims dims, int64_t rows, int layer);
/* policy_act on N frame stacks obs_dev (N, in_c, in_h, in_w): mode 0 sample / 1 argmax /
 * 2 replay (as gs_policy_act); masked actions are never drawn.  obs_store_dev (may be NULL): the
 * rollout buffer's obs row, receives a copy of obs_dev (written by the first convolution from the
 * frames it loads, no separate copy launch). */
int gs_cnn_policy_act(const float *params_dev, gs_cnn_dims dims, const uint8_t *obs_dev, int64_t N, int mode,
                      uint64_t rng_seed, uint64_t rng_counter, int64_t *actions_dev, float *logp_dev,
                      float *value_dev, uint8_t *obs_store_dev, void *workspace_dev, const uint64_t *clock_dev,
                      void *stream);
/* losses_for_batch on one minibatch: metrics record + (optional) dLoss/dlogits (B, A+1). */
int gs_cnn_ppo_loss(const float *params_dev, gs_cnn_dims dims, gs_ppo_hparams hp, gs_rollout_view_u8 rollout,
                    const int32_t *idx_dev, int64_t batch, float *metrics_dev, float *dlogits_dev,
                    void *workspace_dev, void *stream);
/* Activation statistics of the NatureCNN on one minibatch (the reference's forward hooks,
 * utils/models.py:121-147, registered on cnn.0 / cnn.2 / cnn.4 / mlp.0 at :419-422 and recorded
 * per training step at agents/base_agent.py:335-347): stats_out_dev receives 16 doubles, per
 * layer in that order {mean, std (unbiased), dead_pct, dead_max} of the layer's pre-activation
 * output over the batch rows (dead: |z| < 1e-6, per-neuron fraction of rows; dead_pct its mean
 * over neurons, dead_max its max).  fp32 (the reference's precision) whatever the update's mode;
 * uses the update's workspace (gs_cnn_workspace_bytes(dims, batch)). */
int gs_cnn_activation_stats(const float *params_dev, gs_cnn_dims dims, gs_rollout_view_u8 rollout,
                            const int32_t *idx_dev, int64_t batch, double *stats_out_dev, void *workspace_dev,
                            void *stream);
/* n_minibatches fused steps (forward, loss, backward, optional all-reduce, clip, Adam).
 * params / grads / adam_m / adam_v: 16-byte aligned (the clip + Adam kernel moves float4s). */
int gs_cnn_ppo_update(float *params_dev, float *grads_dev, float *adam_m_dev, float *adam_v_dev, gs_cnn_dims dims,
                      gs_ppo_hparams hp, gs_rollout_view_u8 rollout, const int32_t *idx_dev, int64_t batch,
                      int64_t n_minibatches, int64_t adam_step0, float *metrics_dev, int32_t *stop_flag_dev,
                      void *workspace_dev, struct gs_comm *comm, void *stream);
/* Global-minibatch mode of the NatureCNN update (dp_mode "global", the MLP's gs_ppo_update_global
 * for NatureCNN): idx = this rank's rows of every global minibatch (-1 = another rank's row),
 * frame_idx = the same with -1 replaced by a valid sample (those rows are read but dead: zero
 * dLoss/dz, so every gradient gets exact zeros from them); advantage statistics from
 * glob->adv_stats (gs_ppo_global_adv_stats), the loss averaged over glob->batch_global rows, the
 * exchange summing the ranks' shares (no 1/world), and this rank's raw loss sums in
 * glob->metric_sums (14 per minibatch, slot 13 zero) for gs_ppo_global_records.  No KL early
 * stop (target_kl must be unset).  Replaces agents/base_agent.py:591-621 over the reference's
 * single-process minibatches (utils/samplers.py:25-34, utils/torch.py:97-99). */
int gs_cnn_ppo_update_global(float *params_dev, float *grads_dev, float *adam_m_dev, float *adam_v_dev,
                             gs_cnn_dims dims, gs_ppo_hparams hp, gs_rollout_view_u8 rollout, const int32_t *idx_dev,
                             const int32_t *frame_idx_dev, int64_t batch, int64_t n_minibatches, int64_t adam_step0,
                             float *metrics_dev, int32_t *stop_flag_dev, void *workspace_dev, struct gs_comm *comm,
                             const gs_ppo_global *glob, void *stream);

/* ---------------------------------------------------------------- CartPole-v1 dynamics (f1)
 * gymnasium 1.x CartPoleEnv.step restated on device (double-precision state, Euler, tau 0.02,
 * TimeLimit max_steps, NEXT_STEP autoreset), for training on real CartPole dynamics without a
 * host round trip.  state_dev: 4 doubles per env; meta_dev: 3 int32 per env; actions_dev: the
 * (N) int64 actions of this step (ignored on autoreset steps).  Rows/counters as gs_env_step.
 * Reset draws come from a counter hash (gymnasium's PCG64 stream is not reproduced). */
int gs_cartpole_reset(double *state_dev, int32_t *meta_dev, float *ep_ret_dev, float *obs_dev, int64_t N,
                      uint64_t seed, int64_t env_offset, void *stream);
int gs_cartpole_step(double *state_dev, int32_t *meta_dev, float *ep_ret_dev, float *obs_dev,
                     const int64_t *actions_dev, int64_t N, int32_t max_steps, uint64_t seed, int64_t env_offset,
                     float *rewards_row_dev, uint8_t *dones_row_dev, uint8_t *timeouts_row_dev,
                     int32_t *ep_done_count_dev, float *ep_ret_sum_dev, float *ep_len_sum_dev, void *stream);

/* The fp32 MFMA GEMM under the CNN path (convolutions as GEMMs, fc, heads), exported for its
 * tests: row-major C[M][N] = op(A) op(B) + beta C (+ bias[n]) (ReLU if relu), op(X) = X^T
 * when t* != 0 (A stored K x M, B stored N x K). */
int gs_gemm_f32(int ta, int tb, int64_t M, int64_t N, int64_t K, const float *A_dev, int64_t lda,
                const float *B_dev, int64_t ldb, float *C_dev, int64_t ldc, float beta, const float *bias_dev,
                int relu, void *stream);
/* The NatureCNN fc layer's three GEMMs (utils/models.py:56-110: h = relu(a3 Wf^T + bf) and its
 * backward) on the hand-written MFMA kernels the update runs (csrc/gs_fc.hip), exposed for
 * parity tests: op 0 C[M][N] = relu(A[M][K] B[N][K]^T + aux[N]); op 1 C = A^T B with A [K][M],
 * B [K][N]; op 2 C = (A B) .* (aux > 0) with A [M][K], B [K][N], aux [M][ldc].  bf16 != 0: bf16
 * operands (round to nearest even), fp32 accumulation.  GS_E_INVALID for shapes outside
 * K % 64 == 0, 16-B aligned rows (and M, N % 4 == 0 for K-strided operands).  parts_dev (may be NULL;
 * 2 M N floats): with it the fp32 forward runs the update's split-K form (two K halves summed in
 * order, then the bias + ReLU epilogue), without it the single-pass form (ABI 6 added it). */
int gs_fc_gemm(int op, int bf16, int64_t M, int64_t N, int64_t K, const float *A, int64_t lda, const float *B,
               int64_t ldb, float *C, int64_t ldc, const float *aux, float *parts_dev, void *stream);

/* ---------------------------------------------------------------- Atari pixel path (a13)
 * The observation pipeline of ale-py's AtariVectorEnv / gymnasium AtariPreprocessing +
 * FrameStackObservation (utils/environment.py:240-303, :362-385), on device: two raw
 * 210x160x3 u8 frames per env step -> OpenCV-RGB2GRAY grayscale -> max of the two -> area
 * resize to out_h x out_w -> stack of stack_n frames, newest last, zero padding after reset.
 * The frame source is synthetic (hash of seed, env, frame, byte): ALE itself is not
 * available offline.  frames_dev: (N, 2, 210, 160, 3) u8 scratch; stack_dev: (N, stack_n,
 * out_h, out_w) u8 = the observation; state_dev: 4 int32 per env; counters and rows as
 * gs_env_step. */
int gs_atari_preprocess(const uint8_t *frames_dev, int64_t N, int32_t out_h, int32_t out_w, uint8_t *out_dev,
                        void *stream);
int gs_atari_render(uint8_t *frames_dev, int64_t N, uint64_t seed, int64_t env_offset, uint64_t step_count,
                    void *stream);
int gs_atari_env_reset(int32_t *state_dev, float *ep_ret_dev, uint8_t *stack_dev, uint8_t *frames_dev, int64_t N,
                       int32_t stack_n, int32_t out_h, int32_t out_w, int32_t episode_len, uint64_t seed,
                       int64_t env_offset, void *stream);
int gs_atari_env_step(int32_t *state_dev, float *ep_ret_dev, uint8_t *stack_dev, uint8_t *frames_dev, int64_t N,
                      int32_t stack_n, int32_t out_h, int32_t out_w, int32_t episode_len, int32_t truncate_every,
                      uint64_t seed, int64_t env_offset, uint64_t step_count, float *rewards_row_dev,
                      uint8_t *dones_row_dev, uint8_t *timeouts_row_dev, int32_t *ep_done_count_dev,
                      float *ep_ret_sum_dev, float *ep_len_sum_dev, const uint64_t *clock_dev, void *stream);

/* ---------------------------------------------------------------- multi-GPU (xGMI / RCCL)
 * One process per GPU; replaces the reference's single-process gradient step
 * (agents/base_agent.py:331-355 manual_backward + optimizer.step) with a data-parallel
 * mean over ranks.  Two transports behind the same handle:
 *   RCCL: rank 0 creates the 128-byte unique id, the launcher broadcasts it
 *         (torch.distributed), every rank calls gs_comm_init.
 *   xGMI one-shot (default for the update): every rank calls gs_comm_xgmi_create (allocates
 *         and IPC-exports its exchange region, max_count = largest exchange in floats),
 *         the launcher all-gathers the 64-byte handles in rank order, every rank calls
 *         gs_comm_xgmi_connect; after a barrier the communicator is ready.  A wait that
 *         exceeds GS_XGMI_TIMEOUT_S (default 120 s) sets a sticky error that
 *         gs_comm_status reports (GS_E_COMM); later exchanges then fail fast. */
int gs_comm_unique_id(uint8_t out_id[128]);
int gs_comm_init(const uint8_t id[128], int nranks, int rank, struct gs_comm **out);
int gs_comm_xgmi_create(int nranks, int rank, int64_t max_count, uint8_t out_handle[64], struct gs_comm **out);
int gs_comm_xgmi_connect(struct gs_comm *comm, const uint8_t *handles);
int gs_comm_status(struct gs_comm *comm);
/* The first timeout's record (host-only read of the region, synchronous): *timed_out = 1 when a
 * wait gave up; then *workgroup = the exchange workgroup that waited, *peer = the rank it waited
 * for, *site = where (1 exchange launch, 2 / 3 reduce-scatter / all-gather flags of the rsag
 * launch, 4 / 5 push / result flags of the exchange inside k_bwd); -1 / 0 when none.  Any out
 * pointer may be NULL.  gs_comm_status's message carries the same record. */
int gs_comm_error_record(struct gs_comm *comm, int *timed_out, int *workgroup, int *peer, int *site);
/* The MLP update's exchange runs inside the backward kernel (every workgroup waits for the
 * same workgroup of its peers), which needs the peers' workgroups to be resident together.
 * That always holds with one rank per GPU (a node); with c ranks sharing a GPU it needs
 * (c - 1) backward grids to leave a free workgroup slot, and even then the ranks are separate
 * processes, which the GPU time-slices rather than co-schedules.  The launcher reports the
 * largest number of ranks sharing one GPU here; until it does (more than one rank) the
 * colocation counts as unknown and the update exchanges with a separate launch after the
 * backward, as it does from 2 ranks per GPU (GS_XGMI_BWD=1 forces the in-backward form where the
 * grids fit: correct, but paced by the time-slicing).  Host-only, no GPU call. */
int gs_comm_xgmi_set_colocation(struct gs_comm *comm, int ranks_per_device);
/* Where the MLP update exchanges on this communicator: mode 0 = always a separate exchange
 * launch after the backward, 1 = inside the backward where one rank runs per GPU (the default),
 * 2 = inside the backward also for ranks sharing a GPU (GS_XGMI_BWD=1).  The launcher's
 * connect-time self-test (gsamd.distributed.init_xgmi_comm) runs the in-backward form on the
 * job's shapes and sets mode 0 on every rank when it fails.  Every rank must set the same mode
 * before its next update; captured update graphs are keyed by it.  Host-only, no GPU call. */
int gs_comm_xgmi_set_bwd_exchange(struct gs_comm *comm, int mode);
/* Back to the connect-time protocol state after a failed or timed-out exchange: this rank's flag
 * banks, sticky error word and sequence counters are zeroed (synchronous).  Collective in the
 * caller's protocol: every rank drains its device work, meets the others at a host barrier, calls
 * this, and meets them again before the next exchange (gsamd.distributed.xgmi_reset). */
int gs_comm_xgmi_reset(struct gs_comm *comm);
int gs_comm_allreduce_mean_f32(struct gs_comm *comm, float *buf_dev, int64_t count, void *stream);
/* Sum of `count` doubles over ranks, in place (16-B aligned buffer), the same result bits on every
 * rank: xGMI sums the sources in rank order in double (pieces of the communicator's capacity),
 * RCCL runs ncclAllReduce(ncclFloat64, ncclSum).  Stream-ordered. */
int gs_comm_allreduce_sum_f64(struct gs_comm *comm, double *buf_dev, int64_t count, void *stream);
/* What a communicator is: its rank count, this process's rank and the transport
 * (GS_COMM_RCCL / GS_COMM_XGMI).  Any out pointer may be NULL.  Host-only, no GPU call. */
#define GS_COMM_RCCL 0
#define GS_COMM_XGMI 1
int gs_comm_info(struct gs_comm *comm, int *nranks, int *rank, int *transport);
int gs_comm_destroy(struct gs_comm *comm);

#ifdef __cplusplus
}
#endif
#endif /* GSAMD_H */
