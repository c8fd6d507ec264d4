"""GPU: the drop-in plugin surface against the reference's own outputs.

* losses_for_batch / training_step on the reference's tensor batch (agents/ppo/ppo_agent.py:21-152,
  base_agent.py:330-366) with metrics_recorder.record("train", ...) (ppo_agent.py:131-146);
* the rollout collector's get_metrics() after every rollout (utils/rollout_collector.py:686-760)
  and evaluate_episodes (:570-655), against the reference collector driven by the same
  synthetic env (tests/golden/trajectory.npz);
* the sticky KL early stop (base_agent.py:60,330-366; tests/golden/trajectory_kl.npz);
* a checkpoint written by the reference's BaseAgent.save_checkpoint (tests/golden/ref_ckpt/);
* build_agent from the Config the reference's load_config resolves (tests/golden/configs_full.json).

Tolerances: one-minibatch loss and metrics 2e-6 (+1e-5 relative); trajectory-level losses and
per-minibatch metrics 1e-4 (the north-star bar); collector statistics 1e-5 relative where they
depend only on the env / replayed actions, 1e-3 relative where they depend on the policy's
values (the trained weights agree to ~1e-5 relative), counts exactly.
"""
import json
import os
from types import SimpleNamespace

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _agent_for_step(cuda, tag):
    from gsamd.config import load_config
    from gsamd.ppo_agent import DevicePPOAgent
    torch.manual_seed(42)
    if tag == "cartpole":
        cfg = load_config("CartPole-v1", "ppo", overrides=dict(env_dynamics="synthetic", n_envs=8))
    else:
        cfg = load_config("LunarLander-v3", "ppo", overrides=dict(env_dynamics="synthetic", n_envs=1, n_steps=64, ent_coef=0.01))
    return DevicePPOAgent(cfg, device=cuda, use_graph=False)


@pytest.mark.parametrize("tag", ["cartpole", "lunar_ent"])
def test_losses_for_batch_on_reference_tensor_batch(golden, cuda, tag):
    """The reference's batch (CPU tensors in a SimpleNamespace, as its tests pass it) through
    DevicePPOAgent.losses_for_batch: loss and every recorded metric equal the reference's
    record; then training_step on the same batch gives the reference's clipped-Adam update."""
    from gsamd.metrics import ppo_keys
    z = golden("ppo_step.npz")
    agent = _agent_for_step(cuda, tag)
    agent.policy_model.load_flat(z[f"{tag}/params0"])
    batch = SimpleNamespace(observations=torch.as_tensor(z[f"{tag}/obs"]),
                            actions=torch.as_tensor(z[f"{tag}/actions"]),
                            logprobs=torch.as_tensor(z[f"{tag}/old_logprobs"]),
                            values=torch.as_tensor(z[f"{tag}/old_values"]),
                            advantages=torch.as_tensor(z[f"{tag}/advantages"]),
                            returns=torch.as_tensor(z[f"{tag}/returns"]))
    agent.metrics_recorder.reset_epoch("train")
    out = agent.losses_for_batch(batch, 0)
    assert set(out) == {"loss", "early_stop_epoch"} and out["early_stop_epoch"] is False
    assert out["loss"].dim() == 0 and out["loss"].is_cuda
    np.testing.assert_allclose(float(out["loss"]), float(z[f"{tag}/loss"]), atol=2e-6, rtol=1e-5)
    got = agent.metrics_recorder.compute_epoch_means("train")
    ref = dict(zip([str(x) for x in z[f"{tag}/metric_names"]], z[f"{tag}/metric_values"]))
    assert set(got) == set(ref) == set(ppo_keys(True))
    for k in ref:
        np.testing.assert_allclose(got[k], ref[k], atol=2e-6, rtol=1e-5, err_msg=k)
    agent.metrics_recorder.reset_epoch("train")
    agent.training_step(batch, 0)
    torch.cuda.synchronize()
    np.testing.assert_allclose(agent.policy_model.params.cpu().numpy(), z[f"{tag}/params1"], atol=2e-6, rtol=0)
    assert agent.adam_step == 1
    # the pre-clip gradient norms the reference's compute_grad_norms records (utils/models.py:196-230,
    # base_agent.py:607-608): all, backbone, policy_head, value_head
    got = agent.metrics_recorder.compute_epoch_means("train")
    gn = dict(zip([str(x) for x in z[f"{tag}/grad_norm_names"]], z[f"{tag}/grad_norm_values"]))
    assert set(gn) <= set(got), set(gn) - set(got)
    for k in gn:
        np.testing.assert_allclose(got[k], gn[k], rtol=1e-5, err_msg=k)
    # training_step's forward-hook record (base_agent.py:335-347): the single-step chain writes the
    # minibatch's activation statistics into its record (GS_HP_ACT_STATS)
    acts = dict(zip([str(x) for x in z[f"{tag}/activation_names"]], z[f"{tag}/activation_values"]))
    assert set(acts) <= set(got), set(acts) - set(got)
    B = len(z[f"{tag}/actions"])
    for k, want in acts.items():
        tol = 1.0 / B if k.endswith(("dead_pct", "dead_max")) else 1e-5 + 1e-5 * abs(want)
        assert abs(got[k] - want) <= tol, (k, got[k], want)


def _replay_trajectory(agent, z, cuda, check_metrics=True):
    """Replay the fixture's three rollouts (recorded actions) and updates through the agent's
    collector and gs_ppo_update; returns the per-minibatch device records."""
    from gsamd._lib import M, check, lib
    N, T, E, B, D, A = (int(x) for x in z["dims"])
    coll = agent.get_rollout_collector("train")
    names = [str(x) for x in z["roll_metric_names"]]
    recs = []
    for ep in range(3):
        acts = torch.as_tensor(z["actions"][ep].reshape(N, T).T.copy()).to(cuda)
        traj = coll.collect(replay_actions=acts)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(traj.observations.cpu().numpy(), z["obs"][ep])
        np.testing.assert_array_equal(traj.dones.cpu().numpy().astype(np.uint8), z["dones"][ep])
        np.testing.assert_allclose(traj.advantages.cpu().numpy(), z["adv"][ep], atol=1e-5, rtol=0)
        np.testing.assert_allclose(traj.returns.cpu().numpy(), z["ret"][ep], atol=1e-5, rtol=0)
        if check_metrics:
            m = coll.get_metrics()
            assert set(names) <= set(m), set(names) - set(m)
            np.testing.assert_array_equal(m["action_dist"], z["action_dist"][ep])
            for j, k in enumerate(names):
                want = z["roll_metric_values"][ep][j]
                if k.startswith("cnt/") or k in ("roll/env_steps", "roll/vec_steps", "roll/episodes") or \
                        k.startswith("roll/ep_") or k.startswith("roll/baseline"):
                    assert m[k] == want, (ep, k, m[k], want)
                elif k.startswith(("roll/adv", "roll/return")):
                    np.testing.assert_allclose(m[k], want, rtol=1e-3, atol=1e-5, err_msg=f"{ep} {k}")
                else:
                    np.testing.assert_allclose(m[k], want, rtol=1e-5, atol=1e-6, err_msg=f"{ep} {k}")
        idx = agent.prefetcher.upload(ep)
        check(lib.gs_ppo_update(agent.policy_model.params.data_ptr(), agent.grads.data_ptr(), agent.adam_m.data_ptr(),
                                agent.adam_v.data_ptr(), agent.policy_model.dims, agent.hparams(), coll.buffer.view(),
                                idx.data_ptr(), B, agent.n_minibatches, agent.adam_step, agent.metrics_buf.data_ptr(),
                                agent.stop_flag.data_ptr(), agent.workspace.data_ptr(), agent.workspace.numel(), None,
                                0, torch.cuda.current_stream().cuda_stream))
        torch.cuda.synchronize()
        rec = agent.metrics_buf.cpu().numpy().copy()
        agent.adam_step += int((rec[:, M["skipped"]] == 0).sum())
        recs.append(rec)
    return np.concatenate(recs)


def _trajectory_agent(cuda, z, host_env=False, **over):
    from gsamd.config import load_config
    from gsamd.ppo_agent import DevicePPOAgent
    from gsamd.synthetic_env import SyntheticVecEnv
    N, T, E, B, D, A = (int(x) for x in z["dims"])
    L, seed, trunc = (int(x) for x in z["env"])
    torch.manual_seed(42)
    cfg = load_config("CartPole-v1", "ppo", overrides=dict(env_dynamics="synthetic", episode_len=L, truncate_every=trunc, obs_dim=D,
                                                           n_actions=A, **over))
    # host_env: a gymnasium-style host vector env (reset / 5-tuple step / RecordEpisodeStatistics
    # infos) -> the collector's host branch: one H2D of obs and one D2H of actions per step
    env = SyntheticVecEnv(n_envs=N, obs_dim=D, n_actions=A, episode_len=L, seed=seed, truncate_every=trunc) \
        if host_env else None
    agent = DevicePPOAgent(cfg, env=env, device=cuda, use_graph=False)
    agent.policy_model.load_flat(z["params0"])
    return agent


@pytest.mark.parametrize("host_env", [False, True])
def test_collector_metrics_and_evaluation_vs_reference(golden, cuda, host_env):
    """get_metrics() after each of the three replayed rollouts (counters, running statistics,
    action histogram, rolling episode window, best / last episode), the per-minibatch
    metrics_recorder records of the update, and evaluate_episodes(20, deterministic) on the val
    collector after training — all against the reference collector's own outputs; with the
    device env and with a host env (the collector's per-step H2D/D2H branch)."""
    from gsamd.metrics import ppo_keys, ppo_records
    z = golden("trajectory.npz")
    agent = _trajectory_agent(cuda, z, host_env=host_env)
    rec = _replay_trajectory(agent, z, cuda)
    names = [str(x) for x in z["train_metric_names"]]
    keys = list(ppo_keys(True))
    dev = ppo_records(rec, 0.5, 0.0, True)
    ref = z["train_metric_values"]
    assert set(names) == set(keys) and dev.shape == ref.shape
    for j, k in enumerate(keys):
        np.testing.assert_allclose(dev[:, j], ref[:, names.index(k)], atol=1e-4, rtol=1e-4, err_msg=k)
    ev = agent.get_rollout_collector("val").evaluate_episodes(n_episodes=20, deterministic=True)
    en = [str(x) for x in z["eval_metric_names"]]
    assert set(en) <= set(ev), set(en) - set(ev)
    for j, k in enumerate(en):
        want = z["eval_metric_values"][0][j]
        if k.startswith(("roll/adv", "roll/return")):
            np.testing.assert_allclose(ev[k], want, rtol=1e-3, atol=1e-5, err_msg=k)
        else:
            np.testing.assert_allclose(ev[k], want, rtol=1e-5, atol=1e-6, err_msg=k)


def test_kl_early_stop_vs_reference(golden, cuda):
    """target_kl set so the reference's sticky early stop fires in the second rollout's update
    (minibatch 37 of 60): the same minibatches are evaluated, the same ones step, their losses
    agree within 1e-4, and the final weights match."""
    from gsamd._lib import M
    z = golden("trajectory_kl.npz")
    agent = _trajectory_agent(cuda, z, target_kl=float(z["target_kl"]))
    rec = _replay_trajectory(agent, z, cuda, check_metrics=False)
    evaluated = (rec[:, M["unevaluated"]] == 0).astype(np.uint8)
    stepped = (rec[:, M["skipped"]] == 0).astype(np.uint8)
    np.testing.assert_array_equal(evaluated, z["evaluated"])
    np.testing.assert_array_equal(stepped, z["stepped"])
    ev = z["evaluated"].astype(bool)
    np.testing.assert_allclose(rec[ev, M["loss"]], z["losses"][ev], atol=1e-4, rtol=0)
    p_dev = agent.policy_model.params.cpu().numpy().astype(np.float64)
    p_ref = z["params_final"].astype(np.float64)
    assert np.linalg.norm(p_dev - p_ref) / np.linalg.norm(p_ref) < 1e-4
    # the recorder books the evaluated minibatches (the tripping one included), as the reference
    agent.record_epoch_metrics()
    assert agent._early_stop_epoch
    assert agent.adam_step == int(z["stepped"].sum())


def test_reference_checkpoint_resumes(cuda):
    """model.pt / optimizer.pt / state.json written by the reference's BaseAgent.save_checkpoint
    after the trajectory run: weights, Adam moments, step count, lr, counters load exactly,
    and training continues from them."""
    from gsamd.config import load_config
    from gsamd.ppo_agent import DevicePPOAgent
    d = os.path.join(GOLDEN, "ref_ckpt")
    sd = torch.load(os.path.join(d, "model.pt"), map_location="cpu", weights_only=True)
    opt = torch.load(os.path.join(d, "optimizer.pt"), map_location="cpu", weights_only=True)
    state = json.load(open(os.path.join(d, "state.json")))
    torch.manual_seed(0)
    cfg = load_config("CartPole-v1", "ppo", overrides=dict(env_dynamics="synthetic", n_envs=8, n_epochs=2))
    agent = DevicePPOAgent(cfg, device=cuda, use_graph=False, track_stats=False)
    agent.load_checkpoint(d)
    torch.cuda.synchronize()
    flat = np.concatenate([t.reshape(-1).numpy() for t in sd.values()])
    assert np.array_equal(agent.policy_model.params.cpu().numpy(), flat)
    st = opt[0]["state"]
    m = np.concatenate([st[i]["exp_avg"].reshape(-1).numpy() for i in sorted(st)])
    v = np.concatenate([st[i]["exp_avg_sq"].reshape(-1).numpy() for i in sorted(st)])
    assert np.array_equal(agent.adam_m.cpu().numpy(), m) and np.array_equal(agent.adam_v.cpu().numpy(), v)
    assert agent.adam_step == int(float(st[0]["step"]))
    assert agent.policy_lr == opt[0]["param_groups"][0]["lr"]
    assert agent.current_epoch == state["epoch"]
    coll = agent.get_rollout_collector("train")
    assert coll.total_steps == state["total_env_steps"] and coll.total_vec_steps == state["total_vec_steps"]
    assert coll._best_episode_reward == state["best_train_reward"]
    agent.train_epoch()
    torch.cuda.synchronize()
    assert np.isfinite(agent.minibatch_losses()).all()
    assert agent.adam_step == int(float(st[0]["step"])) + agent.n_minibatches


@pytest.mark.parametrize("key", ["CartPole-v1:ppo", "ALE-Breakout-v5:rgb_ppo"])
def test_build_agent_from_reference_config(cuda, key):
    """agents.build_agent(config) with the Config object train.py would pass (every field the
    reference's load_config resolved): the device agent's hyper-parameters are the reference's,
    and the env is the one the config names — CartPole-v1 on the device CartPole dynamics; an
    ALE config (no device emulator) only with an explicit env_dynamics='synthetic'."""
    from gsamd import build_agent
    from gsamd.rollout import DeviceCartPoleVecEnv
    full = json.load(open(os.path.join(GOLDEN, "configs_full.json")))[key]
    want = json.load(open(os.path.join(GOLDEN, "configs.json")))[key]
    ref_cfg = SimpleNamespace(**full)
    small = dict(n_envs=8, n_steps=128, batch_size=1024, env_dynamics="synthetic") if "ALE" in key else {}
    torch.manual_seed(42)
    agent = build_agent(ref_cfg, device=cuda, track_stats=False) if not small else None
    if agent is None:
        from gsamd.config import from_reference_config
        from gsamd.ppo_agent import DevicePPOAgent
        with pytest.raises(ValueError, match="no device dynamics"):
            build_agent(ref_cfg, device=cuda, track_stats=False)
        agent = DevicePPOAgent(from_reference_config(ref_cfg, **small), device=cuda, track_stats=False)
    else:
        assert isinstance(agent.get_env("train"), DeviceCartPoleVecEnv)
    c = agent.config
    for k in ("n_epochs", "gamma", "gae_lambda", "clip_range", "clip_range_vf", "ent_coef", "vf_coef",
              "policy_lr", "max_grad_norm", "seed", "target_kl", "normalize_advantages", "model_id"):
        assert getattr(c, k) == want[k], k
    if not small:
        assert (c.n_envs, c.n_steps, c.batch_size) == (want["n_envs"], want["n_steps"], want["batch_size"])
    assert tuple(c.hidden_dims) == tuple(want["hidden_dims"])
    hp = agent.hparams()
    assert hp.clip_range == np.float32(want["clip_range"]) and hp.lr == np.float32(want["policy_lr"])
    agent.train_epoch()
    torch.cuda.synchronize()
    assert np.isfinite(agent.minibatch_losses()).all()


def test_build_agent_with_host_env_vs_reference_trajectory(golden, cuda):
    """The drop-in's env hand-off: build_agent(reference Config, env=<host
    VectorEnv>) — the env build_env_from_config would return, here the host twin of the synthetic
    env the fixture's reference RolloutCollector stepped — runs the host-env branch of the
    collector (one H2D of obs and one D2H of actions per step) and reproduces the reference's
    trajectory.npz: rollout tensors, per-minibatch losses within 1e-4 (the north-star bar)."""
    from gsamd import build_agent
    from gsamd.synthetic_env import SyntheticVecEnv
    z = golden("trajectory.npz")
    N, T, E, B, D, A = (int(x) for x in z["dims"])
    L, seed, trunc = (int(x) for x in z["env"])
    full = json.load(open(os.path.join(GOLDEN, "configs_full.json")))["CartPole-v1:ppo"]
    assert (full["n_envs"], full["n_steps"], full["batch_size"], full["n_epochs"]) == (N, T, B, E)
    torch.manual_seed(42)
    env = SyntheticVecEnv(n_envs=N, obs_dim=D, n_actions=A, episode_len=L, seed=seed, truncate_every=trunc)
    agent = build_agent(SimpleNamespace(**full), env=env, device=cuda, use_graph=False)
    assert agent.get_env("train") is env
    agent.policy_model.load_flat(z["params0"])
    recs = _replay_trajectory(agent, z, cuda, check_metrics=False)
    np.testing.assert_allclose(recs[:, 0], z["losses"], atol=1e-4, rtol=0)


def test_rollout_advantage_normalisation_vs_reference(golden, cuda):
    """normalize_advantages: rollout (utils/rollout_collector.py:441-448 with
    utils/returns_advantages.py:61-64): the collector normalises every rollout's advantages over
    the whole (T, N) buffer after GAE (gs_normalize_advantages) and the loss takes them as they
    are (no per-minibatch normalisation, utils/torch.py:148-173).  Replays trajectory_rollnorm.npz
    (the reference collector + losses_for_batch with that setting): the normalised advantages
    1e-5, get_metrics incl. roll/adv_norm/{mean,std}, every minibatch record with losses_for_batch's
    keys for that mode, per-minibatch losses 1e-4 (the north-star bar) and the final weights."""
    from gsamd.metrics import ppo_keys, ppo_records
    z = golden("trajectory_rollnorm.npz")
    agent = _trajectory_agent(cuda, z, normalize_advantages="rollout")
    assert agent.hparams().normalize_adv == 0
    assert agent.get_rollout_collector("train").normalize_advantages
    rec = _replay_trajectory(agent, z, cuda)
    names = [str(x) for x in z["train_metric_names"]]
    keys = list(ppo_keys(False))
    dev = ppo_records(rec, 0.5, 0.0, False)
    ref = z["train_metric_values"]
    assert set(names) == set(keys) and dev.shape == ref.shape
    for j, k in enumerate(keys):
        np.testing.assert_allclose(dev[:, j], ref[:, names.index(k)], atol=1e-4, rtol=1e-4, err_msg=k)
    np.testing.assert_allclose(rec[:, 0], z["losses"], atol=1e-4, rtol=0)
    p = agent.policy_model.params.cpu().numpy().astype(np.float64)
    p_ref = z["params_final"].astype(np.float64)
    assert np.linalg.norm(p - p_ref) / np.linalg.norm(p_ref) < 1e-4


@pytest.mark.parametrize("case", ["normal", "offset", "skewed", "constant", "single"])
def test_normalize_advantages_kernel_vs_reference(golden, cuda, case):
    """gs_normalize_advantages against the reference's _normalize_advantages outputs
    (adv_norm.npz), bit-exact: the kernel reproduces numpy's float32 pairwise sums over its
    8192-element chunks, so the applied mean / std and every normalised element are numpy's bits —
    also for the large-offset case, where numpy's float32 mean is 6e-5 off the exact one and a
    double-precision normalisation would differ by 6e-3.  The std = 0 cases give 0 as numpy's
    (a - mean) / 1e-8.  Plus a C2-sized (32 x 4096 = 16 chunks) and a ragged 3-chunk array against
    numpy directly, and one of 2^24 + 4096 elements (numpy divides the float32 sums by the count in
    float64)."""
    from gsamd._lib import check, lib, ptr, stream_handle
    from oracle.ppo_ref import normalize_advantages_rollout

    def run(arr):
        x = torch.as_tensor(arr).to(cuda).contiguous()
        scratch = torch.zeros(int(lib.gs_normalize_advantages_scratch_bytes(x.numel())) // 4, dtype=torch.float32,
                              device=cuda)
        ms = torch.zeros(2, dtype=torch.float32, device=cuda)
        check(lib.gs_normalize_advantages(ptr(x), x.numel(), 1e-8, ptr(scratch), ptr(ms), stream_handle()),
              "gs_normalize_advantages")
        torch.cuda.synchronize()
        return x.cpu().numpy(), ms.cpu().numpy()

    z = golden("adv_norm.npz")
    y, ms = run(z[f"{case}/in"])
    assert np.array_equal(ms.view(np.uint32), z[f"{case}/mean_std"].view(np.uint32)), (ms, z[f"{case}/mean_std"])
    assert np.array_equal(y.view(np.uint32), z[f"{case}/out"].view(np.uint32))
    if case in ("constant", "single"):
        assert (y == 0).all()
    if case == "offset":
        rng = np.random.default_rng(3)
        # (4097, 4096): n > 2^24, where numpy's float64 division by the count differs from a
        # float32 one (the count is no longer a float32)
        for shape in ((32, 4096), (3, 6000), (4097, 4096)):
            a = (rng.standard_normal(shape) * 1.5 + 4.0).astype(np.float32)
            y, _ = run(a)
            assert np.array_equal(y.view(np.uint32), normalize_advantages_rollout(a).view(np.uint32)), shape


def test_training_diagnostics_vs_reference(golden, cuda):
    """The per-epoch diagnostics the reference's BaseAgent records (trajectory_stats.npz, made by
    the reference's own code): opt/activations/* as the epoch mean over every evaluated minibatch's
    forward-hook values (utils/models.py:121-147 via training_step, base_agent.py:335-347 — the
    device update writes each minibatch's statistics into its record, GS_HP_ACT_STATS),
    opt/grads/norm/* over the stepped minibatches (base_agent.py:607-608), and hp/* logged at every
    epoch start (base_agent.py:302, hyperparameter_mixin.py:90-103) under a linear policy_lr schedule
    (HyperparameterSchedulerCallback -> _change_optimizers_lr), so hp/policy_lr and the Adam step
    size change between epochs.  Bars: activation mean / std 1e-5 (+1e-5 relative), dead fractions
    1/B, grad norms 1e-4 relative, hp exact, losses 1e-4 (the north-star bar)."""
    from gsamd._lib import M
    z = golden("trajectory_stats.npz")
    N, T, E, B, D, A = (int(x) for x in z["dims"])
    sv, ev, s0, s1 = (float(x) for x in z["lr_schedule"])
    sched = {"policy_lr": {"schedule": "linear", "start_value": sv, "end_value": ev, "start": None,
                           "end": s1 * N, "warmup": 0.0}}
    agent = _trajectory_agent(cuda, z, schedules=sched)
    assert agent.device_activation_stats
    coll = agent.get_rollout_collector("train")
    hp_names, act_names, gn_names = ([str(x) for x in z[k]] for k in ("hp_names", "act_names", "gn_names"))
    losses = []
    for ep in range(3):
        acts = torch.as_tensor(z["actions"][ep].reshape(N, T).T.copy()).to(cuda)
        coll.collect(replay_actions=acts)
        agent.update_phase()
        torch.cuda.synchronize()
        losses.append(agent.metrics_buf[:, M["loss"]].cpu().numpy().astype(np.float64))
        got = agent.epoch_metrics()
        for j, k in enumerate(hp_names):
            assert got[k] == z["hp_values"][ep][j], (ep, k, got[k], z["hp_values"][ep][j])
        for j, k in enumerate(act_names):
            want = z["act_epoch_means"][ep][j]
            tol = 1.0 / B if k.endswith(("dead_pct", "dead_max")) else 1e-5 + 1e-5 * abs(want)
            assert abs(got[k] - want) <= tol, (ep, k, got[k], want)
        for j, k in enumerate(gn_names):
            np.testing.assert_allclose(got[k], z["gn_epoch_means"][ep][j], rtol=1e-4, err_msg=f"{ep} {k}")
    np.testing.assert_allclose(np.concatenate(losses), z["losses"], atol=1e-4, rtol=0)
    p = agent.policy_model.params.cpu().numpy().astype(np.float64)
    p_ref = z["params_final"].astype(np.float64)
    assert np.linalg.norm(p - p_ref) / np.linalg.norm(p_ref) < 1e-4
