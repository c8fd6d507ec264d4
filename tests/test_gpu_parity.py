"""Parity of the HIP path (through the C-ABI) with the reference's golden vectors and the oracle.

Tolerances (BASELINE.json north_star): GAE and sampler indices bit-exact; advantages /
returns / log-probs / values within 1e-5 fp32; PPO loss trajectory within 1e-4.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _dev(a, cuda, dtype=None):
    t = torch.as_tensor(np.ascontiguousarray(a))
    if dtype is not None:
        t = t.to(dtype)
    return t.to(cuda).contiguous()


# ------------------------------------------------------------------------------- GAE
def test_gae_bit_exact_vs_reference_fixtures(golden, cuda):
    from gsamd.rollout import compute_batched_gae_advantages_and_returns as gae
    g = golden("gae.npz")
    names = sorted({k.split("/")[0] for k in g.files})
    assert len(names) >= 10
    for n in names:
        c = {k.split("/", 1)[1]: g[k] for k in g.files if k.startswith(n + "/")}
        boot = None if "no_boot" in c else _dev(c["bootstrap"], cuda)
        adv, ret = gae(_dev(c["values"], cuda), _dev(c["rewards"], cuda), _dev(c["dones"], cuda),
                       _dev(c["timeouts"], cuda), _dev(c["last_values"], cuda), boot, float(c["gamma"]),
                       float(c["lam"]))
        torch.cuda.synchronize()
        assert np.array_equal(adv.cpu().numpy().view(np.uint32), c["adv"].view(np.uint32)), n
        assert np.array_equal(ret.cpu().numpy().view(np.uint32), c["ret"].view(np.uint32)), n


# staged kernel: EW 16 (N % 16 == 0), 8, 4 with full / partial / half chunks; per-lane
# kernel: N % 4 != 0 (and forced through GS_GAE_KERNEL=lane below); with and without the
# bootstrap buffer
@pytest.mark.parametrize("T,N,boot", [(32, 4096, True), (2048, 1024, True), (7, 3000, True), (1, 1, True),
                                      (130, 1028, True), (64, 16, True), (65, 32, False), (200, 4104, False),
                                      (97, 4098, True), (40, 6, False)])
def test_gae_bit_exact_vs_c_oracle_full_size(cuda, T, N, boot):
    import oracle
    from gsamd.rollout import compute_batched_gae_advantages_and_returns as gae
    rng = np.random.default_rng(T * 7 + N)
    v = rng.standard_normal((T, N)).astype(np.float32)
    r = rng.standard_normal((T, N)).astype(np.float32)
    d = (rng.random((T, N)) < 0.05).astype(np.uint8)
    to = (d.astype(bool) & (rng.random((T, N)) < 0.3)).astype(np.uint8)
    lv = rng.standard_normal(N).astype(np.float32)
    b = rng.standard_normal((T, N)).astype(np.float32) if boot else None
    a_ref, r_ref = oracle.gae_c(v, r, d, to, lv, b if boot else np.zeros((T, N), np.float32), 0.99, 0.95)
    if not boot:   # without the buffer the reference's timeouts bootstrap from v[t+1] (oracle: b = v shifted)
        nv = np.concatenate([v[1:], lv[None]], 0)
        a_ref, r_ref = oracle.gae_c(v, r, d, to, lv, nv, 0.99, 0.95)
    adv, ret = gae(_dev(v, cuda), _dev(r, cuda), _dev(d, cuda), _dev(to, cuda), _dev(lv, cuda),
                   _dev(b, cuda) if boot else None, 0.99, 0.95)
    assert np.array_equal(adv.cpu().numpy().view(np.uint32), a_ref.view(np.uint32))
    assert np.array_equal(ret.cpu().numpy().view(np.uint32), r_ref.view(np.uint32))


def test_gae_lane_and_staged_kernels_agree(cuda, monkeypatch):
    """Both device kernels on the same inputs (the per-lane one forced): bitwise equal."""
    from gsamd.rollout import compute_batched_gae_advantages_and_returns as gae
    rng = np.random.default_rng(5)
    T, N = 300, 2048
    arrs = [rng.standard_normal((T, N)).astype(np.float32) for _ in range(3)]
    d = (rng.random((T, N)) < 0.05).astype(np.uint8)
    to = (d.astype(bool) & (rng.random((T, N)) < 0.5)).astype(np.uint8)
    lv = rng.standard_normal(N).astype(np.float32)
    args = [_dev(arrs[0], cuda), _dev(arrs[1], cuda), _dev(d, cuda), _dev(to, cuda), _dev(lv, cuda),
            _dev(arrs[2], cuda), 0.98, 0.8]
    a1, r1 = gae(*args)
    monkeypatch.setenv("GS_GAE_KERNEL", "lane")
    a2, r2 = gae(*args)
    assert torch.equal(a1.view(torch.int32), a2.view(torch.int32))
    assert torch.equal(r1.view(torch.int32), r2.view(torch.int32))


def test_gae_empty_is_noop(cuda):
    from gsamd._lib import check, lib
    check(lib.gs_gae_f32(None, None, None, None, None, None, 0, 5, 0.99, 0.95, None, None, None))


# ------------------------------------------------------------------------------- policy forward
def test_policy_forward_vs_reference(golden, cuda):
    from gsamd.policy import DeviceMLPActorCritic
    z = golden("policy_fwd.npz")
    pm = DeviceMLPActorCritic(4, (256, 256), 2, device=cuda, init=False)
    pm.load_flat(z["params"])
    obs = _dev(z["obs"], cuda)
    acts = _dev(z["actions"], cuda, torch.int64)
    a, lp, v = pm.act(obs, mode=2, actions=acts.clone())
    torch.cuda.synchronize()
    np.testing.assert_allclose(v.cpu().numpy(), z["values"], atol=1e-5, rtol=0)
    np.testing.assert_allclose(lp.cpu().numpy(), z["logp"], atol=1e-5, rtol=0)
    a_det, lp_det, _ = pm.act(obs, mode=1)
    probs = z["probs"]
    np.testing.assert_array_equal(a_det.cpu().numpy(), probs.argmax(axis=1))
    vv = pm.predict_values(obs)
    np.testing.assert_allclose(vv.cpu().numpy(), z["values"], atol=1e-5, rtol=0)


def test_policy_sampling_follows_probs(cuda):
    from gsamd.policy import DeviceMLPActorCritic
    torch.manual_seed(3)
    pm = DeviceMLPActorCritic(8, (128, 128), 4, device=cuda)
    obs = torch.rand(1, 8, device=cuda).repeat(8192, 1).contiguous()
    counts = np.zeros(4)
    for k in range(8):
        a, lp, _ = pm.act(obs, mode=0, rng_seed=42, rng_counter=k)
        counts += np.bincount(a.cpu().numpy(), minlength=4)
    # probabilities of the single repeated row from the replay path
    probs = np.zeros(4)
    for act in range(4):
        _, lpa, _ = pm.act(obs[:1].contiguous(), mode=2, actions=torch.tensor([act], device=cuda))
        probs[act] = float(np.exp(lpa.cpu().numpy()[0]))
    freq = counts / counts.sum()
    assert np.abs(freq - probs).max() < 0.01, (freq, probs)


def _mix64(x):
    """SplitMix64 finaliser on uint64 numpy arrays (csrc/gs_mlp.hip mix64), wrapping arithmetic"""
    x = x + np.uint64(0x9E3779B97F4A7C15)
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def test_policy_sampling_inverse_cdf_rows(cuda):
    """Row-exact check of the default sampling path: every row's action is the first a with
    u < cdf[a], u = the row's counter-based uniform (host restatement of the kernel's SplitMix64
    draw) and cdf the running sum of that row's probabilities (from the replay path's log-probs).
    Rows whose u lies within 2e-5 of a CDF boundary are left out (the host's exp(logp) and the
    kernel's softmax differ in the last bits); near-tie rows — two actions with probabilities
    within 1e-3 of each other — are generated on purpose and must be checked like the others."""
    from gsamd.policy import DeviceMLPActorCritic
    torch.manual_seed(5)
    pm = DeviceMLPActorCritic(8, (128, 128), 4, device=cuda)
    n = 8192
    obs = (torch.rand(n, 8, device=cuda) * 4 - 2).contiguous()
    seed, ctr = 1234, 7
    a, _, _ = pm.act(obs, mode=0, rng_seed=seed, rng_counter=ctr)
    a = a.cpu().numpy()
    lp = np.zeros((n, 4), np.float32)
    for act in range(4):
        _, lpa, _ = pm.act(obs, mode=2, actions=torch.full((n,), act, device=cuda, dtype=torch.int64))
        lp[:, act] = lpa.cpu().numpy()
    probs = np.exp(lp.astype(np.float64))
    cdf = np.cumsum(probs, axis=1)
    with np.errstate(over="ignore"):
        h = _mix64(_mix64(_mix64(np.uint64(seed)) ^ np.uint64(ctr)) ^ np.arange(n, dtype=np.uint64))
    u = (h >> np.uint64(40)).astype(np.float64) / 16777216.0
    want = np.minimum((u[:, None] >= cdf).sum(axis=1), 3)
    clear = np.abs(u[:, None] - cdf[:, :3]).min(axis=1) > 2e-5
    assert clear.sum() > n - 16, clear.sum()
    np.testing.assert_array_equal(a[clear], want[clear])
    srt = np.sort(probs, axis=1)
    ties = (np.diff(srt, axis=1) < 1e-3).any(axis=1) & clear
    assert ties.sum() >= 8, ties.sum()       # near-tie rows were checked above


# ------------------------------------------------------------------------------- synthetic env
def test_device_env_matches_host_env(cuda):
    from gsamd.rollout import DeviceSyntheticVecEnv
    from gsamd.synthetic_env import SyntheticVecEnv
    host = SyntheticVecEnv(n_envs=37, obs_dim=5, n_actions=2, episode_len=7, seed=42, truncate_every=2, env_offset=11)
    dev = DeviceSyntheticVecEnv(n_envs=37, obs_dim=5, n_actions=2, episode_len=7, seed=42, truncate_every=2,
                                env_offset=11, device=cuda)
    o_h, _ = host.reset()
    o_d, _ = dev.reset()
    assert np.array_equal(o_d.cpu().numpy(), o_h)
    rew = torch.zeros(37, device=cuda)
    dn = torch.zeros(37, dtype=torch.uint8, device=cuda)
    to = torch.zeros(37, dtype=torch.uint8, device=cuda)
    for _ in range(20):
        o_h, r_h, te, tr, _ = host.step(np.zeros(37, np.int64))
        dev.step_into(rew, dn, to)
        assert np.array_equal(dev.obs.cpu().numpy(), o_h)
        assert np.array_equal(rew.cpu().numpy(), r_h)
        assert np.array_equal(dn.cpu().numpy().astype(bool), te | tr)
        assert np.array_equal(to.cpu().numpy().astype(bool), tr)


# ------------------------------------------------------------------------------- one PPO step
def _rollout_view_from_batch(z, tag, cuda):
    from gsamd._lib import RolloutView
    B = int(z[f"{tag}/dims"][-1])
    t = dict(obs=_dev(z[f"{tag}/obs"][None], cuda), actions=_dev(z[f"{tag}/actions"][None], cuda, torch.int64),
             logprobs=_dev(z[f"{tag}/old_logprobs"][None], cuda), values=_dev(z[f"{tag}/old_values"][None], cuda),
             advantages=_dev(z[f"{tag}/advantages"][None], cuda), returns=_dev(z[f"{tag}/returns"][None], cuda))
    view = RolloutView(t["obs"].data_ptr(), t["actions"].data_ptr(), t["logprobs"].data_ptr(),
                       t["values"].data_ptr(), t["advantages"].data_ptr(), t["returns"].data_ptr(), 1, B)
    return t, view


@pytest.mark.parametrize("tag", ["cartpole", "lunar_ent"])
def test_ppo_step_vs_reference(golden, cuda, tag):
    from gsamd._lib import GS_NUM_METRICS, M, MlpDims, PPOHparams, check, lib
    z = golden("ppo_step.npz")
    D, H1, H2, A, B = (int(x) for x in z[f"{tag}/dims"])
    clip, cvf, vf, ent, lr = (float(x) for x in z[f"{tag}/hparams"])
    dims = MlpDims(D, H1, H2, A)
    keep, view = _rollout_view_from_batch(z, tag, cuda)
    P = int(lib.gs_mlp_param_count(dims))
    params = _dev(z[f"{tag}/params0"], cuda)
    assert params.numel() == P
    grads = torch.zeros(P, device=cuda)
    m = torch.zeros(P, device=cuda)
    v = torch.zeros(P, device=cuda)
    ws = torch.zeros(int(lib.gs_ppo_workspace_bytes(dims, B)), dtype=torch.uint8, device=cuda)
    idx = torch.arange(B, dtype=torch.int32, device=cuda)
    met = torch.zeros(GS_NUM_METRICS, device=cuda)
    stop = torch.zeros(1, dtype=torch.int32, device=cuda)
    hp = PPOHparams(clip, cvf, vf, ent, 0.5, lr, 0.9, 0.999, 1e-8, 0.0, 1, 0)
    s = torch.cuda.current_stream().cuda_stream
    check(lib.gs_ppo_loss(params.data_ptr(), dims, hp, view, idx.data_ptr(), B, met.data_ptr(), ws.data_ptr(), s))
    torch.cuda.synchronize()
    np.testing.assert_allclose(float(met[M["loss"]]), float(z[f"{tag}/loss"]), atol=1e-6, rtol=1e-6)
    names = [str(x) for x in z[f"{tag}/metric_names"]]
    ref = dict(zip(names, z[f"{tag}/metric_values"]))
    mm = met.cpu().numpy()
    for key, slot in [("opt/loss/policy", "policy_loss"), ("opt/loss/value", "value_loss"),
                      ("opt/policy/entropy", "entropy"), ("opt/ppo/clip_fraction", "clip_fraction"),
                      ("opt/ppo/clip_fraction_vf", "clip_fraction_vf"), ("opt/value/explained_var", "explained_var"),
                      ("opt/ppo/kl", "kl"), ("opt/ppo/approx_kl", "approx_kl"),
                      ("roll/adv/norm/std", "adv_norm_std")]:
        np.testing.assert_allclose(mm[M[slot]], ref[key], atol=2e-6, rtol=1e-5, err_msg=key)
    # the backbone's activation statistics (utils/models.py:120-190), as the reference's hooks
    # recorded them on this batch (tests/golden/make_golden.py: compute_activation_stats)
    from gsamd.metrics import activation_stats
    nparts = (B + 15) // 16
    parts = torch.zeros(nparts * 2 * (2 + max(H1, H2)), dtype=torch.float64, device=cuda)
    check(lib.gs_mlp_activation_stats(params.data_ptr(), dims, view, idx.data_ptr(), B, parts.data_ptr(), s),
          "gs_mlp_activation_stats")
    torch.cuda.synchronize()
    acts = activation_stats(parts.cpu().numpy().reshape(nparts, -1), B, (H1, H2))
    aref = dict(zip([str(x) for x in z[f"{tag}/activation_names"]], z[f"{tag}/activation_values"]))
    assert set(acts) == set(aref)
    for key, val in aref.items():
        np.testing.assert_allclose(acts[key], val, rtol=2e-5, atol=1e-7, err_msg=key)
    check(lib.gs_ppo_minibatch_step(params.data_ptr(), grads.data_ptr(), m.data_ptr(), v.data_ptr(), dims, hp, view,
                                    idx.data_ptr(), B, 1, met.data_ptr(), stop.data_ptr(), ws.data_ptr(), None, s))
    torch.cuda.synchronize()
    np.testing.assert_allclose(float(met[M["grad_norm"]]), float(z[f"{tag}/total_norm"]), rtol=1e-5)
    g_ref = z[f"{tag}/grads_clipped"]
    np.testing.assert_allclose(grads.cpu().numpy(), g_ref, atol=2e-6 * max(1.0, np.abs(g_ref).max()), rtol=0)
    np.testing.assert_allclose(params.cpu().numpy(), z[f"{tag}/params1"], atol=2e-6, rtol=0)
    del keep


# ------------------------------------------------------------------------------- full trajectory
def test_trajectory_replay_vs_reference(golden, cuda):
    """3 CartPole-shaped rollouts (N=8, T=32, B=256, E=20) replaying the reference's
    sampled actions: rollout tensors, sampler order, all 60 minibatch losses, final weights."""
    from gsamd.config import load_config
    from gsamd.ppo_agent import DevicePPOAgent
    z = golden("trajectory.npz")
    N, T, E, B, D, A = (int(x) for x in z["dims"])
    L, seed, trunc = (int(x) for x in z["env"])
    torch.manual_seed(42)
    cfg = load_config("CartPole-v1", "ppo", overrides=dict(env_dynamics="synthetic", episode_len=L, truncate_every=trunc, obs_dim=D,
                                                           n_actions=A))
    agent = DevicePPOAgent(cfg, device=cuda, use_graph=False)
    # initial weights come from the fixture: orthogonal_ init goes through LAPACK QR, whose
    # last bits depend on the host CPU (tests/test_host_cpu.py checks the init rule itself)
    agent.policy_model.load_flat(z["params0"])
    coll = agent.get_rollout_collector("train")
    losses = []
    for ep in range(3):
        acts = _dev(z["actions"][ep].reshape(N, T).T, cuda, torch.int64)
        traj = coll.collect(replay_actions=acts)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(traj.observations.cpu().numpy(), z["obs"][ep])
        np.testing.assert_allclose(traj.logprobs.cpu().numpy(), z["logp"][ep], atol=1e-5, rtol=0)
        np.testing.assert_allclose(traj.values.cpu().numpy(), z["values"][ep], atol=1e-5, rtol=0)
        np.testing.assert_allclose(traj.advantages.cpu().numpy(), z["adv"][ep], atol=1e-5, rtol=0)
        np.testing.assert_allclose(traj.returns.cpu().numpy(), z["ret"][ep], atol=1e-5, rtol=0)
        np.testing.assert_array_equal(traj.rewards.cpu().numpy(), z["rewards"][ep])
        np.testing.assert_array_equal(traj.dones.cpu().numpy().astype(np.uint8), z["dones"][ep])
        idx = agent.prefetcher.upload(ep)
        np.testing.assert_array_equal(idx.cpu().numpy(), z["order"][ep])
        from gsamd._lib import check, lib
        check(lib.gs_ppo_update(agent.policy_model.params.data_ptr(), agent.grads.data_ptr(), agent.adam_m.data_ptr(),
                                agent.adam_v.data_ptr(), agent.policy_model.dims, agent.hparams(), coll.buffer.view(),
                                idx.data_ptr(), B, agent.n_minibatches, agent.adam_step, agent.metrics_buf.data_ptr(),
                                agent.stop_flag.data_ptr(), agent.workspace.data_ptr(), agent.workspace.numel(), None,
                                0, torch.cuda.current_stream().cuda_stream))
        agent.adam_step += agent.n_minibatches
        losses.append(agent.minibatch_losses())
    losses = np.concatenate(losses)
    assert losses.shape == z["losses"].shape
    np.testing.assert_allclose(losses, z["losses"], atol=1e-4, rtol=0)
    # weights after 60 Adam steps: Adam's m/sqrt(v) amplifies last-bit gradient differences
    # for near-zero-gradient weights, so the weight check is relative (the bar is the loss)
    p_dev = agent.policy_model.params.cpu().numpy().astype(np.float64)
    p_ref = z["params_final"].astype(np.float64)
    assert np.linalg.norm(p_dev - p_ref) / np.linalg.norm(p_ref) < 1e-4
    assert np.abs(p_dev - p_ref).max() < 1e-3


# ------------------------------------------------------------------------------- full-size properties
# (env, variant, n_envs): C2 at full size; C3 shape (T=2048, B=64, E=10) at 32 envs
CASES = [("CartPole-v1", "ppo", 4096), ("LunarLander-v3", "ppo", 32)]


@pytest.mark.parametrize("env,variant,n_envs", CASES)
def test_update_graph_equals_eager_and_is_deterministic(cuda, env, variant, n_envs):
    """BASELINE configs C2/C3 shapes: chunked graph replay == eager launches, bitwise, and a
    rerun is identical (C3: 10 240 minibatches = 20 replays of a 512-step chunk)."""
    from gsamd.config import load_config
    from gsamd.ppo_agent import DevicePPOAgent
    results = []
    for use_graph in (False, True, True):
        torch.manual_seed(42)
        cfg = load_config(env, variant, overrides=dict(env_dynamics="synthetic", n_envs=n_envs))
        agent = DevicePPOAgent(cfg, device=cuda, use_graph=use_graph, track_stats=False)
        agent.train_epoch()
        agent.train_epoch()
        torch.cuda.synchronize()
        results.append((agent.policy_model.params.cpu().numpy(), agent.minibatch_losses()))
        assert np.isfinite(results[-1][1]).all()
        del agent
    for p, l in results[1:]:
        assert np.array_equal(p.view(np.uint32), results[0][0].view(np.uint32))
        assert np.array_equal(l, results[0][1])


@pytest.mark.parametrize("env,variant,n_envs", CASES)
def test_minibatch_step_vs_numpy_oracle(cuda, env, variant, n_envs):
    """One C2/C3-shaped minibatch of a device rollout against the numpy oracle (loss 1e-5 rel,
    clipped grads 1e-6 of max, params after Adam 5e-6)."""
    from oracle import ppo_ref as R
    from gsamd.config import load_config
    from gsamd.ppo_agent import DevicePPOAgent
    torch.manual_seed(42)
    cfg = load_config(env, variant, overrides=dict(env_dynamics="synthetic", n_envs=n_envs))
    agent = DevicePPOAgent(cfg, device=cuda, use_graph=False, track_stats=False)
    batches = agent.train_dataloader()
    traj = agent._trajectories
    p0 = agent.policy_model.params.cpu().numpy()
    b = batches[5]
    idx = b.idx.cpu().numpy().astype(np.int64)
    obs = traj.observations.cpu().numpy()[idx]
    args = [traj.actions.cpu().numpy()[idx], traj.logprobs.cpu().numpy()[idx], traj.values.cpu().numpy()[idx],
            traj.advantages.cpu().numpy()[idx], traj.returns.cpu().numpy()[idx]]
    pm = agent.policy_model
    dims = (pm.obs_dim, pm.hidden_dims[0], pm.hidden_dims[1], pm.n_actions)
    loss, met, g = R.ppo_loss_and_grads(p0, dims, obs, *args, clip=cfg.clip_range, clip_vf=cfg.clip_range_vf,
                                        vf_coef=cfg.vf_coef, ent_coef=cfg.ent_coef)
    gc, total = R.clip_grad_norm(g, dims, cfg.max_grad_norm)
    p1, _, _ = R.adam_step(p0, gc, np.zeros_like(gc), np.zeros_like(gc), 1, cfg.policy_lr)
    agent.training_step(b, 0)
    torch.cuda.synchronize()
    rec = agent.metrics_buf[0].cpu().numpy()
    np.testing.assert_allclose(rec[0], loss, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(agent.grads.cpu().numpy(), gc, atol=1e-6 * max(1, np.abs(gc).max()), rtol=0)
    np.testing.assert_allclose(agent.policy_model.params.cpu().numpy(), p1, atol=5e-6, rtol=0)


@pytest.mark.parametrize("use_graph", [False, True])
def test_update_first_minibatches_vs_numpy_oracle(cuda, use_graph):
    """The default update chain at the full C2 size (4096 envs x 32 steps, the lagged fused
    chain: each minibatch's clip + Adam inside the next forward) over the first 8 minibatches of
    the sampler stream, against 8 sequential numpy-oracle steps on the same rows: every
    minibatch loss within 1e-5 relative, the parameters after the 8th step within 1e-5
    relative L2 (Adam turns last-bit gradient differences of near-zero-gradient weights into up
    to lr-sized moves, hence the norm bar)."""
    from oracle import ppo_ref as R
    from gsamd._lib import check, lib
    from gsamd.config import load_config
    from gsamd.ppo_agent import DevicePPOAgent
    torch.manual_seed(42)
    cfg = load_config("CartPole-v1", "ppo", overrides=dict(env_dynamics="synthetic", n_envs=4096))
    agent = DevicePPOAgent(cfg, device=cuda, use_graph=use_graph, track_stats=False)
    agent.train_dataloader()
    traj = agent._trajectories
    coll = agent.get_rollout_collector("train")
    idx_dev = agent.prefetcher.upload(0)
    pm = agent.policy_model
    dims = (pm.obs_dim, pm.hidden_dims[0], pm.hidden_dims[1], pm.n_actions)
    p = pm.params.cpu().numpy()
    n, B = 8, agent.batch_size
    from gsamd._lib import GS_HP_ACT_STATS, ACT_SLOT
    hp = agent.hparams()
    hp.flags |= GS_HP_ACT_STATS          # every minibatch's activation statistics into its record
    check(lib.gs_ppo_update(pm.params.data_ptr(), agent.grads.data_ptr(), agent.adam_m.data_ptr(),
                            agent.adam_v.data_ptr(), pm.dims, hp, coll.buffer.view(), idx_dev.data_ptr(),
                            B, n, 0, agent.metrics_buf.data_ptr(), agent.stop_flag.data_ptr(),
                            agent.workspace.data_ptr(), agent.workspace.numel(), None, 1 if use_graph else 0,
                            torch.cuda.current_stream().cuda_stream), "gs_ppo_update")
    torch.cuda.synchronize()
    losses = agent.metrics_buf[:n, 0].cpu().numpy()
    stream = idx_dev.cpu().numpy().astype(np.int64)
    fields = [traj.observations.cpu().numpy(), traj.actions.cpu().numpy(), traj.logprobs.cpu().numpy(),
              traj.values.cpu().numpy(), traj.advantages.cpu().numpy(), traj.returns.cpu().numpy()]
    m = np.zeros_like(p)
    v = np.zeros_like(p)
    from gsamd._lib import M
    rec = agent.metrics_buf[:n].cpu().numpy()
    D_, H1, H2, A_ = dims
    o_pol = H1 * D_ + H1 + H2 * H1 + H2
    o_val = o_pol + A_ * H2 + A_
    for k in range(n):
        rows = stream[k * B:(k + 1) * B]
        loss, _, g = R.ppo_loss_and_grads(p, dims, *(f[rows] for f in fields), clip=cfg.clip_range,
                                          clip_vf=cfg.clip_range_vf, vf_coef=cfg.vf_coef, ent_coef=cfg.ent_coef)
        np.testing.assert_allclose(losses[k], loss, rtol=1e-5, atol=1e-6, err_msg=f"minibatch {k}")
        # the forward hooks' statistics of this step's rows under the parameters its loss used
        # (utils/models.py:121-147): mean / std 1e-5, dead fractions 1/B
        st = R.activation_stats(p, dims, fields[0][rows])
        got = rec[k, ACT_SLOT:ACT_SLOT + 8]
        for j in range(8):
            tol = 1.0 / B if j % 4 >= 2 else 1e-5 * (1.0 + abs(st[j]))
            assert abs(got[j] - st[j]) <= tol, (k, j, got[j], st[j])
        # per-component pre-clip norms (utils/models.py:196-230), written by the next forward's
        # lagged step (the last one by k_clip_adam)
        g64 = g.astype(np.float64)
        for slot, part in (("gn_backbone", g64[:o_pol]), ("gn_policy_head", g64[o_pol:o_val]),
                           ("gn_value_head", g64[o_val:])):
            np.testing.assert_allclose(rec[k, M[slot]], np.linalg.norm(part), rtol=2e-5, err_msg=f"{slot} {k}")
        gc, _ = R.clip_grad_norm(g, dims, cfg.max_grad_norm)
        p, m, v = R.adam_step(p, gc, m, v, k + 1, cfg.policy_lr)
    p_dev = pm.params.cpu().numpy().astype(np.float64)
    assert np.linalg.norm(p_dev - p) / np.linalg.norm(p) < 1e-5
    assert np.abs(p_dev - p).max() < 1e-3


@pytest.mark.parametrize("env,variant,n_envs", CASES)
@pytest.mark.parametrize("use_graph", [False, True])
def test_fused_update_chain_equals_unfused(cuda, env, variant, n_envs, use_graph):
    """gs_ppo_update's fused chain (gathered fields, head combine + loss rows inside the
    forward) against the 4-launch chain on the same rollout: bit-identical parameters and
    minibatch losses within 1e-6 relative (metric sums are added in another order)."""
    from gsamd._lib import ACT_SLOT, GS_HP_ACT_STATS, check, lib
    from gsamd.config import load_config
    from gsamd.ppo_agent import DevicePPOAgent
    out = []
    for fused in (True, False):
        torch.manual_seed(42)
        cfg = load_config(env, variant, overrides=dict(env_dynamics="synthetic", n_envs=n_envs // 8 if env == "CartPole-v1" else n_envs,
                                                       n_epochs=2))
        agent = DevicePPOAgent(cfg, device=cuda, use_graph=use_graph, track_stats=False)
        coll = agent.get_rollout_collector("train")
        coll.collect()
        idx = agent.prefetcher.upload(0)
        small = int(lib.gs_ppo_workspace_bytes(agent.policy_model.dims, agent.batch_size))
        assert agent.workspace.numel() > small      # the BASELINE shapes have a fused chain
        hp = agent.hparams()
        hp.flags |= GS_HP_ACT_STATS      # both chains record the activation statistics
        check(lib.gs_ppo_update(agent.policy_model.params.data_ptr(), agent.grads.data_ptr(), agent.adam_m.data_ptr(),
                                agent.adam_v.data_ptr(), agent.policy_model.dims, hp, coll.buffer.view(),
                                idx.data_ptr(), agent.batch_size, agent.n_minibatches, 0, agent.metrics_buf.data_ptr(),
                                agent.stop_flag.data_ptr(), agent.workspace.data_ptr(),
                                agent.workspace.numel() if fused else small, None, 1 if use_graph else 0,
                                torch.cuda.current_stream().cuda_stream), "gs_ppo_update")
        torch.cuda.synchronize()
        rec = agent.metrics_buf.cpu().numpy()
        out.append((agent.policy_model.params.cpu().numpy(), rec))
        del agent
    (p0, m0), (p1, m1) = out
    assert np.array_equal(p0.view(np.uint32), p1.view(np.uint32))
    # per-component gradient norms: the fused chain sums role C's fp32 head sums per step, the
    # 4-launch chain re-reads the head gradients in double (k_component_norms)
    from gsamd._lib import M
    gn = [M[k] for k in ("gn_backbone", "gn_policy_head", "gn_value_head")]
    act = list(range(ACT_SLOT, ACT_SLOT + 8))
    rest = [c for c in range(m0.shape[1]) if c not in gn + act]
    np.testing.assert_allclose(m0[:, rest], m1[:, rest], rtol=1e-6, atol=1e-7)
    # activation statistics: the fused forward's epilogue (float partial sums per workgroup, its
    # MFMA's z2) against the unfused chain's k_mlp_act_stats (double sums, sequential z2)
    B = 256 if env == "CartPole-v1" else 64
    assert np.abs(m0[:, act]).sum() > 0
    for j, c in enumerate(act):
        tol = 1.0 / B if j % 4 >= 2 else 1e-5 * (1.0 + np.abs(m1[:, c]))
        assert (np.abs(m0[:, c] - m1[:, c]) <= tol).all(), (c, np.abs(m0[:, c] - m1[:, c]).max())
    bad = np.argwhere(~np.isclose(m0[:, gn], m1[:, gn], rtol=1e-4, atol=1e-7))
    assert len(bad) == 0, [(int(r), gn[c], m0[r], m1[r]) for r, c in bad[:4]]


@pytest.mark.parametrize("transport", ["rccl", "xgmi"])
@pytest.mark.parametrize("use_graph", [False, True])
def test_comm_update_path_matches_single_gpu(cuda, use_graph, transport):
    """The multi-GPU kernel chain (dW1 partial fold -> exchange over a one-rank communicator
    (RCCL all-reduce, or the xGMI exchange kernel) -> flat norm -> clip+Adam scaled by 1/G)
    gives the single-GPU update: identical losses for the
    first minibatch, losses within 1e-4 (the north-star bar) after one rollout x 2 epochs = 128
    minibatch steps, final params within 1e-3 relative L2.  The clip norm's summation order
    differs between the chains, so the two trajectories drift apart at ulp level; Adam turns
    that into up to ±lr per step on parameters whose gradient is near zero (m/sqrt(v) ≈ ±1),
    which is why the parameter bar is looser than the loss bar."""
    from gsamd.config import load_config
    from gsamd.distributed import destroy_comm, init_local_comm
    from gsamd.ppo_agent import DevicePPOAgent
    out = []
    for with_comm in (False, True):
        comm = init_local_comm(transport, 70_000) if with_comm else None
        torch.manual_seed(42)
        cfg = load_config("CartPole-v1", "ppo", overrides=dict(env_dynamics="synthetic", n_envs=512, n_epochs=2))
        agent = DevicePPOAgent(cfg, device=cuda, use_graph=use_graph, track_stats=False, comm=comm)
        agent.train_epoch()
        torch.cuda.synchronize()
        out.append((agent.policy_model.params.cpu().numpy().astype(np.float64), agent.minibatch_losses()))
        del agent
        destroy_comm(comm)
    (p0, l0), (p1, l1) = out
    assert np.isfinite(l1).all()
    assert l0[0] == l1[0]
    np.testing.assert_allclose(l1, l0, rtol=1e-4, atol=1e-5)
    assert np.linalg.norm(p1 - p0) / np.linalg.norm(p0) < 1e-3
