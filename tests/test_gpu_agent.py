"""GPU: agent-level surface — checkpoint files in the reference's format (agents/base_agent.py:
658-885) round-trip bit-exactly for both policy families, and device evaluate_episodes
(utils/rollout_collector.py:570-655) returns the reference's keys and episode counts."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _agent(cuda, env="CartPole-v1", variant="ppo", seed=42, **over):
    from gsamd.config import load_config
    from gsamd.ppo_agent import DevicePPOAgent
    torch.manual_seed(seed)
    base = dict(n_envs=64, n_epochs=2) if variant == "ppo" else dict(n_envs=8, n_steps=16, batch_size=64, n_epochs=1)
    cfg = load_config(env, variant, overrides=dict(dict(base, env_dynamics="synthetic"), **over))
    return DevicePPOAgent(cfg, device=cuda, track_stats=False)


@pytest.mark.parametrize("env,variant", [("CartPole-v1", "ppo"), ("ALE-Pong-v5", "rgb_ppo")])
def test_checkpoint_round_trip(cuda, tmp_path, env, variant):
    a = _agent(cuda, env, variant)
    a.train_epoch()
    torch.cuda.synchronize()
    a.set_hyperparameter("policy_lr", 5e-4)        # e.g. where a schedule had moved it
    a.set_hyperparameter("clip_range", 0.15)
    a.save_checkpoint(tmp_path)
    sd = torch.load(tmp_path / "model.pt", map_location="cpu", weights_only=True)
    assert list(sd) == [n for n, _ in a.policy_model.shapes()]
    assert all(tuple(sd[n].shape) == tuple(s) for n, s in a.policy_model.shapes())
    opt = torch.load(tmp_path / "optimizer.pt", map_location="cpu", weights_only=True)
    assert isinstance(opt, list) and set(opt[0]) == {"state", "param_groups"}
    assert len(opt[0]["state"]) == len(sd)
    b = _agent(cuda, env, variant, seed=7)
    assert not torch.equal(a.policy_model.params, b.policy_model.params)
    b.load_checkpoint(tmp_path)
    torch.cuda.synchronize()
    for x, y in ((a.policy_model.params, b.policy_model.params), (a.adam_m, b.adam_m), (a.adam_v, b.adam_v)):
        assert torch.equal(x, y)
    assert b.adam_step == a.adam_step and b.current_epoch == a.current_epoch
    assert b.policy_lr == 5e-4 and b.clip_range == 0.15      # resumed with the values in effect
    assert b.get_rollout_collector("train").total_steps == a.get_rollout_collector("train").total_steps
    # the state_dict is the reference's layout (the CNN stores conv2/3 and fc permuted inside)
    for n, t in b.policy_model.state_dict().items():
        assert torch.equal(t, sd[n])


def test_evaluate_episodes_keys_and_counts(cuda):
    a = _agent(cuda, episode_len=9)
    out = a.get_rollout_collector("val").evaluate_episodes(n_episodes=100, deterministic=True)
    assert out["cnt/total_episodes"] == 100
    assert {"roll/ep_rew/mean", "roll/ep_len/mean", "cnt/total_env_steps", "cnt/total_vec_steps"} <= set(out)
    assert 1 <= out["roll/ep_len/mean"] <= 9 and out["roll/ep_rew/mean"] == pytest.approx(out["roll/ep_len/mean"])


def test_device_cartpole_matches_numpy_twin(cuda):
    """f1: device CartPole-v1 dynamics vs the float64 numpy restatement over 300 steps of
    random actions (done/reward rows exact; observations to 1e-5: device cos/sin are not
    glibc's correctly rounded ones)."""
    from oracle.cartpole_ref import CartPoleTwin
    from gsamd.rollout import DeviceCartPoleVecEnv
    N = 64
    env = DeviceCartPoleVecEnv(N, seed=3, env_offset=5, max_steps=60, device=cuda)
    twin = CartPoleTwin(N, seed=3, env_offset=5, max_steps=60)
    env.reset()
    rng = np.random.default_rng(0)
    r = torch.zeros(N, device=cuda)
    d = torch.zeros(N, dtype=torch.uint8, device=cuda)
    to = torch.zeros(N, dtype=torch.uint8, device=cuda)
    n_done = 0
    for _ in range(300):
        a = rng.integers(0, 2, N)
        env.step_into(r, d, to, actions=torch.as_tensor(a).to(cuda))
        rr, dd, tt = twin.step(a)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(d.cpu().numpy().astype(bool), dd)
        np.testing.assert_array_equal(to.cpu().numpy().astype(bool), tt)
        np.testing.assert_array_equal(r.cpu().numpy(), rr)
        np.testing.assert_allclose(env.obs.cpu().numpy(), twin.obs(), atol=1e-5, rtol=0)
        n_done += int(dd.sum())
    assert n_done > N     # episodes ended by both termination and truncation


def test_agent_trains_on_device_cartpole(cuda):
    a = _agent(cuda, env_dynamics="cartpole")
    for _ in range(3):
        a.train_epoch()
    torch.cuda.synchronize()
    assert np.isfinite(a.minibatch_losses()).all()
    m = a.get_rollout_collector("train").get_metrics()
    assert m["cnt/total_episodes"] > 0 and m["roll/ep_len/mean"] > 0


def test_schedules_applied_between_epochs(cuda):
    """A cosine policy_lr schedule and a linear ent_coef schedule move the next epoch's kernel
    arguments exactly as HyperparameterSchedulerCallback.on_train_epoch_end would;
    a manual set_hyperparameter wins until the next epoch end."""
    import torch
    from gsamd.config import load_config
    from gsamd.ppo_agent import DevicePPOAgent
    from gsamd.schedules import build_schedulers
    torch.manual_seed(42)
    cfg = load_config("CartPole-v1", "ppo", overrides=dict(env_dynamics="synthetic", n_envs=8, n_epochs=1, max_env_steps=8 * 32 * 4))
    cfg.schedules = {"policy_lr": {"schedule": "cosine", "start_value": 1e-3, "end_value": 1e-4, "start": 0.0,
                                   "end": 1.0, "warmup": 0.0},
                     "ent_coef": {"schedule": "linear", "start_value": 0.02, "end_value": 0.0, "start": 0.25,
                                  "end": 0.75, "warmup": 0.0}}
    agent = DevicePPOAgent(cfg, device=cuda, track_stats=False)
    ref = {s.parameter: s for s in build_schedulers(cfg.schedules, cfg.max_env_steps, cfg.n_envs)}
    for epoch in range(4):
        agent.train_epoch()
        t = agent.get_rollout_collector("train").total_vec_steps
        assert t == 32 * (epoch + 1)
        hp = agent.hparams()
        assert hp.lr == float(np.float32(ref["policy_lr"].value(t)))          # kernel args are f32
        assert hp.ent_coef == float(np.float32(ref["ent_coef"].value(t)))
    assert abs(agent.policy_lr - 1e-4) < 1e-12            # the schedule's end
    agent.set_hyperparameter("clip_range", 0.15)
    assert abs(agent.hparams().clip_range - 0.15) < 1e-7 and cfg.clip_range == 0.15
    assert np.isfinite(agent.minibatch_losses()).all()


def test_scheduled_lr_reuses_the_update_graph(cuda):
    """a policy_lr schedule changes lr every epoch; the captured update graph must be
    replayed (lr reaches it through the per-step table), not re-captured, and device memory must
    not grow.  A scheduled clip_range re-captures in place (same entry count)."""
    import ctypes
    from gsamd._lib import lib
    from gsamd.config import load_config
    from gsamd.ppo_agent import DevicePPOAgent

    def info():
        n, c = ctypes.c_int64(), ctypes.c_int64()
        assert lib.gs_ppo_graph_cache_info(ctypes.byref(n), ctypes.byref(c)) == 0
        return n.value, c.value

    torch.manual_seed(42)
    cfg = load_config("CartPole-v1", "ppo", overrides=dict(env_dynamics="synthetic", n_envs=64, n_epochs=1, max_env_steps=64 * 32 * 8))
    cfg.schedules = {"policy_lr": {"schedule": "linear", "start_value": 1e-3, "end_value": 1e-4, "start": 0.0,
                                   "end": 1.0, "warmup": 0.0}}
    agent = DevicePPOAgent(cfg, device=cuda, track_stats=False)
    agent.train_epoch()
    agent.train_epoch()        # the rollout graph is captured on the second rollout
    torch.cuda.synchronize()
    n0, c0 = info()
    mem0 = torch.cuda.memory_allocated()
    lrs = []
    for _ in range(3):
        lrs.append(agent.hparams().lr)
        agent.train_epoch()
    torch.cuda.synchronize()
    assert len(set(lrs)) == 3                     # the schedule really moved lr
    assert info() == (n0, c0)                     # no new entry, no re-capture
    assert torch.cuda.memory_allocated() == mem0
    # a baked hyper-parameter change re-captures into the same entry
    agent.set_hyperparameter("clip_range", 0.15)
    agent.train_epoch()
    torch.cuda.synchronize()
    assert info() == (n0, c0 + 1)
    assert np.isfinite(agent.minibatch_losses()).all()


@pytest.mark.parametrize("env,variant,over", [
    ("CartPole-v1", "ppo", dict(n_envs=256)),
    ("CartPole-v1", "ppo", dict(n_envs=128, env_dynamics="cartpole")),
    ("LunarLander-v3", "ppo", dict(n_envs=64, n_steps=256, batch_size=64)),
    ("ALE-Breakout-v5", "rgb_ppo", dict(n_envs=8, n_steps=16, batch_size=64, n_epochs=1))])
def test_rollout_graph_equals_eager(cuda, env, variant, over):
    """The captured T-step rollout (policy act + env step per vector step, replayed with the
    rollout clock) writes bit for bit the rollout of the eager per-step launches — sampled and
    deterministic actions, over several rollouts, between updates that move the weights."""
    from gsamd.config import load_config
    from gsamd.ppo_agent import DevicePPOAgent
    runs = []
    for use_graph in (False, True):
        torch.manual_seed(42)
        cfg = load_config(env, variant, overrides=dict({"env_dynamics": "synthetic"}, **over))
        agent = DevicePPOAgent(cfg, device=cuda, use_graph=use_graph, track_stats=True, one_launch=False)
        coll = agent.get_rollout_collector("train")
        rec = []
        for k in range(4):
            agent.train_epoch()
            b = coll.buffer
            rec.append([t.clone() for t in (b.obs, b.actions, b.logprobs, b.values, b.rewards, b.dones, b.timeouts,
                                            b.advantages, b.returns)])
        coll.collect(deterministic=True)
        coll.collect(deterministic=True)
        rec.append([coll.buffer.actions.clone(), coll.buffer.values.clone()])
        torch.cuda.synchronize()
        runs.append((rec, coll.get_metrics(), coll.total_vec_steps))
        assert (coll._graphs.get(0) is not None) == use_graph
        del agent
    (r0, m0, n0), (r1, m1, n1) = runs
    assert n0 == n1
    for k, (a, b) in enumerate(zip(r0, r1)):
        for x, y in zip(a, b):
            assert torch.equal(x, y), k
    assert m0["cnt/total_episodes"] == m1["cnt/total_episodes"]
    assert m0.get("roll/ep_rew/mean") == m1.get("roll/ep_rew/mean")


@pytest.mark.parametrize("env,variant,over", [
    ("LunarLander-v3", "ppo", dict(n_envs=72, n_steps=96, batch_size=64, n_epochs=2)),
    ("CartPole-v1", "ppo", dict(n_envs=40, n_steps=64, batch_size=64, n_epochs=2, model_id="mlp_small"))])
def test_one_launch_rollout_equals_step_loop(cuda, env, variant, over):
    """gs_rollout_synth (the whole rollout in one launch, envs resident in LDS) writes bit for bit
    the rows of the per-step loop (gs_policy_act + gs_env_step launches): sampled, deterministic
    and replayed actions, over rollouts separated by updates, a ragged last workgroup (N % 16 != 0),
    and leaves the same env state, observations and episode counters."""
    from gsamd.config import load_config
    from gsamd.ppo_agent import DevicePPOAgent
    runs = []
    for one in (False, True):
        torch.manual_seed(42)
        cfg = load_config(env, variant, overrides=dict({"env_dynamics": "synthetic"}, **over))
        agent = DevicePPOAgent(cfg, device=cuda, use_graph=False, track_stats=True, one_launch=one)
        coll = agent.get_rollout_collector("train")
        assert coll.one_launch == one
        rec = []
        for k in range(3):
            agent.train_epoch()
            b = coll.buffer
            rec.append([t.clone() for t in (b.obs, b.actions, b.logprobs, b.values, b.rewards, b.dones, b.timeouts,
                                            b.advantages, b.returns)])
        coll.collect(deterministic=True)
        rec.append([t.clone() for t in (coll.buffer.actions, coll.buffer.logprobs, coll.buffer.values)])
        replay = torch.randint(0, coll.env.n_actions, coll.buffer.actions.shape, device=coll.buffer.actions.device,
                               generator=torch.Generator(device=coll.buffer.actions.device).manual_seed(7))
        coll.collect(replay_actions=replay)
        rec.append([t.clone() for t in (coll.buffer.actions, coll.buffer.logprobs, coll.buffer.values)])
        e = coll.env
        rec.append([t.clone() for t in (e.state, e.ep_ret, e.obs, e.ep_count, e.ep_ret_sum, e.ep_len_sum)])
        torch.cuda.synchronize()
        runs.append((rec, coll.get_metrics(), coll.total_vec_steps, e.step_count))
        del agent
    (r0, m0, n0, s0), (r1, m1, n1, s1) = runs
    assert (n0, s0) == (n1, s1)
    for k, (a, b) in enumerate(zip(r0, r1)):
        for j, (x, y) in enumerate(zip(a, b)):
            assert torch.equal(x, y), (k, j)
    assert m0["cnt/total_episodes"] == m1["cnt/total_episodes"]


@pytest.mark.parametrize("over", [dict(n_envs=256, episode_len=50), dict(n_envs=8, episode_len=7)])
def test_untracked_collector_keeps_the_rolling_window(cuda, over):
    """track_stats=False (the bench path) still reports the reference's rolling window
    (rollout_collector.py:242-294, 753-758: the last 100 finished episodes, best and last episode),
    kept on the device: equal to the tracked collector's host deques over several rollouts, with
    many episodes per rollout (256 envs) and with fewer than the window per rollout (8 envs)."""
    from gsamd.config import load_config
    from gsamd.ppo_agent import DevicePPOAgent
    out = []
    for track in (True, False):
        torch.manual_seed(42)
        cfg = load_config("CartPole-v1", "ppo", overrides=dict(env_dynamics="synthetic", n_epochs=1, **over))
        agent = DevicePPOAgent(cfg, device=cuda, use_graph=False, track_stats=track)
        coll = agent.get_rollout_collector("train")
        ms = []
        for _ in range(4):
            agent.train_epoch()
            ms.append(coll.get_metrics())
        out.append(ms)
        del agent
    for mt, mu in zip(*out):
        assert mt["cnt/total_episodes"] == mu["cnt/total_episodes"]
        for k in ("roll/ep_rew/mean", "roll/ep_rew/best", "roll/ep_rew/last", "roll/ep_len/mean", "roll/ep_len/last"):
            assert (k in mt) == (k in mu), k
            if k in mt:
                np.testing.assert_allclose(mu[k], mt[k], rtol=1e-6, atol=1e-6, err_msg=k)


@pytest.mark.parametrize("shape,p,W", [((32, 4096), 0.01, 100), ((32, 4096), 0.3, 2048), ((7, 33), 0.2, 5),
                                       ((3, 7), 0.5, 1), ((1, 1), 1.0, 3), ((2048, 64), 0.02, 100),
                                       ((512, 1024), 0.01, 100), ((4, 16), 0.5, 7), ((1, 16), 0.0, 4)])
def test_episode_window_kernel_vs_model(cuda, shape, p, W):
    """gs_episode_window (the track_stats=False rolling window, rollout_collector.py:242-294,
    753-758) against its definition: the window is the last W entries of (previous window ++ this
    rollout's finished episodes in (step, env) order), meta = {count so far, best return}; three
    calls in a row carry the window, with negative returns, a ragged sample count (n % 4 != 0) and
    a dones buffer at an odd address (the scalar path of the kernel's 4-sample groups)."""
    from gsamd._lib import check, lib, ptr, stream_handle
    T, N = shape
    rng = np.random.default_rng(T * 1000 + N)
    win = torch.zeros(2, W, dtype=torch.float64, device=cuda)
    meta = torch.tensor([0.0, -np.inf, 0.0], dtype=torch.float64, device=cuda)
    tot = torch.zeros((), dtype=torch.int64, device=cuda)
    m_win, m_cnt, m_best = np.zeros((2, W)), 0.0, -np.inf
    for call in range(3):
        d = (rng.random((T, N)) < p).astype(np.uint8)
        r = (rng.standard_normal((T, N)) * 50).astype(np.float32)
        ln = rng.integers(1, 500, (T, N)).astype(np.int32)
        if call == 2:                      # odd address: the scalar path
            dd = torch.zeros(T * N + 1, dtype=torch.uint8, device=cuda)
            dd[1:] = torch.as_tensor(d.reshape(-1)).to(cuda)
            dv = dd[1:]
        else:
            dv = torch.as_tensor(d).to(cuda)
        rt, lt = torch.as_tensor(r).to(cuda), torch.as_tensor(ln).to(cuda)
        check(lib.gs_episode_window(ptr(dv), ptr(rt), ptr(lt), T, N, W, ptr(win), ptr(meta), ptr(tot),
                                    stream_handle()), "gs_episode_window")
        torch.cuda.synchronize()
        at = np.flatnonzero(d.reshape(-1))
        m_win = np.concatenate([m_win, np.stack([r.reshape(-1)[at].astype(np.float64),
                                                 ln.reshape(-1)[at].astype(np.float64)])], axis=1)[:, -W:]
        m_cnt += at.size
        if at.size:
            m_best = max(m_best, float(r.reshape(-1)[at].max()))
        assert int(tot.item()) == at.size
        np.testing.assert_array_equal(win.cpu().numpy(), m_win)
        mm = meta.cpu().numpy()
        assert mm[0] == m_cnt and mm[1] == m_best
