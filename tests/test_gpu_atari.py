"""GPU: the Atari pixel path (a13) bit-exact against oracle/atari_ref.py, and the pixel PPO
agent (C4/C5 shapes, NatureCNN + masked actions) end to end.  Tolerances as
tests/test_gpu_cnn.py; preprocessing and the env twin are integer work: bit-exact."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_atari_preprocess_bit_exact(cuda):
    from oracle import atari_ref as A
    from gsamd.atari_env import atari_preprocess
    fr = A.render(42, np.arange(5), 3)
    rng = np.random.default_rng(0)
    noise = rng.integers(0, 256, (3, 2, 210, 160, 3), dtype=np.uint8)
    flat = np.zeros((1, 2, 210, 160, 3), np.uint8)
    flat[0, 0, 100:150, 30:90] = [200, 40, 90]      # a sprite in one of the two frames only
    for frames in (fr, noise, flat):
        dev = atari_preprocess(torch.as_tensor(frames).to(cuda).contiguous())
        torch.cuda.synchronize()
        assert np.array_equal(dev.cpu().numpy(), A.preprocess(frames))


def test_device_atari_env_matches_twin(cuda):
    from oracle import atari_ref as A
    from gsamd.atari_env import DeviceAtariVecEnv
    env = DeviceAtariVecEnv(6, episode_len=5, seed=42, truncate_every=2, env_offset=3, device=cuda)
    twin = A.AtariEnvTwin(6, seed=42, env_offset=3, episode_len=5, truncate_every=2)
    env.reset()
    torch.cuda.synchronize()
    assert np.array_equal(env.obs.cpu().numpy(), twin.stack)
    r = torch.zeros(6, device=cuda)
    d = torch.zeros(6, dtype=torch.uint8, device=cuda)
    to = torch.zeros(6, dtype=torch.uint8, device=cuda)
    for _ in range(12):
        env.step_into(r, d, to)
        rr, dd, tt = twin.step()
        torch.cuda.synchronize()
        assert np.array_equal(r.cpu().numpy().view(np.uint32), rr.view(np.uint32))
        assert np.array_equal(d.cpu().numpy().astype(bool), dd)
        assert np.array_equal(to.cpu().numpy().astype(bool), tt)
        assert np.array_equal(env.obs.cpu().numpy(), twin.stack)


def _pixel_agent(cuda, **over):
    from gsamd.config import load_config
    from gsamd.ppo_agent import DevicePPOAgent
    torch.manual_seed(42)
    cfg = load_config("ALE-Pong-v5", "rgb_ppo", overrides=dict(dict(env_dynamics="synthetic", n_envs=8, n_steps=16, batch_size=64, n_epochs=2),
                                                                **over))
    return cfg, DevicePPOAgent(cfg, device=cuda, track_stats=True)


def test_pixel_agent_minibatch_vs_oracle(cuda):
    """First minibatch of a device Atari rollout through the CNN step vs the torch-CPU oracle."""
    from oracle import cnn_ref as C
    cfg, agent = _pixel_agent(cuda)
    batches = agent.train_dataloader()
    traj = agent._trajectories
    pm = agent.policy_model
    p0 = pm.flat_to_reference(pm.params)
    b = batches[3]
    idx = b.idx.cpu().numpy().astype(np.int64)
    obs = traj.observations.cpu().numpy()[idx]
    args = [traj.actions.cpu().numpy()[idx], traj.logprobs.cpu().numpy()[idx], traj.values.cpu().numpy()[idx],
            traj.advantages.cpu().numpy()[idx], traj.returns.cpu().numpy()[idx]]
    assert set(np.unique(args[0])) <= set(cfg.valid_actions)
    shapes = C.cnn_param_shapes()
    logits, values, _ = C.forward(C.unflatten(p0, shapes), obs, cfg.valid_actions)
    ln = (logits - torch.logsumexp(logits, -1, keepdim=True)).numpy()
    np.testing.assert_allclose(args[1], ln[np.arange(len(idx)), args[0]], atol=1e-5, rtol=0)   # rollout logp
    np.testing.assert_allclose(args[2], values.numpy(), atol=1e-5, rtol=0)
    loss, met, g = C.loss_and_grads(p0, shapes, obs, *args, valid=cfg.valid_actions, clip=cfg.clip_range,
                                    clip_vf=cfg.clip_range_vf, vf_coef=cfg.vf_coef, ent_coef=cfg.ent_coef)[:3]
    P = p0.size
    _, _, _, gc, total = C.clip_and_adam(p0, g, shapes, np.zeros(P, np.float32), np.zeros(P, np.float32), 1,
                                         cfg.policy_lr)
    agent.training_step(b, 0)
    torch.cuda.synchronize()
    rec = agent.metrics_buf[0].cpu().numpy()
    assert abs(rec[0] - loss) < 1e-5 * max(1.0, abs(loss))
    assert abs(rec[12] - total) < 1e-5 * total
    np.testing.assert_allclose(pm.flat_to_reference(agent.grads), gc, atol=2e-5 * np.abs(gc).max(), rtol=0)


def test_pixel_agent_epochs_deterministic(cuda):
    out = []
    for _ in range(2):
        cfg, agent = _pixel_agent(cuda)
        agent.train_epoch()
        agent.train_epoch()
        torch.cuda.synchronize()
        out.append((agent.policy_model.params.cpu().numpy(), agent.minibatch_losses(), agent.epoch_metrics(),
                    agent.get_rollout_collector("train").get_metrics()))
        del agent
    (p0, l0, m0, r0), (p1, l1, _, _) = out
    assert np.isfinite(l0).all()
    assert np.array_equal(p0.view(np.uint32), p1.view(np.uint32)) and np.array_equal(l0, l1)
    assert "opt/loss/total" in m0 and "roll/obs/mean" in r0 and 0 <= r0["roll/obs/mean"] <= 255
