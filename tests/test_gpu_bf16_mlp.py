"""GPU: the MLP update's bf16 mode (precision: bf16, GS_HP_BF16) — bf16 MFMA operands in the fused
chain's hidden-to-hidden product, its weight / input gradients and the head-weight gradient, fp32
accumulation, parameters, moments, loss, clip and Adam (DESIGN.md §3 Precision modes).

Bars (written per test): against the bf16 emulation of the numpy oracle (oracle/ppo_ref.py
bf16=True: the operands rounded where the kernels round them), per-minibatch losses within 1e-4
relative and the parameters after 8 lagged-Adam steps within 1e-4 relative L2 — products of bf16
operands are exact in fp32, so what remains is the accumulation order and the odd bf16 rounding
of an h1 / dh2 value the device and numpy compute 1 ulp apart; the device must also sit far
closer to the bf16 emulation than to the fp32 oracle (the mode really rounds).  Against the fp32
path: the mode's whole-update loss deviation bounded (the line bench.py --dtype bf16 reports)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _agent(cuda, precision, n_envs=4096, **over):
    from gsamd.config import load_config
    from gsamd.ppo_agent import DevicePPOAgent
    torch.manual_seed(42)
    cfg = load_config("CartPole-v1", "ppo", overrides=dict(env_dynamics="synthetic", n_envs=n_envs,
                                                           precision=precision, **over))
    return cfg, DevicePPOAgent(cfg, device=cuda, track_stats=False)


@pytest.mark.parametrize("use_graph", [False, True])
def test_mlp_bf16_chain_vs_bf16_oracle(cuda, use_graph):
    from oracle import ppo_ref as R
    from gsamd._lib import check, lib
    cfg, agent = _agent(cuda, "bf16")
    agent.train_dataloader()
    traj = agent._trajectories
    coll = agent.get_rollout_collector("train")
    idx_dev = agent.prefetcher.upload(0)
    pm = agent.policy_model
    dims = (pm.obs_dim, pm.hidden_dims[0], pm.hidden_dims[1], pm.n_actions)
    p0 = pm.params.cpu().numpy()
    n, B = 8, agent.batch_size
    hp = agent.hparams()
    assert hp.flags == 1
    check(lib.gs_ppo_update(pm.params.data_ptr(), agent.grads.data_ptr(), agent.adam_m.data_ptr(),
                            agent.adam_v.data_ptr(), pm.dims, hp, coll.buffer.view(), idx_dev.data_ptr(), B, n, 0,
                            agent.metrics_buf.data_ptr(), agent.stop_flag.data_ptr(), agent.workspace.data_ptr(),
                            agent.workspace.numel(), None, 1 if use_graph else 0,
                            torch.cuda.current_stream().cuda_stream), "gs_ppo_update")
    torch.cuda.synchronize()
    losses = agent.metrics_buf[:n, 0].cpu().numpy()
    stream = idx_dev.cpu().numpy().astype(np.int64)
    fields = [traj.observations.cpu().numpy(), traj.actions.cpu().numpy(), traj.logprobs.cpu().numpy(),
              traj.values.cpu().numpy(), traj.advantages.cpu().numpy(), traj.returns.cpu().numpy()]
    ref = {}
    for bf in (True, False):
        p, m, v = p0.copy(), np.zeros_like(p0), np.zeros_like(p0)
        ls = []
        for k in range(n):
            rows = stream[k * B:(k + 1) * B]
            loss, _, g = R.ppo_loss_and_grads(p, dims, *(f[rows] for f in fields), clip=cfg.clip_range,
                                              clip_vf=cfg.clip_range_vf, vf_coef=cfg.vf_coef, ent_coef=cfg.ent_coef,
                                              bf16=bf)
            ls.append(loss)
            gc, _ = R.clip_grad_norm(g, dims, cfg.max_grad_norm)
            p, m, v = R.adam_step(p, gc, m, v, k + 1, cfg.policy_lr)
        ref[bf] = (np.array(ls), p.astype(np.float64))
    l16, p16 = ref[True]
    _, p32 = ref[False]
    np.testing.assert_allclose(losses, l16, rtol=1e-4, atol=1e-6)
    p_dev = pm.params.cpu().numpy().astype(np.float64)
    d16 = np.linalg.norm(p_dev - p16) / np.linalg.norm(p16)
    d32 = np.linalg.norm(p_dev - p32) / np.linalg.norm(p32)
    assert d16 < 1e-4, d16
    assert d16 < 0.1 * d32, (d16, d32)      # the bf16 mode really rounds its operands


def test_mlp_bf16_mode_deviation_bounded(cuda):
    """One whole C2-shaped update (2 epochs over 512 envs x 32 steps) in the bf16 mode and in fp32
    from the same state, rollout and sampler order: per-minibatch losses within 5e-2 of their
    scale, final parameters within 0.25 relative L2 (Adam's early steps move each weight by about
    lr x sign(g): weights whose small gradients flip sign take opposite steps)."""
    out = {}
    for prec in ("fp32", "bf16"):
        _, agent = _agent(cuda, prec, n_envs=512, n_epochs=2)
        agent.train_epoch()
        torch.cuda.synchronize()
        out[prec] = (agent.minibatch_losses(), agent.policy_model.params.cpu().numpy().astype(np.float64))
        del agent
    (l32, p32), (l16, p16) = out["fp32"], out["bf16"]
    assert np.isfinite(l16).all() and not np.array_equal(l16, l32)
    scale = max(1.0, float(np.abs(l32).max()))
    assert np.abs(l16 - l32).max() / scale < 5e-2
    assert np.linalg.norm(p16 - p32) / np.linalg.norm(p32) < 0.25


def test_mlp_bf16_refuses_unsupported_chain(cuda):
    """precision bf16 runs on the fused chain of the compile-time shapes only: a shape without it
    raises ValueError (GS_E_INVALID) instead of silently training in fp32."""
    from gsamd.config import load_config
    from gsamd.ppo_agent import DevicePPOAgent
    torch.manual_seed(42)
    cfg = load_config("CartPole-v1", "ppo", overrides=dict(env_dynamics="synthetic", n_envs=64, precision="bf16",
                                                           model_id="mlp_large"))
    agent = DevicePPOAgent(cfg, device=cuda, track_stats=False)
    with pytest.raises(ValueError, match="bf16"):
        agent.train_epoch()


def test_mlp_bf16_refuses_single_step_entries(cuda):
    """The single-step entries (training_step -> gs_ppo_minibatch_step, losses_for_batch ->
    gs_ppo_loss, the unfused gs_ppo_stage stages) run fp32 kernels: with precision bf16 they raise
    ValueError instead of training in fp32 silently; the fused chain's stages keep the
    bf16 mode (bench.py times them)."""
    from gsamd._lib import check, lib, ptr, stream_handle
    from gsamd.config import load_config
    from gsamd.ppo_agent import DevicePPOAgent
    torch.manual_seed(42)
    cfg = load_config("CartPole-v1", "ppo", overrides=dict(env_dynamics="synthetic", n_envs=64, precision="bf16"))
    agent = DevicePPOAgent(cfg, device=cuda, track_stats=False)
    batches = agent.train_dataloader()
    with pytest.raises(ValueError, match="bf16"):
        agent.training_step(batches[0], 0)
    with pytest.raises(ValueError, match="bf16"):
        agent.losses_for_batch(batches[0], 0)
    pm, hp = agent.policy_model, agent.hparams()
    view = agent.get_rollout_collector("train").buffer.view()
    idx = batches[0].idx

    def stage(k):
        return lib.gs_ppo_stage(k, ptr(pm.params), ptr(agent.grads), ptr(agent.adam_m), ptr(agent.adam_v), pm.dims, hp,
                                view, ptr(idx), agent.batch_size, 1, ptr(agent.metrics_buf), ptr(agent.workspace),
                                stream_handle())
    with pytest.raises(ValueError, match="bf16"):
        check(stage(0), "gs_ppo_stage")
    check(stage(6), "gs_ppo_stage")      # the fused chain's gather stage accepts the mode
    torch.cuda.synchronize()
