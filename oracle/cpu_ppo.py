"""ORACLE — test infrastructure only (bench.py's cpu_baseline leg and tests).

torch-CPU restatement of the reference's training loop for the PPO path, used as the
CPU baseline timed on the GPU box's host cores (SURVEY.md §8d "CPU baseline"):
  per-step rollout loop        utils/rollout_collector.py:459-567 (torch policy_act on CPU,
                               numpy env step, numpy buffer rows, .cpu() round trips)
  GAE                          oracle/ppo_ref.gae_numpy == utils/returns_advantages.py:115-155
  env-major flatten            utils/rollout_buffer.py:105-173
  sampler                      torch.rand + argsort per epoch (utils/samplers.py:25-34)
  minibatch loop               9-field gather (rollout_collector.py:657-682), activation-stat
                               hooks (models.py:121-147), losses_for_batch + metric .item()s
                               (ppo_agent.py:21-152), backward, compute_grad_norms
                               (models.py:196-230), clip_grad_norm_(0.5), torch.optim.Adam
                               (base_agent.py:591-621)
It is a restatement (no reference code is imported), timed on synthetic env steps.
"""
from __future__ import annotations

import time

import numpy as np
import torch
import torch.nn as nn

from . import ppo_ref


class _MLPActorCritic(nn.Module):
    def __init__(self, D, H, A):
        super().__init__()
        layers, last = [], D
        for h in H:
            layers += [nn.Linear(last, h), nn.ReLU()]
            last = h
        self.backbone = nn.Sequential(*layers)
        self.policy_head = nn.Linear(last, A)
        self.value_head = nn.Linear(last, 1)

    def forward(self, obs):
        x = self.backbone(obs)
        return torch.distributions.Categorical(logits=self.policy_head(x)), self.value_head(x).squeeze(-1)


def _activation_stats(model, obs):
    """The reference's forward hooks on backbone Linear layers (utils/models.py:121-147):
    mean/std/dead_pct/dead_max per layer, each forced to a Python float."""
    x = obs
    for m in model.backbone:
        x = m(x)
        if isinstance(m, nn.Linear):
            with torch.no_grad():
                flat = x.flatten(start_dim=1)
                dead = (flat.abs() < 1e-6).float().mean(dim=0)
                flat.mean().item(), flat.std().item(), dead.mean().item(), dead.max().item()


def _grad_norms(model):
    """compute_grad_norms (utils/models.py:196-230): per-parameter .item() norms."""
    for group in (list(model.parameters()), list(model.backbone.parameters()), list(model.policy_head.parameters()),
                  list(model.value_head.parameters())):
        float(sum(p.grad.detach().norm(2).item() ** 2 for p in group)) ** 0.5


def _losses(model, obs, actions, old_lp, old_v, adv, ret, clip, clip_vf, vf_coef, ent_coef):
    adv = (adv - adv.mean()) / (adv.std() + 1e-8)
    _activation_stats(model, obs)
    dist, v = model(obs)
    lp = dist.log_prob(actions)
    ratio = torch.exp(lp - old_lp)
    pl = -torch.min(adv * ratio, adv * torch.clamp(ratio, 1 - clip, 1 + clip)).mean()
    vd = v - old_v
    vl = torch.max((v - ret) ** 2, (old_v + torch.clamp(vd, -clip_vf, clip_vf) - ret) ** 2).mean()
    ent = dist.entropy().mean()
    loss = pl + vf_coef * vl - ent_coef * ent
    with torch.no_grad():   # the reference's per-minibatch metrics (each forces .item() there)
        ((ratio < 1 - clip) | (ratio > 1 + clip)).float().mean().item()
        ((vd < -clip_vf) | (vd > clip_vf)).float().mean().item()
        (1 - torch.var(ret - v) / torch.var(ret)).item()
        d = torch.clamp(lp - old_lp, -20, 20)
        r2 = torch.exp(d)
        ((r2 - 1) - torch.log(r2)).mean().item()
    return loss


def run_cpu_baseline(n_envs=4096, n_steps=32, batch=256, n_epochs=20, obs_dim=4, hidden=(256, 256), n_actions=2,
                     gamma=0.98, lam=0.8, clip=0.1, lr=1e-3, max_minibatches=2000, threads=None, seed=42):
    """Time one rollout + GAE + `max_minibatches` of the update; extrapolate to the full
    update (n_envs*n_steps/batch*n_epochs minibatches).  Returns a dict."""
    from gsamd.synthetic_env import SyntheticVecEnv     # shared env spec (host numpy twin)
    if threads:
        torch.set_num_threads(int(threads))
    torch.manual_seed(seed)
    model = _MLPActorCritic(obs_dim, hidden, n_actions)
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    env = SyntheticVecEnv(n_envs=n_envs, obs_dim=obs_dim, n_actions=n_actions, episode_len=200, seed=seed)
    obs, _ = env.reset()
    T, N = n_steps, n_envs
    bufs = {k: np.zeros((T, N), np.float32) for k in ("logp", "values", "rewards")}
    obs_buf = np.zeros((T, N, obs_dim), np.float32)
    act_buf = np.zeros((T, N), np.int64)
    dones = np.zeros((T, N), bool)
    touts = np.zeros((T, N), bool)
    t0 = time.perf_counter()
    with torch.inference_mode():
        for t in range(T):
            dist, v = model(torch.as_tensor(obs))
            a = dist.sample()
            lp = dist.log_prob(a)
            a_np = a.cpu().numpy()
            nobs, r, te, tr, _ = env.step(a_np)
            obs_buf[t], act_buf[t] = obs, a_np
            bufs["logp"][t], bufs["values"][t], bufs["rewards"][t] = lp.numpy(), v.numpy(), r
            dones[t], touts[t] = te | tr, tr
            obs = nobs
        _, last_v = model(torch.as_tensor(obs))
    t1 = time.perf_counter()
    adv, ret = ppo_ref.gae_numpy(bufs["values"], bufs["rewards"], dones, touts, last_v.numpy(),
                                 np.zeros((T, N), np.float32), gamma, lam)
    t2 = time.perf_counter()

    def em(x):
        return torch.as_tensor(np.ascontiguousarray(x.swapaxes(0, 1)).reshape(N * T, *x.shape[2:]))
    tr_obs, tr_act, tr_lp, tr_v, tr_adv, tr_ret = (em(obs_buf), em(act_buf), em(bufs["logp"]), em(bufs["values"]),
                                                    em(adv), em(ret))
    tr_rew, tr_done, tr_nobs = em(bufs["rewards"]), em(dones), em(obs_buf)
    g = torch.Generator()
    g.manual_seed(seed)
    order = torch.argsort(torch.rand((n_epochs, N * T), generator=g), dim=1).reshape(-1)
    t3 = time.perf_counter()
    n_total = N * T // batch * n_epochs
    n_run = min(max_minibatches, n_total)
    for k in range(n_run):
        idx = order[k * batch:(k + 1) * batch]
        # collate: the reference slices all 9 trajectory fields per minibatch
        # (utils/rollout_collector.py:672-682), incl. rewards/dones/next_obs PPO never reads
        b_obs, b_act, b_lp, b_v, b_adv, b_ret = (tr_obs[idx], tr_act[idx], tr_lp[idx], tr_v[idx], tr_adv[idx],
                                                 tr_ret[idx])
        tr_rew[idx], tr_done[idx], tr_nobs[idx]
        loss = _losses(model, b_obs, b_act, b_lp, b_v, b_adv, b_ret, clip, 0.2, 0.5, 0.0)
        opt.zero_grad()
        loss.backward()
        _grad_norms(model)
        torch.nn.utils.clip_grad_norm_(model.parameters(), 0.5)
        opt.step()
    t4 = time.perf_counter()
    per_mb = (t4 - t3) / max(n_run, 1)
    rollout_s = (t1 - t0) + (t2 - t1) + (t3 - t2) + per_mb * n_total
    return dict(env_steps_per_s=N * T / rollout_s, collect_s=t1 - t0, gae_s=t2 - t1, sampler_s=t3 - t2,
                minibatch_s=per_mb, minibatches_timed=n_run, minibatches_per_rollout=n_total,
                wall_s=t4 - t0, threads=torch.get_num_threads())


_ = ppo_ref
