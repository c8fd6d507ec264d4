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
                     gamma=0.98, lam=0.8, clip=0.1, lr=1e-3, max_minibatches=None, threads=None, seed=42):
    """Time one rollout + GAE + the update (all n_envs*n_steps/batch*n_epochs minibatches, or the
    first `max_minibatches` extrapolated).  Returns a dict; window_minibatch_s holds the mean
    minibatch time of each tenth of the timed minibatches."""
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
    n_run = n_total if max_minibatches is None else min(int(max_minibatches), n_total)
    marks = [time.perf_counter()]
    edges = {int(round(n_run * j / 10)) for j in range(1, 11)}
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
        if k + 1 in edges:
            marks.append(time.perf_counter())
    t4 = time.perf_counter()
    per_mb = (t4 - t3) / max(n_run, 1)
    bounds = sorted(edges)
    sizes = [b - a for a, b in zip([0] + bounds[:-1], bounds)]
    windows = [(marks[j + 1] - marks[j]) / s for j, s in enumerate(sizes) if s > 0]
    rollout_s = (t1 - t0) + (t2 - t1) + (t3 - t2) + per_mb * n_total
    return dict(env_steps_per_s=N * T / rollout_s, collect_s=t1 - t0, gae_s=t2 - t1, sampler_s=t3 - t2,
                minibatch_s=per_mb, minibatches_timed=n_run, minibatches_per_rollout=n_total,
                window_minibatch_s=windows, wall_s=t4 - t0, threads=torch.get_num_threads())


class _CNNActorCritic(nn.Module):
    """CNNActorCritic restated (utils/models.py:347-455): NatureCNN trunk, fc 512, masked heads."""

    def __init__(self, C, A, hidden, valid):
        super().__init__()
        self.cnn = nn.Sequential(nn.Conv2d(C, 32, 8, 4), nn.ReLU(), nn.Conv2d(32, 64, 4, 2), nn.ReLU(),
                                 nn.Conv2d(64, 64, 3, 1), nn.ReLU(), nn.Flatten())
        self.mlp = nn.Sequential(nn.Linear(64 * 7 * 7, hidden), nn.ReLU())
        self.policy_head = nn.Linear(hidden, A)
        self.value_head = nn.Linear(hidden, 1)
        self.valid = valid

    def forward(self, obs):
        from .cnn_ref import dist_terms  # noqa: F401  (same masked-categorical semantics)
        x = self.mlp(self.cnn(obs.to(torch.float32) / 255.0))
        logits = self.policy_head(x)
        if self.valid is not None:
            mask = torch.ones_like(logits, dtype=torch.bool)
            mask[:, self.valid] = False
            logits = logits.masked_fill(mask, float("-inf"))
        return logits, self.value_head(x).squeeze(-1)


def run_cpu_baseline_cnn(n_envs=256, n_steps=256, batch=1024, n_epochs=15, in_shape=(4, 84, 84), n_actions=18,
                         valid=(0, 3, 4), hidden=512, clip=0.2, ent_coef=0.01, lr=3e-4, sample_steps=64,
                         sample_minibatches=40, threads=None, seed=42):
    """Bounded CPU sample of the pixel path (C4/C5): `sample_steps` vector steps of the rollout
    policy forward + sampling and `sample_minibatches` full minibatch steps (forward, masked PPO
    loss, backward, clip, Adam), each extrapolated to the full rollout / update (defaults: about
    12 s of CPU work at the C4 shapes on 16 cores), after one untimed step of each.  The frame
    source is a pre-made u8 stack (the reference's ALE emulation and preprocessing run in ale-py
    C++, not available here): env cost is EXCLUDED, which flatters the CPU number.  The timed
    minibatches are also reported in windows of `sample_minibatches // 10` (their spread)."""
    from .cnn_ref import dist_terms
    if threads:
        torch.set_num_threads(int(threads))
    torch.manual_seed(seed)
    valid = list(valid) if valid is not None else None
    model = _CNNActorCritic(in_shape[0], n_actions, hidden, valid)
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    g = torch.Generator().manual_seed(seed)
    obs = torch.randint(0, 256, (n_envs, *in_shape), dtype=torch.uint8, generator=g)
    with torch.inference_mode():
        for i in range(sample_steps + 1):
            if i == 1:
                t0 = time.perf_counter()      # after one untimed step
            logits, v = model(obs)
            a = torch.distributions.Categorical(logits=logits).sample()
            dist_terms(logits, a, valid)
            a.numpy(), v.numpy()
    t1 = time.perf_counter()
    mb_obs = torch.randint(0, 256, (batch, *in_shape), dtype=torch.uint8, generator=g)
    va = torch.tensor(valid if valid is not None else list(range(n_actions)))
    act = va[torch.randint(0, len(va), (batch,), generator=g)]
    old_lp = torch.full((batch,), float(np.log(1.0 / len(va))))
    old_v = torch.zeros(batch)
    adv = torch.randn(batch, generator=g)
    ret = adv.clone()
    marks = []
    for i in range(sample_minibatches + 1):
        if i == 1:
            t2 = time.perf_counter()          # after one untimed minibatch
        a_n = (adv - adv.mean()) / (adv.std() + 1e-8)
        logits, v = model(mb_obs)
        lp, H = dist_terms(logits, act, valid)
        ratio = torch.exp(lp - old_lp)
        pl = -torch.min(a_n * ratio, a_n * torch.clamp(ratio, 1 - clip, 1 + clip)).mean()
        vd = v - old_v
        vl = torch.max((v - ret) ** 2, (old_v + torch.clamp(vd, -0.2, 0.2) - ret) ** 2).mean()
        loss = pl + 0.5 * vl - ent_coef * H.mean()
        opt.zero_grad()
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 0.5)
        opt.step()
        loss.item()
        if i >= 1:
            marks.append(time.perf_counter())
    t3 = time.perf_counter()
    per_step = (t1 - t0) / sample_steps
    per_mb = (t3 - t2) / sample_minibatches
    n_mb = n_envs * n_steps // batch * n_epochs
    total = per_step * n_steps + per_mb * n_mb
    w = max(1, sample_minibatches // 10)
    edges = [t2] + marks
    windows = [(edges[min(j + w, len(edges) - 1)] - edges[j]) / (min(j + w, len(edges) - 1) - j)
               for j in range(0, len(edges) - 1, w)]
    return dict(env_steps_per_s=n_envs * n_steps / total, step_s=per_step, minibatch_s=per_mb,
                minibatches_per_rollout=n_mb, wall_s=t3 - t0, threads=torch.get_num_threads(),
                sample_steps=sample_steps, sample_minibatches=sample_minibatches, window_minibatch_s=windows)


_ = ppo_ref
