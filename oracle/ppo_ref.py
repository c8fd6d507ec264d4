"""ORACLE — test infrastructure only.

May be imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg,
as the CHECKER.  The product path (gymnasium-solver_amd/) never imports it.

numpy restatement of the reference's PPO minibatch step with analytic gradients:
  * MLPActorCritic forward                utils/models.py:285-346 (Linear/ReLU backbone, heads)
  * Categorical log_prob / entropy        torch.distributions.Categorical
  * batch advantage normalisation         utils/torch.py:97-99, :148-174
  * PPO clipped surrogate / value / ent   agents/ppo/ppo_agent.py:21-152
  * KL diagnostics                        utils/torch.py:102-119
  * clip_grad_norm_(max_norm=0.5)         agents/base_agent.py:612-617 (Lightning -> torch)
  * torch.optim.Adam defaults             utils/optimizer_factory.py:6-29
Gradients follow torch's autograd conventions, including the tie rules of
torch.min / torch.max (a tie splits the gradient in halves) and clamp's inclusive
pass-through.  Pinned by tests/golden/ppo_step.npz (the reference's own loss/grads).
"""
from __future__ import annotations

import numpy as np

F32 = np.float32


def param_shapes(dims):
    """dims = (D, H1, ..., Hk, A) -> list of (name, shape) in reference parameter order."""
    D, *H, A = dims
    shapes, last = [], D
    for i, h in enumerate(H):
        shapes.append((f"backbone.{2 * i}.weight", (h, last)))
        shapes.append((f"backbone.{2 * i}.bias", (h,)))
        last = h
    shapes += [("policy_head.weight", (A, last)), ("policy_head.bias", (A,)),
               ("value_head.weight", (1, last)), ("value_head.bias", (1,))]
    return shapes


def unflatten(flat, dims):
    out, o = {}, 0
    for name, shp in param_shapes(dims):
        n = int(np.prod(shp))
        out[name] = np.asarray(flat[o:o + n], F32).reshape(shp)
        o += n
    return out


def flatten(d, dims):
    return np.concatenate([np.asarray(d[n], F32).reshape(-1) for n, _ in param_shapes(dims)])


def bf16_round(x):
    """float32 -> nearest bfloat16 (ties to even) -> float32: the device's v_cvt_pk_bf16_f32 on
    finite values (the bf16 mode's MFMA operands)."""
    u = np.ascontiguousarray(x, F32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return r.astype(np.uint32).view(F32).reshape(np.shape(x))


def forward(flat, dims, obs, bf16=False):
    """bf16: the MLP chain's bf16 mode (GS_HP_BF16) — the hidden-to-hidden product takes bf16
    operands with fp32 accumulation (h2 = relu(bf16(h1) bf16(W2)^T + b2)); the first layer and
    the heads stay fp32 (VALU on the device)."""
    P = unflatten(flat, dims)
    nh = len(dims) - 2
    x = np.asarray(obs, F32)
    acts = [x]
    for i in range(nh):
        W = P[f"backbone.{2 * i}.weight"]
        if bf16 and i > 0:
            x = np.maximum((bf16_round(x) @ bf16_round(W).T).astype(F32) + P[f"backbone.{2 * i}.bias"], F32(0))
        else:
            x = np.maximum(x @ W.T + P[f"backbone.{2 * i}.bias"], F32(0))
        acts.append(x)
    logits = x @ P["policy_head.weight"].T + P["policy_head.bias"]
    value = (x @ P["value_head.weight"].T + P["value_head.bias"])[:, 0]
    return logits.astype(F32), value.astype(F32), acts


def activation_stats(flat, dims, obs, bf16=False):
    """The forward hooks' statistics of the backbone's Linear layers (utils/models.py:121-147,
    registered on backbone.0 / backbone.2): for each layer's pre-activation output z (B, H) —
    mean and unbiased std over all of z, and the per-neuron fraction of rows with |z| < 1e-6,
    averaged (dead_pct) and maximised (dead_max) over neurons.  Returns [mean, std, dead_pct,
    dead_max] per layer, flattened (the GS_M_ACT slot order); float64 statistics of the float32 z."""
    P = unflatten(flat, dims)
    x = np.asarray(obs, F32)
    out = []
    for i in range(len(dims) - 2):
        W, b = P[f"backbone.{2 * i}.weight"], P[f"backbone.{2 * i}.bias"]
        if bf16 and i > 0:
            z = ((bf16_round(x) @ bf16_round(W).T).astype(F32) + b).astype(F32)
        else:
            z = (x @ W.T + b).astype(F32)
        zd = z.astype(np.float64)
        dead = (np.abs(z) < F32(1e-6)).mean(axis=0)
        out += [zd.mean(), zd.std(ddof=1), dead.mean(), dead.max()]
        x = np.maximum(z, F32(0))
    return np.array(out, np.float64)


def log_softmax(logits):
    m = logits.max(axis=1, keepdims=True)
    z = logits - m
    lse = np.log(np.exp(z).sum(axis=1, keepdims=True))
    return (z - lse).astype(F32)


def _min_grads(a, b):
    """d min(a,b)/da, d/db with torch's tie rule (halves)."""
    ga = np.where(a < b, 1.0, np.where(a == b, 0.5, 0.0))
    gb = np.where(b < a, 1.0, np.where(a == b, 0.5, 0.0))
    return ga.astype(F32), gb.astype(F32)


def _max_grads(a, b):
    ga = np.where(a > b, 1.0, np.where(a == b, 0.5, 0.0))
    gb = np.where(b > a, 1.0, np.where(a == b, 0.5, 0.0))
    return ga.astype(F32), gb.astype(F32)


def ppo_loss_and_grads(flat, dims, obs, actions, old_logp, old_values, adv, ret, *, clip, clip_vf,
                       vf_coef, ent_coef, normalize="batch", bf16=False):
    """Return (loss, metrics, flat_grads) of PPOAgent.losses_for_batch + backward.  bf16: the
    device MLP chain's bf16 mode — bf16-rounded operands (fp32 accumulation) in the hidden-to-
    hidden product, the head-weight gradient (bf16(dz)^T bf16(h2)), the hidden weight gradient
    (bf16(dh2)^T bf16(h1)) and the hidden input gradient (bf16(dh2) bf16(W2)); biases, the first
    layer and everything else fp32."""
    B = obs.shape[0]
    P = unflatten(flat, dims)
    nh = len(dims) - 2
    assert not bf16 or nh == 2, "bf16 emulation: the two-hidden-layer MLP of the device chain"
    bq = bf16_round if bf16 else (lambda v: v)
    logits, value, acts = forward(flat, dims, obs, bf16=bf16)
    adv = np.asarray(adv, F32)
    metrics = {}
    if normalize == "batch":
        mu = adv.mean(dtype=np.float64)
        sd = adv.std(ddof=1, dtype=np.float64)
        adv_n = ((adv - F32(mu)) / (F32(sd) + F32(1e-8))).astype(F32)
        metrics["roll/adv/norm/mean"] = float(adv_n.mean(dtype=np.float64))
        metrics["roll/adv/norm/std"] = float(adv_n.std(ddof=1, dtype=np.float64))
    else:
        adv_n = adv
    ln = log_softmax(logits)
    p = np.exp(ln).astype(F32)
    a = np.asarray(actions, np.int64)
    new_lp = ln[np.arange(B), a]
    ratio = np.exp(new_lp - old_logp).astype(F32)
    rc = np.clip(ratio, F32(1 - clip), F32(1 + clip))
    s1, s2 = adv_n * ratio, adv_n * rc
    pl = -np.minimum(s1, s2).mean(dtype=np.float64)
    vdelta = value - old_values
    vu = (value - ret) ** 2
    vcl = old_values + np.clip(vdelta, -clip_vf, clip_vf)
    vc = (vcl - ret) ** 2
    vl = np.maximum(vu, vc).mean(dtype=np.float64)
    H = -(p * ln).sum(axis=1)
    ent = H.mean(dtype=np.float64)
    loss = pl + vf_coef * vl - ent_coef * ent

    # --- backward (mean over B) ---
    g1, g2 = _min_grads(s1, s2)
    in_clip = ((ratio >= F32(1 - clip)) & (ratio <= F32(1 + clip))).astype(F32)
    dratio = -(adv_n * g1 + adv_n * g2 * in_clip) / B
    dlp = dratio * ratio
    onehot = np.zeros_like(p)
    onehot[np.arange(B), a] = 1.0
    dlogits = dlp[:, None] * (onehot - p)
    # entropy term: loss += -ent_coef * mean(H); dH/dl_b = -p_b (ln_b + H)
    dlogits += (-ent_coef / B) * (-p * (ln + H[:, None]))
    h1, h2 = _max_grads(vu, vc)
    vin = ((vdelta >= -clip_vf) & (vdelta <= clip_vf)).astype(F32)
    dvalue = vf_coef / B * (h1 * 2 * (value - ret) + h2 * 2 * (vcl - ret) * vin)

    G = {}
    x = acts[-1]
    if bf16:
        G["policy_head.weight"] = (bq(dlogits.astype(F32)).T @ bq(x)).astype(F32)
        G["value_head.weight"] = (bq(dvalue.astype(F32))[None, :] @ bq(x)).astype(F32)
    else:
        G["policy_head.weight"] = dlogits.T @ x
        G["value_head.weight"] = (dvalue[:, None] * x).sum(0)[None, :]
    G["policy_head.bias"] = dlogits.sum(0)
    G["value_head.bias"] = np.array([dvalue.sum()], F32)
    dx = dlogits @ P["policy_head.weight"] + dvalue[:, None] * P["value_head.weight"]
    for i in reversed(range(nh)):
        dx = dx * (acts[i + 1] > 0)
        if bf16 and i > 0:
            G[f"backbone.{2 * i}.weight"] = (bq(dx.astype(F32)).T @ bq(acts[i])).astype(F32)
        else:
            G[f"backbone.{2 * i}.weight"] = dx.T @ acts[i]
        G[f"backbone.{2 * i}.bias"] = dx.sum(0)
        if i > 0:
            W = P[f"backbone.{2 * i}.weight"]
            dx = (bq(dx.astype(F32)) @ bq(W)).astype(F32) if bf16 else dx @ W

    with np.errstate(over="ignore"):
        clipfrac = ((ratio < 1 - clip) | (ratio > 1 + clip)).mean()
        clipfrac_vf = ((vdelta < -clip_vf) | (vdelta > clip_vf)).mean()
        ev = 1 - np.var(ret - value, ddof=1) / np.var(ret, ddof=1)
        diff = np.clip(new_lp - old_logp, -20.0, 20.0)
        r2 = np.exp(diff)
        approx_kl = ((r2 - 1) - np.log(r2)).mean()
    metrics.update({
        "opt/loss/total": float(loss), "opt/loss/policy": float(pl), "opt/loss/entropy": float(-ent),
        "opt/policy/entropy": float(ent), "opt/loss/entropy_scaled": float(-ent_coef * ent),
        "opt/loss/value": float(vl), "opt/loss/value_scaled": float(vf_coef * vl),
        "opt/ppo/clip_fraction": float(clipfrac), "opt/ppo/clip_fraction_vf": float(clipfrac_vf),
        "opt/value/explained_var": float(ev), "opt/ppo/kl": float((old_logp - new_lp).mean()),
        "opt/ppo/approx_kl": float(approx_kl), "opt/ppo/kl_stop_triggered": 0.0,
    })
    return float(loss), metrics, flatten(G, dims)


def loss_sums(flat, dims, obs, actions, old_logp, old_values, adv, ret, *, clip, clip_vf, normalize="batch",
              adv_stats=None):
    """The 14 raw per-minibatch sums the device exports in the global-minibatch mode
    (include/gsamd.h gs_ppo_global.metric_sums), over the given rows: sum of min-surrogate,
    clipped value loss, entropy, ratio / value clip counts, kl, approx_kl (utils/torch.py:102-119),
    ret - v and its square, ret and its square, normalised advantage and its square, and one
    unused slot (agents/ppo/ppo_agent.py:53-146).  adv_stats: the (mean, std) to normalise with (a global
    minibatch's); default the rows' own (utils/torch.py:97-99)."""
    adv = np.asarray(adv, F32)
    if normalize == "batch":
        mu, sd = adv_stats if adv_stats is not None else (adv.mean(dtype=np.float64), adv.std(ddof=1, dtype=np.float64))
        adv = ((adv - F32(mu)) / (F32(sd) + F32(1e-8))).astype(F32)
    logits, value, _ = forward(flat, dims, obs)
    ln = log_softmax(logits)
    p = np.exp(ln).astype(F32)
    n = obs.shape[0]
    a = np.asarray(actions, np.int64)
    new_lp = ln[np.arange(n), a]
    ratio = np.exp(new_lp - old_logp).astype(F32)
    rc = np.clip(ratio, F32(1 - clip), F32(1 + clip))
    vdelta = value - old_values
    vu = (value - ret) ** 2
    vc = (old_values + np.clip(vdelta, -clip_vf, clip_vf) - ret) ** 2
    H = -(p * ln).sum(axis=1)
    r2 = np.exp(np.clip(new_lp - old_logp, -20.0, 20.0))
    rv = (ret - value).astype(np.float64)
    d = np.float64
    return np.array([np.minimum(adv * ratio, adv * rc).sum(dtype=d), np.maximum(vu, vc).sum(dtype=d),
                     H.sum(dtype=d), ((ratio < F32(1 - clip)) | (ratio > F32(1 + clip))).sum(dtype=d),
                     ((vdelta < -clip_vf) | (vdelta > clip_vf)).sum(dtype=d), (old_logp - new_lp).sum(dtype=d),
                     ((r2 - 1) - np.log(r2)).sum(dtype=d), rv.sum(), (rv * rv).sum(),
                     np.asarray(ret, d).sum(), (np.asarray(ret, d) ** 2).sum(), adv.sum(dtype=d),
                     (adv.astype(d) ** 2).sum(), 0.0])


def clip_grad_norm(flat_grads, dims, max_norm):
    """torch.nn.utils.clip_grad_norm_: norm of per-parameter norms, coef clamped to 1."""
    P = unflatten(flat_grads, dims)
    norms = [np.linalg.norm(P[n].astype(np.float64)) for n, _ in param_shapes(dims)]
    total = float(np.linalg.norm(norms))
    coef = min(1.0, max_norm / (total + 1e-6))
    return (flat_grads * F32(coef)).astype(F32), total


def adam_step(p, g, m, v, t, lr, b1=0.9, b2=0.999, eps=1e-8):
    """torch.optim.Adam single-tensor step (defaults, no weight decay); t is 1-based."""
    m = (b1 * m + (1 - b1) * g).astype(F32)
    v = (b2 * v + (1 - b2) * g * g).astype(F32)
    bc1 = 1 - b1 ** t
    bc2 = 1 - b2 ** t
    denom = np.sqrt(v) / np.sqrt(bc2) + eps
    p = (p - (lr / bc1) * m / denom).astype(F32)
    return p, m, v


def gae_numpy(values, rewards, dones, timeouts, last_values, bootstrap, gamma, lam):
    """numpy restatement of returns_advantages.py:115-155 (same op order)."""
    values = np.asarray(values, F32)
    T, N = values.shape
    nv = np.empty_like(values)
    nv[:-1] = values[1:]
    nv[-1] = last_values
    dones = np.asarray(dones, bool)
    timeouts = np.asarray(timeouts, bool)
    if bootstrap is not None:
        nv = np.where(timeouts, np.asarray(bootstrap, F32), nv)
    nt = (~(dones & ~timeouts)).astype(F32)
    c1, c2 = F32(gamma), F32(gamma * lam)
    adv = np.zeros_like(values)
    gae = np.zeros(N, F32)
    for t in range(T - 1, -1, -1):
        delta = rewards[t] + (c1 * nv[t]) * nt[t] - values[t]
        gae = delta + (c2 * gae) * nt[t]
        adv[t] = gae
    return adv, adv + values


def numpy_f32_sum(a) -> np.float32:
    """numpy's float32 np.add.reduce of a contiguous array, restated (what gs_normalize_advantages
    reproduces on the device): sequential over 8192-element buffer chunks from 0, each chunk by
    pairwise_sum (numpy/_core/src/umath/loops_utils.h.src): n < 8 a plain loop from 0; n <= 128 eight
    strided accumulators, ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)), then the n % 8 rest;
    else split at n2 = n // 2 - (n // 2) % 8.  Pinned against numpy itself in
    tests/test_oracle_golden.py."""
    a = np.ascontiguousarray(a, F32).reshape(-1)

    def pw(x):
        n = x.size
        if n < 8:
            r = F32(0)
            for v in x:
                r = F32(r + v)
            return r
        if n <= 128:
            r = x[:8].copy()
            m = n - n % 8
            for i in range(8, m, 8):
                r = (r + x[i:i + 8]).astype(F32)
            res = F32(F32(F32(r[0] + r[1]) + F32(r[2] + r[3])) + F32(F32(r[4] + r[5]) + F32(r[6] + r[7])))
            for i in range(m, n):
                res = F32(res + x[i])
            return res
        n2 = n // 2
        n2 -= n2 % 8
        return F32(pw(x[:n2]) + pw(x[n2:]))

    total = F32(0)
    for c in range(0, a.size, 8192):
        total = F32(total + pw(a[c:c + 8192]))
    return total


def normalize_advantages_rollout(adv, eps: float = 1e-8) -> np.ndarray:
    """utils/returns_advantages.py:61-64 (_normalize_advantages), the rollout-level normalisation
    of utils/rollout_collector.py:441-442: (a - mean) / (std + eps) over every element, numpy
    float32 statistics (std biased)."""
    a = np.asarray(adv, F32)
    flat = a.reshape(-1)
    return (a - flat.mean()) / (flat.std() + float(eps))


def normalize_advantages_model(adv, eps: float = 1e-8) -> np.ndarray:
    """normalize_advantages_rollout written out with numpy_f32_sum (the device kernel's steps):
    mean = S / n, std = sqrt(S((a - mean)^2) / n), float32 sums; each division of a float32 sum by
    the integer count in float64, cast back to float32 (numpy's _mean / _var: float32 / np.intp)."""
    a = np.asarray(adv, F32)
    n = np.float64(a.size)
    mean = F32(np.float64(numpy_f32_sum(a)) / n)
    d = (a - mean).astype(F32)
    std = np.sqrt(F32(np.float64(numpy_f32_sum((d * d).astype(F32))) / n)).astype(F32)
    return ((a - mean) / F32(std + F32(eps))).astype(F32)
