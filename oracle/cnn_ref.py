"""ORACLE — test infrastructure only (tests/, smoke(), bench cpu_baseline may import it; the
product path never does).

torch-CPU fp32 restatement of the reference's NatureCNN actor-critic PPO minibatch step, the
floating-point checker for the HIP CNN path (C4/C5 rows of SURVEY.md §8):
  * CNNActorCritic.forward         utils/models.py:424-455 (u8 / 255, conv 8x8s4 / 4x4s2 / 3x3s1,
                                   ReLU, flatten (C,H,W), Linear 3136->512 ReLU, heads)
  * build_cnn                      utils/models.py:56-110 (no padding, ReLU after every conv)
  * action masking                 utils/policy_ops.py:44-75 (masked_fill(-inf) of invalid actions)
  * MaskedCategorical              utils/distributions.py:8-82 (entropy over valid actions with
                                   log(p + 1e-8); log_prob = Categorical's)
  * PPO losses                     agents/ppo/ppo_agent.py:21-152, batch normalisation
                                   utils/torch.py:97-99, KL diagnostics utils/torch.py:102-119
  * clip_grad_norm_ + Adam         agents/base_agent.py:612-617, utils/optimizer_factory.py:6-29
Gradients come from torch autograd on this restatement (so torch's min/max/clamp tie rules hold
by construction).  Pinned by tests/golden/cnn_step.npz, generated from the reference itself.
Parameters are a flat fp32 vector in the reference's state_dict order (cnn.0, cnn.2, cnn.4,
mlp.0, policy_head, value_head; each weight then bias).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

NATURE = dict(channels=(32, 64, 64), kernels=(8, 4, 3), strides=(4, 2, 1), hidden=512)


def cnn_param_shapes(in_shape=(4, 84, 84), n_actions=18, spec=NATURE):
    C, H, W = in_shape
    shapes, c, h, w = [], C, H, W
    for i, (co, k, s) in enumerate(zip(spec["channels"], spec["kernels"], spec["strides"])):
        shapes += [(f"cnn.{2 * i}.weight", (co, c, k, k)), (f"cnn.{2 * i}.bias", (co,))]
        c, h, w = co, (h - k) // s + 1, (w - k) // s + 1
    feat = c * h * w
    shapes += [("mlp.0.weight", (spec["hidden"], feat)), ("mlp.0.bias", (spec["hidden"],)),
               ("policy_head.weight", (n_actions, spec["hidden"])), ("policy_head.bias", (n_actions,)),
               ("value_head.weight", (1, spec["hidden"])), ("value_head.bias", (1,))]
    return shapes


def unflatten(flat, shapes):
    out, o = {}, 0
    for n, s in shapes:
        k = int(np.prod(s))
        out[n] = torch.as_tensor(np.asarray(flat[o:o + k], np.float32).reshape(s))
        o += k
    return out


def _bf(t):
    """round-to-nearest-even to bf16 and back (v_cvt_pk_bf16_f32)."""
    return t.to(torch.bfloat16).to(torch.float32)


class _Bf16Conv(torch.autograd.Function):
    """conv2d with bf16-rounded operands and fp32 accumulation in all three products (forward,
    input gradient, weight gradient); the bias gradient sums the unrounded output gradient."""

    @staticmethod
    def forward(ctx, x, w, b, stride):
        ctx.save_for_backward(x, w)
        ctx.stride = stride
        return F.conv2d(_bf(x), _bf(w), b, stride=stride)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        g = _bf(gy)
        dx = torch.nn.grad.conv2d_input(x.shape, _bf(w), g, stride=ctx.stride) if ctx.needs_input_grad[0] else None
        dw = torch.nn.grad.conv2d_weight(_bf(x), w.shape, g, stride=ctx.stride)
        return dx, dw, gy.sum((0, 2, 3)), None


class _Bf16Linear(torch.autograd.Function):
    """linear with bf16-rounded operands in the products listed in `rounded` ("fwd", "dx", "dw"),
    fp32 in the others: the heads round fwd + dw (their input gradient dh is a plain fp32 kernel);
    the fc layer rounds all three (csrc/gs_fc.hip's bf16 kernels: forward, weight gradient, input
    gradient)."""

    @staticmethod
    def forward(ctx, x, w, b, rounded):
        ctx.save_for_backward(x, w)
        ctx.rounded = rounded
        y = (_bf(x) @ _bf(w).t()) if "fwd" in rounded else (x @ w.t())
        return y + b if b is not None else y

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        r = ctx.rounded
        dx = (_bf(gy) @ _bf(w)) if "dx" in r else (gy @ w)
        dw = (_bf(gy).t() @ _bf(x)) if "dw" in r else (gy.t() @ x)
        return dx, dw, gy.sum(0), None


def forward(params: dict, obs_u8, valid=None, spec=NATURE, bf16=False, fc_mask=None, conv_masks=None):
    """-> (masked logits (B,A) with -inf for invalid actions, value (B,), hidden (B,512)).

    fc_mask: (B, 512) bool, the fc layer's ReLU decisions taken as given (h = u * mask) instead of
    u > 0 — the device's own decisions, for a teacher-forced comparison where a pre-activation
    within rounding of zero has its sign decided by the summation order (see fc_preact); None:
    plain ReLU.  conv_masks: the same for the three convolutions, (B, C, H, W) bool each (see
    relu_decisions).

    bf16=True: the device's GS_HP_BF16 mode (SURVEY.md Appendix A "Precision modes") — every
    convolution product, the fc layer's three products and the heads' forward / weight gradient
    take bf16-rounded operands with fp32 accumulation, at the points the HIP kernels round them
    (u8/255 frames, activations, weights, output gradients); biases, ReLU, the loss, the heads'
    input gradient and Adam stay fp32."""
    x = torch.as_tensor(obs_u8)
    x = x.to(torch.float32) / 255.0 if x.dtype == torch.uint8 else x.to(torch.float32)
    conv = (lambda x, w, b, s: _Bf16Conv.apply(x, w, b, s)) if bf16 else (lambda x, w, b, s: F.conv2d(x, w, b, stride=s))
    lin = (lambda x, w, b, r: _Bf16Linear.apply(x, w, b, r)) if bf16 else (lambda x, w, b, r: F.linear(x, w, b))
    for i, s in enumerate(spec["strides"]):
        u = conv(x, params[f"cnn.{2 * i}.weight"], params[f"cnn.{2 * i}.bias"], s)
        if conv_masks is not None:
            x = u * torch.as_tensor(np.asarray(conv_masks[i], bool)).to(u.dtype)
        else:
            x = F.relu(u)
    x = x.flatten(1)
    u = lin(x, params["mlp.0.weight"], params["mlp.0.bias"], ("fwd", "dx", "dw"))
    if fc_mask is not None:
        h = u * torch.as_tensor(np.asarray(fc_mask, bool)).to(u.dtype)
    else:
        h = F.relu(u)
    logits = lin(h, params["policy_head.weight"], params["policy_head.bias"], ("fwd", "dw"))
    if valid is not None:
        mask = torch.ones_like(logits, dtype=torch.bool)
        mask[:, list(valid)] = False
        logits = logits.masked_fill(mask, float("-inf"))
    value = lin(h, params["value_head.weight"], params["value_head.bias"], ("fwd", "dw")).squeeze(-1)
    return logits, value, h


def dist_terms(logits, actions, valid):
    """log_prob of actions and entropy: Categorical / MaskedCategorical semantics."""
    ln = logits - torch.logsumexp(logits, dim=-1, keepdim=True)
    lp = ln.gather(1, torch.as_tensor(actions, dtype=torch.int64)[:, None]).squeeze(1)
    p = torch.softmax(logits, dim=-1)
    if valid is None:
        fmin = torch.finfo(ln.dtype).min
        ent = -(p * ln.clamp(min=fmin)).sum(-1)
    else:
        vm = torch.isfinite(logits)
        ent = -(p * torch.where(vm, torch.log(p + 1e-8), torch.zeros_like(p))).sum(-1)
    return lp, ent


def fc_preact(flat, shapes, obs_u8, spec=NATURE):
    """(u, mag): the fc layer's fp32 pre-activations u = a3 Wf^T + bf as forward computes them, and
    the float64 sums of its terms' magnitudes |a3| |Wf|^T + |bf| (a ReLU decision with |u| far
    below ~1e-6 mag is decided by the summation order)."""
    params = unflatten(flat, shapes)
    with torch.no_grad():
        x = torch.as_tensor(obs_u8)
        x = x.to(torch.float32) / 255.0
        for i, st in enumerate(spec["strides"]):
            x = F.relu(F.conv2d(x, params[f"cnn.{2 * i}.weight"], params[f"cnn.{2 * i}.bias"], stride=st))
        x = x.flatten(1)
        w, b = params["mlp.0.weight"], params["mlp.0.bias"]
        u = F.linear(x, w, b)
        mag = x.to(torch.float64).abs() @ w.to(torch.float64).abs().T + b.to(torch.float64).abs()
    return u.numpy(), mag.numpy()


def relu_decisions(flat, shapes, obs_u8, masks, spec=NATURE):
    """Teacher-forced ReLU decisions: masks = the device's (conv1, conv2, conv3 as (B, C, H, W) bool,
    fc as (B, 512) bool).  Walks the fp32 forward with each layer's input built from the given
    decisions of the layers before it, and returns per layer (n, rel): the number of units whose
    given decision differs from the sign of the oracle's own fp32 pre-activation u, and the
    largest |u| / mag over them, mag the float64 sum of the pre-activation's term magnitudes
    (|x| |w| over the receptive field + |b|) — a decision with rel far below 1e-5 is one the
    summation order decides (the fc layer: as fc_preact)."""
    params = unflatten(flat, shapes)
    out = []
    with torch.no_grad():
        x = torch.as_tensor(obs_u8).to(torch.float32) / 255.0
        for i, st in enumerate(spec["strides"]):
            w, b = params[f"cnn.{2 * i}.weight"], params[f"cnn.{2 * i}.bias"]
            u = F.conv2d(x, w, b, stride=st)
            m = torch.as_tensor(np.asarray(masks[i], bool))
            diff = ((u > 0) != m).nonzero().tolist()
            rel = 0.0
            k = w.shape[-1]
            for (r, c, y, xx) in diff:
                patch = x[r, :, y * st:y * st + k, xx * st:xx * st + k].to(torch.float64).abs()
                mag = float((patch * w[c].to(torch.float64).abs()).sum() + abs(float(b[c])))
                rel = max(rel, abs(float(u[r, c, y, xx])) / max(mag, 1e-30))
            out.append((len(diff), rel))
            x = u * m.to(u.dtype)
        x = x.flatten(1)
        w, b = params["mlp.0.weight"], params["mlp.0.bias"]
        u = F.linear(x, w, b)
        m = torch.as_tensor(np.asarray(masks[3], bool))
        diff = ((u > 0) != m).nonzero().tolist()
        rel = 0.0
        for (r, j) in diff:
            mag = float((x[r].to(torch.float64).abs() * w[j].to(torch.float64).abs()).sum() + abs(float(b[j])))
            rel = max(rel, abs(float(u[r, j])) / max(mag, 1e-30))
        out.append((len(diff), rel))
    return out


def loss_and_grads(flat, shapes, obs_u8, actions, old_logp, old_values, adv, ret, *, valid, clip, clip_vf,
                   vf_coef, ent_coef, normalize="batch", bf16=False, fc_mask=None, conv_masks=None):
    """(loss, metrics, flat grads, logits, values) of losses_for_batch + backward (bf16: see forward)."""
    params = {k: v.clone().requires_grad_(True) for k, v in unflatten(flat, shapes).items()}
    adv = torch.as_tensor(np.asarray(adv, np.float32))
    old_logp = torch.as_tensor(np.asarray(old_logp, np.float32))
    old_values = torch.as_tensor(np.asarray(old_values, np.float32))
    ret = torch.as_tensor(np.asarray(ret, np.float32))
    metrics = {}
    if normalize == "batch":
        adv_n = (adv - adv.mean()) / (adv.std() + 1e-8)
        metrics["roll/adv/norm/mean"] = float(adv_n.mean())
        metrics["roll/adv/norm/std"] = float(adv_n.std())
    else:
        adv_n = adv
    logits, value, _ = forward(params, obs_u8, valid, bf16=bf16, fc_mask=fc_mask, conv_masks=conv_masks)
    new_lp, H = dist_terms(logits, actions, valid)
    ratio = torch.exp(new_lp - old_logp)
    pl = -torch.min(adv_n * ratio, adv_n * torch.clamp(ratio, 1.0 - clip, 1.0 + clip)).mean()
    vdelta = value - old_values
    vl = torch.max((value - ret) ** 2, (old_values + torch.clamp(vdelta, -clip_vf, clip_vf) - ret) ** 2).mean()
    ent = H.mean()
    loss = pl + vf_coef * vl + ent_coef * (-ent)
    loss.backward()
    g = np.concatenate([params[n].grad.reshape(-1).numpy() for n, _ in shapes]).astype(np.float32)
    with torch.no_grad():
        diff = torch.clamp(new_lp - old_logp, -20.0, 20.0)
        r2 = torch.exp(diff)
        metrics.update({
            "opt/loss/total": float(loss), "opt/loss/policy": float(pl), "opt/loss/entropy": float(-ent),
            "opt/policy/entropy": float(ent), "opt/loss/value": float(vl),
            "opt/ppo/clip_fraction": float(((ratio < 1 - clip) | (ratio > 1 + clip)).float().mean()),
            "opt/ppo/clip_fraction_vf": float(((vdelta < -clip_vf) | (vdelta > clip_vf)).float().mean()),
            "opt/value/explained_var": float(1 - torch.var(ret - value) / torch.var(ret)),
            "opt/ppo/kl": float((old_logp - new_lp).mean()),
            "opt/ppo/approx_kl": float(((r2 - 1) - torch.log(r2)).mean()),
        })
    return float(loss.detach()), metrics, g, logits.detach().numpy(), value.detach().numpy()


def clip_and_adam(flat, g, shapes, m, v, t, lr, max_norm=0.5, b1=0.9, b2=0.999, eps=1e-8):
    """clip_grad_norm_ (norm of per-tensor norms) then torch Adam; returns (p, m, v, gc, total)."""
    norms = []
    o = 0
    for _, s in shapes:
        k = int(np.prod(s))
        norms.append(np.linalg.norm(g[o:o + k].astype(np.float64)))
        o += k
    total = float(np.linalg.norm(norms))
    coef = min(np.float32(max_norm) / (np.float32(total) + np.float32(1e-6)), np.float32(1.0))
    gc = (g * np.float32(coef)).astype(np.float32)
    p = torch.as_tensor(np.array(flat, np.float32)).requires_grad_(True)
    opt = torch.optim.Adam([p], lr=lr, betas=(b1, b2), eps=eps, foreach=False)
    st = opt.state[p]
    if t > 1:
        st["step"] = torch.tensor(float(t - 1))
        st["exp_avg"] = torch.as_tensor(np.array(m, np.float32))
        st["exp_avg_sq"] = torch.as_tensor(np.array(v, np.float32))
    p.grad = torch.as_tensor(gc)
    opt.step()
    st = opt.state[p]
    return (p.detach().numpy().copy(), st["exp_avg"].numpy().copy(), st["exp_avg_sq"].numpy().copy(), gc, total)
