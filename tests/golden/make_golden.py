"""Generate golden fixtures for the hot-path parity tests FROM THE REFERENCE ITSELF.

Runs ONLY in the build container, where the reference tree is mounted read-only at
/root/reference (it never travels to the GPU box).  It imports the reference's own
Python modules (third-party packages that are not installed -- gymnasium, wandb,
pytorch_lightning, ale_py ... -- are replaced by inert stubs, exactly the trick the
reference's own tests/conftest.py:14-81 uses for Lightning) and records inputs and
outputs as small .npz / .json files next to this script.  Those files are DATA:
inputs plus the reference's outputs on them.  The test-suite compares the oracle
(oracle/) and the HIP path against them.

Fixtures written:
  gae.npz          compute_batched_gae_advantages_and_returns  (utils/returns_advantages.py:115-155)
  sampler.npz      MultiPassRandomSampler index streams        (utils/samplers.py:7-37)
  ppo_step.npz     PPOAgent.losses_for_batch + backward + clip_grad_norm_ + Adam
                   (agents/ppo/ppo_agent.py:21-152, agents/base_agent.py:591-621)
  trajectory.npz   3 rollouts x 20 passes of CartPole-shaped training through the
                   reference RolloutCollector (utils/rollout_collector.py:459-567) on the
                   synthetic fixed-length env below; recorded actions, logp, values,
                   adv, ret, sampler order, per-minibatch losses, final params
  policy_fwd.npz   MLPActorCritic forward (utils/models.py:285-346) + Categorical log_prob/entropy
  configs.json     load_config(...) resolution for the BASELINE.json configs C1-C5
  configs_full.json  every field of those Config objects (what agents.build_agent receives)
  trajectory_kl.npz  the trajectory with target_kl set: the sticky KL early stop
                   (agents/base_agent.py:330-366) fires in the second rollout's update
  ref_ckpt/        model.pt / optimizer.pt / state.json written by BaseAgent.save_checkpoint
                   (agents/base_agent.py:658-732) after the trajectory run
  synth_env.npz    the synthetic env's hashed observations (spec below, not a reference artefact)
  adv_norm.npz     _normalize_advantages (utils/returns_advantages.py:61-64) on a few arrays,
                   the rollout-level advantage normalisation (normalize_advantages "rollout")
  trajectory_rollnorm.npz  the trajectory with normalize_advantages "rollout": the collector
                   normalises each rollout's advantages (utils/rollout_collector.py:441-448) and
                   losses_for_batch does not (utils/torch.py:148-173)

Usage:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import importlib.abc
import importlib.machinery
import json
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.path.insert(0, REF)
sys.path.insert(0, os.path.join(HERE, "..", ".."))

# ----------------------------------------------------------------------------------------
# Stub finder for third-party packages that the reference imports but the image lacks.
# ----------------------------------------------------------------------------------------
_STUB_ROOTS = {
    "gymnasium", "wandb", "ale_py", "dotenv", "ruamel", "watchdog", "cv2", "PIL", "ocatari",
    "pytorch_lightning", "lightning", "vizdoom", "retro", "stable_retro", "gradio", "mcp",
    "modal", "Box2D", "shimmy", "moviepy", "imageio", "pygame", "matplotlib",
}


class _AnyMeta(type):
    def __getattr__(cls, name):
        if name.startswith("__"):
            raise AttributeError(name)
        return _mk(name)


def _mk(name):
    return _AnyMeta(name, (object,), {"__init__": lambda self, *a, **k: None})


class _StubModule(types.ModuleType):
    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        if name[:1].isupper():
            v = _mk(name)
        else:
            v = _StubModule(self.__name__ + "." + name)
            v.__path__ = []
        setattr(self, name, v)
        return v


class _Finder(importlib.abc.MetaPathFinder, importlib.abc.Loader):
    def find_spec(self, fullname, path, target=None):
        if fullname.split(".")[0] in _STUB_ROOTS:
            return importlib.machinery.ModuleSpec(fullname, self, is_package=True)
        return None

    def create_module(self, spec):
        m = _StubModule(spec.name)
        m.__path__ = []
        return m

    def exec_module(self, module):
        pass


sys.meta_path.insert(0, _Finder())

import torch  # noqa: E402

_pl = types.ModuleType("pytorch_lightning")


class _LightningModule(torch.nn.Module):
    def __init__(self, *a, **k):
        super().__init__()

    def save_hyperparameters(self, *a, **k):
        return None


_pl.LightningModule = _LightningModule
_pl.Callback = object
_pl.Trainer = object
sys.modules["pytorch_lightning"] = _pl

from utils.returns_advantages import compute_batched_gae_advantages_and_returns  # noqa: E402
from utils.returns_advantages import _normalize_advantages  # noqa: E402
from utils.samplers import MultiPassRandomSampler  # noqa: E402
from utils.models import MLPActorCritic, CNNActorCritic  # noqa: E402
from utils.rollout_collector import RolloutCollector  # noqa: E402
from utils.dataloaders import build_index_collate_loader_from_collector  # noqa: E402
from utils.random import set_random_seed  # noqa: E402
from utils.config import load_config  # noqa: E402
from agents.ppo.ppo_agent import PPOAgent  # noqa: E402

# The synthetic env spec lives in the product package (shared by CPU tests, GPU kernel
# and this generator); it is NOT a reference artefact.
sys.path.insert(0, os.path.join(HERE, "..", "..", "gymnasium-solver_amd"))
from gsamd.synthetic_env import SyntheticVecEnv, synth_obs  # noqa: E402
# deterministic (LAPACK-free) CNN parameters / batches: test infrastructure, shared with tests
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from oracle.cnn_case import cnn_batch, cnn_params  # noqa: E402

CNN_CASES = {  # tag: (valid actions, clip, ent_coef, lr, B, params seed, batch seed) — C4 / C5 configs
    "pong": ([0, 3, 4], 0.2, 0.01, 3e-4, 48, 1, 3),
    "breakout": ([0, 1, 3, 4], 0.1, 0.01, 3e-4, 40, 2, 5),
}
CNN_SAMPLE = 8192   # grad / param entries stored per case (indices from PCG64 seed 11)


def _gae_case(rng, T, N, p_done, p_timeout_of_done, gamma, lam, with_boot=True):
    values = rng.standard_normal((T, N)).astype(np.float32)
    rewards = rng.standard_normal((T, N)).astype(np.float32)
    dones = rng.random((T, N)) < p_done
    timeouts = dones & (rng.random((T, N)) < p_timeout_of_done)
    last_values = rng.standard_normal(N).astype(np.float32)
    boot = rng.standard_normal((T, N)).astype(np.float32) if with_boot else np.zeros((T, N), np.float32)
    adv, ret = compute_batched_gae_advantages_and_returns(
        values=values, rewards=rewards, dones=dones, timeouts=timeouts,
        last_values=last_values, bootstrapped_next_values=boot, gamma=gamma, gae_lambda=lam)
    return dict(values=values, rewards=rewards, dones=dones.astype(np.uint8),
                timeouts=timeouts.astype(np.uint8), last_values=last_values, bootstrap=boot,
                gamma=np.float64(gamma), lam=np.float64(lam),
                adv=adv.astype(np.float32), ret=ret.astype(np.float32))


def make_gae():
    rng = np.random.default_rng(1234)
    cases = {
        "t1_n1": (1, 1, 0.5, 0.3, 0.98, 0.8),
        "t3_n1": (3, 1, 0.3, 0.3, 0.99, 0.95),
        "t32_n8_c1": (32, 8, 0.05, 0.3, 0.98, 0.8),
        "t32_n1024_c2": (32, 1024, 0.05, 0.3, 0.98, 0.8),
        "t2048_n16_c3": (2048, 16, 0.05, 0.3, 0.99, 0.95),
        "t256_n64_c4": (256, 64, 0.02, 0.3, 0.99, 0.95),
        "t128_n33_ragged": (128, 33, 0.1, 0.5, 0.99, 0.95),
        "t17_n5_alldone": (17, 5, 1.0, 0.5, 0.98, 0.8),
        "t9_n7_alltimeout": (9, 7, 1.0, 1.0, 0.98, 0.8),
        "t64_n3_nodone": (64, 3, 0.0, 0.0, 0.97, 0.9),
    }
    out = {}
    for name, (T, N, pd, pt, g, l) in cases.items():
        c = _gae_case(rng, T, N, pd, pt, g, l)
        for k, v in c.items():
            out[f"{name}/{k}"] = v
    # the reference's call site with no bootstrap array (bootstrapped_next_values=None)
    c = _gae_case(rng, 16, 4, 0.2, 0.5, 0.98, 0.8, with_boot=False)
    adv, ret = compute_batched_gae_advantages_and_returns(
        values=c["values"], rewards=c["rewards"], dones=c["dones"].astype(bool),
        timeouts=c["timeouts"].astype(bool), last_values=c["last_values"],
        bootstrapped_next_values=None, gamma=0.98, gae_lambda=0.8)
    c["adv"], c["ret"] = adv.astype(np.float32), ret.astype(np.float32)
    c["no_boot"] = np.uint8(1)
    for k, v in c.items():
        out[f"t16_n4_noboot/{k}"] = v
    np.savez_compressed(os.path.join(HERE, "gae.npz"), **out)
    print("gae.npz:", len(cases) + 1, "cases")


def _sampler_stream(data_len, passes, epoch):
    torch.manual_seed(42)   # set_random_seed(42) -> torch.initial_seed() == 42
    s = MultiPassRandomSampler(data_len=data_len, num_passes=passes, generator=torch.Generator())
    s.set_epoch(epoch)
    return np.asarray(list(iter(s)), dtype=np.int64)


def make_sampler():
    out = {}
    for ep in range(4):
        out[f"n256_p20_e{ep}"] = _sampler_stream(256, 20, ep)
    out["n7_p2_e0"] = _sampler_stream(7, 2, 0)
    out["n1_p5_e0"] = _sampler_stream(1, 5, 0)
    big = _sampler_stream(131072, 2, 0)
    out["n131072_p2_e0/head"] = big[:4096]
    out["n131072_p2_e3/head"] = _sampler_stream(131072, 2, 3)[:4096]
    out["n131072_p2_e0/sha256"] = np.frombuffer(hashlib.sha256(big.tobytes()).digest(), np.uint8)
    # the first pass of the C2 shape (N*T = 131072, 20 passes): hash of the whole stream
    c2 = _sampler_stream(131072, 20, 0)
    out["n131072_p20_e0/sha256"] = np.frombuffer(hashlib.sha256(c2.tobytes()).digest(), np.uint8)
    out["n131072_p20_e0/tail"] = c2[-4096:]
    np.savez_compressed(os.path.join(HERE, "sampler.npz"), **out)
    print("sampler.npz written")


def _flat_params(model):
    return np.concatenate([p.detach().reshape(-1).numpy() for p in model.parameters()]).astype(np.float32)


def _flat_grads(model):
    return np.concatenate([p.grad.detach().reshape(-1).numpy() for p in model.parameters()]).astype(np.float32)


def _agent(model, cfg):
    """A PPOAgent with just the attributes losses_for_batch reads (as test_ppo.py:73-98 builds
    one); metrics_recorder.record collects every record."""
    agent = object.__new__(PPOAgent)
    torch.nn.Module.__init__(agent)
    agent.config = types.SimpleNamespace(normalize_advantages=cfg["normalize"], target_kl=cfg.get("target_kl"))
    agent.clip_range = cfg["clip"]
    agent.clip_range_vf = cfg["clip_vf"]
    agent.vf_coef = cfg["vf_coef"]
    agent.ent_coef = cfg["ent_coef"]
    agent.policy_model = model
    recs = []
    agent.metrics_recorder = types.SimpleNamespace(record=lambda ns, d: recs.append(dict(d)))
    return agent, recs


def make_ppo_step():
    out = {}
    for tag, (D, H, A, B, clip, ent) in {
        "cartpole": (4, (256, 256), 2, 256, 0.1, 0.0),
        "lunar_ent": (8, (128, 128), 4, 64, 0.2, 0.01),
    }.items():
        torch.manual_seed(42)
        model = MLPActorCritic(input_shape=(D,), hidden_dims=H, output_shape=(A,), activation="relu")
        g = torch.Generator().manual_seed(7)
        obs = torch.randn(B, D, generator=g)
        actions = torch.randint(0, A, (B,), generator=g)
        with torch.no_grad():
            dist, v = model(obs)
            lp = dist.log_prob(actions)
        old_lp = (lp + 0.05 * torch.randn(B, generator=g)).float()
        old_v = (v + 0.1 * torch.randn(B, generator=g)).float()
        adv = torch.randn(B, generator=g) * 2.0 + 0.3
        ret = old_v + adv
        p0 = _flat_params(model)
        cfg = dict(normalize="batch", clip=clip, clip_vf=0.2, vf_coef=0.5, ent_coef=ent)
        agent, recs = _agent(model, cfg)
        batch = types.SimpleNamespace(observations=obs, actions=actions, logprobs=old_lp, values=old_v,
                                      advantages=adv, returns=ret)
        opt = torch.optim.Adam(model.parameters(), lr=1e-3 if tag == "cartpole" else 3e-4)
        opt.zero_grad()
        model._track_activations = True          # BaseAgent.training_step (base_agent.py:336-347)
        res = agent.losses_for_batch(batch, 0)
        acts = model.compute_activation_stats()
        model._track_activations = False
        res["loss"].backward()
        g_raw = _flat_grads(model)
        gnorms = model.compute_grad_norms()      # BaseAgent._backpropagate_and_step (base_agent.py:607-608)
        total = torch.nn.utils.clip_grad_norm_(model.parameters(), 0.5)
        g_clip = _flat_grads(model)
        opt.step()
        p1 = _flat_params(model)
        metrics = {k: float(v) for k, v in recs[0].items()}
        out.update({f"{tag}/obs": obs.numpy(), f"{tag}/actions": actions.numpy(),
                    f"{tag}/old_logprobs": old_lp.numpy(), f"{tag}/old_values": old_v.numpy(),
                    f"{tag}/advantages": adv.numpy(), f"{tag}/returns": ret.numpy(),
                    f"{tag}/params0": p0, f"{tag}/grads_raw": g_raw, f"{tag}/grads_clipped": g_clip,
                    f"{tag}/params1": p1, f"{tag}/loss": np.float32(res["loss"].item()),
                    f"{tag}/total_norm": np.float32(total.item()),
                    f"{tag}/dims": np.array([D, *H, A, B], np.int64),
                    f"{tag}/hparams": np.array([clip, 0.2, 0.5, ent, opt.param_groups[0]["lr"]], np.float64),
                    f"{tag}/metric_names": np.array(sorted(metrics)),
                    f"{tag}/metric_values": np.array([metrics[k] for k in sorted(metrics)], np.float64),
                    f"{tag}/grad_norm_names": np.array(sorted(gnorms)),
                    f"{tag}/grad_norm_values": np.array([gnorms[k] for k in sorted(gnorms)], np.float64),
                    f"{tag}/activation_names": np.array(sorted(acts)),
                    f"{tag}/activation_values": np.array([acts[k] for k in sorted(acts)], np.float64)})
    np.savez_compressed(os.path.join(HERE, "ppo_step.npz"), **out)
    print("ppo_step.npz written")


def make_cnn_step():
    """The reference's CNNActorCritic (NatureCNN, masked actions) through
    PPOAgent.losses_for_batch + backward + clip_grad_norm_ + Adam.  Params/obs are regenerated
    from oracle.cnn_case, so only outputs are stored (per-tensor grad norms + sampled entries)."""
    out = {}
    for tag, (valid, clip, ent, lr, B, pseed, bseed) in CNN_CASES.items():
        model = CNNActorCritic(input_shape=(4, 84, 84), hidden_dims=(512,), output_shape=(18,),
                               valid_actions=valid)
        flat = cnn_params(pseed)
        o = 0
        with torch.no_grad():
            for _, prm in model.named_parameters():
                n = prm.numel()
                prm.copy_(torch.as_tensor(flat[o:o + n]).reshape(prm.shape))
                o += n
        assert o == flat.size
        obs, actions, old_lp, old_v, adv, ret = cnn_batch(bseed, B, valid)
        cfg = dict(normalize="batch", clip=clip, clip_vf=0.2, vf_coef=0.5, ent_coef=ent)
        agent, recs = _agent(model, cfg)
        t = torch.as_tensor
        batch = types.SimpleNamespace(observations=t(obs), actions=t(actions), logprobs=t(old_lp), values=t(old_v),
                                      advantages=t(adv), returns=t(ret))
        with torch.no_grad():
            dist, v = model(t(obs))
            logits = dist.logits.numpy()
        opt = torch.optim.Adam(model.parameters(), lr=lr)
        opt.zero_grad()
        model._track_activations = True          # BaseAgent.training_step (base_agent.py:336-347)
        res = agent.losses_for_batch(batch, 0)
        acts = model.compute_activation_stats()
        model._track_activations = False
        res["loss"].backward()
        g_raw = _flat_grads(model)
        gnorms = model.compute_grad_norms()      # BaseAgent._backpropagate_and_step (base_agent.py:607-608)
        norms = np.array([p.grad.double().norm().item() for p in model.parameters()], np.float64)
        total = torch.nn.utils.clip_grad_norm_(model.parameters(), 0.5)
        opt.step()
        p1 = _flat_params(model)
        sel = np.sort(np.random.default_rng(11).choice(flat.size, CNN_SAMPLE, replace=False))
        metrics = {k: float(v) for k, v in recs[0].items()}
        out.update({f"{tag}/loss": np.float32(res["loss"].item()), f"{tag}/total_norm": np.float32(total.item()),
                    f"{tag}/tensor_norms": norms, f"{tag}/sel": sel.astype(np.int64),
                    f"{tag}/grads_sel": g_raw[sel], f"{tag}/params1_sel": p1[sel],
                    f"{tag}/logits": logits, f"{tag}/values": v.numpy(),
                    f"{tag}/metric_names": np.array(sorted(metrics)),
                    f"{tag}/metric_values": np.array([metrics[k] for k in sorted(metrics)], np.float64),
                    f"{tag}/grad_norm_names": np.array(sorted(gnorms)),
                    f"{tag}/grad_norm_values": np.array([gnorms[k] for k in sorted(gnorms)], np.float64),
                    f"{tag}/activation_names": np.array(sorted(acts)),
                    f"{tag}/activation_values": np.array([acts[k] for k in sorted(acts)], np.float64)})
    np.savez_compressed(os.path.join(HERE, "cnn_step.npz"), **out)
    print("cnn_step.npz written")


def make_policy_fwd():
    out = {}
    torch.manual_seed(42)
    model = MLPActorCritic(input_shape=(4,), hidden_dims=(256, 256), output_shape=(2,), activation="relu")
    g = torch.Generator().manual_seed(11)
    obs = torch.rand(512, 4, generator=g) * 2 - 1
    actions = torch.randint(0, 2, (512,), generator=g)
    with torch.no_grad():
        dist, v = model(obs)
        out.update(params=_flat_params(model), obs=obs.numpy(), actions=actions.numpy(),
                   logits=dist.logits.numpy(), values=v.numpy(), logp=dist.log_prob(actions).numpy(),
                   entropy=dist.entropy().numpy(), probs=dist.probs.numpy())
    np.savez_compressed(os.path.join(HERE, "policy_fwd.npz"), **out)
    print("policy_fwd.npz written")


class _RefVecEnvAdapter:
    """gymnasium-1.x-shaped wrapper around the synthetic env for the reference collector."""

    def __init__(self, env):
        self._env = env
        self.num_envs = env.num_envs
        self.single_action_space = types.SimpleNamespace(sample=lambda: 0, n=env.n_actions)

    def reset(self):
        return self._env.reset()

    def step(self, actions):
        return self._env.step(actions)


# get_metrics() keys that are wall-clock or object-valued (compared separately or not at all)
_METRIC_SKIP = ("roll/fps", "action_dist")


def _metrics_arrays(dicts):
    """A list of metric dicts with identical keys -> (sorted key names, values [n, K])."""
    keys = sorted(k for k in dicts[0] if k not in _METRIC_SKIP)
    return np.array(keys), np.array([[float(d[k]) for k in keys] for d in dicts], np.float64)


def make_adv_norm():
    """_normalize_advantages on (T, N) float32 arrays: the C2 shape's scale, a (64, 256) normal
    case, a large common offset (cancellation in the mean), a constant array (std 0: the result is
    (a - mean) / 1e-8 = 0) and a single element."""
    rng = np.random.default_rng(7)
    cases = {
        "normal": (rng.standard_normal((64, 256)) * 2.0 + 0.3).astype(np.float32),
        "offset": (1000.0 + rng.standard_normal((32, 64)) * 0.01).astype(np.float32),
        "skewed": np.exp(rng.standard_normal((48, 40)) * 1.5).astype(np.float32),
        "constant": np.full((4, 8), 1.5, np.float32),
        "single": np.array([[3.25]], np.float32),
    }
    out = {}
    for k, a in cases.items():
        flat = a.reshape(-1)
        out[f"{k}/in"] = a
        out[f"{k}/out"] = _normalize_advantages(a)
        out[f"{k}/mean_std"] = np.array([flat.mean(), flat.std()], np.float32)
    np.savez_compressed(os.path.join(HERE, "adv_norm.npz"), **out)
    print("adv_norm.npz written")


def make_trajectory_rollnorm():
    make_trajectory(out_name="trajectory_rollnorm.npz", normalize="rollout")


def make_trajectory_stats():
    """The trajectory with the reference's per-training-step diagnostics recorded as
    BaseAgent.training_step records them (agents/base_agent.py:330-366): the forward hooks'
    activation statistics of every evaluated minibatch (utils/models.py:121-147, 184-190) and the
    pre-clip gradient norms of every stepped one (base_agent.py:607-608); the hyper-parameters
    logged at every epoch start (_log_hyperparameters, base_agent.py:302,
    hyperparameter_mixin.py:90-103); and a linear policy_lr schedule applied by the reference's
    HyperparameterSchedulerCallback through _change_optimizers_lr (callback_builder.py:108-113),
    so hp/policy_lr and the Adam step size change between epochs."""
    make_trajectory(out_name="trajectory_stats.npz", stats=True, lr_schedule=(1e-3, 2e-4, 0.0, 96.0))


def make_trajectory(target_kl=None, out_name="trajectory.npz", normalize="batch", stats=False, lr_schedule=None):
    """CartPole-v1:ppo shapes (C1: N=8, T=32, B=256, E=20) for 3 rollouts, through the
    reference's own training-step logic (agents/base_agent.py:330-366): the sticky KL early
    stop (`_early_stop_epoch`, never reset) skips the triggering minibatch's optimizer step and
    every minibatch after it.  Also records, per rollout, the collector's get_metrics()
    (utils/rollout_collector.py:686-760), every metrics_recorder record of losses_for_batch
    (agents/ppo/ppo_agent.py:131-146) and, for the plain run, evaluate_episodes
    (rollout_collector.py:570-655) on a second collector and a checkpoint written by
    BaseAgent.save_checkpoint (agents/base_agent.py:658-732)."""
    N, T, E, B, D, A = 8, 32, 20, 256, 4, 2
    set_random_seed(42)
    model = MLPActorCritic(input_shape=(D,), hidden_dims=(256, 256), output_shape=(A,), activation="relu")
    params0 = _flat_params(model)
    env = SyntheticVecEnv(n_envs=N, obs_dim=D, n_actions=A, episode_len=20, seed=42, truncate_every=3)
    collector = RolloutCollector(_RefVecEnvAdapter(env), model, n_steps=T, gamma=0.98, gae_lambda=0.8,
                                 returns_type="gae:rtg", advantages_type="gae",
                                 normalize_advantages=normalize == "rollout")
    cfg = dict(normalize=normalize, clip=0.1, clip_vf=0.2, vf_coef=0.5, ent_coef=0.0, target_kl=target_kl)
    agent, recs = _agent(model, cfg)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    traj_holder = {}
    hp_recs, act_recs, gn_recs, bounds = [], [], [], []
    sched = None
    if stats:
        # the agent attributes _log_hyperparameters / _change_optimizers_lr read
        agent.n_epochs, agent.policy_lr = E, opt.param_groups[0]["lr"]
        agent.optimizers = lambda: opt
        recorder = agent.metrics_recorder
        rec_hp = types.SimpleNamespace(record=lambda ns, d: hp_recs.append(dict(d)))
    if lr_schedule is not None:
        from trainer_callbacks.hyperparameter_scheduler import HyperparameterSchedulerCallback
        sv, ev, s0, s1 = lr_schedule
        sched = HyperparameterSchedulerCallback(schedule="linear", parameter="policy_lr", start_value=sv, end_value=ev,
                                                start_step=s0, end_step=s1,
                                                set_value_fn=lambda m, v: m._change_optimizers_lr(v))
        sched_module = types.SimpleNamespace(get_rollout_collector=lambda stage: collector,
                                             _change_optimizers_lr=agent._change_optimizers_lr)
    from utils.random import get_global_torch_generator
    loader = None
    rec = {k: [] for k in ["actions", "logp", "values", "adv", "ret", "obs", "rewards", "dones", "order", "losses"]}
    evaluated, stepped, roll_metrics, action_dist = [], [], [], []
    early_stop = False                 # BaseAgent._early_stop_epoch: set once, never reset
    for epoch in range(3):
        if stats:               # on_train_epoch_start -> _log_hyperparameters (base_agent.py:302)
            agent.metrics_recorder = rec_hp
            agent._log_hyperparameters()
            agent.metrics_recorder = recorder
            bounds.append((len(act_recs), len(gn_recs)))
        traj = collector.collect()
        traj_holder["t"] = traj
        m = collector.get_metrics()
        roll_metrics.append(m)
        action_dist.append(np.asarray(m["action_dist"], np.int64))
        if loader is None:
            loader = build_index_collate_loader_from_collector(
                collector=collector, trajectories_getter=lambda: traj_holder["t"], batch_size=B,
                num_passes=E, generator=get_global_torch_generator(42))
        loader.sampler.set_epoch(epoch)        # Lightning fit_loop._set_sampler_epoch
        for bi, batch in enumerate(loader):
            if early_stop:                     # training_step returns before losses_for_batch
                evaluated.append(0)
                stepped.append(0)
                rec["losses"].append(np.nan)
                continue
            opt.zero_grad()
            model._track_activations = stats         # BaseAgent.training_step (base_agent.py:336-347)
            res = agent.losses_for_batch(batch, bi)
            if stats:
                act_recs.append(model.compute_activation_stats())
                model._track_activations = False
            evaluated.append(1)
            rec["losses"].append(float(res["loss"].item()))
            if res["early_stop_epoch"]:
                early_stop = True
                stepped.append(0)
                continue
            res["loss"].backward()
            if stats:                                # _backpropagate_and_step (base_agent.py:607-608)
                gn_recs.append(model.compute_grad_norms())
            torch.nn.utils.clip_grad_norm_(model.parameters(), 0.5)
            opt.step()
            stepped.append(1)
        if sched is not None:      # HyperparameterSchedulerCallback.on_train_epoch_end
            sched.on_train_epoch_end(None, sched_module)
        loader.sampler.set_epoch(epoch)
        order = np.asarray(list(iter(loader.sampler)), np.int64)
        rec["order"].append(order)
        rec["actions"].append(traj.actions.numpy())
        rec["logp"].append(traj.logprobs.numpy())
        rec["values"].append(traj.values.numpy())
        rec["adv"].append(traj.advantages.numpy())
        rec["ret"].append(traj.returns.numpy())
        rec["obs"].append(traj.observations.numpy())
        rec["rewards"].append(traj.rewards.numpy())
        rec["dones"].append(traj.dones.numpy().astype(np.uint8))
    out = {k: np.asarray(v) for k, v in rec.items()}
    out["losses"] = np.asarray(rec["losses"], np.float64)
    out["evaluated"] = np.asarray(evaluated, np.uint8)
    out["stepped"] = np.asarray(stepped, np.uint8)
    out["params0"] = params0
    out["params_final"] = _flat_params(model)
    out["dims"] = np.array([N, T, E, B, D, A], np.int64)
    out["env"] = np.array([20, 42, 3], np.int64)
    out["target_kl"] = np.float64(target_kl if target_kl is not None else 0.0)
    out["roll_metric_names"], out["roll_metric_values"] = _metrics_arrays(roll_metrics)
    out["action_dist"] = np.asarray(action_dist)
    out["train_metric_names"], out["train_metric_values"] = _metrics_arrays(recs)
    if stats:
        # per-record values and the per-epoch means of each key (MetricsRecorder.compute_epoch_means)
        out["hp_names"], out["hp_values"] = _metrics_arrays(hp_recs)
        out["act_names"], out["act_values"] = _metrics_arrays(act_recs)
        out["gn_names"], out["gn_values"] = _metrics_arrays(gn_recs)
        ends = bounds[1:] + [(len(act_recs), len(gn_recs))]
        out["act_epoch_means"] = np.stack([out["act_values"][a0:a1].mean(axis=0)
                                           for (a0, _), (a1, _) in zip(bounds, ends)])
        out["gn_epoch_means"] = np.stack([out["gn_values"][g0:g1].mean(axis=0) for (_, g0), (_, g1) in zip(bounds, ends)])
        out["lr_schedule"] = np.array(lr_schedule if lr_schedule is not None else (0.0,) * 4, np.float64)
    if target_kl is None and normalize == "batch" and not stats:
        # evaluate_episodes on a second collector (the device agent's "val" stage: same env
        # shape, seed + 1000), deterministic, 20 episodes over 8 envs
        eval_env = SyntheticVecEnv(n_envs=N, obs_dim=D, n_actions=A, episode_len=20, seed=42 + 1000,
                                   truncate_every=3)
        eval_coll = RolloutCollector(_RefVecEnvAdapter(eval_env), model, n_steps=T, gamma=0.98, gae_lambda=0.8,
                                     returns_type="gae:rtg", advantages_type="gae", normalize_advantages=False)
        ev = eval_coll.evaluate_episodes(n_episodes=20, deterministic=True)
        out["eval_metric_names"], out["eval_metric_values"] = _metrics_arrays([ev])
        _write_reference_checkpoint(model, opt, collector)
    np.savez_compressed(os.path.join(HERE, out_name), **out)
    print(f"{out_name} written: losses", int(out["evaluated"].sum()), "of", len(evaluated), "evaluated")
    return out


def _write_reference_checkpoint(model, opt, collector):
    """BaseAgent.save_checkpoint (agents/base_agent.py:658-732) on the trained trajectory model:
    model.pt, optimizer.pt, state.json written by the reference's own code into ref_ckpt/."""
    from agents.base_agent import BaseAgent
    d = os.path.join(HERE, "ref_ckpt")
    os.makedirs(d, exist_ok=True)
    this = types.SimpleNamespace(
        policy_model=model, optimizers=lambda: opt, current_epoch=3, run=None,
        config=load_config("CartPole-v1", "ppo"),
        get_rollout_collector=lambda stage: collector if stage == "train" else types.SimpleNamespace(
            _best_episode_reward=float("-inf")))
    torch.manual_seed(1234)            # the RNG state the file records (any fixed state)
    BaseAgent.save_checkpoint(this, d)
    print("ref_ckpt/ written:", sorted(os.listdir(d)))


def make_trajectory_kl():
    """The trajectory with target_kl set so that the sticky early stop fires in the middle of
    the second rollout's update: the threshold sits halfway between the first approx_kl that
    exceeds it and the largest one before."""
    base = np.load(os.path.join(HERE, "trajectory.npz"))
    names = [str(x) for x in base["train_metric_names"]]
    ak = base["train_metric_values"][:, names.index("opt/ppo/approx_kl")]
    best = None
    for first in range(20, 45):
        lo, hi = float(ak[:first].max()), float(ak[first])
        if hi > lo * 1.05:
            best = (first, 0.5 * (lo + hi))
            break
    assert best is not None, "no clean early-stop threshold in 20..45"
    out = make_trajectory(target_kl=best[1], out_name="trajectory_kl.npz")
    assert int(out["evaluated"].sum()) == best[0] + 1, (out["evaluated"].sum(), best)


def make_configs_full():
    """Every field of the Config object the reference's load_config resolves for C1-C5
    (utils/config.py:887-889; dataclasses.asdict, enums as their values): what
    agents.build_agent receives from train.py."""
    import dataclasses
    out = {}
    for env, var in [("CartPole-v1", "ppo"), ("LunarLander-v3", "ppo"), ("ALE-Pong-v5", "rgb_ppo"),
                     ("ALE-Breakout-v5", "rgb_ppo")]:
        c = load_config(env, var)
        d = {k: getattr(v, "value", v) for k, v in dataclasses.asdict(c).items()}
        d["algo_id"] = c.algo_id
        out[f"{env}:{var}"] = json.loads(json.dumps(d, default=lambda o: getattr(o, "value", str(o))))
    with open(os.path.join(HERE, "configs_full.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("configs_full.json written")


def make_configs():
    out = {}
    for cid, env, var in [("C1", "CartPole-v1", "ppo"), ("C3", "LunarLander-v3", "ppo"),
                          ("C4", "ALE-Pong-v5", "rgb_ppo"), ("C5", "ALE-Breakout-v5", "rgb_ppo")]:
        c = load_config(env, var)
        out[f"{env}:{var}"] = dict(
            env_id=c.env_id, algo_id=c.algo_id, n_envs=int(c.n_envs), n_steps=int(c.n_steps),
            batch_size=int(c.batch_size), n_epochs=int(c.n_epochs), gamma=float(c.gamma),
            gae_lambda=float(c.gae_lambda), clip_range=float(c.clip_range), clip_range_vf=float(c.clip_range_vf),
            ent_coef=float(c.ent_coef), vf_coef=float(c.vf_coef), policy_lr=float(c.policy_lr),
            max_grad_norm=float(c.max_grad_norm), model_id=c.model_id, hidden_dims=list(c.hidden_dims),
            activation=c.activation, normalize_advantages=str(getattr(c.normalize_advantages, "value", c.normalize_advantages)),
            target_kl=c.target_kl, seed=int(c.seed), obs_type=str(getattr(c.obs_type, "value", c.obs_type)),
            frame_stack=c.frame_stack, valid_actions=c.spec.get("action_space", {}).get("valid"),
            n_actions=c.spec.get("action_space", {}).get("discrete"),
            policy_kwargs={k: list(v) for k, v in c.policy_kwargs.items()},
            max_env_steps=c.max_env_steps)
    with open(os.path.join(HERE, "configs.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("configs.json written")


def make_synth_env():
    env = SyntheticVecEnv(n_envs=6, obs_dim=4, n_actions=2, episode_len=5, seed=42, truncate_every=2)
    obs0, _ = env.reset()
    rows = [obs0]
    rews, terms, truncs = [], [], []
    for _ in range(12):
        o, r, te, tr, _ = env.step(np.zeros(6, np.int64))
        rows.append(o); rews.append(r); terms.append(te); truncs.append(tr)
    np.savez_compressed(os.path.join(HERE, "synth_env.npz"), obs=np.asarray(rows), rewards=np.asarray(rews),
                        terminated=np.asarray(terms), truncated=np.asarray(truncs),
                        probe=synth_obs(42, np.arange(3, dtype=np.uint64)[:, None],
                                        np.uint64(77), np.arange(8, dtype=np.uint64)[None, :]))
    print("synth_env.npz written")


def make_schedules():
    """Reference scheduler callback + position resolver on a grid of cases
    (trainer_callbacks/hyperparameter_scheduler.py, utils/schedule_resolver.py)."""
    from trainer_callbacks.hyperparameter_scheduler import HyperparameterSchedulerCallback
    from utils.schedule_resolver import schedule_pos_to_vec_steps

    class _Coll:
        total_vec_steps = 0

    class _Mod:
        def __init__(self):
            self.coll, self.got = _Coll(), None

        def get_rollout_collector(self, stage):
            return self.coll

    steps = np.array([0, 5, 10, 37, 50, 64, 99, 100, 101, 150, 200, 250, 400], np.float64)
    cases, values = [], []
    for kind in ("linear", "cosine", "exponential"):
        for warm in (0.0, 0.25):
            for (sv, ev, s0, s1) in ((1e-3, 1e-4, 10.0, 200.0), (0.2, 0.05, 0.0, 100.0), (0.0, 0.01, 50.0, 50.0)):
                cb = HyperparameterSchedulerCallback(schedule=kind, parameter="p", start_value=sv, end_value=ev,
                                                     start_step=s0, end_step=s1, warmup_fraction=warm,
                                                     set_value_fn=lambda m, v: setattr(m, "got", v))
                mod, row = _Mod(), []
                for t in steps:
                    mod.coll.total_vec_steps = float(t)
                    cb.on_train_epoch_end(None, mod)
                    row.append(mod.got)
                cases.append(f"{kind}|{warm}|{sv}|{ev}|{s0}|{s1}")
                values.append(row)
    pos = []
    for raw, dmax, mx, n in ((None, False, 1e6, 8), (None, True, 1e6, 8), (0.5, False, 1e6, 8), (1.0, True, 2e5, 16),
                             (4096.0, False, None, 8), (123456.0, True, 1e6, 32)):
        pos.append([schedule_pos_to_vec_steps(raw, param="p", default_to_max=dmax, max_env_steps=mx, n_envs=n)])
    out = {"cases": np.array(cases), "steps": steps, "values": np.array(values, np.float64),
           "pos": np.array(pos, np.float64)}
    np.savez_compressed(os.path.join(HERE, "schedules.npz"), **out)
    print("schedules.npz written")


if __name__ == "__main__":
    if len(sys.argv) > 1:
        for name in sys.argv[1:]:
            globals()[f"make_{name}"]()
        sys.exit(0)
    make_cnn_step()
    make_gae()
    make_sampler()
    make_ppo_step()
    make_policy_fwd()
    make_configs()
    make_synth_env()
    make_trajectory()
    make_trajectory_kl()
    make_configs_full()
    make_schedules()
    make_adv_norm()
    make_trajectory_rollnorm()
