"""Config entry point for the device path — same `<env>:<variant>` ids and resolution rules
as the reference's utils/config.py (Config/PPOConfig :17-885, build_from_yaml :363-445,
load_config :887-889), restricted to the fields the rollout + GAE + PPO-update path reads.

Two sources:
  * ``config_dir`` = the reference's ``config/environments`` directory (drop-in mode):
    the YAML files are parsed with the reference's rules (``_base``/anchors, variant
    dicts inheriting file-level fields, ``project_id_variant`` / ``env_id_variant``
    aliases, numeric-string coercion :588-592, fractional batch size :594-607,
    unknown keys dropped :354-357);
  * otherwise the resolved presets of the BASELINE.json configs (gsamd/presets.py).
The BASELINE ids ``LunarLander-v2`` and ``ALE/*:ppo`` are accepted as aliases of
``LunarLander-v3`` and ``ALE-*:rgb_ppo``.
"""
from __future__ import annotations

import dataclasses
import glob
import os
import re
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple

import yaml

from .presets import MODEL_REGISTRY, PRESETS


@dataclass
class PPOConfig:
    env_id: str = ""
    project_id: str = ""
    algo_id: str = "ppo"
    n_envs: int = 8
    n_steps: int = 2048
    batch_size: Any = 64
    n_epochs: int = 10
    max_epochs: Optional[int] = None
    max_env_steps: Optional[float] = None
    seed: int = 42
    gamma: float = 0.99
    gae_lambda: float = 0.95
    clip_range: float = 0.2
    clip_range_vf: float = 0.2
    target_kl: Optional[float] = None
    ent_coef: float = 0.0
    vf_coef: float = 0.5
    max_grad_norm: float = 0.5
    policy_lr: float = 3e-4
    optimizer: str = "adam"
    normalize_advantages: str = "batch"
    model_id: str = "mlp_medium"
    obs_type: str = "vector"
    frame_stack: Optional[int] = None
    accelerator: str = "auto"
    spec: Dict[str, Any] = field(default_factory=dict)
    # env construction fields the env choice depends on (utils/config.py:96-151, get_env_args :676-696)
    max_episode_steps: Optional[int] = None
    seed_train: int = 42
    seed_val: int = 1042
    seed_test: int = 2042
    env_wrappers: List[Any] = field(default_factory=list)
    env_kwargs: Dict[str, Any] = field(default_factory=dict)
    normalize_obs: Any = False
    # device-path extras (not reference fields): synthetic env shape for bench / tests
    obs_dim: Optional[int] = None
    n_actions: Optional[int] = None
    episode_len: int = 200
    truncate_every: int = 0
    # which env the agent steps when the caller passes none (device_env_kind):
    #   "auto"      the env_id's own dynamics where the device implements them (CartPole-v1),
    #               otherwise the caller must pass the host VectorEnv (raises if not)
    #   "synthetic" the fixed-length-episode synthetic env of SURVEY §8d (bench / tests), or the
    #               synthetic Atari frame source for rgb configs
    #   "cartpole"  device CartPole-v1 dynamics
    env_dynamics: str = "auto"
    # data-parallel semantics of a multi-rank update:
    #   "local"  every rank takes B-row minibatches of its own samples (weak scaling, global batch G·B)
    #   "global" every rank takes its share of the reference's global minibatches (the single-GPU
    #            math on G GPUs: global sampler, normalisation and KL stop; gs_ppo_update_global)
    dp_mode: str = "local"
    # MFMA operand precision of the NatureCNN update (include/gsamd.h GS_HP_BF16): "fp32" (the
    # parity path, default) or "bf16" (bf16 operands, fp32 accumulation / parameters / Adam)
    precision: str = "fp32"
    # {param: {schedule, start_value, end_value, start, end, warmup}} (gsamd.schedules)
    schedules: Dict[str, Dict[str, Any]] = field(default_factory=dict)

    def __post_init__(self):
        self._resolve_schedules()
        self._resolve_numeric_strings()
        self._resolve_batch_size()
        self.validate()

    # --- reference-equivalent resolution -------------------------------------------
    def _resolve_schedules(self):
        """utils/config.py:626-655: dict-valued policy_lr / ent_coef start at their 'start'."""
        from .schedules import parse_schedule_dict
        self.schedules = dict(self.schedules or {})
        for p in ("policy_lr", "ent_coef"):
            v = getattr(self, p)
            if isinstance(v, dict):
                spec = parse_schedule_dict(v)
                self.schedules[p] = spec
                setattr(self, p, spec["start_value"])

    def _resolve_numeric_strings(self):
        for f in dataclasses.fields(self):
            v = getattr(self, f.name)
            if isinstance(v, str):
                try:
                    setattr(self, f.name, float(v))
                except ValueError:
                    pass

    def _resolve_batch_size(self):
        if self.batch_size is not None and self.batch_size <= 1:
            self.batch_size = max(1, int(self.n_envs * self.n_steps * self.batch_size))
        self.batch_size = int(self.batch_size)

    def validate(self):
        for k in ("n_envs", "n_steps", "batch_size", "n_epochs", "policy_lr"):
            if getattr(self, k) is not None and getattr(self, k) <= 0:
                raise ValueError(f"{k} must be positive, got {getattr(self, k)}")
        if not (0 < self.gamma <= 1):
            raise ValueError("gamma must be in (0, 1]")
        rollout = self.n_envs * self.n_steps
        if self.dp_mode == "global":
            pass        # minibatches span every rank's rollout: DevicePPOAgent checks them with the world size
        elif self.batch_size > rollout:
            raise ValueError(f"batch_size ({self.batch_size}) should not exceed n_envs ({self.n_envs}) * "
                             f"n_steps ({self.n_steps}).")
        if self.dp_mode != "global" and rollout % self.batch_size != 0:
            raise ValueError("batch_size must divide (n_envs * n_steps) exactly to yield uniform minibatches: "
                             f"rollout_size={rollout}, batch_size={self.batch_size}.")
        if self.normalize_advantages not in ("batch", "rollout", "off", False, None, ""):
            raise ValueError("normalize_advantages must be 'rollout', 'batch', or 'off'.")
        if self.precision not in ("fp32", "bf16"):
            raise ValueError(f"precision must be 'fp32' or 'bf16', got {self.precision!r}")
        if self.precision == "bf16" and self.obs_type != "rgb" and self.target_kl is not None:
            raise ValueError("precision 'bf16' of the MLP update runs on its fused chain, which has no KL early "
                             "stop: unset target_kl or use precision 'fp32'")
        if self.dp_mode not in ("local", "global"):
            raise ValueError(f"dp_mode must be 'local' or 'global', got {self.dp_mode!r}")
        if str(self.env_dynamics or "auto") not in ENV_DYNAMICS:
            raise ValueError(f"env_dynamics must be one of {ENV_DYNAMICS}, got {self.env_dynamics!r}")

    # --- derived -----------------------------------------------------------------------
    @property
    def hidden_dims(self) -> Tuple[int, ...]:
        return tuple(MODEL_REGISTRY[self.model_id]["hidden_dims"])

    @property
    def activation(self) -> str:
        return MODEL_REGISTRY[self.model_id].get("activation", "relu")

    @property
    def valid_actions(self) -> Optional[List[int]]:
        return (self.spec or {}).get("action_space", {}).get("valid")

    def resolved_n_actions(self) -> int:
        if self.n_actions:
            return int(self.n_actions)
        return int((self.spec or {}).get("action_space", {}).get("discrete", 2))

    def resolved_obs_dim(self) -> int:
        if self.obs_dim:
            return int(self.obs_dim)
        obs = (self.spec or {}).get("observation_space", {})
        variants = obs.get("variants", {})
        default = variants.get(obs.get("default", "state"), {})
        shape = default.get("shape") or [4]
        return int(shape[0])

    def get_rollout_collector_kwargs(self) -> Dict[str, Any]:
        """utils/config.py:698-718."""
        return dict(n_steps=self.n_steps, gamma=self.gamma, gae_lambda=self.gae_lambda,
                    normalize_returns=False, returns_type="gae:rtg", advantages_type="gae",
                    normalize_advantages=self.normalize_advantages == "rollout")


_FIELDS = {f.name for f in dataclasses.fields(PPOConfig)}
_ALIASES = {"LunarLander-v2": "LunarLander-v3"}

ENV_DYNAMICS = ("auto", "synthetic", "cartpole")
# env ids whose dynamics the device implements, as BaseAgent.build_env would build them from a
# config without wrappers / env kwargs / observation normalisation
DEVICE_DYNAMICS = {"CartPole-v1": "cartpole"}


def device_env_kind(cfg) -> Optional[str]:
    """The device env a config trains on when the caller passes no env: "synthetic",
    "cartpole", or None when the config names an env the device does not simulate — the
    caller then passes the host VectorEnv the reference would build
    (agents/base_agent.py:129-192 → utils/environment.py:421-425 build_env_from_config)."""
    mode = str(getattr(cfg, "env_dynamics", None) or "auto")
    if mode != "auto":
        return mode
    if str(getattr(cfg, "obs_type", "vector")) == "rgb":
        return None
    kind = DEVICE_DYNAMICS.get(str(getattr(cfg, "env_id", "")))
    plain = (not getattr(cfg, "env_wrappers", None) and not getattr(cfg, "env_kwargs", None)
             and not getattr(cfg, "normalize_obs", False) and getattr(cfg, "frame_stack", None) in (None, 0, 1))
    return kind if plain else None


def needs_host_env(cfg) -> bool:
    """True when build_agent(cfg) needs env= (a gymnasium VectorEnv built on the host)."""
    return device_env_kind(from_reference_config(cfg)) is None


def _sanitize(name: str) -> str:
    return re.sub(r"[^A-Za-z0-9_.-]", "-", name)


def canonical_id(env_id: str, variant: Optional[str]) -> Tuple[str, str]:
    """Map BASELINE.json ids onto the reference's config ids."""
    if variant is None and ":" in env_id:
        env_id, variant = env_id.split(":", 1)
    env_id = _ALIASES.get(env_id, env_id)
    if env_id.startswith("ALE/"):
        env_id = "ALE-" + env_id[4:]
        if variant == "ppo":
            variant = "rgb_ppo"
    return env_id, variant or "ppo"


def _collect_yaml(config_dir: str) -> Dict[str, Dict[str, Any]]:
    out: Dict[str, Dict[str, Any]] = {}
    for path in sorted(glob.glob(os.path.join(config_dir, "*.yaml"))):
        with open(path) as f:
            doc = yaml.safe_load(f) or {}
        base: Dict[str, Any] = {}
        if isinstance(doc.get("_base"), dict):
            base.update({k: v for k, v in doc["_base"].items() if k in _FIELDS})
        base.update({k: v for k, v in doc.items() if k in _FIELDS})
        for k, v in doc.items():
            if k in _FIELDS or not isinstance(v, dict) or str(k).startswith("_"):
                continue
            cfg = dict(base)
            cfg.update(v)
            if not cfg.get("project_id"):
                env = cfg.get("env_id", "")
                cfg["project_id"] = f"{env}_{cfg.get('obs_type', 'rgb')}" if env else os.path.splitext(
                    os.path.basename(path))[0]
            keys = {f"{cfg['project_id']}_{k}", f"{_sanitize(cfg['project_id'])}_{k}"}
            if cfg.get("env_id"):
                keys |= {f"{cfg['env_id']}_{k}", f"{_sanitize(cfg['env_id'])}_{k}"}
            for key in keys:
                out.setdefault(key, cfg)
    return out


def load_config(env_id: str, variant: Optional[str] = None, config_dir: Optional[str] = None,
                overrides: Optional[Dict[str, Any]] = None) -> PPOConfig:
    env_id, variant = canonical_id(env_id, variant)
    if config_dir:
        table = _collect_yaml(config_dir)
        raw = dict(table[f"{env_id}_{variant}"])
        if raw.get("algo_id", "ppo") != "ppo":
            raise ValueError(f"device path implements algo_id 'ppo' only, got {raw.get('algo_id')}")
    else:
        key = f"{env_id}:{variant}"
        if key not in PRESETS:
            raise KeyError(f"no bundled preset for {key}; pass config_dir=<reference>/config/environments")
        raw = dict(PRESETS[key])
    raw = {k: v for k, v in raw.items() if k in _FIELDS}
    cfg = PPOConfig(**raw)
    if overrides:
        cfg = apply_overrides(cfg, overrides)
    return cfg


def apply_overrides(cfg: PPOConfig, overrides: Dict[str, Any]) -> PPOConfig:
    """`--override K=V` (utils/train_launcher.py:81-98): applied after resolution, like the
    reference, but re-validated here (the reference skips re-validation)."""
    for k, v in overrides.items():
        if k not in _FIELDS:
            raise KeyError(f"unknown config field {k!r}")
        cur = getattr(cfg, k)
        if isinstance(v, str) and isinstance(cur, (int, float)) and not isinstance(cur, bool):
            v = type(cur)(float(v)) if isinstance(cur, int) else float(v)
        setattr(cfg, k, v)
    cfg._resolve_numeric_strings()
    cfg._resolve_batch_size()
    cfg.validate()
    return cfg


def from_reference_config(cfg: Any, **extras) -> PPOConfig:
    """Adapt the reference's own Config/PPOConfig object (utils/config.py:17-885) — whatever
    ``agents.build_agent`` received from ``train.py`` — into a PPOConfig, reading the
    fields this path uses by name (enums are reduced to their ``value``)."""
    if isinstance(cfg, PPOConfig):
        return apply_overrides(cfg, extras) if extras else cfg
    from .schedules import SCHEDULABLE, from_attributes
    kw: Dict[str, Any] = {}
    for name in _FIELDS:
        if hasattr(cfg, name) and name != "schedules":
            v = getattr(cfg, name)
            kw[name] = getattr(v, "value", v)
    sched = {p: spec for p in SCHEDULABLE if (spec := from_attributes(cfg, p)) is not None}
    if sched:
        kw["schedules"] = sched
    kw.update(extras)
    return PPOConfig(**kw)
