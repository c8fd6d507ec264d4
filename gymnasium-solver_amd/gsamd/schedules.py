"""Hyper-parameter schedules of the update.

Restates trainer_callbacks/hyperparameter_scheduler.py (linear / cosine / exponential curves,
optional linear warmup, `on_train_epoch_end` fraction from the train collector's
`total_vec_steps`) and utils/schedule_resolver.py (`schedule_pos_to_vec_steps`: positions as
fractions of `max_env_steps` or absolute env steps, converted to vector steps).  The values
land in the next epoch's kernel arguments (`DevicePPOAgent.hparams()`): `policy_lr` becomes
Adam's step size, `clip_range` / `clip_range_vf` / `vf_coef` / `ent_coef` the loss
constants — the device path has no other state to update."""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Any, Dict, List, Optional

SCHEDULABLE = ("policy_lr", "ent_coef", "clip_range", "clip_range_vf", "vf_coef")


def linear(start_value: float, end_value: float, fraction: float) -> float:
    """hyperparameter_scheduler.py:8-11."""
    f = max(0.0, min(fraction, 1.0))
    return start_value + (end_value - start_value) * f


def cosine(start_value: float, end_value: float, fraction: float) -> float:
    """hyperparameter_scheduler.py:14-18."""
    f = max(0.0, min(fraction, 1.0))
    return end_value + (start_value - end_value) * (0.5 * (1 + math.cos(math.pi * f)))


def exponential(start_value: float, end_value: float, fraction: float) -> float:
    """hyperparameter_scheduler.py:21-30: decay rate 2, normalised to hit both end points."""
    f = max(0.0, min(fraction, 1.0))
    k = 2.0
    norm = (math.exp(-k * f) - math.exp(-k)) / (1.0 - math.exp(-k))
    return end_value + (start_value - end_value) * norm


CURVES = {"linear": linear, "cosine": cosine, "exponential": exponential}


def schedule_pos_to_vec_steps(raw: Optional[float], *, param: str, default_to_max: bool,
                              max_env_steps: Optional[float], n_envs: int) -> float:
    """utils/schedule_resolver.py:8-51: None -> 0 or the whole budget; <= 1 -> fraction of
    max_env_steps; > 1 -> absolute env steps; always returned in vector steps."""
    if raw is None:
        if default_to_max:
            if max_env_steps is None:
                raise ValueError(f"{param}_schedule requires config.max_env_steps or an explicit {param}_schedule_end.")
            return float(max_env_steps) / n_envs
        return 0.0
    v = float(raw)
    if v < 0.0:
        raise ValueError(f"{param}_schedule start/end must be non-negative.")
    if v <= 1.0:
        if max_env_steps is None:
            raise ValueError(f"{param}_schedule uses fractional start/end but config.max_env_steps is not set.")
        return v * float(max_env_steps) / n_envs
    return v / n_envs


@dataclass
class Scheduler:
    """One HyperparameterSchedulerCallback (hyperparameter_scheduler.py:40-116)."""
    parameter: str
    schedule: str
    start_value: float
    end_value: float
    start_step: float
    end_step: float
    warmup_fraction: float = 0.0

    def __post_init__(self):
        if self.schedule not in CURVES:
            raise ValueError(f"invalid schedule: {self.schedule}")
        if self.end_step < self.start_step:
            raise ValueError("schedule end_step must be >= start_step")
        if not 0.0 <= self.warmup_fraction < 1.0:
            raise ValueError(f"warmup_fraction must be in [0, 1), got {self.warmup_fraction}")

    def fraction(self, total_vec_steps: float) -> float:
        if total_vec_steps <= self.start_step:
            return 0.0
        if total_vec_steps >= self.end_step or self.end_step == self.start_step:
            return 1.0
        return (total_vec_steps - self.start_step) / (self.end_step - self.start_step)

    def value(self, total_vec_steps: float) -> float:
        f = self.fraction(float(total_vec_steps))
        w = self.warmup_fraction
        if w > 0.0 and f < w:          # linear warmup from end_value to start_value
            return self.end_value + (self.start_value - self.end_value) * (f / w)
        g = (f - w) / (1.0 - w) if w > 0.0 else f
        return CURVES[self.schedule](self.start_value, self.end_value, g)


def parse_schedule_dict(value: Dict[str, Any]) -> Dict[str, Any]:
    """utils/config.py:626-655: {start, end=0, from=0, to=1, schedule='linear', warmup=0}."""
    if value.get("start") is None:
        raise ValueError("schedule dict must have 'start' key")
    return {"schedule": value.get("schedule", "linear"), "start_value": float(value["start"]),
            "end_value": float(value.get("end", 0.0)), "start": float(value.get("from", 0.0)),
            "end": float(value.get("to", 1.0)), "warmup": float(value.get("warmup", 0.0))}


def from_attributes(cfg: Any, param: str) -> Optional[Dict[str, Any]]:
    """The resolved attribute form a reference Config carries (`<p>_schedule`,
    `<p>_schedule_start_value`, ... utils/config.py:188-196, 657-674)."""
    kind = getattr(cfg, f"{param}_schedule", None)
    if not kind:
        return None
    sv = getattr(cfg, f"{param}_schedule_start_value", None)
    ev = getattr(cfg, f"{param}_schedule_end_value", None)
    return {"schedule": str(kind), "start_value": float(sv if sv is not None else getattr(cfg, param)),
            "end_value": float(ev if ev is not None else 0.0),
            "start": getattr(cfg, f"{param}_schedule_start", None),
            "end": getattr(cfg, f"{param}_schedule_end", None),
            "warmup": float(getattr(cfg, f"{param}_schedule_warmup", 0.0) or 0.0)}


def build_schedulers(schedules: Dict[str, Dict[str, Any]], max_env_steps: Optional[float],
                     n_envs: int) -> List[Scheduler]:
    """utils/schedule_resolver.py:54-124 over a {param: spec} table."""
    out = []
    for param, s in schedules.items():
        if param not in SCHEDULABLE:
            raise ValueError(f"{param} is not a schedulable hyper-parameter of the device path")
        start = schedule_pos_to_vec_steps(s.get("start"), param=param, default_to_max=False,
                                          max_env_steps=max_env_steps, n_envs=n_envs)
        end = schedule_pos_to_vec_steps(s.get("end"), param=param, default_to_max=True,
                                        max_env_steps=max_env_steps, n_envs=n_envs)
        out.append(Scheduler(param, s["schedule"], float(s["start_value"]), float(s["end_value"]), start, end,
                             float(s.get("warmup", 0.0))))
    return out
