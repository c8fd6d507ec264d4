"""Device-resident MLP actor-critic (utils/models.py:285-346 MLPActorCritic).

Parameters live in ONE flat fp32 HBM buffer in the reference's state_dict order, so the
optimizer, gradient clip and the multi-GPU all-reduce each touch a single contiguous
vector.  ``state_dict()`` / ``load_state_dict()`` speak the reference's key names
(``backbone.0.weight`` ... ``value_head.bias``) so checkpoints interoperate.
Initialisation reproduces utils/torch.py:204-258 (orthogonal, gain sqrt(2) for
ReLU-followed layers, 0.01 policy head, 1.0 value head, zero bias) with the same torch
CPU RNG consumption as the reference's module construction, so a given torch seed gives
bit-identical initial weights.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, Sequence, Tuple

import torch
import torch.nn as nn

from . import _lib
from ._lib import MlpDims, check, lib, ptr, stream_handle


def param_shapes(obs_dim: int, hidden: Sequence[int], n_actions: int):
    shapes, last = [], obs_dim
    for i, h in enumerate(hidden):
        shapes.append((f"backbone.{2 * i}.weight", (h, last)))
        shapes.append((f"backbone.{2 * i}.bias", (h,)))
        last = h
    shapes += [("policy_head.weight", (n_actions, last)), ("policy_head.bias", (n_actions,)),
               ("value_head.weight", (1, last)), ("value_head.bias", (1,))]
    return shapes


def reference_init(obs_dim: int, hidden: Sequence[int], n_actions: int) -> "OrderedDict[str, torch.Tensor]":
    """Same module construction order + init rules as MLPActorCritic (consumes the torch
    CPU default generator exactly like the reference)."""
    layers, last = [], obs_dim
    for h in hidden:
        layers += [nn.Linear(last, h), nn.ReLU()]
        last = h
    backbone = nn.Sequential(*layers)
    policy_head = nn.Linear(last, n_actions)
    value_head = nn.Linear(last, 1)
    gain = nn.init.calculate_gain("relu")
    with torch.no_grad():
        for m in backbone:
            if isinstance(m, nn.Linear):
                nn.init.orthogonal_(m.weight, gain=gain)
                nn.init.constant_(m.bias, 0.0)
        nn.init.orthogonal_(policy_head.weight, gain=0.01)
        nn.init.constant_(policy_head.bias, 0.0)
        nn.init.orthogonal_(value_head.weight, gain=1.0)
        nn.init.constant_(value_head.bias, 0.0)
    sd = OrderedDict()
    for i, m in enumerate(backbone):
        if isinstance(m, nn.Linear):
            sd[f"backbone.{i}.weight"] = m.weight.detach().clone()
            sd[f"backbone.{i}.bias"] = m.bias.detach().clone()
    sd["policy_head.weight"] = policy_head.weight.detach().clone()
    sd["policy_head.bias"] = policy_head.bias.detach().clone()
    sd["value_head.weight"] = value_head.weight.detach().clone()
    sd["value_head.bias"] = value_head.bias.detach().clone()
    return sd


class DeviceMLPActorCritic:
    """Two-hidden-layer ReLU actor-critic whose forward runs in libgsamd kernels."""

    def __init__(self, obs_dim: int, hidden_dims: Tuple[int, ...], n_actions: int, device="cuda",
                 init: bool = True):
        if len(hidden_dims) != 2:
            raise ValueError(f"device MLP path implements two hidden layers, got {hidden_dims}")
        self.obs_dim, self.hidden_dims, self.n_actions = int(obs_dim), tuple(int(h) for h in hidden_dims), int(n_actions)
        self.dims = MlpDims(self.obs_dim, self.hidden_dims[0], self.hidden_dims[1], self.n_actions)
        self.n_params = int(lib.gs_mlp_param_count(self.dims))
        self.device = torch.device(device)
        self.params = torch.zeros(self.n_params, dtype=torch.float32, device=self.device)
        self._scratch = {}
        if init:
            self.load_state_dict(reference_init(self.obs_dim, self.hidden_dims, self.n_actions))

    # --- state dict in the reference's key order -----------------------------------------
    def shapes(self):
        return param_shapes(self.obs_dim, self.hidden_dims, self.n_actions)

    def state_dict(self) -> "OrderedDict[str, torch.Tensor]":
        out, o = OrderedDict(), 0
        flat = self.params.detach().cpu()
        for name, shp in self.shapes():
            n = 1
            for s in shp:
                n *= s
            out[name] = flat[o:o + n].view(shp).clone()
            o += n
        return out

    def load_state_dict(self, sd: Dict[str, torch.Tensor]) -> None:
        parts = []
        for name, shp in self.shapes():
            t = torch.as_tensor(sd[name], dtype=torch.float32)
            if tuple(t.shape) != tuple(shp):
                raise ValueError(f"{name}: expected shape {shp}, got {tuple(t.shape)}")
            parts.append(t.reshape(-1))
        self.params.copy_(torch.cat(parts).to(self.device))

    def load_flat(self, flat) -> None:
        self.params.copy_(torch.as_tensor(flat, dtype=torch.float32).to(self.device))

    # --- forward --------------------------------------------------------------------------
    def scratch(self, n: int) -> torch.Tensor:
        t = self._scratch.get(n)
        if t is None:
            nbytes = int(lib.gs_policy_scratch_bytes(self.dims, n))
            t = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
            self._scratch[n] = t
        return t

    def act(self, obs: torch.Tensor, *, mode: int = 0, rng_seed: int = 0, rng_counter: int = 0,
            actions: torch.Tensor = None, logp: torch.Tensor = None, values: torch.Tensor = None,
            obs_store: torch.Tensor = None, clock: torch.Tensor = None):
        """policy_act (utils/policy_ops.py:14-34): returns (actions int64, logp, values).  clock:
        optional (2,) uint64 device tensor whose [0] is added to rng_counter on device."""
        n = obs.shape[0]
        assert obs.is_contiguous() and obs.dtype == torch.float32 and obs.device == self.device
        if actions is None:
            actions = torch.empty(n, dtype=torch.int64, device=self.device)
        if logp is None:
            logp = torch.empty(n, dtype=torch.float32, device=self.device)
        if values is None:
            values = torch.empty(n, dtype=torch.float32, device=self.device)
        check(lib.gs_policy_act(ptr(self.params), self.dims, ptr(obs), n, int(mode), int(rng_seed),
                                int(rng_counter), ptr(actions), ptr(logp), ptr(values), ptr(obs_store),
                                ptr(self.scratch(n)), ptr(clock), stream_handle()), "gs_policy_act")
        return actions, logp, values

    def predict_values(self, obs: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
        """policy_predict_values (utils/policy_ops.py:37-42)."""
        n = obs.shape[0]
        if out is None:
            out = torch.empty(n, dtype=torch.float32, device=self.device)
        check(lib.gs_policy_value(ptr(self.params), self.dims, ptr(obs), n, ptr(out), ptr(self.scratch(n)),
                                  stream_handle()), "gs_policy_value")
        return out

    def parameters(self):
        return [self.params]


_ = _lib  # keep the binding module referenced
