"""Device-resident NatureCNN actor-critic (utils/models.py:347-455 CNNActorCritic) with
optional action masking (utils/policy_ops.py:44-75, utils/distributions.py:8-82).

Parameters live in ONE flat fp32 HBM buffer in the reference's tensor order (cnn.0, cnn.2,
cnn.4, mlp.0, policy_head, value_head).  Inside that order the kernels want NHWC: conv2 /
conv3 weights are stored (out, ky, kx, in) and the fc weight (hidden, y, x, c), so
``state_dict()`` / ``load_state_dict()`` permute to and from the reference's
(out, in, ky, kx) / (hidden, c*y*x) layouts; every other tensor is stored as is.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, Optional, Sequence

import numpy as np
import torch
import torch.nn as nn

from ._lib import CnnDims, check, lib, ptr, stream_handle

CHANNELS, KERNELS, STRIDES = (32, 64, 64), (8, 4, 3), (4, 2, 1)


def cnn_param_shapes(in_shape=(4, 84, 84), n_actions: int = 18, hidden: int = 512):
    C, H, W = in_shape
    shapes, c, h, w = [], C, H, W
    for i, (co, k, s) in enumerate(zip(CHANNELS, KERNELS, STRIDES)):
        shapes += [(f"cnn.{2 * i}.weight", (co, c, k, k)), (f"cnn.{2 * i}.bias", (co,))]
        c, h, w = co, (h - k) // s + 1, (w - k) // s + 1
    shapes += [("mlp.0.weight", (hidden, c * h * w)), ("mlp.0.bias", (hidden,)),
               ("policy_head.weight", (n_actions, hidden)), ("policy_head.bias", (n_actions,)),
               ("value_head.weight", (1, hidden)), ("value_head.bias", (1,))]
    return shapes, (c, h, w)


def valid_mask(valid_actions: Optional[Sequence[int]], n_actions: int) -> int:
    if valid_actions is None:
        return 0
    m = 0
    for a in valid_actions:
        if not 0 <= int(a) < n_actions:
            raise ValueError(f"valid action {a} outside [0, {n_actions})")
        m |= 1 << int(a)
    return m


def reference_init(in_shape=(4, 84, 84), n_actions: int = 18, hidden: int = 512) -> "OrderedDict[str, torch.Tensor]":
    """Module construction order + init_model_weights rules of CNNActorCritic (utils/torch.py:204-258):
    orthogonal gain sqrt(2) for ReLU-followed convs / fc, 0.01 policy head, 1.0 value head,
    zero biases; consumes the torch CPU generator like the reference."""
    C = in_shape[0]
    convs, c = [], C
    for co, k, s in zip(CHANNELS, KERNELS, STRIDES):
        convs.append(nn.Conv2d(c, co, k, s))
        c = co
    shapes, (c3, h3, w3) = cnn_param_shapes(in_shape, n_actions, hidden)
    fc = nn.Linear(c3 * h3 * w3, hidden)
    policy_head = nn.Linear(hidden, n_actions)
    value_head = nn.Linear(hidden, 1)
    gain = nn.init.calculate_gain("relu")
    with torch.no_grad():
        for m in convs + [fc]:
            nn.init.orthogonal_(m.weight, gain=gain)
            nn.init.constant_(m.bias, 0.0)
        nn.init.orthogonal_(policy_head.weight, gain=0.01)
        nn.init.constant_(policy_head.bias, 0.0)
        nn.init.orthogonal_(value_head.weight, gain=1.0)
        nn.init.constant_(value_head.bias, 0.0)
    mods = convs + [fc, policy_head, value_head]
    sd = OrderedDict()
    for (name, _), t in zip(shapes, [p for m in mods for p in (m.weight, m.bias)]):
        sd[name] = t.detach().clone()
    return sd


class DeviceCNNActorCritic:
    """NatureCNN actor-critic whose forward/backward run in libgsamd (gs_cnn_*)."""

    def __init__(self, in_shape=(4, 84, 84), n_actions: int = 18, hidden: int = 512,
                 valid_actions: Optional[Sequence[int]] = None, device="cuda", init: bool = True):
        self.in_shape = tuple(int(x) for x in in_shape)
        self.n_actions, self.hidden = int(n_actions), int(hidden)
        self.valid_actions = None if valid_actions is None else [int(a) for a in valid_actions]
        self.dims = CnnDims(*self.in_shape, self.n_actions, self.hidden, valid_mask(self.valid_actions, self.n_actions))
        self.n_params = int(lib.gs_cnn_param_count(self.dims))
        if self.n_params <= 0:
            raise ValueError(f"unsupported CNN input {self.in_shape} / {self.n_actions} actions")
        self._shapes, self.feat_chw = cnn_param_shapes(self.in_shape, self.n_actions, self.hidden)
        self.device = torch.device(device)
        self.params = torch.zeros(self.n_params, dtype=torch.float32, device=self.device)
        self._scratch = {}
        if init:
            self.load_state_dict(reference_init(self.in_shape, self.n_actions, self.hidden))

    def shapes(self):
        return self._shapes

    # --- reference layout <-> internal layout -------------------------------------------------
    def _to_internal(self, name, t: torch.Tensor) -> torch.Tensor:
        if name in ("cnn.2.weight", "cnn.4.weight"):
            return t.permute(0, 2, 3, 1)                      # (out, ky, kx, in)
        if name == "mlp.0.weight":
            c, h, w = self.feat_chw
            return t.reshape(self.hidden, c, h, w).permute(0, 2, 3, 1)   # (hidden, y, x, c)
        return t

    def _from_internal(self, name, t: torch.Tensor, shp) -> torch.Tensor:
        if name in ("cnn.2.weight", "cnn.4.weight"):
            o, i, k, _ = shp
            return t.reshape(o, k, k, i).permute(0, 3, 1, 2)
        if name == "mlp.0.weight":
            c, h, w = self.feat_chw
            return t.reshape(self.hidden, h, w, c).permute(0, 3, 1, 2).reshape(shp)
        return t.reshape(shp)

    def flat_from_reference(self, flat_ref) -> torch.Tensor:
        """Flat vector in the reference's layout -> internal flat vector (host)."""
        flat_ref = torch.as_tensor(np.asarray(flat_ref, np.float32))
        parts, o = [], 0
        for name, shp in self._shapes:
            n = int(np.prod(shp))
            parts.append(self._to_internal(name, flat_ref[o:o + n].reshape(shp)).reshape(-1))
            o += n
        return torch.cat(parts)

    def flat_to_reference(self, flat_int) -> np.ndarray:
        flat_int = torch.as_tensor(flat_int).detach().cpu()
        parts, o = [], 0
        for name, shp in self._shapes:
            n = int(np.prod(shp))
            parts.append(self._from_internal(name, flat_int[o:o + n], shp).reshape(-1))
            o += n
        return torch.cat(parts).numpy()

    def state_dict(self) -> "OrderedDict[str, torch.Tensor]":
        flat = torch.as_tensor(self.flat_to_reference(self.params))
        out, o = OrderedDict(), 0
        for name, shp in self._shapes:
            n = int(np.prod(shp))
            out[name] = flat[o:o + n].view(shp).clone()
            o += n
        return out

    def load_state_dict(self, sd: Dict[str, torch.Tensor]) -> None:
        parts = []
        for name, shp in self._shapes:
            t = torch.as_tensor(sd[name], dtype=torch.float32)
            if tuple(t.shape) != tuple(shp):
                raise ValueError(f"{name}: expected shape {shp}, got {tuple(t.shape)}")
            parts.append(self._to_internal(name, t).reshape(-1))
        self.params.copy_(torch.cat(parts).to(self.device))

    def load_reference_flat(self, flat_ref) -> None:
        self.params.copy_(self.flat_from_reference(flat_ref).to(self.device))

    # --- forward ------------------------------------------------------------------------------
    def workspace(self, rows: int) -> torch.Tensor:
        t = self._scratch.get(rows)
        if t is None:
            nbytes = int(lib.gs_cnn_workspace_bytes(self.dims, rows))
            t = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
            self._scratch[rows] = t
        return t

    def act(self, obs: torch.Tensor, *, mode: int = 0, rng_seed: int = 0, rng_counter: int = 0,
            actions: torch.Tensor = None, logp: torch.Tensor = None, values: torch.Tensor = None,
            obs_store: torch.Tensor = None, clock: torch.Tensor = None):
        """policy_act (utils/policy_ops.py:14-34) on u8 frame stacks (N, C, H, W); obs_store
        (the rollout row) receives a copy of the observation (written by the first convolution)."""
        n = obs.shape[0]
        if not (obs.is_contiguous() and obs.dtype == torch.uint8 and obs.device == self.device):
            raise ValueError("obs must be a contiguous uint8 device tensor (N, C, H, W)")
        if obs_store is not None and not (obs_store.is_contiguous() and obs_store.dtype == torch.uint8
                                          and obs_store.shape == obs.shape and obs_store.device == obs.device):
            raise ValueError("obs_store must be a contiguous uint8 device tensor shaped like obs")
        if actions is None:
            actions = torch.empty(n, dtype=torch.int64, device=self.device)
        if logp is None:
            logp = torch.empty(n, dtype=torch.float32, device=self.device)
        if values is None:
            values = torch.empty(n, dtype=torch.float32, device=self.device)
        check(lib.gs_cnn_policy_act(ptr(self.params), self.dims, ptr(obs), n, int(mode), int(rng_seed),
                                    int(rng_counter), ptr(actions), ptr(logp), ptr(values),
                                    ptr(obs_store) if obs_store is not None else None, ptr(self.workspace(n)),
                                    ptr(clock), stream_handle()), "gs_cnn_policy_act")
        return actions, logp, values

    def predict_values(self, obs: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
        n = obs.shape[0]
        if out is None:
            out = torch.empty(n, dtype=torch.float32, device=self.device)
        check(lib.gs_cnn_policy_act(ptr(self.params), self.dims, ptr(obs), n, 0, 0, 0, None, None, ptr(out), None,
                                    ptr(self.workspace(n)), None, stream_handle()), "gs_cnn_policy_act")
        return out

    def parameters(self):
        return [self.params]
