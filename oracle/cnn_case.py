"""ORACLE — test infrastructure only.  Deterministic CNN PPO cases without LAPACK: parameters
and observations come from the SplitMix64 counter hash (identical on every host), the rest
from numpy's PCG64 with a fixed seed.  Used by tests/golden/make_golden.py (reference outputs)
and by the CPU/GPU tests (inputs regenerated, never stored)."""
from __future__ import annotations

import numpy as np

from .cnn_ref import NATURE, cnn_param_shapes

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _mix64(z):
    z = (z + np.uint64(0x9E3779B97F4A7C15)) & M64
    z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & M64
    z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & M64
    return z ^ (z >> np.uint64(31))


def hash_uniform(seed: int, n: int) -> np.ndarray:
    """n floats uniform in [-1, 1) from mix64(seed * 2^32 + i)."""
    with np.errstate(over="ignore"):
        i = np.arange(n, dtype=np.uint64) + (np.uint64(seed) << np.uint64(32))
        h = _mix64(i)
    return ((h >> np.uint64(40)).astype(np.float64) * 2.0 ** -23 - 1.0).astype(np.float32)


def hash_u8(seed: int, n: int) -> np.ndarray:
    with np.errstate(over="ignore"):
        i = np.arange(n, dtype=np.uint64) + (np.uint64(seed) << np.uint64(32))
        return (_mix64(i) >> np.uint64(56)).astype(np.uint8)


def cnn_params(seed: int = 1, in_shape=(4, 84, 84), n_actions=18, spec=NATURE) -> np.ndarray:
    """Flat params: each tensor uniform in +-sqrt(3 / fan_in) (unit-variance activations)."""
    out = []
    for k, (name, s) in enumerate(cnn_param_shapes(in_shape, n_actions, spec)):
        n = int(np.prod(s))
        fan_in = int(np.prod(s[1:])) if len(s) > 1 else 1
        scale = np.sqrt(3.0 / fan_in) if name.endswith("weight") else 0.05
        if name.startswith("policy_head.weight"):
            scale *= 0.1
        out.append(hash_uniform(seed * 1000 + k, n) * np.float32(scale))
    return np.concatenate(out).astype(np.float32)


def cnn_batch(seed: int, B: int, valid, in_shape=(4, 84, 84), n_actions=18):
    """(obs u8 (B,C,H,W), actions, old_logp, old_values, adv, ret) — old_logp near uniform over
    the valid actions; actions drawn from the valid set."""
    rng = np.random.default_rng(seed)
    obs = hash_u8(seed, B * int(np.prod(in_shape))).reshape(B, *in_shape)
    va = np.asarray(valid if valid is not None else range(n_actions))
    actions = va[rng.integers(0, len(va), B)].astype(np.int64)
    old_logp = (np.log(1.0 / len(va)) + 0.05 * rng.standard_normal(B)).astype(np.float32)
    old_values = (0.1 * rng.standard_normal(B)).astype(np.float32)
    adv = (rng.standard_normal(B) * 2.0 + 0.3).astype(np.float32)
    ret = (old_values + adv).astype(np.float32)
    return obs, actions, old_logp, old_values, adv, ret
