"""Metrics recording for the device agent, behind the reference's recorder surface
(utils/metrics_recorder.py:11-76, utils/metrics_buffer.py:8-31): ``record(namespace, metrics)``
appends one record, ``compute_epoch_means(namespace)`` averages every key over its records,
``reset_epoch(namespace)`` clears them.

The device update writes one 24-float record per minibatch (include/gsamd.h GS_M_* slots) and
the host reads them once per epoch; ``ppo_records`` turns such records into the reference's
``losses_for_batch`` keys (agents/ppo/ppo_agent.py:131-146, utils/torch.py:170-173), and
``record_rows`` books a whole block of them at once (no per-minibatch Python on the fast path).
"""
from __future__ import annotations

import math
from typing import Dict, List, Mapping

import numpy as np

from ._lib import M

# losses_for_batch's record, in the order ppo_agent.py builds it
PPO_KEYS = ("opt/loss/total", "opt/loss/policy", "opt/loss/entropy", "opt/policy/entropy",
            "opt/loss/entropy_scaled", "opt/loss/value", "opt/loss/value_scaled", "opt/ppo/clip_fraction",
            "opt/ppo/clip_fraction_vf", "opt/value/explained_var", "opt/ppo/kl_stop_triggered", "opt/ppo/kl",
            "opt/ppo/approx_kl")
ADV_NORM_KEYS = ("roll/adv/norm/mean", "roll/adv/norm/std")


def ppo_records(rows: np.ndarray, vf_coef: float, ent_coef: float, normalize_batch: bool) -> np.ndarray:
    """(n, GS_NUM_METRICS) device records -> (n, K) values for PPO_KEYS (+ ADV_NORM_KEYS).  The
    derived terms are formed in f32 as the reference's tensors are."""
    r = np.asarray(rows, np.float32).reshape(-1, rows.shape[-1])
    ent = r[:, M["entropy"]]
    ent_loss = -ent
    vl = r[:, M["value_loss"]]
    cols = [r[:, M["loss"]], r[:, M["policy_loss"]], ent_loss, ent, np.float32(ent_coef) * ent_loss, vl,
            np.float32(vf_coef) * vl, r[:, M["clip_fraction"]], r[:, M["clip_fraction_vf"]],
            r[:, M["explained_var"]], r[:, M["kl_stop"]], r[:, M["kl"]], r[:, M["approx_kl"]]]
    if normalize_batch:
        cols += [r[:, M["adv_norm_mean"]], r[:, M["adv_norm_std"]]]
    return np.stack(cols, axis=1).astype(np.float64)


NUM_SUMS = 14      # raw loss sums per minibatch (include/gsamd.h gs_ppo_global.metric_sums)


def records_from_sums(sums: np.ndarray, rows: int, vf_coef: float, ent_coef: float, normalize: bool) -> np.ndarray:
    """(n, 14) raw loss sums of whole minibatches (every rank's added) -> the (n, 24) loss slots of
    the device records, with the arithmetic of csrc/gs_mlp.hip write_metrics (f32 terms from
    double sums; torch.var's unbiased variance for explained_var, utils/torch.py:97-99 statistics
    for the normalised advantages).  The KL / skip / grad-norm slots are left at zero."""
    t = np.asarray(sums, np.float64).reshape(-1, NUM_SUMS)
    Bd = float(rows)
    out = np.zeros((t.shape[0], len(M)), np.float32)
    pl = (-t[:, 0] / Bd).astype(np.float32)
    vl = (t[:, 1] / Bd).astype(np.float32)
    ent = (t[:, 2] / Bd).astype(np.float32)
    loss = (pl + np.float32(vf_coef) * vl) + np.float32(ent_coef) * (-ent)
    with np.errstate(divide="ignore", invalid="ignore"):
        var_rv = (t[:, 8] - t[:, 7] * t[:, 7] / Bd) / (Bd - 1.0)
        var_r = (t[:, 10] - t[:, 9] * t[:, 9] / Bd) / (Bd - 1.0)
        out[:, M["explained_var"]] = (1.0 - var_rv / var_r).astype(np.float32)
    out[:, M["loss"]], out[:, M["policy_loss"]], out[:, M["value_loss"]], out[:, M["entropy"]] = loss, pl, vl, ent
    out[:, M["clip_fraction"]] = (t[:, 3] / Bd).astype(np.float32)
    out[:, M["clip_fraction_vf"]] = (t[:, 4] / Bd).astype(np.float32)
    out[:, M["kl"]] = (t[:, 5] / Bd).astype(np.float32)
    out[:, M["approx_kl"]] = (t[:, 6] / Bd).astype(np.float32)
    if normalize:
        out[:, M["adv_norm_mean"]] = (t[:, 11] / Bd).astype(np.float32)
        out[:, M["adv_norm_std"]] = np.sqrt(np.maximum(0.0, (t[:, 12] - t[:, 11] ** 2 / Bd) / (Bd - 1.0))
                                            ).astype(np.float32)
    return out


def ppo_keys(normalize_batch: bool):
    return PPO_KEYS + (ADV_NORM_KEYS if normalize_batch else ())


class MetricsRecorder:
    def __init__(self):
        self._sums: Dict[str, Dict[str, float]] = {}
        self._counts: Dict[str, Dict[str, int]] = {}

    def record(self, namespace: str, metrics: Mapping[str, object]) -> None:
        """One record; values are reduced to Python scalars (torch / numpy one-element values
        included) and must be finite numbers, as the reference asserts."""
        if not metrics:
            raise AssertionError("metrics cannot be empty")
        s, c = self._ns(namespace)
        for k, v in metrics.items():
            x = _scalar(v)
            if x is None:
                continue
            if math.isnan(x) or math.isinf(x):
                raise AssertionError(f"metric '{k}' is not finite: {x}")
            s[k] = s.get(k, 0.0) + x
            c[k] = c.get(k, 0) + 1

    def record_rows(self, namespace: str, keys, values: np.ndarray) -> None:
        """len(values) records at once (rows of `values`, columns named by `keys`)."""
        v = np.asarray(values, np.float64).reshape(-1, len(keys))
        if v.shape[0] == 0:
            return
        if not np.isfinite(v).all():
            raise AssertionError(f"non-finite metric in {namespace} records")
        s, c = self._ns(namespace)
        tot = v.sum(axis=0)
        for j, k in enumerate(keys):
            s[k] = s.get(k, 0.0) + float(tot[j])
            c[k] = c.get(k, 0) + v.shape[0]

    def compute_epoch_means(self, namespace: str) -> Dict[str, float]:
        s, c = self._ns(namespace)
        return {k: s[k] / c[k] for k in s if c[k]}

    def sums_counts(self, namespace: str, keys) -> np.ndarray:
        """(2, len(keys)) float64: the sum and the record count of each key (zeros for a key with
        no record) — a fixed-length vector a multi-rank job can all-reduce."""
        s, c = self._ns(namespace)
        return np.array([[s.get(k, 0.0) for k in keys], [float(c.get(k, 0)) for k in keys]], np.float64)

    def reset_epoch(self, namespace: str) -> None:
        s, c = self._ns(namespace)
        s.clear()
        c.clear()

    def namespaces(self) -> List[str]:
        return sorted(self._sums)

    def _ns(self, namespace: str):
        if not namespace:
            raise AssertionError("namespace cannot be empty")
        return self._sums.setdefault(namespace, {}), self._counts.setdefault(namespace, {})


def _scalar(v):
    if isinstance(v, bool):
        return float(v)
    if isinstance(v, (int, float)):
        return float(v)
    if hasattr(v, "numel") and v.numel() == 1:        # torch tensor
        return float(v.item())
    a = np.asarray(v)
    if a.size == 1 and a.dtype.kind in "biuf":
        return float(a.reshape(()).item())
    return None


def activation_stats(parts: np.ndarray, rows: int, hidden: tuple, prefix: str = "backbone",
                     layer_ids: tuple = (0, 2)) -> Dict[str, float]:
    """gs_mlp_activation_stats parts (n_parts, 2 * (2 + max(H))) -> the reference's
    ``opt/activations/<prefix>.<i>/{mean,std,dead_pct,dead_max}`` (utils/models.py:120-145,184-190:
    mean and unbiased std over all of a Linear layer's outputs, dead_pct / dead_max the mean / max
    over neurons of the fraction of rows with |z| < 1e-6)."""
    p = np.asarray(parts, np.float64).reshape(parts.shape[0], 2, -1).sum(axis=0)
    out: Dict[str, float] = {}
    for layer, (lid, H) in enumerate(zip(layer_ids, hidden)):
        n = float(rows) * H
        s1, s2 = p[layer, 0], p[layer, 1]
        dead = p[layer, 2:2 + H] / float(rows)
        name = f"opt/activations/{prefix}.{lid}"
        out[f"{name}/mean"] = s1 / n
        out[f"{name}/std"] = math.sqrt(max(0.0, (s2 - s1 * s1 / n) / (n - 1.0)))
        out[f"{name}/dead_pct"] = float(dead.mean())
        out[f"{name}/dead_max"] = float(dead.max())
    return out

