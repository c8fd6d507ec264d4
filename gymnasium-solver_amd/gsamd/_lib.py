"""ctypes binding of libgsamd.so (the C-ABI declared in include/gsamd.h).

The library is built in-tree by ``__graft_entry__.build()`` and linked against the same
HIP runtime soname torch loads (libamdhip64.so.7), so importing torch first makes both
share one runtime.  There is no fallback: if the library is missing, importing any
device module raises, loudly.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (load torch's HIP runtime before the library)

# GSAMD_LIB selects a diagnostic build of the same library (tools/ phase-timer variant)
LIB_PATH = os.environ.get("GSAMD_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libgsamd.so")

GS_OK, GS_E_INVALID, GS_E_HIP, GS_E_COMM = 0, -1, -2, -3
GS_ABI_VERSION = 7          # include/gsamd.h: the argument lists this binding declares
GS_NUM_METRICS = 40
METRIC_SLOTS = (
    "loss", "policy_loss", "value_loss", "entropy", "clip_fraction", "clip_fraction_vf",
    "explained_var", "kl", "approx_kl", "adv_norm_mean", "adv_norm_std", "kl_stop", "grad_norm",
    "skipped", "unevaluated", "res1",
    # pre-clip per-component gradient norms (utils/models.py:196-230)
    "gn_backbone", "gn_policy_head", "gn_value_head", "gn_mlp", "res20", "res21", "res22", "res23",
    # GS_HP_ACT_STATS: per hooked layer {mean, std, dead_pct, dead_max} (utils/models.py:121-147)
    *(f"act{l}_{k}" for l in range(4) for k in ("mean", "std", "dead_pct", "dead_max")),
)
ACT_SLOT = 24                # GS_M_ACT
M = {name: i for i, name in enumerate(METRIC_SLOTS)}


class MlpDims(ctypes.Structure):
    _fields_ = [("obs_dim", ctypes.c_int32), ("hidden1", ctypes.c_int32), ("hidden2", ctypes.c_int32),
                ("n_actions", ctypes.c_int32)]


class PPOHparams(ctypes.Structure):
    _fields_ = [("clip_range", ctypes.c_float), ("clip_range_vf", ctypes.c_float), ("vf_coef", ctypes.c_float),
                ("ent_coef", ctypes.c_float), ("max_grad_norm", ctypes.c_float), ("lr", ctypes.c_float),
                ("adam_beta1", ctypes.c_float), ("adam_beta2", ctypes.c_float), ("adam_eps", ctypes.c_float),
                ("target_kl", ctypes.c_float), ("normalize_adv", ctypes.c_int32), ("flags", ctypes.c_int32)]


GS_HP_BF16 = 1      # include/gsamd.h: bf16 MFMA operands in the NatureCNN update
GS_HP_ACT_STATS = 2  # include/gsamd.h: per-minibatch activation statistics into the records (GS_M_ACT)


class RolloutView(ctypes.Structure):
    _fields_ = [("obs", ctypes.c_void_p), ("actions", ctypes.c_void_p), ("logprobs", ctypes.c_void_p),
                ("values", ctypes.c_void_p), ("advantages", ctypes.c_void_p), ("returns", ctypes.c_void_p),
                ("T", ctypes.c_int64), ("N", ctypes.c_int64)]


class PPOGlobal(ctypes.Structure):
    """gs_ppo_global (include/gsamd.h): the global-minibatch mode's extra arguments."""
    _fields_ = [("batch_global", ctypes.c_int64), ("adv_stats", ctypes.c_void_p), ("metric_sums", ctypes.c_void_p)]


class CnnDims(ctypes.Structure):
    _fields_ = [("in_c", ctypes.c_int32), ("in_h", ctypes.c_int32), ("in_w", ctypes.c_int32),
                ("n_actions", ctypes.c_int32), ("hidden", ctypes.c_int32), ("valid_mask", ctypes.c_uint32)]


class RolloutViewU8(ctypes.Structure):
    _fields_ = RolloutView._fields_


class GsError(RuntimeError):
    pass


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is not built: the device path has no CPU fallback. "
            "Run `python -c 'import __graft_entry__ as g; g.build()'` from the repo root.")
    L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    vp, i32, i64, u64, f32, f64, sz = (ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64,
                                       ctypes.c_float, ctypes.c_double, ctypes.c_size_t)
    sig = {
        "gs_abi_version": (ctypes.c_int, []),
        "gs_last_error": (ctypes.c_char_p, []),
        "gs_build_source_hash": (ctypes.c_char_p, [ctypes.c_char_p]),
        "gs_normalize_advantages_scratch_bytes": (sz, [i64]),
        "gs_normalize_advantages": (ctypes.c_int, [vp, i64, f32, vp, vp, vp]),
        "gs_cnn_activation_stats": (ctypes.c_int, [vp, CnnDims, RolloutViewU8, vp, i64, vp, vp, vp]),
        "gs_gae_f32": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, i64, i64, f64, f64, vp, vp, vp]),
        "gs_sampler_stream_i32": (ctypes.c_int, [i64, i64, u64, vp, ctypes.c_int]),
        "gs_mlp_param_count": (i64, [MlpDims]),
        "gs_policy_scratch_bytes": (sz, [MlpDims, i64]),
        "gs_policy_act": (ctypes.c_int, [vp, MlpDims, vp, i64, ctypes.c_int, u64, u64, vp, vp, vp, vp, vp, vp, vp]),
        "gs_policy_value": (ctypes.c_int, [vp, MlpDims, vp, i64, vp, vp, vp]),
        "gs_rollout_synth_supported": (ctypes.c_int, [MlpDims, vp]),
        "gs_rollout_synth": (ctypes.c_int, [vp, MlpDims, i64, i64, ctypes.c_int, u64, u64, vp, vp, vp, i32, i32, f32,
                                            u64, i64, u64, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
        "gs_env_reset": (ctypes.c_int, [vp, vp, vp, i64, i32, i32, u64, i64, vp]),
        "gs_env_step": (ctypes.c_int, [vp, vp, vp, i64, i32, i32, i32, f32, u64, i64, u64, vp, vp, vp, vp, vp,
                                       vp, vp, vp]),
        "gs_episode_stats": (ctypes.c_int, [vp, vp, i64, i64, vp, vp, vp, vp, vp]),
        "gs_episode_window": (ctypes.c_int, [vp, vp, vp, i64, i64, i64, vp, vp, vp, vp]),
        "gs_ppo_workspace_bytes": (sz, [MlpDims, i64]),
        "gs_ppo_minibatch_step": (ctypes.c_int, [vp, vp, vp, vp, MlpDims, PPOHparams, RolloutView, vp, i64, i64,
                                                 vp, vp, vp, vp, vp]),
        "gs_ppo_loss": (ctypes.c_int, [vp, MlpDims, PPOHparams, RolloutView, vp, i64, vp, vp, vp]),
        "gs_mlp_activation_stats": (ctypes.c_int, [vp, MlpDims, RolloutView, vp, i64, vp, vp]),
        "gs_ppo_stage": (ctypes.c_int, [ctypes.c_int, vp, vp, vp, vp, MlpDims, PPOHparams, RolloutView, vp, i64,
                                        i64, vp, vp, vp]),
        "gs_ppo_update": (ctypes.c_int, [vp, vp, vp, vp, MlpDims, PPOHparams, RolloutView, vp, i64, i64, i64, vp,
                                         vp, vp, sz, vp, ctypes.c_int, vp]),
        "gs_ppo_update_global": (ctypes.c_int, [vp, vp, vp, vp, MlpDims, PPOHparams, RolloutView, vp, i64, i64, i64,
                                                vp, vp, vp, sz, vp, ctypes.c_int, ctypes.POINTER(PPOGlobal), vp]),
        "gs_ppo_update_workspace_bytes": (sz, [MlpDims, i64, i64]),
        "gs_ppo_graph_cache_info": (ctypes.c_int, [vp, vp]),
        "gs_ppo_exchange_inside_bwd": (ctypes.c_int, [vp, MlpDims, ctypes.c_int64, vp]),
        "gs_cnn_param_count": (i64, [CnnDims]),
        "gs_cnn_workspace_bytes": (sz, [CnnDims, i64]),
        "gs_cnn_workspace_hidden_offset": (i64, [CnnDims, i64]),
        "gs_cnn_workspace_act_offset": (i64, [CnnDims, i64, ctypes.c_int]),
        "gs_cnn_policy_act": (ctypes.c_int, [vp, CnnDims, vp, i64, ctypes.c_int, u64, u64, vp, vp, vp, vp, vp, vp, vp]),
        "gs_cnn_ppo_loss": (ctypes.c_int, [vp, CnnDims, PPOHparams, RolloutViewU8, vp, i64, vp, vp, vp, vp]),
        "gs_cnn_ppo_update": (ctypes.c_int, [vp, vp, vp, vp, CnnDims, PPOHparams, RolloutViewU8, vp, i64, i64, i64,
                                             vp, vp, vp, vp, vp]),
        "gs_cnn_ppo_update_global": (ctypes.c_int, [vp, vp, vp, vp, CnnDims, PPOHparams, RolloutViewU8, vp, vp, i64, i64,
                                                    i64, vp, vp, vp, vp, ctypes.POINTER(PPOGlobal), vp]),
        "gs_gemm_f32": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, i64, i64, i64, vp, i64, vp, i64, vp, i64,
                                       f32, vp, ctypes.c_int, vp]),
        "gs_fc_gemm": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, i64, i64, i64, vp, i64, vp, i64, vp, i64, vp, vp,
                                      vp]),
        "gs_cartpole_reset": (ctypes.c_int, [vp, vp, vp, vp, i64, u64, i64, vp]),
        "gs_cartpole_step": (ctypes.c_int, [vp, vp, vp, vp, vp, i64, i32, u64, i64, vp, vp, vp, vp, vp, vp, vp]),
        "gs_atari_preprocess": (ctypes.c_int, [vp, i64, i32, i32, vp, vp]),
        "gs_atari_render": (ctypes.c_int, [vp, i64, u64, i64, u64, vp]),
        "gs_atari_env_reset": (ctypes.c_int, [vp, vp, vp, vp, i64, i32, i32, i32, i32, u64, i64, vp]),
        "gs_atari_env_step": (ctypes.c_int, [vp, vp, vp, vp, i64, i32, i32, i32, i32, i32, u64, i64, u64, vp, vp, vp,
                                             vp, vp, vp, vp, vp]),
        "gs_comm_unique_id": (ctypes.c_int, [vp]),
        "gs_comm_init": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp)]),
        "gs_comm_xgmi_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, i64, vp, ctypes.POINTER(vp)]),
        "gs_comm_xgmi_connect": (ctypes.c_int, [vp, vp]),
        "gs_comm_status": (ctypes.c_int, [vp]),
        "gs_comm_error_record": (ctypes.c_int, [vp, vp, vp, vp, vp]),
        "gs_comm_xgmi_set_colocation": (ctypes.c_int, [vp, ctypes.c_int]),
        "gs_comm_xgmi_set_bwd_exchange": (ctypes.c_int, [vp, ctypes.c_int]),
        "gs_comm_xgmi_reset": (ctypes.c_int, [vp]),
        "gs_comm_allreduce_mean_f32": (ctypes.c_int, [vp, vp, i64, vp]),
        "gs_comm_allreduce_sum_f64": (ctypes.c_int, [vp, vp, i64, vp]),
        "gs_ppo_global_adv_stats": (ctypes.c_int, [vp, i64, i64, i64, vp, i64, i64, vp, vp, vp, vp]),
        "gs_ppo_global_records": (ctypes.c_int, [ctypes.POINTER(PPOHparams), i64, i64, vp, vp, vp, vp]),
        "gs_comm_info": (ctypes.c_int, [vp, vp, vp, vp]),
        "gs_comm_destroy": (ctypes.c_int, [vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    if L.gs_abi_version() != GS_ABI_VERSION:
        raise ImportError(f"{LIB_PATH} implements C-ABI version {L.gs_abi_version()}, this binding version "
                          f"{GS_ABI_VERSION}: rebuild the library (__graft_entry__.build())")
    return L


lib = _load()
EXPORTED = ("gs_abi_version", "gs_last_error", "gs_build_source_hash", "gs_normalize_advantages_scratch_bytes", "gs_normalize_advantages",
            "gs_cnn_activation_stats", "gs_gae_f32", "gs_sampler_stream_i32", "gs_mlp_param_count",
            "gs_policy_scratch_bytes", "gs_policy_act", "gs_policy_value", "gs_rollout_synth_supported",
            "gs_rollout_synth", "gs_env_reset", "gs_env_step",
            "gs_episode_stats", "gs_episode_window",
            "gs_ppo_workspace_bytes", "gs_ppo_minibatch_step", "gs_ppo_loss", "gs_mlp_activation_stats", "gs_ppo_stage", "gs_ppo_update",
            "gs_ppo_update_global", "gs_ppo_update_workspace_bytes",
            "gs_ppo_graph_cache_info", "gs_ppo_exchange_inside_bwd",
            "gs_cnn_param_count", "gs_cnn_workspace_bytes", "gs_cnn_workspace_hidden_offset", "gs_cnn_workspace_act_offset", "gs_cnn_policy_act", "gs_cnn_ppo_loss", "gs_cnn_ppo_update",
            "gs_cnn_ppo_update_global",
            "gs_gemm_f32", "gs_fc_gemm", "gs_cartpole_reset", "gs_cartpole_step", "gs_atari_preprocess", "gs_atari_render", "gs_atari_env_reset", "gs_atari_env_step", "gs_comm_unique_id",
            "gs_comm_init", "gs_comm_xgmi_create", "gs_comm_xgmi_connect", "gs_comm_status", "gs_comm_error_record",
            "gs_comm_xgmi_set_colocation", "gs_comm_xgmi_set_bwd_exchange", "gs_comm_xgmi_reset",
            "gs_comm_allreduce_mean_f32", "gs_comm_allreduce_sum_f64", "gs_ppo_global_adv_stats",
            "gs_ppo_global_records", "gs_comm_info", "gs_comm_destroy")


def check(rc: int, what: str = "") -> None:
    """Raise on a non-zero status: ValueError for bad arguments (the reference's error
    type for shape/config problems), GsError for runtime/RCCL failures."""
    if rc == GS_OK:
        return
    msg = (lib.gs_last_error() or b"").decode(errors="replace")
    if rc == GS_E_INVALID:
        raise ValueError(f"{what}: {msg}")
    raise GsError(f"{what} failed ({rc}): {msg}")


def ptr(t) -> int | None:
    """Device/host address of a torch tensor (None passes NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_handle(stream=None) -> int | None:
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream
