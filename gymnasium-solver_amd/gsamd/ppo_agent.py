"""Device PPO agent — the drop-in for the reference's PPOAgent/BaseAgent plugin surface.

Reference surface mirrored (agents/__init__.py:1-8, agents/base_agent.py:26-885,
agents/ppo/ppo_agent.py:10-152):
  build_agent(config)                         -> DevicePPOAgent when config.algo_id == "ppo"
  train_dataloader()                          first rollout + minibatch index stream  (base_agent.py:253-283)
  on_train_epoch_start()                      re-collect from epoch 1 on             (base_agent.py:284-328)
  training_step(batch, batch_idx)             one fused minibatch step               (base_agent.py:330-366)
  losses_for_batch(batch, batch_idx)          {loss, early_stop_epoch}               (ppo_agent.py:21-152)
  configure_optimizers()                      Adam(lr=policy_lr) state in HBM         (base_agent.py:633-639)
  get_rollout_collector(stage)                DeviceRolloutCollector
and the fast path the trainer uses instead of per-minibatch Python:
  train_epoch()                               rollout + the whole update phase in one C-ABI call
Metrics are kept on device, one 40-float record per minibatch, and converted to the
reference's metric keys once per epoch (the reference pays ~20 .item() syncs per
minibatch, SURVEY.md §3 Boundaries).
"""
from __future__ import annotations

from typing import Any, Dict, Optional

import numpy as np
import torch

import ctypes

from ._lib import ACT_SLOT, GS_HP_ACT_STATS, GS_HP_BF16, GS_NUM_METRICS, M, PPOGlobal, PPOHparams, RolloutView, RolloutViewU8, check, lib, ptr, stream_handle
from .atari_env import DeviceAtariVecEnv
from .config import device_env_kind
from .cnn import DeviceCNNActorCritic
from .policy import DeviceMLPActorCritic
from .rollout import DeviceCartPoleVecEnv, DeviceRolloutCollector, DeviceSyntheticVecEnv
from .samplers import IndexStreamPrefetcher, MultiPassRandomSampler, index_stream, rank_share
from .distributed import allreduce_sum_f64, broadcast_int, check_replicas, comm_status, world_active
from . import distributed as _dist
from .metrics import NUM_SUMS, MetricsRecorder, ppo_keys, ppo_records
from .schedules import SCHEDULABLE, build_schedulers

STAGES = ("train",)


class MinibatchIndices:
    """A minibatch as the device sees it: B env-major sample indices (int32, in HBM)."""

    def __init__(self, idx: torch.Tensor, trajectories=None):
        self.idx = idx
        self.trajectories = trajectories

    def __len__(self):
        return int(self.idx.numel())


class DevicePPOAgent:
    def __init__(self, config, env=None, device: Optional[str] = None, rank: int = 0, world_size: int = 1,
                 comm=None, use_graph: bool = True, track_stats: bool = True, one_launch: bool = True,
                 env_factory=None):
        self.config = config
        self.env_factory = env_factory       # stage -> host VectorEnv (configs without device dynamics)
        self.device = torch.device(device or f"cuda:{torch.cuda.current_device()}")
        self.rank, self.world_size, self.comm = int(rank), int(world_size), comm
        self.use_graph = bool(use_graph)
        self.one_launch = bool(one_launch)      # synthetic env + LDS-sized MLP: one-launch rollouts
        self.track_stats = bool(track_stats)
        # schedulable hyper-parameters (base_agent.py:72-77)
        self.policy_lr = config.policy_lr
        self.clip_range = config.clip_range
        self.clip_range_vf = config.clip_range_vf
        self.vf_coef = config.vf_coef
        self.ent_coef = config.ent_coef
        # HyperparameterSchedulerCallback equivalents (schedule_resolver.py:54-124); positions
        # in vector steps of the whole job (all ranks step in lockstep)
        self.schedulers = build_schedulers(config.schedules, config.max_env_steps, config.n_envs * int(world_size))
        self.n_epochs = config.n_epochs
        self.current_epoch = 0
        self._early_stop_epoch = False
        self._envs: Dict[str, Any] = {}
        self._rollout_collectors: Dict[str, DeviceRolloutCollector] = {}
        self.metrics_history = []
        self.metrics_recorder = MetricsRecorder()    # base_agent.py:85
        self._staged = None                          # a tensor batch's T=1 rollout view (losses_for_batch)
        # optional per-epoch (start, update-start, end) events on the launch stream (bench.py)
        self.phase_events = None
        self.build_env("train", env)
        self.build_models()
        self.build_rollout_collector("train")
        self.configure_optimizers()

    # ---- construction (base_agent.py:103-222) -------------------------------------------
    def build_env(self, stage: str, env=None):
        """BaseAgent.build_env (base_agent.py:129-192): the env the config names.  A passed env
        (the host VectorEnv build_env_from_config returns, or a device env) is used as is;
        otherwise env_factory(stage) when given, otherwise the device dynamics of
        config.device_env_kind — and a config naming an env the device does not simulate
        raises instead of training on a stand-in."""
        c = self.config
        if env is None and self.env_factory is not None and device_env_kind(c) is None:
            env = self.env_factory(stage)
        if env is None:
            env = self._device_env(stage)
        if int(getattr(env, "num_envs", c.n_envs)) != int(c.n_envs):
            raise ValueError(f"env has {env.num_envs} envs, config.n_envs is {c.n_envs}")
        self._envs[stage] = env

    def _device_env(self, stage: str):
        c = self.config
        kind = device_env_kind(c)
        if kind is None:
            raise ValueError(
                f"env_id {c.env_id!r} (obs_type {c.obs_type!r}) has no device dynamics: pass env=<the gymnasium "
                f"VectorEnv build_env_from_config(config, seed=config.seed_train) returns> (or env_factory=), or "
                f"set env_dynamics='synthetic' for the fixed-length synthetic env of the benchmark")
        off = self.rank * c.n_envs
        train = stage == "train"
        if kind == "cartpole":
            if self.is_pixel or c.resolved_obs_dim() != 4 or c.resolved_n_actions() != 2:
                raise ValueError("env_dynamics='cartpole' needs vector observations of dim 4 and 2 actions")
            return DeviceCartPoleVecEnv(c.n_envs, seed=c.seed_train if train else c.seed_val, env_offset=off,
                                        max_steps=int(c.max_episode_steps or 500), device=self.device)
        seed = c.seed if train else c.seed + 1000
        if self.is_pixel:
            return DeviceAtariVecEnv(n_envs=c.n_envs, n_actions=c.resolved_n_actions(), episode_len=c.episode_len,
                                     seed=seed, truncate_every=c.truncate_every, env_offset=off,
                                     frame_stack=int(c.frame_stack or 4), device=self.device)
        return DeviceSyntheticVecEnv(n_envs=c.n_envs, obs_dim=c.resolved_obs_dim(), n_actions=c.resolved_n_actions(),
                                     episode_len=c.episode_len, seed=seed, truncate_every=c.truncate_every,
                                     env_offset=off, device=self.device)

    def get_env(self, stage: str):
        return self._envs[stage]

    @property
    def is_pixel(self) -> bool:
        """rgb observations -> NatureCNN + Atari pipeline (C4/C5), else the MLP path."""
        return str(getattr(self.config, "obs_type", "vector")) == "rgb"

    def _env_shapes(self):
        """(observation shape, action count) of the train env: a device env's own attributes, a
        host VectorEnv's single spaces (build_policy_from_env_and_config, policy_factory.py:79-130),
        else the config's spec."""
        c, env = self.config, self.get_env("train")
        shape = getattr(env, "obs_shape", None)
        n_act = getattr(env, "n_actions", None)
        osp, asp = getattr(env, "single_observation_space", None), getattr(env, "single_action_space", None)
        if shape is None and getattr(env, "obs_dim", None) is not None:
            shape = (int(env.obs_dim),)
        if shape is None and getattr(osp, "shape", None) is not None:
            shape = tuple(int(x) for x in osp.shape)
        if n_act is None and getattr(asp, "n", None) is not None:
            n_act = int(asp.n)
        shape = tuple(shape) if shape is not None else (c.resolved_obs_dim(),)
        return shape, int(n_act if n_act is not None else c.resolved_n_actions())

    def build_models(self):
        c = self.config
        shape, n_act = self._env_shapes()
        if self.is_pixel:
            self.policy_model = DeviceCNNActorCritic(in_shape=shape, n_actions=n_act, hidden=int(c.hidden_dims[0]),
                                                     valid_actions=c.valid_actions, device=self.device)
        else:
            if len(shape) != 1:
                raise ValueError(f"the MLP policy needs flat observations, the env gives {shape}")
            self.policy_model = DeviceMLPActorCritic(int(shape[0]), c.hidden_dims, n_act, device=self.device)

    def build_rollout_collector(self, stage: str):
        c = self.config
        self._rollout_collectors[stage] = DeviceRolloutCollector(
            self.get_env(stage), self.policy_model, c.n_steps, gamma=c.gamma, gae_lambda=c.gae_lambda,
            rng_seed=c.seed + 7919 * self.rank, track_stats=self.track_stats, use_graph=self.use_graph,
            one_launch=self.one_launch, normalize_advantages=self._rollout_adv_norm())

    def _rollout_adv_norm(self) -> bool:
        """normalize_advantages == "rollout": the collector normalises each rollout's advantages
        (utils/config.py:709-710 hands the collector that flag); "batch" is the loss's own
        per-minibatch normalisation (hparams().normalize_adv), "off" neither."""
        return str(getattr(self.config, "normalize_advantages", "batch")) == "rollout"

    def get_rollout_collector(self, stage: str) -> DeviceRolloutCollector:
        if stage not in self._rollout_collectors and stage in ("val", "test"):
            # evaluation collector: its own env instance (the stage's seed), same policy
            c = self.config
            self.build_env(stage)
            env = self._envs[stage]
            self._rollout_collectors[stage] = DeviceRolloutCollector(
                env, self.policy_model, c.n_steps, gamma=c.gamma, gae_lambda=c.gae_lambda,
                rng_seed=c.seed + 1000 + 7919 * self.rank, track_stats=True,
                normalize_advantages=self._rollout_adv_norm())
        return self._rollout_collectors[stage]

    # ---- checkpoints (agents/base_agent.py:658-885) -----------------------------------------
    def _adam_state_dicts(self):
        """Flat HBM moments -> torch.optim.Adam state_dict layout (one entry per tensor in
        the reference's parameter order)."""
        pm = self.policy_model
        to_ref = getattr(pm, "flat_to_reference", None)
        m = to_ref(self.adam_m) if to_ref else self.adam_m.cpu().numpy()
        v = to_ref(self.adam_v) if to_ref else self.adam_v.cpu().numpy()
        state, o = {}, 0
        for i, (_, shp) in enumerate(pm.shapes()):
            n = int(np.prod(shp))
            state[i] = {"step": torch.tensor(float(self.adam_step)),
                        "exp_avg": torch.as_tensor(m[o:o + n]).reshape(shp).clone(),
                        "exp_avg_sq": torch.as_tensor(v[o:o + n]).reshape(shp).clone()}
            o += n
        group = {"lr": float(self.policy_lr), "betas": (0.9, 0.999), "eps": 1e-8, "weight_decay": 0,
                 "amsgrad": False, "maximize": False, "foreach": None, "capturable": False,
                 "differentiable": False, "fused": None, "params": list(range(len(state)))}
        return [{"state": state, "param_groups": [group]}]

    def save_checkpoint(self, checkpoint_dir) -> None:
        """model.pt (reference state_dict keys), optimizer.pt (torch Adam state_dict list),
        state.json (epoch, counters, config, RNG) — the reference's checkpoint files."""
        import dataclasses
        import json
        import random
        from pathlib import Path
        d = Path(checkpoint_dir)
        d.mkdir(parents=True, exist_ok=True)
        torch.save(self.policy_model.state_dict(), d / "model.pt")
        torch.save(self._adam_state_dicts(), d / "optimizer.pt")
        coll = self.get_rollout_collector("train")
        np_state = np.random.get_state()
        state = {
            "epoch": int(self.current_epoch),
            "total_env_steps": int(coll.total_steps), "total_vec_steps": int(coll.total_vec_steps),
            "adam_step": int(self.adam_step), "run_id": None,
            "config": {k: (list(v) if isinstance(v, tuple) else v) for k, v in dataclasses.asdict(self.config).items()},
            "best_train_reward": float(coll._best_episode_reward),
            # the schedulable hyper-parameters in effect (a resumed run continues from these)
            "hyperparameters": {k: float(getattr(self, k)) for k in SCHEDULABLE},
            "rng_states": {"torch": torch.get_rng_state().tolist(),
                           "numpy": {"state_type": np_state[0], "state_keys": np_state[1].tolist(),
                                     "state_pos": int(np_state[2]), "state_has_gauss": int(np_state[3]),
                                     "state_cached_gaussian": float(np_state[4])},
                           "random": random.getstate()},
        }
        (d / "state.json").write_text(json.dumps(state, default=float))

    def load_checkpoint(self, checkpoint_dir, resume_training: bool = True, strict: bool = True) -> None:
        """Restore model (and, when resuming, Adam state, counters and RNG) from a checkpoint
        directory written by save_checkpoint or by the reference (weights_only loads only)."""
        import json
        import random
        from pathlib import Path
        d = Path(checkpoint_dir)
        sd = torch.load(d / "model.pt", map_location="cpu", weights_only=True)
        if strict:
            self.policy_model.load_state_dict(sd)
        else:
            cur = self.policy_model.state_dict()
            cur.update({k: v for k, v in sd.items() if k in cur and tuple(v.shape) == tuple(cur[k].shape)})
            self.policy_model.load_state_dict(cur)
        state = json.loads((d / "state.json").read_text()) if (d / "state.json").exists() else None
        if not (resume_training and state):
            return
        opt_path = d / "optimizer.pt"
        if opt_path.exists():
            opt = torch.load(opt_path, map_location="cpu", weights_only=True)
            opt = opt[0] if isinstance(opt, (list, tuple)) else opt
            st = opt["state"]
            m = np.concatenate([np.asarray(st[i]["exp_avg"], np.float32).reshape(-1) for i in sorted(st)])
            v = np.concatenate([np.asarray(st[i]["exp_avg_sq"], np.float32).reshape(-1) for i in sorted(st)])
            from_ref = getattr(self.policy_model, "flat_from_reference", None)
            mt = from_ref(m) if from_ref else torch.as_tensor(m)
            vt = from_ref(v) if from_ref else torch.as_tensor(v)
            self.adam_m.copy_(mt.to(self.device))
            self.adam_v.copy_(vt.to(self.device))
            steps = {int(float(st[i]["step"])) for i in st}
            self.adam_step = int(state.get("adam_step", max(steps) if steps else 0))
            groups = opt.get("param_groups") or []
            if groups and "lr" in groups[0]:      # torch's Adam.load_state_dict restores lr too
                self.set_hyperparameter("policy_lr", float(groups[0]["lr"]))
        for k, v in (state.get("hyperparameters") or {}).items():
            if k in SCHEDULABLE:
                self.set_hyperparameter(k, float(v))
        self.current_epoch = int(state.get("epoch", 0))
        coll = self.get_rollout_collector("train")
        coll.total_steps = int(state.get("total_env_steps", 0))
        coll.total_vec_steps = int(state.get("total_vec_steps", 0))
        if state.get("best_train_reward") is not None:
            coll._best_episode_reward = float(state["best_train_reward"])
        rng = state.get("rng_states")
        if rng:
            torch.set_rng_state(torch.ByteTensor(rng["torch"]))
            n = rng["numpy"]
            np.random.set_state((n["state_type"], np.array(n["state_keys"], dtype=np.uint32), n["state_pos"],
                                 n["state_has_gauss"], n["state_cached_gaussian"]))
            r = rng["random"]
            random.setstate((r[0], tuple(r[1]), r[2]))

    def configure_optimizers(self):
        """Adam(params, lr=policy_lr) (utils/optimizer_factory.py:6-29): state in HBM."""
        if str(getattr(self.config, "optimizer", "adam")).lower() != "adam":
            raise ValueError("device path implements the reference's default optimizer 'adam' only")
        P = self.policy_model.n_params
        z = dict(dtype=torch.float32, device=self.device)
        self.grads = torch.zeros(P, **z)
        self.adam_m = torch.zeros(P, **z)
        self.adam_v = torch.zeros(P, **z)
        self.adam_step = 0
        c = self.config
        self.batch_size = int(c.batch_size)
        self.data_len = c.n_envs * c.n_steps
        if str(getattr(c, "dp_mode", "local")) == "global":
            total = self.data_len * self.world_size
            if self.batch_size > total or total % self.batch_size != 0:
                raise ValueError(f"batch_size ({self.batch_size}) must divide the job's rollout of {total} samples "
                                 f"({self.world_size} ranks x {c.n_envs} envs x {c.n_steps} steps) in global mode")
        elif self.data_len % self.batch_size != 0:
            raise ValueError(f"Batch size must divide rollout size exactly: data_len={self.data_len}, "
                             f"batch_size={self.batch_size}.")
        self.n_minibatches = self.data_len // self.batch_size * c.n_epochs
        # global-minibatch mode (dp_mode "global"): every rank runs the reference's
        # minibatches of the whole job's rollout, its own rows of each padded to B
        self.global_mode = str(getattr(c, "dp_mode", "local")) == "global"
        if self.global_mode:
            if self.is_pixel and c.target_kl is not None:
                raise ValueError("dp_mode 'global' of the NatureCNN update has no KL early stop: unset target_kl")
            if self._rollout_adv_norm() and self.world_size > 1:
                # the reference normalises over the single process's whole rollout; each rank here
                # holds a share of it, and the statistics are not summed over ranks
                raise ValueError("dp_mode 'global' with normalize_advantages='rollout' is not supported over "
                                 "several ranks: use 'batch' (whole-global-minibatch statistics) or dp_mode 'local'")
            self.n_minibatches = self.data_len * self.world_size // self.batch_size * c.n_epochs
            z64 = dict(dtype=torch.float64, device=self.device)
            self._gsums = torch.zeros(self.n_minibatches, NUM_SUMS, **z64)
            self._adv_stats = torch.zeros(self.n_minibatches, 2, dtype=torch.float32, device=self.device)
            self._adv_sums = torch.zeros(self.n_minibatches, 2, **z64)
            self._gidx = torch.empty(self.n_minibatches * self.batch_size, dtype=torch.int32, device=self.device)
            if self.is_pixel:     # frame reads of another rank's rows go to sample 0 (dead rows)
                self._fidx = torch.empty_like(self._gidx)
        self._base_seed = int(torch.initial_seed())
        if self.global_mode and self.world_size > 1 and world_active():
            # every rank must cut its shares from the SAME global permutation (samplers.py:25-34,
            # seed initial_seed + epoch): launchers often seed ranks differently (seed + rank), so
            # rank 0's seed is the job's sampler seed
            seed0 = broadcast_int(self._base_seed, 0)
            if seed0 != self._base_seed:
                import warnings
                warnings.warn(f"dp_mode 'global': rank {self.rank} was seeded {self._base_seed}, using rank 0's "
                              f"sampler seed {seed0} so every rank draws the same global minibatches")
            self._base_seed = seed0
        if self.is_pixel:
            ws = int(lib.gs_cnn_workspace_bytes(self.policy_model.dims, self.batch_size))
        else:   # the whole update's workspace (fused chain: per-update gathered minibatch fields)
            ws = int(lib.gs_ppo_update_workspace_bytes(self.policy_model.dims, self.batch_size, self.n_minibatches))
        self.workspace = torch.zeros(ws, dtype=torch.uint8, device=self.device)
        self.stop_flag = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.metrics_buf = torch.zeros(self.n_minibatches, GS_NUM_METRICS, **z)
        self._step_metrics = torch.zeros(GS_NUM_METRICS, **z)
        self.prefetcher = IndexStreamPrefetcher(self.data_len, c.n_epochs, int(torch.initial_seed()), self.device)
        return None

    @property
    def device_activation_stats(self) -> bool:
        """The update records every evaluated minibatch's activation statistics into its record
        (GS_HP_ACT_STATS: the reference's forward hooks, utils/models.py:121-147, recorded by every
        training_step, base_agent.py:335-347; MLP: backbone.{0,2}, NatureCNN: cnn.{0,2,4} and mlp.0,
        models.py:419-422) — with track_stats, not in global mode (a rank holds a share of each
        global minibatch)."""
        return self.track_stats and not getattr(self, "global_mode", False)

    def hparams(self) -> PPOHparams:
        c = self.config
        tkl = c.target_kl if c.target_kl is not None else 0.0
        flags = GS_HP_BF16 if str(getattr(c, "precision", "fp32")) == "bf16" else 0
        if self.device_activation_stats:
            flags |= GS_HP_ACT_STATS
        return PPOHparams(float(self.clip_range), float(self.clip_range_vf), float(self.vf_coef), float(self.ent_coef),
                          float(c.max_grad_norm if c.max_grad_norm is not None else 0.0), float(self.policy_lr),
                          0.9, 0.999, 1e-8, float(tkl), 1 if c.normalize_advantages == "batch" else 0, flags)

    # ---- Lightning-style hooks ------------------------------------------------------------
    def train_dataloader(self):
        """Collect the first rollout and return the minibatch index loader of epoch 0."""
        self._trajectories = self.get_rollout_collector("train").collect()
        return self._epoch_batches(0)

    def _epoch_batches(self, epoch: int):
        if self.global_mode:
            raise NotImplementedError("dp_mode 'global' runs whole updates (train_epoch), not per-minibatch "
                                      "training_step calls")
        idx = self.prefetcher.upload(epoch)
        self.prefetcher.prefetch(epoch + 1)
        B = self.batch_size
        return [MinibatchIndices(idx[k * B:(k + 1) * B], self._trajectories) for k in range(self.n_minibatches)]

    def on_train_epoch_start(self):
        if self.current_epoch > 0:
            self._trajectories = self.get_rollout_collector("train").collect()

    def _stage_batch(self, batch):
        """A tensor batch (RolloutTrajectory or any object with observations / actions /
        logprobs / values / advantages / returns, rollout_buffer.py:16-25; the reference's tests
        pass SimpleNamespace) -> device copies laid out as a one-step rollout of B envs, so the
        env-major indices 0..B-1 select the rows in order.  Returns (view, idx, B)."""
        obs = torch.as_tensor(batch.observations)
        B = int(obs.shape[0])
        pix = self.is_pixel
        st = self._staged
        if st is None or st["B"] != B:
            dev = self.device
            st = {"B": B, "idx": torch.arange(B, dtype=torch.int32, device=dev),
                  "obs": torch.empty((1, *obs.shape), dtype=torch.uint8 if pix else torch.float32, device=dev),
                  "act": torch.empty(1, B, dtype=torch.int64, device=dev),
                  **{k: torch.empty(1, B, dtype=torch.float32, device=dev) for k in ("lp", "v", "adv", "ret")}}
            ws_need = int(lib.gs_cnn_workspace_bytes(self.policy_model.dims, B) if pix else
                          lib.gs_ppo_workspace_bytes(self.policy_model.dims, B))
            st["ws"] = self.workspace if ws_need <= self.workspace.numel() else \
                torch.zeros(ws_need, dtype=torch.uint8, device=dev)
            self._staged = st
        st["obs"][0].copy_(obs.to(st["obs"].dtype).reshape(st["obs"].shape[1:]))
        st["act"][0].copy_(torch.as_tensor(batch.actions).reshape(B).to(torch.int64))
        for k, f in (("lp", "logprobs"), ("v", "values"), ("adv", "advantages"), ("ret", "returns")):
            st[k][0].copy_(torch.as_tensor(getattr(batch, f)).reshape(B).to(torch.float32))
        V = RolloutViewU8 if pix else RolloutView
        view = V(ptr(st["obs"]), ptr(st["act"]), ptr(st["lp"]), ptr(st["v"]), ptr(st["adv"]), ptr(st["ret"]), 1, B)
        return view, st["idx"], B, st["ws"]

    def _batch_view(self, batch):
        if isinstance(batch, MinibatchIndices):
            return self.get_rollout_collector("train").buffer.view(), batch.idx, len(batch), self.workspace
        return self._stage_batch(batch)

    def _record_step(self, rec: torch.Tensor) -> np.ndarray:
        """metrics_recorder.record("train", ...) with losses_for_batch's keys (ppo_agent.py:131-146)."""
        row = rec.detach().cpu().numpy().reshape(1, GS_NUM_METRICS)
        norm = self.config.normalize_advantages == "batch"
        vals = ppo_records(row, float(self.vf_coef), float(self.ent_coef), norm)[0]
        self.metrics_recorder.record("train", dict(zip(ppo_keys(norm), vals)))
        return row[0]

    def losses_for_batch(self, batch, batch_idx: int):
        """PPOAgent.losses_for_batch (agents/ppo/ppo_agent.py:21-152): forward + loss + metrics of
        one minibatch, no optimizer step.  `batch` is the reference's tensor batch or this
        agent's MinibatchIndices.  Returns {loss: 0-d device tensor, early_stop_epoch: bool} and
        records the metrics under "train"."""
        view, idx, B, ws = self._batch_view(batch)
        if self.is_pixel:
            check(lib.gs_cnn_ppo_loss(ptr(self.policy_model.params), self.policy_model.dims, self.hparams(), view,
                                      ptr(idx), B, ptr(self._step_metrics), None, ptr(ws), stream_handle()),
                  "gs_cnn_ppo_loss")
        else:
            check(lib.gs_ppo_loss(ptr(self.policy_model.params), self.policy_model.dims, self.hparams(), view,
                                  ptr(idx), B, ptr(self._step_metrics), ptr(ws), stream_handle()), "gs_ppo_loss")
        row = self._record_step(self._step_metrics)
        early = self.config.target_kl is not None and bool(row[M["kl_stop"]])
        return dict(loss=self._step_metrics[M["loss"]].clone(), early_stop_epoch=early)

    def _require_exchange(self) -> None:
        """A data-parallel job (world_size > 1) trains ONE model only through the gradient
        exchange: without a communicator every rank would step on its own shard's gradient and the
        replicas would drift apart silently (local mode) or train on a share of each global
        minibatch (global mode).  Raised before any device work of the step, on every rank."""
        if self.world_size > 1 and not self.comm:
            mode = "dp_mode 'global'" if getattr(self, "global_mode", False) else "dp_mode 'local'"
            raise ValueError(f"{mode} with world_size={self.world_size} needs a communicator: set agent.comm = "
                             f"init_xgmi_comm(...) or init_device_comm(...) before training (rank {self.rank})")

    def training_step(self, batch, batch_idx: int):
        """BaseAgent.training_step (base_agent.py:330-366) fused: forward, loss, backward,
        clip_grad_norm_(max_grad_norm), Adam.step.  The KL early stop is sticky as in the
        reference: the minibatch that trips it takes no step, nor does any later one."""
        if self._early_stop_epoch:
            return None
        self._require_exchange()
        view, idx, B, ws = self._batch_view(batch)
        self.adam_step += 1
        rec = self.metrics_buf[batch_idx % self.n_minibatches]
        if self.is_pixel:
            check(lib.gs_cnn_ppo_update(ptr(self.policy_model.params), ptr(self.grads), ptr(self.adam_m),
                                        ptr(self.adam_v), self.policy_model.dims, self.hparams(), view,
                                        ptr(idx), B, 1, self.adam_step - 1, ptr(rec),
                                        ptr(self.stop_flag), ptr(ws), self.comm, stream_handle()),
                  "gs_cnn_ppo_update")
        else:
            check(lib.gs_ppo_minibatch_step(ptr(self.policy_model.params), ptr(self.grads), ptr(self.adam_m),
                                            ptr(self.adam_v), self.policy_model.dims, self.hparams(), view,
                                            ptr(idx), B, self.adam_step, ptr(rec), ptr(self.stop_flag),
                                            ptr(ws), self.comm, stream_handle()), "gs_ppo_minibatch_step")
        row = self._record_step(rec)
        if self.device_activation_stats:         # training_step's hook record (base_agent.py:340-343)
            keys = self.activation_keys()
            self.metrics_recorder.record("train", dict(zip(keys, row[ACT_SLOT:ACT_SLOT + len(keys)].tolist())))
        if self.config.target_kl is not None and row[M["kl_stop"]]:
            self._early_stop_epoch = True
            self.adam_step -= 1              # the tripping minibatch took no optimizer step
        else:
            keys, slots = self.grad_norm_keys()
            self.metrics_recorder.record("train", {k: float(row[j]) for k, j in zip(keys, slots)})
        return None

    def grad_norm_keys(self):
        """compute_grad_norms' keys (utils/models.py:196-230, base_agent.py:607-608) and their record
        slots: "all", then the model's components in the reference's discovery order."""
        comps = ("cnn", "mlp", "policy_head", "value_head") if self.is_pixel else ("backbone", "policy_head", "value_head")
        slot = {"backbone": M["gn_backbone"], "cnn": M["gn_backbone"], "mlp": M["gn_mlp"],
                "policy_head": M["gn_policy_head"], "value_head": M["gn_value_head"]}
        return (("opt/grads/norm/all",) + tuple(f"opt/grads/norm/{c}" for c in comps),
                [M["grad_norm"]] + [slot[c] for c in comps])

    # ---- fused epoch (the trainer's path) -------------------------------------------------------
    def train_epoch(self) -> None:
        """One reference epoch: rollout (epoch > 0) + n_epochs passes of minibatch steps."""
        epoch = self.current_epoch
        collector = self.get_rollout_collector("train")
        ev = self.phase_events
        if ev is not None:
            ev.append([torch.cuda.Event(enable_timing=True) for _ in range(3)])
            ev[-1][0].record()
        if epoch == 0 and collector.total_rollouts == 0:
            self._trajectories = collector.collect()
        elif epoch > 0:
            self._trajectories = collector.collect()
        self.update_phase(ev)

    def update_phase(self, ev=None) -> None:
        """The update half of an epoch on the train collector's current rollout (the n_epochs
        passes of minibatch steps, then the epoch's bookkeeping) — train_epoch after its collect;
        callers that collect themselves (e.g. a replayed rollout) call it directly."""
        self._require_exchange()
        # the hyper-parameters this update runs with, as the reference logs them at the epoch's
        # start (on_train_epoch_start -> _log_hyperparameters, base_agent.py:302): booked with the
        # update's records by record_epoch_metrics (the scheduler changes them at the epoch's end)
        self._epoch_hp = self.hyperparameter_record()
        epoch = self.current_epoch
        collector = self.get_rollout_collector("train")
        # the epoch's minibatch indices go up on the update's own stream: a side-stream upload
        # overlapping the rollout (tried: C3 collect -2 ms) made every minibatch step of the
        # update that followed ~1.4 us slower (same-box A/B on C2: 16.8 vs 15.3 us), with the
        # update waiting on the copy's event on the device or on the host alike
        idx = None if self.global_mode else self.prefetcher.upload(epoch)
        if not self.global_mode:
            self.prefetcher.prefetch(epoch + 1)
        buf = collector.buffer
        if self.world_size > 1:
            self._verify_exchange()
        if ev:
            ev[-1][1].record()
        if self.global_mode:
            self._global_update(epoch, buf)
        elif self.is_pixel:
            check(lib.gs_cnn_ppo_update(ptr(self.policy_model.params), ptr(self.grads), ptr(self.adam_m),
                                        ptr(self.adam_v), self.policy_model.dims, self.hparams(), buf.view(), ptr(idx),
                                        self.batch_size, self.n_minibatches, self.adam_step, ptr(self.metrics_buf),
                                        ptr(self.stop_flag), ptr(self.workspace), self.comm, stream_handle()),
                  "gs_cnn_ppo_update")
        else:
            check(lib.gs_ppo_update(ptr(self.policy_model.params), ptr(self.grads), ptr(self.adam_m),
                                    ptr(self.adam_v), self.policy_model.dims, self.hparams(), buf.view(), ptr(idx),
                                    self.batch_size, self.n_minibatches, self.adam_step, ptr(self.metrics_buf),
                                    ptr(self.stop_flag), ptr(self.workspace), self.workspace.numel(), self.comm,
                                    1 if self.use_graph else 0, stream_handle()), "gs_ppo_update")
        if ev:
            ev[-1][2].record()
        if self.comm:
            # the exchange's sticky timeout record, read once per epoch (one 8-byte D2H after the
            # update): a peer that never arrived leaves this update on a non-mean gradient, so
            # training stops here with the workgroup and peer that timed out
            comm_status(self.comm)
            # replica check: every rank must hold the same parameter bits after the update (the
            # exchange is the only thing that keeps them equal; a stale-but-finite slot would let
            # them drift silently) — two float64 checksums all-reduced as min / max, GsError on
            # a mismatch (DESIGN §5 Failure surfacing)
            if self.world_size > 1:
                check_replicas(self.policy_model.params)
                self._exchange_canary()
        if self.config.target_kl is None:
            self.adam_step += self.n_minibatches
        else:       # minibatches from the sticky KL stop on took no optimizer step
            self.adam_step += int((self.metrics_buf[:, M["skipped"]] == 0).sum().item())
        self.current_epoch += 1
        self.on_train_epoch_end()

    def _verify_exchange(self) -> None:
        """Before the first update with an xGMI communicator attached (every rank reaches it
        together): the in-backward exchange of the MLP chain is self-tested on THIS job's shapes and
        precision (gsamd.distributed.bwd_exchange_self_test: replicas bit-identical, agreement
        with the exchange launch; on failure every rank switches to the launch form together),
        unless the launcher's init_xgmi_comm(verify_shapes=...) already did; the result is kept in
        self.exchange_self_test.  The NatureCNN update exchanges with a launch only, which
        init_xgmi_comm's full-capacity vector self-test covers."""
        if getattr(self, "_exchange_checked", False):
            return
        self._exchange_checked = True
        self.exchange_self_test = None
        if _dist.comm_info(self.comm)["transport"] != "xgmi" or self.is_pixel:
            return
        dims, flags = self.policy_model.dims, int(self.hparams().flags)
        if _dist.verified(self.comm, dims, self.batch_size, flags):
            self.exchange_self_test = dict(_dist.LAST_SELF_TEST)
            return
        self.exchange_self_test = _dist.bwd_exchange_self_test(self.comm, self.rank, self.world_size, dims,
                                                               self.batch_size, self.device, flags=flags)

    def _exchange_canary(self) -> None:
        """Once per epoch, after the replica check: one exchange of a known, epoch-dependent
        pattern over the whole parameter count through the job's xGMI communicator, compared bit
        for bit on every rank with the exact rank-order answer.  The replica check sees only
        asymmetric faults; a slot read stale identically on every rank keeps the replicas equal
        but fails this.  GsError on every rank on a mismatch."""
        if _dist.comm_info(self.comm)["transport"] != "xgmi":
            return
        self._canary_round = getattr(self, "_canary_round", 0) + 1
        # a rank whose exchange call raises (GsError) still meets the others in _agree, so every
        # rank raises together instead of its peers blocking in the all-reduce until it times out
        try:
            ok = _dist.xgmi_self_test(self.comm, self.rank, self.world_size, self.policy_model.n_params, self.device,
                                      rounds=1, salt=self._canary_round)
        except RuntimeError:
            ok = False
        if not _dist._agree(ok, self.device):
            from ._lib import GsError
            raise GsError(f"exchange canary failed on epoch {self.current_epoch} (rank {self.rank}): a known "
                          f"vector did not come back as its exact rank-order mean through the xGMI exchange")

    CNN_ACTIVATION_LAYERS = ("cnn.0", "cnn.2", "cnn.4", "mlp.0")

    def activation_keys(self):
        if self.global_mode or not self.track_stats:
            return ()
        layers = self.CNN_ACTIVATION_LAYERS if self.is_pixel else ("backbone.0", "backbone.2")
        return tuple(f"opt/activations/{n}/{k}" for n in layers for k in ("mean", "std", "dead_pct", "dead_max"))

    def global_shares(self, epoch: int) -> np.ndarray:
        """This rank's rows of every global minibatch of `epoch` (padded with -1): the reference's
        sampler over the whole job's rollout (utils/samplers.py:25-34, seed initial_seed + epoch,
        global env g = rank * n_envs + local env)."""
        stream = index_stream(self.data_len * self.world_size, self.config.n_epochs, self._base_seed + int(epoch))
        return rank_share(stream, self.batch_size, self.rank, self.data_len)

    def _global_update(self, epoch: int, buf) -> None:
        """gs_ppo_update_global (MLP) / gs_cnn_ppo_update_global (NatureCNN) on this rank's shares
        of the global minibatches, with the mode's
        statistics kept on the device: gs_ppo_global_adv_stats (this rank's per-minibatch advantage
        sums, one f64 sum over ranks through the communicator, the whole minibatch's mean / std),
        the update, then gs_ppo_global_records (the ranks' raw loss sums added through the
        communicator, every evaluated record rewritten from them) — identical on every rank, no
        host round trip."""
        c, B, n, T = self.config, self.batch_size, self.n_minibatches, self.config.n_steps
        self._gidx.copy_(torch.from_numpy(self.global_shares(epoch)))
        norm = c.normalize_advantages == "batch"
        Bg = B   # batch_size is the global minibatch size
        comm = self.comm if self.world_size > 1 else None
        st = stream_handle()
        if norm:     # utils/torch.py:97-99 over the whole global minibatch
            check(lib.gs_ppo_global_adv_stats(ptr(self._gidx), n, B, Bg, ptr(buf.advantages), T, c.n_envs, comm,
                                              ptr(self._adv_sums), ptr(self._adv_stats), st), "gs_ppo_global_adv_stats")
        glob = PPOGlobal(Bg, ptr(self._adv_stats) if norm else None, ptr(self._gsums))
        hp = self.hparams()
        if self.is_pixel:
            torch.clamp(self._gidx, min=0, out=self._fidx)
            check(lib.gs_cnn_ppo_update_global(ptr(self.policy_model.params), ptr(self.grads), ptr(self.adam_m),
                                               ptr(self.adam_v), self.policy_model.dims, hp, buf.view(),
                                               ptr(self._gidx), ptr(self._fidx), B, n, self.adam_step,
                                               ptr(self.metrics_buf), ptr(self.stop_flag), ptr(self.workspace),
                                               self.comm, ctypes.byref(glob), st), "gs_cnn_ppo_update_global")
        else:
            check(lib.gs_ppo_update_global(ptr(self.policy_model.params), ptr(self.grads), ptr(self.adam_m),
                                           ptr(self.adam_v), self.policy_model.dims, hp, buf.view(),
                                           ptr(self._gidx), B, n, self.adam_step, ptr(self.metrics_buf),
                                           ptr(self.stop_flag), ptr(self.workspace), self.workspace.numel(),
                                           self.comm, 1 if self.use_graph else 0, ctypes.byref(glob), st),
                  "gs_ppo_update_global")
        check(lib.gs_ppo_global_records(ctypes.byref(hp), n, Bg, comm, ptr(self._gsums), ptr(self.metrics_buf), st),
              "gs_ppo_global_records")

    def set_hyperparameter(self, param: str, value: float) -> None:
        """hyperparameter_mixin.py:105-114 (+ the policy_lr setter of callback_builder.py:108-113:
        the next update's Adam step size is the attribute itself)."""
        setattr(self, param, value)
        if hasattr(self.config, param):
            setattr(self.config, param, value)

    HP_KEYS = ("n_epochs", "ent_coef", "vf_coef", "clip_range", "policy_lr", "clip_range_vf")

    def hyperparameter_record(self) -> Dict[str, float]:
        """HyperparameterMixin._log_hyperparameters (agents/hyperparameter_mixin.py:90-103): the
        tunable values in effect, under hp/<name> (clip_range_vf: PPO's; a None value is dropped as
        the recorder drops non-scalars)."""
        return {f"hp/{k}": getattr(self, k) for k in self.HP_KEYS if getattr(self, k, None) is not None}

    def on_train_epoch_end(self) -> None:
        """HyperparameterSchedulerCallback.on_train_epoch_end for every configured schedule."""
        if not self.schedulers:
            return
        total = self.get_rollout_collector("train").total_vec_steps
        for s in self.schedulers:
            self.set_hyperparameter(s.parameter, s.value(total))

    def record_epoch_metrics(self) -> np.ndarray:
        """Book the last update's per-minibatch records into metrics_recorder["train"] with
        losses_for_batch's keys — only the minibatches whose loss was evaluated, as the
        reference records them (the one that trips the KL stop included) — plus
        opt/grads/norm/all of the minibatches that stepped (base_agent.py:607-608).  One D2H."""
        rec = self.metrics_buf.cpu().numpy()
        norm = self.config.normalize_advantages == "batch"
        live = rec[rec[:, M["unevaluated"]] == 0]
        self.metrics_recorder.record_rows("train", ppo_keys(norm),
                                          ppo_records(live, float(self.vf_coef), float(self.ent_coef), norm))
        if getattr(self, "_epoch_hp", None):
            self.metrics_recorder.record("train", self._epoch_hp)
        stepped = rec[rec[:, M["skipped"]] == 0]
        keys, slots = self.grad_norm_keys()
        self.metrics_recorder.record_rows("train", keys, stepped[:, slots])
        if self.device_activation_stats:
            # every evaluated minibatch's statistics (the update's GS_M_ACT slots), as the reference
            # records them once per training_step — their epoch mean is the recorder's
            keys = self.activation_keys()
            self.metrics_recorder.record_rows("train", keys, live[:, ACT_SLOT:ACT_SLOT + len(keys)])
        if self.config.target_kl is not None and (rec[:, M["kl_stop"]] != 0).any():
            self._early_stop_epoch = True        # sticky, as BaseAgent._early_stop_epoch
        return rec

    def epoch_metric_keys(self):
        """The fixed key list of epoch_metrics (every rank sends the same vector)."""
        norm = self.config.normalize_advantages == "batch"
        hp = tuple(f"hp/{k}" for k in self.HP_KEYS if getattr(self, k, None) is not None)
        return tuple(ppo_keys(norm)) + self.grad_norm_keys()[0] + self.activation_keys() + hp

    def epoch_metrics(self) -> Dict[str, float]:
        """The last update's epoch means under the reference's metric keys (ppo_agent.py:131-146,
        torch.py:170-173, base_agent.py:607-608); the recorder's "train" namespace is reset
        first, so this is exactly one update.  In a multi-rank job every rank all-reduces the same
        fixed key list as (sum, count) pairs — a rank whose KL stop left a key without records adds
        0 to both — and the means are pooled over all ranks' records."""
        self.metrics_recorder.reset_epoch("train")
        self.record_epoch_metrics()
        if not world_active():
            out = self.metrics_recorder.compute_epoch_means("train")
            return {k: float(v) for k, v in out.items()}
        keys = self.epoch_metric_keys()
        sc = allreduce_sum_f64(self.metrics_recorder.sums_counts("train", keys).reshape(-1)).reshape(2, -1)
        return {k: float(sc[0, j] / sc[1, j]) for j, k in enumerate(keys) if sc[1, j] > 0}

    def minibatch_losses(self) -> np.ndarray:
        return self.metrics_buf[:, M["loss"]].cpu().numpy().astype(np.float64)

    def learn(self, max_epochs: Optional[int] = None, log=None) -> None:
        """Lightning-free fit loop: max_env_steps guard (base_agent.py:306-320) + epochs.
        The run is bounded as the reference's Trainer bounds it (utils/trainer_factory.py:33:
        `max_epochs=config.max_epochs`, -1 = unbounded when None): training stops once
        current_epoch reaches config.max_epochs (Lightning counts epochs from the run's start, a
        resumed run included).  An explicit `max_epochs` runs at most that many more epochs in
        this call, inside the config's bound."""
        c = self.config
        cap = getattr(c, "max_epochs", None)
        if cap is not None and int(cap) < 0:
            cap = None
        epochs = 0
        while max_epochs is None or epochs < max_epochs:
            if cap is not None and self.current_epoch >= int(cap):
                break
            if c.max_env_steps is not None:
                done = self.get_rollout_collector("train").total_steps
                if done + c.n_envs * c.n_steps * self.world_size > c.max_env_steps:
                    break
            self.train_epoch()
            epochs += 1
            if log is not None:
                m = self.get_rollout_collector("train").get_metrics()
                m.pop("action_dist", None)
                log({**m, **self.epoch_metrics()})

    # ---- misc -----------------------------------------------------------------------------------
    def make_sampler(self) -> MultiPassRandomSampler:
        return MultiPassRandomSampler(self.data_len, self.config.n_epochs)


def build_agent(config, *args, **kwargs):
    """agents/__init__.py:1-8 for the device path.  Accepts a gsamd PPOConfig or the
    reference's own Config object (adapted by name, gsamd.config.from_reference_config).
    The env is the one the config names (DevicePPOAgent.build_env): CartPole-v1 steps on the
    device CartPole dynamics; any other env_id needs env= / env_factory= (the host VectorEnv
    the reference's build_env_from_config returns); the synthetic env only with
    env_dynamics='synthetic'."""
    from .config import from_reference_config
    algo = getattr(getattr(config, "algo_id", None), "value", getattr(config, "algo_id", None))
    if algo != "ppo":
        raise ValueError(f"device path implements algo_id 'ppo' only, got {algo!r}")
    return DevicePPOAgent(from_reference_config(config), *args, **kwargs)

