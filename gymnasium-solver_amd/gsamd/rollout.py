"""Device-resident rollout: SoA buffer in HBM, fused policy-act kernels, GAE scan.

Mirrors the reference's RolloutBuffer (utils/rollout_buffer.py:28-173) and
RolloutCollector (utils/rollout_collector.py:22-777) for the PPO path
(returns_type "gae:rtg", advantages_type "gae"):

  * buffers are allocated once, time-major ``(T, N, ...)`` like the reference's numpy
    buffers, but in HBM; a rollout never copies them to the host;
  * per step: ``gs_policy_act`` (MLP forward + categorical sample + log_prob, writes
    the step's obs/action/logp/value rows) then the env step;  with the device
    synthetic env (``env.device_native``) the env step is a kernel writing the
    reward/done/timeout rows, so the whole rollout is stream-ordered kernels;  a host
    gymnasium-style env goes through one H2D/D2H per step as in the reference;
  * last-obs value + ``gs_gae_f32`` produce advantages/returns in place;
  * ``bootstrapped_values`` stays all-zero: with gymnasium 1.x vector envs the
    reference never receives ``final_observation``, so its
    ``bootstrapped_values_buf`` is never written yet IS read at timeouts; this
    reproduces that behaviour (pass ``bootstrap_timeouts=True`` to opt out is future work).

The returned trajectory keeps the reference's field names; env-major ``(N*T, ...)``
views (utils/rollout_buffer.py:105-173) are materialised only when accessed — the
device update reads the time-major buffers directly through sampler indices.
"""
from __future__ import annotations

import ctypes
import time
from typing import Optional

import numpy as np
import torch

from ._lib import check, lib, ptr, stream_handle
from .distributed import allreduce_sum_f64
from .rollout_stats import RollingWindow


class DeviceSyntheticVecEnv:
    """Device twin of gsamd.synthetic_env.SyntheticVecEnv (same hash, same episodes)."""

    device_native = True

    def __init__(self, n_envs, obs_dim, n_actions, episode_len=200, seed=42, truncate_every=0, env_offset=0,
                 reward=1.0, device="cuda"):
        self.num_envs, self.obs_dim, self.n_actions = int(n_envs), int(obs_dim), int(n_actions)
        self.episode_len, self.seed, self.truncate_every = int(episode_len), int(seed), int(truncate_every)
        self.env_offset, self.reward = int(env_offset), float(reward)
        self.obs_shape, self.obs_dtype = (self.obs_dim,), torch.float32
        self.device = torch.device(device)
        N = self.num_envs
        self.state = torch.zeros(4 * N, dtype=torch.int32, device=self.device)
        self.ep_ret = torch.zeros(N, dtype=torch.float32, device=self.device)
        self.obs = torch.zeros(N, self.obs_dim, dtype=torch.float32, device=self.device)
        self.ep_count = torch.zeros(N, dtype=torch.int32, device=self.device)
        self.ep_ret_sum = torch.zeros(N, dtype=torch.float32, device=self.device)
        self.ep_len_sum = torch.zeros(N, dtype=torch.float32, device=self.device)
        self.step_count = 0

    def reset(self):
        self.step_count = 0
        check(lib.gs_env_reset(ptr(self.state), ptr(self.ep_ret), ptr(self.obs), self.num_envs, self.obs_dim,
                               self.episode_len, self.seed, self.env_offset, stream_handle()), "gs_env_reset")
        return self.obs, {}

    def step_into(self, rewards_row, dones_row, timeouts_row, actions=None, clock=None, step=None):
        """One vector step into the rollout rows.  clock/step: inside a captured rollout the
        step count is clock[1] (device) + step instead of the host counter."""
        if clock is None:
            self.step_count += 1
        check(lib.gs_env_step(ptr(self.state), ptr(self.ep_ret), ptr(self.obs), self.num_envs, self.obs_dim,
                              self.episode_len, self.truncate_every, self.reward, self.seed, self.env_offset,
                              self.step_count if clock is None else int(step), ptr(rewards_row), ptr(dones_row),
                              ptr(timeouts_row), ptr(self.ep_count), ptr(self.ep_ret_sum), ptr(self.ep_len_sum),
                              ptr(clock), stream_handle()), "gs_env_step")


class DeviceCartPoleVecEnv:
    """CartPole-v1 on device (gymnasium 1.x dynamics restated in
    csrc/gs_cartpole.hip, NEXT_STEP autoreset, TimeLimit 500).  Parity with gymnasium's own
    episodes is unpinned (reset draws use a counter hash, not PCG64)."""

    device_native = True

    def __init__(self, n_envs, seed=42, env_offset=0, max_steps=500, device="cuda", **_):
        self.num_envs, self.obs_dim, self.n_actions = int(n_envs), 4, 2
        self.seed, self.env_offset, self.max_steps = int(seed), int(env_offset), int(max_steps)
        self.obs_shape, self.obs_dtype = (4,), torch.float32
        self.device = torch.device(device)
        N, z = self.num_envs, dict(device=self.device)
        self.state = torch.zeros(N, 4, dtype=torch.float64, **z)
        self.meta = torch.zeros(N, 3, dtype=torch.int32, **z)
        self.ep_ret = torch.zeros(N, dtype=torch.float32, **z)
        self.obs = torch.zeros(N, 4, dtype=torch.float32, **z)
        self.ep_count = torch.zeros(N, dtype=torch.int32, **z)
        self.ep_ret_sum = torch.zeros(N, dtype=torch.float32, **z)
        self.ep_len_sum = torch.zeros(N, dtype=torch.float32, **z)

    def reset(self):
        check(lib.gs_cartpole_reset(ptr(self.state), ptr(self.meta), ptr(self.ep_ret), ptr(self.obs), self.num_envs,
                                    self.seed, self.env_offset, stream_handle()), "gs_cartpole_reset")
        return self.obs, {}

    def step_into(self, rewards_row, dones_row, timeouts_row, actions=None, clock=None, step=None):
        if actions is None:
            raise ValueError("CartPole dynamics need the step's actions")
        check(lib.gs_cartpole_step(ptr(self.state), ptr(self.meta), ptr(self.ep_ret), ptr(self.obs), ptr(actions),
                                   self.num_envs, self.max_steps, self.seed, self.env_offset, ptr(rewards_row),
                                   ptr(dones_row), ptr(timeouts_row), ptr(self.ep_count), ptr(self.ep_ret_sum),
                                   ptr(self.ep_len_sum), stream_handle()), "gs_cartpole_step")


class DeviceRolloutBuffer:
    """Preallocated time-major SoA rollout storage in HBM (utils/rollout_buffer.py:28-80)."""

    def __init__(self, n_envs: int, obs_shape, n_steps: int, device, obs_dtype=torch.float32):
        T, N = int(n_steps), int(n_envs)
        self.obs_shape = (int(obs_shape),) if isinstance(obs_shape, int) else tuple(int(x) for x in obs_shape)
        self.T, self.N, self.device, self.obs_dtype = T, N, torch.device(device), obs_dtype
        self.obs_dim = self.obs_shape[0]
        z = dict(device=self.device)
        # (T, N, *obs_shape): f32 vectors, or the u8 frame stacks of the pixel path
        self.obs = torch.zeros(T, N, *self.obs_shape, dtype=obs_dtype, **z)
        self.actions = torch.zeros(T, N, dtype=torch.int64, **z)
        self.logprobs = torch.zeros(T, N, dtype=torch.float32, **z)
        self.values = torch.zeros(T, N, dtype=torch.float32, **z)
        self.rewards = torch.zeros(T, N, dtype=torch.float32, **z)
        self.dones = torch.zeros(T, N, dtype=torch.uint8, **z)
        self.timeouts = torch.zeros(T, N, dtype=torch.uint8, **z)
        self.bootstrapped_values = torch.zeros(T, N, dtype=torch.float32, **z)
        self.advantages = torch.zeros(T, N, dtype=torch.float32, **z)
        self.returns = torch.zeros(T, N, dtype=torch.float32, **z)
        self.last_values = torch.zeros(N, dtype=torch.float32, **z)

    def view(self):
        from ._lib import RolloutView, RolloutViewU8
        V = RolloutViewU8 if self.obs_dtype == torch.uint8 else RolloutView
        return V(ptr(self.obs), ptr(self.actions), ptr(self.logprobs), ptr(self.values),
                           ptr(self.advantages), ptr(self.returns), self.T, self.N)


def _env_major(t: torch.Tensor) -> torch.Tensor:
    T, N = t.shape[0], t.shape[1]
    return t.transpose(0, 1).reshape(N * T, *t.shape[2:])


class DeviceTrajectory:
    """RolloutTrajectory-compatible (utils/rollout_buffer.py:16-25) view of a device rollout."""

    _FIELDS = ("observations", "actions", "rewards", "dones", "logprobs", "values", "advantages", "returns",
               "next_observations")

    def __init__(self, buf: DeviceRolloutBuffer):
        self.buffer = buf

    def __len__(self):
        return self.buffer.T * self.buffer.N

    @property
    def observations(self):
        return _env_major(self.buffer.obs)

    @property
    def actions(self):
        return _env_major(self.buffer.actions)

    @property
    def rewards(self):
        return _env_major(self.buffer.rewards)

    @property
    def dones(self):
        return _env_major(self.buffer.dones).bool()

    @property
    def logprobs(self):
        return _env_major(self.buffer.logprobs)

    @property
    def values(self):
        return _env_major(self.buffer.values)

    @property
    def advantages(self):
        return _env_major(self.buffer.advantages)

    @property
    def returns(self):
        return _env_major(self.buffer.returns)

    @property
    def next_observations(self):
        raise NotImplementedError("next_observations are never read by PPO and are not stored on device")


def compute_batched_gae_advantages_and_returns(values, rewards, dones, timeouts, last_values,
                                               bootstrapped_next_values, gamma, gae_lambda, adv_out=None,
                                               ret_out=None):
    """Same signature and result as utils/returns_advantages.py:115-155, on device tensors
    (T, N); bit-exact with the reference's numpy float32 loop."""
    T, N = values.shape
    dev = values.device
    dones = dones.to(torch.uint8) if dones.dtype != torch.uint8 else dones
    timeouts = timeouts.to(torch.uint8) if timeouts.dtype != torch.uint8 else timeouts
    adv = adv_out if adv_out is not None else torch.empty(T, N, dtype=torch.float32, device=dev)
    ret = ret_out if ret_out is not None else torch.empty(T, N, dtype=torch.float32, device=dev)
    args = [values, rewards, dones, timeouts, bootstrapped_next_values, last_values]
    for a in args:
        if a is not None and not (a.is_cuda and a.is_contiguous()):
            raise ValueError("GAE inputs must be contiguous device tensors")
    check(lib.gs_gae_f32(ptr(values), ptr(rewards), ptr(dones), ptr(timeouts), ptr(bootstrapped_next_values),
                         ptr(last_values), T, N, float(gamma), float(gae_lambda), ptr(adv), ptr(ret),
                         stream_handle()), "gs_gae_f32")
    return adv, ret


class DeviceRolloutCollector:
    """RolloutCollector (utils/rollout_collector.py:22-777) for the device path."""

    def __init__(self, env, policy_model, n_steps, *, gamma: float = 0.99, gae_lambda: float = 0.95,
                 stats_window_size: int = 100, rng_seed: int = 42, track_stats: bool = True,
                 use_graph: bool = True, one_launch: bool = True, normalize_advantages: bool = False, **kwargs):
        self.env = env
        self.policy_model = policy_model
        self.n_steps = int(n_steps)
        self.gamma, self.gae_lambda = float(gamma), float(gae_lambda)
        self.n_envs = int(env.num_envs)
        self.device = policy_model.device
        self.rng_seed = int(rng_seed)
        self.track_stats = bool(track_stats)
        # the rollout-level advantage normalisation (normalize_advantages == "rollout":
        # utils/rollout_collector.py:441-442 with returns_advantages.py:61-64), after GAE on the device
        self.normalize_advantages = bool(normalize_advantages)
        self._adv_scratch = None
        # device envs: the T-step loop (policy act + env step per vector step) is captured once
        # per sampling mode into a hipGraph and replayed; the per-rollout counters reach the
        # kernels through a 2-word device clock (include/gsamd.h "Rollout clock")
        self.use_graph = bool(use_graph)
        # the synthetic device env with a policy that fits in LDS: the whole rollout is one
        # launch (gs_rollout_synth, rows bit-identical to the step-wise loop)
        self.one_launch = bool(one_launch) and isinstance(env, DeviceSyntheticVecEnv) and \
            hasattr(policy_model, "dims") and self._synth_supported(policy_model)
        self._graphs = {}
        self._clock = None
        self.total_rollouts = self.total_steps = self.total_vec_steps = self.total_episodes = 0
        self.rollout_steps = self.rollout_vec_steps = self.rollout_episodes = 0
        self.stats_window_size = int(stats_window_size)
        self.rollout_fpss = RollingWindow(stats_window_size)
        # finished-episode statistics in the reference's processing order (step, then env):
        # rolling windows, best / last episode (utils/rollout_collector.py:93-98, 210-294)
        self.episode_reward_deque = RollingWindow(stats_window_size)
        self.episode_length_deque = RollingWindow(stats_window_size)
        self._best_episode_reward = -float("inf")
        self._last_episode_reward, self._last_episode_length = 0.0, 0
        self._recent_episodes = []       # (env, return, length, timeout) since the last consumer
        self._buffer: Optional[DeviceRolloutBuffer] = None
        self._started = False
        self._stats = None
        self._action_counts = None       # device int64 histogram of taken actions

    # ---- phases --------------------------------------------------------------------
    def _prepare(self):
        if self._started:
            return
        if getattr(self.env, "device_native", False):
            self.env.reset()
            obs_shape, obs_dtype = tuple(self.env.obs_shape), self.env.obs_dtype
        else:
            obs, _ = self.env.reset()
            obs = np.asarray(obs)
            obs_dtype = torch.uint8 if obs.dtype == np.uint8 else torch.float32
            self._host_obs = obs if obs_dtype == torch.uint8 else obs.astype(np.float32)
            obs_shape = tuple(obs.shape[1:])
        self._buffer = DeviceRolloutBuffer(self.n_envs, obs_shape, self.n_steps, self.device, obs_dtype)
        self._obs_dev = torch.zeros(self.n_envs, *obs_shape, dtype=obs_dtype, device=self.device)
        # running episode return / length per env (carried across rollouts) and this rollout's
        # completed-episode rows (gs_episode_stats)
        z = dict(device=self.device)
        self._run_ret = torch.zeros(self.n_envs, dtype=torch.float32, **z)
        self._run_len = torch.zeros(self.n_envs, dtype=torch.int32, **z)
        self._ep_ret_rows = torch.zeros(self.n_steps, self.n_envs, dtype=torch.float32, **z)
        self._ep_len_rows = torch.zeros(self.n_steps, self.n_envs, dtype=torch.int32, **z)
        self._started = True

    def _reset_env(self):
        """Fresh episodes on every env (evaluate_episodes; the reference sets obs = None)."""
        self._prepare()
        if getattr(self.env, "device_native", False):
            self.env.reset()
        else:
            obs, _ = self.env.reset()
            self._host_obs = np.asarray(obs, dtype=self._host_obs.dtype)
        self._run_ret.zero_()
        self._run_len.zero_()

    @property
    def buffer(self) -> DeviceRolloutBuffer:
        self._prepare()
        return self._buffer

    def collect(self, deterministic: bool = False, replay_actions: Optional[torch.Tensor] = None):
        """One rollout of n_steps vector steps; returns a DeviceTrajectory.

        replay_actions: optional (T, N) int64 device tensor of actions to take instead of
        sampling (parity tests replay a recorded reference rollout)."""
        self._prepare()
        buf, pm, N, T = self._buffer, self.policy_model, self.n_envs, self.n_steps
        t0 = time.time()
        mode = 2 if replay_actions is not None else (1 if deterministic else 0)
        native = getattr(self.env, "device_native", False)
        self.rollout_episodes = 0
        if self.one_launch:
            if replay_actions is not None:
                buf.actions.copy_(replay_actions)
            self._collect_one_launch(mode)
            T = 0                               # the steps ran inside the launch
        elif native and replay_actions is None and self.use_graph:
            self._collect_steps_graph(mode)
            T = 0                               # the steps ran inside the graph
        for t in range(T):
            if replay_actions is not None:
                buf.actions[t].copy_(replay_actions[t])
            counter = self.total_vec_steps + t
            if native:
                pm.act(self.env.obs, mode=mode, rng_seed=self.rng_seed, rng_counter=counter, actions=buf.actions[t],
                       logp=buf.logprobs[t], values=buf.values[t], obs_store=buf.obs[t])
                self.env.step_into(buf.rewards[t], buf.dones[t], buf.timeouts[t], actions=buf.actions[t])
            else:
                self._obs_dev.copy_(torch.from_numpy(self._host_obs))
                pm.act(self._obs_dev, mode=mode, rng_seed=self.rng_seed, rng_counter=counter, actions=buf.actions[t],
                       logp=buf.logprobs[t], values=buf.values[t], obs_store=buf.obs[t])
                actions_np = buf.actions[t].cpu().numpy()
                next_obs, rew, term, trunc, infos = self.env.step(actions_np)
                done = np.logical_or(term, trunc)
                buf.rewards[t].copy_(torch.from_numpy(np.asarray(rew, np.float32)))
                buf.dones[t].copy_(torch.from_numpy(done.astype(np.uint8)))
                buf.timeouts[t].copy_(torch.from_numpy(np.asarray(trunc).astype(np.uint8)))
                self._host_episode_infos(done, np.asarray(trunc, bool), infos)
                self._host_obs = np.asarray(next_obs, dtype=self._host_obs.dtype)
        T = self.n_steps
        last_obs = self.env.obs if native else self._obs_dev.copy_(torch.from_numpy(self._host_obs))
        pm.predict_values(last_obs, out=buf.last_values)
        compute_batched_gae_advantages_and_returns(buf.values, buf.rewards, buf.dones, buf.timeouts,
                                                   buf.last_values, buf.bootstrapped_values, self.gamma,
                                                   self.gae_lambda, adv_out=buf.advantages, ret_out=buf.returns)
        self.rollout_steps, self.rollout_vec_steps = N * T, T
        self.total_steps += N * T
        self.total_vec_steps += T
        self.total_rollouts += 1
        if self.track_stats:
            self._accumulate_stats()
            if native:
                self._episode_records()
        elif native:
            self._episode_window()
        if self.normalize_advantages:
            self._normalize_rollout_advantages()
        if not native:
            self.total_episodes += self.rollout_episodes
        self.rollout_fpss.append(N * T / max(time.time() - t0, 1e-9))
        return DeviceTrajectory(buf)

    @staticmethod
    def _synth_supported(pm) -> bool:
        v = ctypes.c_int()
        check(lib.gs_rollout_synth_supported(pm.dims, ctypes.byref(v)), "gs_rollout_synth_supported")
        return bool(v.value)

    def _collect_one_launch(self, mode):
        """The T vector steps as one gs_rollout_synth launch (policy act + env step per step,
        envs resident in LDS); the env's host step counter advances by T."""
        buf, pm, env = self._buffer, self.policy_model, self.env
        check(lib.gs_rollout_synth(ptr(pm.params), pm.dims, self.n_envs, self.n_steps, int(mode), self.rng_seed,
                                   self.total_vec_steps, ptr(env.state), ptr(env.ep_ret), ptr(env.obs),
                                   env.episode_len, env.truncate_every, env.reward, env.seed, env.env_offset,
                                   env.step_count, ptr(env.ep_count), ptr(env.ep_ret_sum), ptr(env.ep_len_sum),
                                   ptr(buf.obs), ptr(buf.actions), ptr(buf.logprobs), ptr(buf.values),
                                   ptr(buf.rewards), ptr(buf.dones), ptr(buf.timeouts), stream_handle()),
              "gs_rollout_synth")
        env.step_count += self.n_steps

    def _steps_into_buffer(self, mode, clock=None):
        """The rollout's T vector steps on a device env: policy act (writes the step's obs /
        action / log-prob / value rows) then the env step (reward / done / timeout rows)."""
        buf, pm, env = self._buffer, self.policy_model, self.env
        for t in range(self.n_steps):
            pm.act(env.obs, mode=mode, rng_seed=self.rng_seed, rng_counter=t if clock is not None else
                   self.total_vec_steps + t, actions=buf.actions[t], logp=buf.logprobs[t], values=buf.values[t],
                   obs_store=buf.obs[t], clock=clock)
            env.step_into(buf.rewards[t], buf.dones[t], buf.timeouts[t], actions=buf.actions[t], clock=clock,
                          step=t + 1)

    def _collect_steps_graph(self, mode):
        """Replay the captured T-step graph of this sampling mode (captured on the mode's second
        rollout; the first runs eagerly and allocates every scratch buffer the steps use).  The
        clock holds {rng counter, env step count} at the rollout start."""
        env = self.env
        if self._clock is None:
            self._clock = torch.zeros(2, dtype=torch.int64, device=self.device)
        step0 = int(getattr(env, "step_count", 0))
        g = self._graphs.get(mode)
        if g is None and (mode, "warm") not in self._graphs:
            self._graphs[(mode, "warm")] = True
            self._steps_into_buffer(mode)                       # eager, host counters
            return
        self._clock[0:1].fill_(self.total_vec_steps)
        self._clock[1:2].fill_(step0)
        if g is None:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                self._steps_into_buffer(mode, clock=self._clock)
            self._graphs[mode] = g
        g.replay()
        if hasattr(env, "step_count"):
            env.step_count = step0 + self.n_steps

    def _record_episode(self, env: int, ret: float, length: int, timeout: bool) -> None:
        """One finished episode, as _process_done_infos books it (rollout_collector.py:242-294)."""
        self.episode_reward_deque.append(ret)
        self.episode_length_deque.append(length)
        self._last_episode_reward, self._last_episode_length = ret, length
        self._best_episode_reward = max(self._best_episode_reward, ret)
        self._recent_episodes.append((env, ret, length, timeout))

    def _episode_records(self):
        """This rollout's finished episodes in the reference's order (step, then env), one D2H
        of their (return, length, timeout) records."""
        buf, N, T = self._buffer, self.n_envs, self.n_steps
        check(lib.gs_episode_stats(ptr(buf.rewards), ptr(buf.dones), T, N, ptr(self._run_ret), ptr(self._run_len),
                                   ptr(self._ep_ret_rows), ptr(self._ep_len_rows), stream_handle()),
              "gs_episode_stats")
        at = torch.nonzero(buf.dones.reshape(-1)).squeeze(1)        # time-major = (step, env) order
        rec = torch.stack([at.double(), self._ep_ret_rows.reshape(-1)[at].double(),
                           self._ep_len_rows.reshape(-1)[at].double(),
                           buf.timeouts.reshape(-1)[at].double()]).cpu().numpy()
        for pos, r, length, to in rec.T:
            self._record_episode(int(pos) % N, float(np.float32(r)), int(length), bool(to))
        self.rollout_episodes = rec.shape[1]
        self.total_episodes += self.rollout_episodes

    def _episode_window(self):
        """track_stats=False: the reference's rolling window (the last stats_window_size finished
        episodes, rollout_collector.py:242-294, 753-758) kept on the device with no host sync —
        this rollout's episodes in (step, env) order (gs_episode_stats) are merged behind the
        previous window by index arithmetic; best / last episode and the count ride along."""
        buf, N, T = self._buffer, self.n_envs, self.n_steps
        W = int(self.stats_window_size)
        check(lib.gs_episode_stats(ptr(buf.rewards), ptr(buf.dones), T, N, ptr(self._run_ret), ptr(self._run_len),
                                   ptr(self._ep_ret_rows), ptr(self._ep_len_rows), stream_handle()),
              "gs_episode_stats")
        dev = self.device
        if getattr(self, "_win", None) is None:
            self._win = torch.zeros(2, W, dtype=torch.float64, device=dev)        # returns, lengths
            self._win_meta = torch.zeros(3, dtype=torch.float64, device=dev)      # count, best, -
            self._win_meta[1] = -float("inf")
            self.rollout_episodes_dev = torch.zeros((), dtype=torch.int64, device=dev)
        # one launch (gs_episode_window): the block scan numbers this rollout's episodes in (step,
        # env) order, the last W land behind the shifted previous window
        check(lib.gs_episode_window(ptr(buf.dones), ptr(self._ep_ret_rows), ptr(self._ep_len_rows), T, N, W,
                                    ptr(self._win), ptr(self._win_meta), ptr(self.rollout_episodes_dev),
                                    stream_handle()), "gs_episode_window")

    def _window_metrics(self):
        """roll/ep_rew/{mean,best,last} and roll/ep_len/{mean,last} from the device window (one D2H)."""
        if getattr(self, "_win", None) is None:
            return {}
        w, meta = self._win.cpu().numpy(), self._win_meta.cpu().numpy()
        n = int(min(meta[0], w.shape[1]))
        if n <= 0:
            return {}
        r, ln = w[0, -n:], w[1, -n:]
        return {"roll/ep_rew/mean": float(np.float32(r).mean()), "roll/ep_len/mean": int(ln.mean()),
                "roll/ep_rew/best": float(meta[1]), "roll/ep_rew/last": float(np.float32(r[-1])),
                "roll/ep_len/last": int(ln[-1])}

    def _host_episode_infos(self, done, trunc, infos):
        """A host env's RecordEpisodeStatistics infos (rollout_collector.py:210-294)."""
        ep, mask = infos.get("episode"), infos.get("_episode")
        for e in np.nonzero(done)[0]:
            ok = ep is not None and mask is not None and mask[e]
            self._record_episode(int(e), float(ep["r"][e]) if ok else 0.0, int(ep["l"][e]) if ok else 0,
                                 bool(trunc[e]))
        self.rollout_episodes += int(np.count_nonzero(done))

    def _normalize_rollout_advantages(self):
        """adv = (adv - mean) / (std + 1e-8) over the whole rollout in place
        (gs_normalize_advantages; utils/returns_advantages.py:61-64), after the pre-normalisation
        advantage statistics were taken; with track_stats the normalised advantages feed the
        roll/adv_norm/* running statistics (utils/rollout_collector.py:441-448)."""
        buf = self._buffer
        if self._adv_scratch is None:
            nb = int(lib.gs_normalize_advantages_scratch_bytes(buf.advantages.numel()))
            self._adv_scratch = torch.zeros(max(1, nb // 4), dtype=torch.float32, device=self.device)
            self.adv_mean_std = torch.zeros(2, dtype=torch.float32, device=self.device)
        check(lib.gs_normalize_advantages(ptr(buf.advantages), buf.advantages.numel(), 1e-8, ptr(self._adv_scratch),
                                          ptr(self.adv_mean_std), stream_handle()), "gs_normalize_advantages")
        if self.track_stats:
            s = self._stats
            s[10] += buf.advantages.sum(dtype=torch.float64)
            s[11] += (buf.advantages.double() ** 2).sum()
            s[12] += buf.advantages.numel()

    def _accumulate_stats(self):
        """Device-side RunningStats sums (utils/rollout_stats.py:34-67) for get_metrics (slots 10-12:
        the normalised advantages, filled by _normalize_rollout_advantages)."""
        buf = self._buffer
        if self._stats is None:
            self._stats = torch.zeros(13, dtype=torch.float64, device=self.device)
        s = self._stats
        s[0] += buf.obs.numel()
        if buf.obs.dtype == torch.uint8:     # exact, without a float copy of the frames
            cnt = torch.bincount(buf.obs.reshape(-1), minlength=256).double()
            v = torch.arange(256, dtype=torch.float64, device=self.device)
            s[1] += (cnt * v).sum()
            s[2] += (cnt * v * v).sum()
        else:
            s[1] += buf.obs.sum(dtype=torch.float64)
            s[2] += (buf.obs.double() ** 2).sum()
        s[3] += buf.rewards.sum(dtype=torch.float64)
        s[4] += (buf.rewards.double() ** 2).sum()
        s[5] += buf.advantages.sum(dtype=torch.float64)
        s[6] += (buf.advantages.double() ** 2).sum()
        s[7] += buf.returns.sum(dtype=torch.float64)
        s[8] += (buf.returns.double() ** 2).sum()
        s[9] += buf.rewards.numel()
        # action histogram (rollout_collector.py:189-199), on device
        n_act = int(getattr(self.policy_model, "n_actions", 0)) or int(buf.actions.max().item()) + 1
        h = torch.bincount(buf.actions.reshape(-1), minlength=n_act)
        if self._action_counts is None or self._action_counts.numel() < h.numel():
            grown = torch.zeros(h.numel(), dtype=torch.int64, device=self.device)
            if self._action_counts is not None:
                grown[:self._action_counts.numel()] += self._action_counts
            self._action_counts = grown
        self._action_counts[:h.numel()] += h

    # ---- evaluation (utils/rollout_collector.py:570-655) -----------------------------
    def evaluate_episodes(self, *, n_episodes: int, deterministic: bool = True,
                          timeout_seconds: Optional[float] = None) -> dict:
        """The reference's protocol on this collector's env: fresh episodes on every env, whole
        rollouts (deterministic: argmax actions) until every env finished its balanced share of
        n_episodes; means over those episodes only, env steps counted per rollout."""
        N = self.n_envs
        base, rem = divmod(int(n_episodes), N)
        targets = [base + (1 if i < rem else 0) for i in range(N)]
        counts = [0] * N
        rew_sum, len_sum, steps, vec_steps = 0.0, 0, 0, 0
        self._reset_env()
        self._recent_episodes = []
        was_tracking, self.track_stats = self.track_stats, True    # episode records are needed
        t0 = time.time()
        try:
            while any(c < t for c, t in zip(counts, targets)):
                self.collect(deterministic=deterministic)
                steps += N * self.n_steps
                vec_steps += self.rollout_vec_steps
                recent, self._recent_episodes = self._recent_episodes, []
                for env, r, length, _ in recent:
                    if counts[env] >= targets[env]:
                        continue
                    rew_sum += float(r)
                    len_sum += int(length)
                    counts[env] += 1
                if timeout_seconds is not None and time.time() - t0 >= float(timeout_seconds):
                    break
        finally:
            self.track_stats = was_tracking
        total = int(sum(counts))
        m = self.get_metrics()
        m.pop("action_dist", None)
        m.update({"cnt/total_episodes": total, "cnt/total_env_steps": int(steps), "cnt/total_vec_steps": int(vec_steps)})
        if total > 0:
            m["roll/ep_rew/mean"] = float(rew_sum / total)
            m["roll/ep_len/mean"] = float(len_sum / total)
        return m

    # ---- API parity ------------------------------------------------------------------
    def slice_trajectories(self, trajectories, idxs):
        """utils/rollout_collector.py:657-682 — index the env-major views."""
        idx = torch.as_tensor(idxs, dtype=torch.int64, device=self.device)
        from types import SimpleNamespace
        return SimpleNamespace(**{f: getattr(trajectories, f)[idx] for f in DeviceTrajectory._FIELDS[:-1]})

    def get_metrics(self):
        """utils/rollout_collector.py:686-760: counters, running obs / reward / return /
        advantage statistics, the action histogram and its moments, baseline statistics (PPO's
        GAE targets never update them: zeros), and — once an episode has finished — the rolling
        window means, best and last episode.  In a multi-rank job the additive sums (steps,
        episodes, statistics, action counts) are summed over ranks before the means; the rolling
        window and best/last episode are this rank's."""
        part = [self.rollout_steps, self.total_episodes, self.rollout_episodes]
        n_stats = 0
        if self._stats is not None:
            st = list(self._stats.cpu().numpy().astype(np.float64))
            n_stats = len(st)
            part += st
        counts = self._action_counts.cpu().numpy() if self._action_counts is not None else np.zeros(0, np.int64)
        part += list(counts.astype(np.float64))
        env = self.env
        native = getattr(env, "device_native", False)
        dev_eps = native and not self.track_stats      # episode sums from the env's device counters
        if dev_eps:
            part += [float(env.ep_count.sum().item()), float(env.ep_ret_sum.sum().item()),
                     float(env.ep_len_sum.sum().item())]
        part = allreduce_sum_f64(part)
        scale = part[0] / max(self.rollout_steps, 1)
        m = {"cnt/total_env_steps": int(round(self.total_steps * scale)), "cnt/total_vec_steps": self.total_vec_steps,
             "cnt/total_episodes": int(part[1]), "cnt/total_rollouts": self.total_rollouts,
             "roll/env_steps": int(part[0]), "roll/vec_steps": self.rollout_vec_steps,
             "roll/episodes": int(part[2]), "roll/fps": float(self.rollout_fpss.mean()) if self.rollout_fpss else 0.0}

        def mean_std(sum_, sq, n):      # RunningStats.mean / .std (rollout_stats.py:59-67)
            if n <= 0:
                return 0.0, 0.0
            mean = sum_ / n
            return float(mean), float(np.sqrt(max(0.0, sq / n - mean * mean)))
        zero = (0.0, 0.0)
        if n_stats:
            s = part[3:3 + n_stats]
            obs, rew, adv, ret = (mean_std(s[1], s[2], s[0]), mean_std(s[3], s[4], s[9]), mean_std(s[5], s[6], s[9]),
                                  mean_std(s[7], s[8], s[9]))
        else:
            obs = rew = adv = ret = zero
        m["roll/obs/mean"], m["roll/obs/std"] = obs
        m["roll/reward/mean"], m["roll/reward/std"] = rew
        m["roll/return/mean"], m["roll/return/std"] = ret
        m["roll/adv/mean"], m["roll/adv/std"] = adv
        hist = np.asarray(part[3 + n_stats:3 + n_stats + counts.size], np.int64)
        nz = np.flatnonzero(hist)
        if nz.size:     # the reference's histogram grows to the largest action seen
            hist = hist[:nz[-1] + 1]
            idxs = np.arange(hist.shape[0], dtype=np.float32)
            total = float(hist.sum())
            a_mean = float((idxs * hist).sum() / total)
            a_var = float(((idxs - a_mean) ** 2 * hist).sum() / total)
            m["roll/actions/mean"], m["roll/actions/std"] = a_mean, float(np.sqrt(max(0.0, a_var)))
            m["action_dist"] = hist
        else:
            m["roll/actions/mean"], m["roll/actions/std"], m["action_dist"] = 0.0, 0.0, None
        m["roll/baseline/mean"], m["roll/baseline/std"] = zero
        if self.normalize_advantages and n_stats and s[12] > 0:      # rollout_collector.py:748-750
            m["roll/adv_norm/mean"], m["roll/adv_norm/std"] = mean_std(s[10], s[11], s[12])
        if dev_eps:
            cnt = part[-3]
            m["cnt/total_episodes"] = int(cnt)
            m.update(self._window_metrics())      # this rank's rolling window, as the reference's deques
        elif self.episode_reward_deque:
            m["roll/ep_rew/mean"] = float(self.episode_reward_deque.mean())
            m["roll/ep_len/mean"] = int(self.episode_length_deque.mean())
            m["roll/ep_rew/best"] = float(self._best_episode_reward)
            m["roll/ep_rew/last"] = float(self._last_episode_reward)
            m["roll/ep_len/last"] = int(self._last_episode_length)
        return m
