"""Synthetic fixed-length-episode vector env (SURVEY.md §8d "Synthetic inputs").

The bench and the parity tests have no gymnasium / Box2D / ALE on the GPU box, so the
workload runs on a synthetic env whose observations are a counter-based hash, identical
bit for bit on the host (this module, numpy) and on the device (csrc/gs_env.hip):

    h      = mix(mix(mix(seed) ^ env) ^ step) ^ dim   ; mix = SplitMix64 finaliser
    obs    = f32(h' >> 40) * 2^-23 - 1                 ; h' = mix(h), exact in f32, in [-1, 1)

Episode bookkeeping mirrors gymnasium's RecordEpisodeStatistics vector output
(``info["episode"]{r,l}``, ``info["_episode"]``) that the reference collector consumes at
utils/rollout_collector.py:223-240.  Env ``e`` starts ``e mod L`` steps into its first
episode so that dones spread over steps; an episode lasts ``L`` steps and ends
``terminated``, except every ``truncate_every``-th episode of an env, which ends
``truncated`` (exercises the timeout path of GAE).  Autoreset is same-step: the obs
returned with a done is already the next episode's first obs (obs do not depend on
state, so the reset obs is simply the hash of the next counter).  Actions are ignored.
Env dynamics parity with gymnasium is out of scope ("parity unpinned").
"""
from __future__ import annotations

import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
_GOLD = np.uint64(0x9E3779B97F4A7C15)
_C1 = np.uint64(0xBF58476D1CE4E5B9)
_C2 = np.uint64(0x94D049BB133111EB)


def mix64(x):
    """SplitMix64 step (increment + finaliser) on uint64 arrays, wrapping."""
    with np.errstate(over="ignore"):
        x = np.asarray(x, dtype=np.uint64) + _GOLD
        x = (x ^ (x >> np.uint64(30))) * _C1
        x = (x ^ (x >> np.uint64(27))) * _C2
        return x ^ (x >> np.uint64(31))


def synth_obs(seed, env, step, dim):
    """Observation component ``dim`` of env ``env`` after ``step`` vector steps (broadcasts)."""
    h = mix64(mix64(mix64(np.uint64(seed)) ^ np.asarray(env, np.uint64)) ^ np.asarray(step, np.uint64))
    h = mix64(h ^ np.asarray(dim, np.uint64))
    u24 = (h >> np.uint64(40)).astype(np.float32)
    return (u24 * np.float32(2.0 ** -23) - np.float32(1.0)).astype(np.float32)


class SyntheticVecEnv:
    """gymnasium-1.x VectorEnv-shaped synthetic env: reset() -> (obs, info); step(a) -> 5-tuple."""

    def __init__(self, n_envs, obs_dim, n_actions, episode_len=200, seed=42, truncate_every=0,
                 env_offset=0, reward=1.0):
        self.num_envs = int(n_envs)
        self.n_actions = int(n_actions)
        self.obs_dim = int(obs_dim)
        self.episode_len = int(episode_len)
        self.seed = int(seed)
        self.truncate_every = int(truncate_every)
        self.env_offset = int(env_offset)   # global env id of local env 0 (multi-GPU shards)
        self.reward = float(reward)
        self._env_ids = np.arange(self.num_envs, dtype=np.uint64) + np.uint64(self.env_offset)
        self._dims = np.arange(self.obs_dim, dtype=np.uint64)
        self.reset()

    def _obs(self):
        return synth_obs(self.seed, self._env_ids[:, None], np.uint64(self.step_count), self._dims[None, :])

    def reset(self, *args, **kwargs):
        self.step_count = 0
        self.k = (self._env_ids % np.uint64(self.episode_len)).astype(np.int64)
        self.episode_idx = np.zeros(self.num_envs, np.int64)
        self.ep_ret = np.zeros(self.num_envs, np.float32)
        self.ep_len = np.zeros(self.num_envs, np.int64)
        return self._obs(), {}

    def step(self, actions):
        assert np.asarray(actions).shape[0] == self.num_envs
        self.step_count += 1
        rew = np.full(self.num_envs, self.reward, np.float32)
        self.k += 1
        self.ep_ret += rew
        self.ep_len += 1
        done = self.k >= self.episode_len
        if self.truncate_every > 0:
            trunc_ep = (self.episode_idx % self.truncate_every) == (self.truncate_every - 1)
        else:
            trunc_ep = np.zeros(self.num_envs, bool)
        truncated = done & trunc_ep
        terminated = done & ~trunc_ep
        infos = {}
        if done.any():
            infos["episode"] = {"r": np.where(done, self.ep_ret, 0.0).astype(np.float32),
                                "l": np.where(done, self.ep_len, 0).astype(np.int64)}
            infos["_episode"] = done.copy()
            self.k[done] = 0
            self.episode_idx[done] += 1
            self.ep_ret[done] = 0.0
            self.ep_len[done] = 0
        return self._obs(), rew, terminated, truncated, infos
