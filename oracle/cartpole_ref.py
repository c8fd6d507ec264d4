"""ORACLE — test infrastructure only.

numpy float64 twin of the device CartPole-v1 dynamics (gymnasium-solver_amd/csrc/gs_cartpole.hip),
SURVEY.md §8 f1.  gymnasium 1.1.1 (the reference's CartPole-v1 provider, un-vendored and not
installed here) is restated from its published CartPoleEnv: masscart 1.0, masspole 0.1,
length 0.5, force 10, tau 0.02, Euler integration, thresholds 2.4 / 12 degrees, reward 1,
TimeLimit 500, vector NEXT_STEP autoreset (reset step: reward 0, no done, action ignored).
Reset draws are the device's counter hash, not numpy's PCG64: parity with the reference's
own episodes is UNPINNED; this twin pins the kernel (tolerance: device cos/sin are not
correctly rounded like glibc's, so states agree to ~1e-12 and observations to f32 rounding).
"""
from __future__ import annotations

import math

import numpy as np

M64 = (1 << 64) - 1


def _mix64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M64
    return x ^ (x >> 31)


def reset_uniform(seed: int, env: int, episode: int, c: int) -> float:
    h = _mix64(_mix64(_mix64(_mix64(seed) ^ env) ^ episode) ^ (0xC0 + c))
    return -0.05 + 0.1 * ((h >> 11) * (1.0 / 9007199254740992.0))


class CartPoleTwin:
    def __init__(self, n_envs, seed=42, env_offset=0, max_steps=500):
        self.N, self.seed, self.off, self.max_steps = n_envs, seed, env_offset, max_steps
        self.state = [[reset_uniform(seed, env_offset + e, 0, c) for c in range(4)] for e in range(n_envs)]
        self.steps = [0] * n_envs
        self.episodes = [0] * n_envs
        self.pending = [False] * n_envs

    def obs(self):
        return np.array(self.state, dtype=np.float32)

    def step(self, actions):
        rew = np.zeros(self.N, np.float32)
        done = np.zeros(self.N, bool)
        trunc = np.zeros(self.N, bool)
        for e in range(self.N):
            if self.pending[e]:
                self.state[e] = [reset_uniform(self.seed, self.off + e, self.episodes[e], c) for c in range(4)]
                self.steps[e] = 0
                self.pending[e] = False
                continue
            x, x_dot, theta, theta_dot = self.state[e]
            force = 10.0 if int(actions[e]) == 1 else -10.0
            costheta, sintheta = math.cos(theta), math.sin(theta)
            temp = (force + 0.05 * (theta_dot * theta_dot) * sintheta) / 1.1
            thetaacc = (9.8 * sintheta - costheta * temp) / (0.5 * (4.0 / 3.0 - 0.1 * (costheta * costheta) / 1.1))
            xacc = temp - 0.05 * thetaacc * costheta / 1.1
            x, x_dot = x + 0.02 * x_dot, x_dot + 0.02 * xacc
            theta, theta_dot = theta + 0.02 * theta_dot, theta_dot + 0.02 * thetaacc
            self.state[e] = [x, x_dot, theta, theta_dot]
            th = 12.0 * 2.0 * math.pi / 360.0
            term = x < -2.4 or x > 2.4 or theta < -th or theta > th
            self.steps[e] += 1
            tr = (not term) and self.steps[e] >= self.max_steps
            rew[e] = 1.0
            done[e], trunc[e] = term or tr, tr
            if term or tr:
                self.episodes[e] += 1
                self.pending[e] = True
        return rew, done, trunc
