"""ORACLE — test infrastructure only (tests/, smoke(), bench cpu_baseline).

numpy restatement of the device Atari observation pipeline (gymnasium-solver_amd/csrc/
gs_atari.hip), the a13 row of SURVEY.md §8:
  * frame source: synthetic ALE-shaped frames, two 210x160x3 u8 frames per env step
    (the last two frames of a frameskip), bytes = little-endian words of
    mix64^4(seed, env, 2*step+j, word) — the reference's emulator (ale-py 0.11.2) is not
    vendored and not installed, so frames are synthetic;
  * grayscale: OpenCV COLOR_RGB2GRAY fixed point (4899 R + 9617 G + 1868 B + 2^13) >> 14,
    the conversion gymnasium's AtariPreprocessing applies when it receives RGB frames
    (utils/environment.py:362-385); known answers (255,0,0)->76, (0,255,0)->150,
    (0,0,255)->29;
  * max-pool over the two frames (AtariPreprocessing / ale-py maxpool);
  * INTER_AREA-style box-filter resize to 84x84: fractional source coverage weights
    (double -> f32), row sums then column sum in f32 in a fixed order, times f32(1/area),
    round half to even — OpenCV's exact arithmetic is not available here (cv2 absent):
    parity with the reference's resize is UNPINNED; this restatement pins the device kernel;
  * frame stack of 4, newest last, zero padding after reset (FrameStackObservation
    padding_type="zero"), same-step autoreset with fixed-length episodes.
"""
from __future__ import annotations

import numpy as np

FH, FW, FC = 210, 160, 3
M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def mix64(z):
    with np.errstate(over="ignore"):
        z = (np.asarray(z, np.uint64) + np.uint64(0x9E3779B97F4A7C15)) & M64
        z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & M64
        z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & M64
        return z ^ (z >> np.uint64(31))


def render(seed: int, env_ids, step: int) -> np.ndarray:
    """(len(env_ids), 2, 210, 160, 3) u8 raw frames of vector step `step`."""
    env_ids = np.asarray(env_ids, np.uint64)
    words = np.arange(FH * FW * FC // 8, dtype=np.uint64)
    out = np.empty((len(env_ids), 2, FH * FW * FC // 8), np.uint64)
    for j in range(2):
        h = mix64(mix64(np.uint64(seed)) ^ env_ids)[:, None]
        h = mix64(mix64(h ^ np.uint64(2 * step + j)) ^ words[None, :])
        out[:, j] = h
    return out.view(np.uint8).reshape(len(env_ids), 2, FH, FW, FC)


def gray(frames: np.ndarray) -> np.ndarray:
    f = frames.astype(np.int64)
    return ((f[..., 0] * 4899 + f[..., 1] * 9617 + f[..., 2] * 1868 + (1 << 13)) >> 14).astype(np.int64)


def area_tables(n_out: int, n_in: int):
    sc = n_in / n_out
    starts, weights = [], []
    for o in range(n_out):
        a, b = o * sc, (o + 1) * sc
        i0, i1 = int(np.floor(a)), min(int(np.ceil(b)), n_in)
        starts.append(i0)
        weights.append([np.float32(min(b, i + 1) - max(a, i)) for i in range(i0, i1)])
    return starts, weights, sc


def preprocess(frames: np.ndarray, out_h: int = 84, out_w: int = 84) -> np.ndarray:
    """(N, 2, 210, 160, 3) -> (N, out_h, out_w) u8."""
    g = np.maximum(gray(frames[:, 0]), gray(frames[:, 1])).astype(np.float32)   # (N, H, W)
    ys, wy, sy = area_tables(out_h, FH)
    xs, wx, sx = area_tables(out_w, FW)
    inv_area = np.float32(1.0 / (sy * sx))
    N = frames.shape[0]
    out = np.empty((N, out_h, out_w), np.uint8)
    for oy in range(out_h):
        total = np.zeros((N, out_w), np.float32)
        for iy, w_y in enumerate(wy[oy]):
            src = g[:, ys[oy] + iy, :]
            row = np.zeros((N, out_w), np.float32)
            for ox in range(out_w):
                r = np.float32(0.0) * np.ones(N, np.float32)
                for ix, w_x in enumerate(wx[ox]):
                    r = (r + np.float32(w_x) * src[:, xs[ox] + ix]).astype(np.float32)
                row[:, ox] = r
            total = (total + np.float32(w_y) * row).astype(np.float32)
        out[:, oy, :] = np.clip(np.rint((total * inv_area).astype(np.float32)), 0, 255).astype(np.uint8)
    return out


class AtariEnvTwin:
    """Host twin of the device env (counters, rewards, dones, stacks)."""

    def __init__(self, n_envs, seed=42, env_offset=0, episode_len=27, stack=4, out_hw=(84, 84), truncate_every=0):
        self.N, self.seed, self.off, self.L, self.S = n_envs, seed, env_offset, episode_len, stack
        self.hw, self.trunc_every = out_hw, truncate_every
        self.ge = np.arange(n_envs, dtype=np.uint64) + np.uint64(env_offset)
        self.k = (self.ge % np.uint64(episode_len)).astype(np.int64)
        self.epi = np.zeros(n_envs, np.int64)
        self.stack = np.zeros((n_envs, stack, *out_hw), np.uint8)
        self.stack[:, -1] = preprocess(render(seed, self.ge, 0), *out_hw)
        self.step_count = 0

    def step(self):
        self.step_count += 1
        s = self.step_count
        h = mix64(mix64(mix64(mix64(np.uint64(self.seed)) ^ self.ge) ^ np.uint64(s)) ^ np.uint64(0xA7A7))
        rew = ((h >> np.uint64(40)).astype(np.float32) * np.float32(2.0 ** -23) - np.float32(1.0)).astype(np.float32)
        self.k += 1
        done = self.k >= self.L
        trunc = done & (self.trunc_every > 0) & ((self.epi % max(self.trunc_every, 1)) == self.trunc_every - 1)
        self.k[done] = 0
        self.epi[done] += 1
        new = preprocess(render(self.seed, self.ge, s), *self.hw)
        self.stack[:, :-1] = np.where(done[:, None, None, None], 0, self.stack[:, 1:])
        self.stack[:, -1] = new
        return rew, done, trunc
