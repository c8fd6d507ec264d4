"""Device Atari-shaped vector env: synthetic ALE-sized frames rendered on
the GPU, the AtariVectorEnv observation pipeline (grayscale, max-pool of the last two frames,
84x84 area resize, 4-frame stack) as HIP kernels, fixed-length episodes with same-step
autoreset.  Observations never leave HBM: the rollout collector copies each step's stack
into the u8 rollout buffer and the CNN reads it from there.

Reference: utils/environment.py:240-303 (ale-py AtariVectorEnv: grayscale, img 84x84,
stack_num 4, frameskip, full 18-action space) and :362-385 (AtariPreprocessing +
FrameStackObservation(padding_type="zero")).
"""
from __future__ import annotations

import torch

from ._lib import check, lib, ptr, stream_handle


class DeviceAtariVecEnv:
    device_native = True

    def __init__(self, n_envs, n_actions=18, episode_len=400, seed=42, truncate_every=0, env_offset=0,
                 frame_stack=4, out_hw=(84, 84), device="cuda"):
        self.num_envs, self.n_actions = int(n_envs), int(n_actions)
        self.episode_len, self.seed, self.truncate_every = int(episode_len), int(seed), int(truncate_every)
        self.env_offset, self.frame_stack = int(env_offset), int(frame_stack)
        self.out_h, self.out_w = (int(x) for x in out_hw)
        self.obs_shape = (self.frame_stack, self.out_h, self.out_w)
        self.obs_dtype = torch.uint8
        self.device = torch.device(device)
        N = self.num_envs
        z = dict(device=self.device)
        self.state = torch.zeros(4 * N, dtype=torch.int32, **z)
        self.ep_ret = torch.zeros(N, dtype=torch.float32, **z)
        self.obs = torch.zeros(N, *self.obs_shape, dtype=torch.uint8, **z)
        self.frames = torch.zeros(N, 2, 210, 160, 3, dtype=torch.uint8, **z)
        self.ep_count = torch.zeros(N, dtype=torch.int32, **z)
        self.ep_ret_sum = torch.zeros(N, dtype=torch.float32, **z)
        self.ep_len_sum = torch.zeros(N, dtype=torch.float32, **z)
        self.step_count = 0

    def reset(self):
        self.step_count = 0
        check(lib.gs_atari_env_reset(ptr(self.state), ptr(self.ep_ret), ptr(self.obs), ptr(self.frames),
                                     self.num_envs, self.frame_stack, self.out_h, self.out_w, self.episode_len,
                                     self.seed, self.env_offset, stream_handle()), "gs_atari_env_reset")
        return self.obs, {}

    def step_into(self, rewards_row, dones_row, timeouts_row, actions=None, clock=None, step=None):
        """One vector step; clock/step as DeviceSyntheticVecEnv.step_into (captured rollouts)."""
        if clock is None:
            self.step_count += 1
        check(lib.gs_atari_env_step(ptr(self.state), ptr(self.ep_ret), ptr(self.obs), ptr(self.frames),
                                    self.num_envs, self.frame_stack, self.out_h, self.out_w, self.episode_len,
                                    self.truncate_every, self.seed, self.env_offset,
                                    self.step_count if clock is None else int(step), ptr(rewards_row),
                                    ptr(dones_row), ptr(timeouts_row), ptr(self.ep_count), ptr(self.ep_ret_sum),
                                    ptr(self.ep_len_sum), ptr(clock), stream_handle()), "gs_atari_env_step")


def atari_preprocess(frames: torch.Tensor, out_hw=(84, 84)) -> torch.Tensor:
    """(N, 2, 210, 160, 3) u8 device frames -> (N, 84, 84) u8 observation frames."""
    if not (frames.is_cuda and frames.dtype == torch.uint8 and frames.is_contiguous()
            and tuple(frames.shape[1:]) == (2, 210, 160, 3)):
        raise ValueError("frames must be a contiguous uint8 device tensor (N, 2, 210, 160, 3)")
    out = torch.empty(frames.shape[0], *out_hw, dtype=torch.uint8, device=frames.device)
    check(lib.gs_atari_preprocess(ptr(frames), frames.shape[0], int(out_hw[0]), int(out_hw[1]), ptr(out),
                                  stream_handle()), "gs_atari_preprocess")
    return out
