"""Workload for the a13 evidence (profiles/r04_atari_*): the device Atari env at C4's shape
(256 envs; N from argv) stepped 200 times — counters + synthetic render + the observation
pipeline (k_atari_stack84: grayscale, max-pool, 84x84 area resize, 4-frame stack shift) —
for `rocprofv3 --kernel-trace --stats` and the separate FETCH_SIZE / WRITE_SIZE passes.
Prints the mean step time from HIP events on the launch stream and the stack kernel's
algorithmic bytes per launch (201 600 read + 7 056 written per env step)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gymnasium-solver_amd")]

import torch  # noqa: E402

from gsamd.atari_env import DeviceAtariVecEnv  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    dev = torch.device("cuda:0")
    env = DeviceAtariVecEnv(N, episode_len=400, seed=42, device=dev)
    env.reset()
    r = torch.zeros(N, device=dev)
    d = torch.zeros(N, dtype=torch.uint8, device=dev)
    to = torch.zeros(N, dtype=torch.uint8, device=dev)
    for _ in range(10):
        env.step_into(r, d, to)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(steps):
        env.step_into(r, d, to)
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) * 1e3 / steps
    alg = N * (2 * 210 * 160 * 3 + 84 * 84)
    print(f"N={N} env step (counters + render + stack) {us:.2f} us; stack algorithmic bytes per launch {alg}")


if __name__ == "__main__":
    main()
