"""Workload for the rollout (collect) evidence: one workload's device rollouts only (no update),
for `rocprofv3 --kernel-trace --stats`.  Usage: python tools/collect_run.py [C5|C4|C2] [rollouts]
Prints the mean collect time per rollout from HIP events on the launch stream."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gymnasium-solver_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from gsamd.config import load_config  # noqa: E402
from gsamd.ppo_agent import DevicePPOAgent  # noqa: E402


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "C5"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    env_id, variant, n_envs = bench.WORKLOADS[wl]
    torch.manual_seed(42)
    cfg = load_config(env_id, variant, overrides=dict(n_envs=n_envs, env_dynamics="synthetic"))
    agent = DevicePPOAgent(cfg, device=torch.device("cuda:0"), track_stats=False)
    coll = agent.get_rollout_collector("train")
    coll.collect()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        coll.collect()
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / n
    print(f"{wl}: {n_envs} envs x {cfg.n_steps} steps: collect {ms:.3f} ms per rollout "
          f"({ms * 1e3 / cfg.n_steps:.1f} us per vector step)")


if __name__ == "__main__":
    main()
