"""Where the bench line's collect phase differs from a back-to-back collect (tools/collect_run.py):
one process, the bench's agent and workload, three timings of the same rollout —
  (a) back-to-back collects (collect_run's loop),
  (b) train_epoch's order (collect right after an update, no host sync), split by events into
      the graph replay, the post-graph tail (values, GAE, episode window) and the index upload,
      with the host time of each call,
  (c) as (b) with a device sync between the update and the collect.
Usage: python tools/collect_phase_probe.py [C5|C4] [epochs]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gymnasium-solver_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from gsamd.config import load_config  # noqa: E402
from gsamd.ppo_agent import DevicePPOAgent  # noqa: E402


def ev():
    return torch.cuda.Event(enable_timing=True)


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "C5"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    env_id, variant, n_envs = bench.WORKLOADS[wl]
    torch.manual_seed(42)
    cfg = load_config(env_id, variant, overrides=dict(n_envs=n_envs, env_dynamics="synthetic"))
    agent = DevicePPOAgent(cfg, device=torch.device("cuda:0"), track_stats=False)
    coll = agent.get_rollout_collector("train")
    for _ in range(2):
        agent.train_epoch()
    torch.cuda.synchronize()

    marks = {}
    orig = coll._collect_steps_graph

    def replay(mode):
        marks["g0"].record()
        t = time.perf_counter()
        orig(mode)
        marks["host_replay"] = time.perf_counter() - t
        marks["g1"].record()
    coll._collect_steps_graph = replay

    def one(sync_before):
        for k in ("c0", "g0", "g1", "c1", "u0", "u1"):
            marks[k] = ev()
        if sync_before:
            torch.cuda.synchronize()
        marks["c0"].record()
        t = time.perf_counter()
        agent._trajectories = coll.collect()
        marks["host_collect"] = time.perf_counter() - t
        marks["c1"].record()
        agent.update_phase([[ev(), marks["u0"], marks["u1"]]])   # [1]: after the index upload
        return dict(marks)

    rows = {"after-update": [], "sync-then-collect": []}
    for i in range(n):
        rows["after-update"].append(one(False))
        rows["sync-then-collect"].append(one(True))
    torch.cuda.synchronize()
    for name, rs in rows.items():
        for r in rs:
            print(f"{wl} {name:18s} collect {r['c0'].elapsed_time(r['u0']):7.3f} ms "
                  f"[start->graph {r['c0'].elapsed_time(r['g0']):6.3f}  graph {r['g0'].elapsed_time(r['g1']):7.3f}  "
                  f"tail {r['g1'].elapsed_time(r['c1']):6.3f}  c1->update {r['c1'].elapsed_time(r['u0']):6.3f}] "
                  f"update {r['u0'].elapsed_time(r['u1']):7.3f} ms  host: replay {r['host_replay'] * 1e3:6.3f} "
                  f"collect {r['host_collect'] * 1e3:6.3f} ms")
    e0, e1 = ev(), ev()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(n):
        coll.collect()
    e1.record()
    e1.synchronize()
    print(f"{wl} back-to-back       collect {e0.elapsed_time(e1) / n:7.3f} ms per rollout")


if __name__ == "__main__":
    main()
