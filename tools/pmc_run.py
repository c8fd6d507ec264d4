#!/usr/bin/env python3
"""Workload for the rocprofv3 --pmc passes (profiles/pmc_traffic.json): one C2 rollout, then
`--reps` eager launches of each fused-chain minibatch kernel through gs_ppo_stage (no hipGraph, so
every dispatch is a separate counter record), then the GAE scan at the C2 and C3 shapes.  Run under
  rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d DIR -o pmc_fetch -- python tools/pmc_run.py
  rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d DIR -o pmc_write -- python tools/pmc_run.py
and reduce with tools/pmc_summarize.py."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "gymnasium-solver_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=64)
    ap.add_argument("--n-envs", type=int, default=4096)
    a = ap.parse_args()
    from gsamd._lib import check, lib
    from gsamd.config import load_config
    from gsamd.ppo_agent import DevicePPOAgent
    torch.manual_seed(42)
    cfg = load_config("CartPole-v1", "ppo", overrides=dict(env_dynamics="synthetic", n_envs=a.n_envs, n_epochs=1))
    agent = DevicePPOAgent(cfg, device="cuda:0", use_graph=False, track_stats=False)
    agent.train_epoch()
    pm = agent.policy_model
    idx = agent.prefetcher.device_buf
    def stage(st):
        return lib.gs_ppo_stage(st, pm.params.data_ptr(), agent.grads.data_ptr(), agent.adam_m.data_ptr(),
                                agent.adam_v.data_ptr(), pm.dims, agent.hparams(),
                                agent.get_rollout_collector("train").buffer.view(), idx.data_ptr(),
                                agent.batch_size, 1, agent.metrics_buf.data_ptr(), agent.workspace.data_ptr(),
                                torch.cuda.current_stream().cuda_stream)
    check(stage(6), "gs_ppo_stage")   # the fused chain's per-update gather (what gs_ppo_update runs)
    # the forward carrying the previous step's clip + Adam (stage 7, what gs_ppo_update runs on
    # one GPU) when available, else the plain fused forward (4); k_bwd<fused>; k_clip_adam
    fwd = 7 if stage(7) == 0 else 4
    for st in (fwd, 5, 3):
        for _ in range(a.reps):
            check(stage(st), "gs_ppo_stage")
    # the GAE scan on the C2 rollout buffer, and on a C3-shaped (2048 x 1024) random rollout
    from gsamd.rollout import compute_batched_gae_advantages_and_returns as gae
    buf = agent.get_rollout_collector("train").buffer
    for _ in range(8):
        gae(buf.values, buf.rewards, buf.dones, buf.timeouts, buf.last_values, buf.bootstrapped_values, 0.98, 0.8,
            adv_out=torch.empty_like(buf.advantages), ret_out=torch.empty_like(buf.returns))
    T, N = 2048, 1024
    v, r, b = (torch.randn(T, N, device="cuda:0") for _ in range(3))
    d = (torch.rand(T, N, device="cuda:0") < 0.05).to(torch.uint8)
    to = (d.bool() & (torch.rand(T, N, device="cuda:0") < 0.3)).to(torch.uint8)
    lv = torch.randn(N, device="cuda:0")
    for _ in range(8):
        gae(v, r, d, to, lv, b, 0.99, 0.95)
    torch.cuda.synchronize()
    print("pmc_run done")


if __name__ == "__main__":
    main()
