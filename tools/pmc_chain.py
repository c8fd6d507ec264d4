#!/usr/bin/env python3
"""Workload for chain-context PMC passes: the C2 update chain as it runs in gs_ppo_update
(lagged forward -> backward, minibatch after minibatch), launched eagerly so every dispatch is
its own counter record.  Run under `rocprofv3 --pmc <counters> --kernel-trace ...`; reduce with
tools/pmc_chain_summary.py."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "gymnasium-solver_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402


def main(n=96):
    from gsamd._lib import check, lib
    from gsamd.config import load_config
    from gsamd.ppo_agent import DevicePPOAgent
    torch.manual_seed(42)
    cfg = load_config("CartPole-v1", "ppo", overrides=dict(env_dynamics="synthetic", n_envs=4096, n_epochs=1))
    agent = DevicePPOAgent(cfg, device="cuda:0", use_graph=False, track_stats=False)
    agent.train_epoch()
    coll = agent.get_rollout_collector("train")
    idx = agent.prefetcher.upload(1)
    pm = agent.policy_model
    check(lib.gs_ppo_update(pm.params.data_ptr(), agent.grads.data_ptr(), agent.adam_m.data_ptr(),
                            agent.adam_v.data_ptr(), pm.dims, agent.hparams(), coll.buffer.view(), idx.data_ptr(),
                            agent.batch_size, n, agent.adam_step, agent.metrics_buf.data_ptr(),
                            agent.stop_flag.data_ptr(), agent.workspace.data_ptr(), agent.workspace.numel(), None, 0,
                            torch.cuda.current_stream().cuda_stream), "gs_ppo_update")
    torch.cuda.synchronize()
    print("pmc_chain done")


if __name__ == "__main__":
    main()
