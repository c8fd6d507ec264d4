#!/usr/bin/env python3
"""Workload for the per-kernel C4 evidence (profiles/r03_c4_kernels.json): one C4-shaped rollout
(Pong rgb_ppo, 256 envs x 256 steps, NatureCNN, B = 1024), then `--mb` eager minibatch steps of the
update (gs_cnn_ppo_update over the first mb minibatches: no hipGraph, so every dispatch is its own
record).  Run it under
  rocprofv3 --kernel-trace --stats --output-format csv -d DIR -o cnn -- python tools/cnn_kernel_run.py
  rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d DIR -o fetch -- python tools/cnn_kernel_run.py
  rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d DIR -o write -- python tools/cnn_kernel_run.py
and reduce with tools/cnn_kernel_summary.py."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "gymnasium-solver_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=6)
    ap.add_argument("--n-envs", type=int, default=256)
    ap.add_argument("--workload", default="ALE-Pong-v5")
    ap.add_argument("--bf16", action="store_true", help="GS_HP_BF16 (bf16 MFMA operands)")
    a = ap.parse_args()
    from gsamd._lib import GS_HP_BF16, check, lib, ptr, stream_handle
    from gsamd.config import load_config
    from gsamd.ppo_agent import DevicePPOAgent
    torch.manual_seed(42)
    cfg = load_config(a.workload, "rgb_ppo", overrides=dict(env_dynamics="synthetic", n_envs=a.n_envs))
    agent = DevicePPOAgent(cfg, device="cuda:0", use_graph=False, track_stats=False)
    coll = agent.get_rollout_collector("train")
    coll.collect()
    idx = agent.prefetcher.upload(0)
    pm = agent.policy_model
    hp = agent.hparams()
    if a.bf16:
        hp.flags = GS_HP_BF16
    for n in (1, a.mb):     # one warm minibatch, then the measured ones
        check(lib.gs_cnn_ppo_update(ptr(pm.params), ptr(agent.grads), ptr(agent.adam_m), ptr(agent.adam_v), pm.dims,
                                    hp, coll.buffer.view(), ptr(idx), agent.batch_size, n, 0,
                                    ptr(agent.metrics_buf), ptr(agent.stop_flag), ptr(agent.workspace), None,
                                    stream_handle()), "gs_cnn_ppo_update")
    torch.cuda.synchronize()
    print(f"cnn kernel run: {1 + a.mb} minibatches of B={agent.batch_size}, loss {float(agent.metrics_buf[0, 0]):.5f}")


if __name__ == "__main__":
    main()
