#!/usr/bin/env python3
"""Diagnostic: phase stamps of the rollout act's conv2 / conv3 forward (k_conv_fwd, fp32, 4
workgroups per sample; workgroup 0, thread 0, s_memtime) over C5 collects, from the GS_STAMPS build
of tools/cnn_stamp_run.py --build (ab_libs/libgsamd_cnnstamps.so).  Never part of the product.
GPU box:  python tools/act_stamp_run.py [rollouts]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gymnasium-solver_amd")]
os.environ["GSAMD_LIB"] = os.path.join(ROOT, "ab_libs", "libgsamd_cnnstamps.so")

PHASES = ["weights + staging burst + LDS stores", "barrier", "MFMAs", "k-range partials via LDS", "epilogue"]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    import numpy as np
    import torch
    import bench
    from gsamd._lib import lib
    from gsamd.config import load_config
    from gsamd.ppo_agent import DevicePPOAgent
    lib.gs_debug_conv_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    env_id, variant, n_envs = bench.WORKLOADS["C5"]
    torch.manual_seed(42)
    cfg = load_config(env_id, variant, overrides=dict(n_envs=n_envs, env_dynamics="synthetic"))
    agent = DevicePPOAgent(cfg, device=torch.device("cuda:0"), track_stats=False)
    coll = agent.get_rollout_collector("train")
    coll.collect()
    torch.cuda.synchronize()
    a0, c0 = np.zeros(40, np.uint64), np.zeros(5, np.uint64)
    lib.gs_debug_conv_stamps(a0.ctypes.data, c0.ctypes.data)
    for _ in range(n):
        coll.collect()
    torch.cuda.synchronize()
    a1, c1 = np.zeros(40, np.uint64), np.zeros(5, np.uint64)
    lib.gs_debug_conv_stamps(a1.ctypes.data, c1.ctypes.data)
    acc = (a1 - a0).reshape(5, 8).astype(np.float64)
    for k, name in ((3, "conv2 forward (act, FS 4)"), (4, "conv3 forward (act, FS 4)")):
        cn = float(c1[k] - c0[k])
        if cn <= 0:
            continue
        per = acc[k, :len(PHASES)] / cn
        print(f"{name} workgroup 0 over {int(cn)} launches: {per.sum():8.0f} cyc = {per.sum() / 2.4e3:6.2f} us")
        for ph, v in zip(PHASES, per):
            print(f"    {ph:38s} {v:8.0f} cyc  {v / 2.4e3:6.2f} us")


if __name__ == "__main__":
    main()
