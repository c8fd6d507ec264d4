#!/usr/bin/env python3
"""Diagnostic: per-phase cycle breakdown of the NatureCNN update's fused head + loss kernel
(k_cnn_head_loss, workgroup 0) from a GS_STAMPS build (s_memtime stamps of thread 0: shader
clock cycles, printed as us at 2.4 GHz).  Never part of the product library.

Here (CPU):        python tools/cnn_stamp_run.py --build      -> ab_libs/libgsamd_cnnstamps.so
GPU box:           python tools/cnn_stamp_run.py [--bf16] [--mb 8]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gymnasium-solver_amd")]
VARIANT = os.path.join(ROOT, "ab_libs", "libgsamd_cnnstamps.so")   # travels (tools/*.so do not)

PHASES = ["staging loads + LDS stores", "advantage statistics", "z partials", "z slice sums",
          "loss rows", "loss-sum reduction", "dh + dWh partials", "bias column"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--bf16", action="store_true")
    ap.add_argument("--mb", type=int, default=8)
    a = ap.parse_args()
    if a.build:
        import build_lib
        os.makedirs(os.path.dirname(VARIANT), exist_ok=True)
        build_lib.build_variant(VARIANT, ["GS_STAMPS"], tag="cnn")
        print("built", VARIANT)
        return
    os.environ["GSAMD_LIB"] = VARIANT
    import numpy as np
    import torch
    from gsamd._lib import GS_HP_BF16, check, lib, ptr, stream_handle
    from gsamd.config import load_config
    from gsamd.ppo_agent import DevicePPOAgent
    lib.gs_debug_cnn_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    torch.manual_seed(42)
    cfg = load_config("ALE-Pong-v5", "rgb_ppo", overrides=dict(env_dynamics="synthetic", n_envs=256))
    agent = DevicePPOAgent(cfg, device="cuda:0", use_graph=False, track_stats=False)
    coll = agent.get_rollout_collector("train")
    coll.collect()
    idx = agent.prefetcher.upload(0)
    pm = agent.policy_model
    hp = agent.hparams()
    if a.bf16:
        hp.flags = GS_HP_BF16

    def run(n):
        check(lib.gs_cnn_ppo_update(ptr(pm.params), ptr(agent.grads), ptr(agent.adam_m), ptr(agent.adam_v), pm.dims,
                                    hp, coll.buffer.view(), ptr(idx), agent.batch_size, n, 0,
                                    ptr(agent.metrics_buf), ptr(agent.stop_flag), ptr(agent.workspace), None,
                                    stream_handle()), "gs_cnn_ppo_update")
        torch.cuda.synchronize()

    run(1)
    acc0, cnt0 = np.zeros(128, np.uint64), np.zeros(8, np.uint64)
    lib.gs_debug_cnn_stamps(acc0.ctypes.data, cnt0.ctypes.data)
    run(a.mb)
    acc, cnt = np.zeros(128, np.uint64), np.zeros(8, np.uint64)
    lib.gs_debug_cnn_stamps(acc.ctypes.data, cnt.ctypes.data)
    acc = (acc - acc0).reshape(8, 16).astype(np.float64)
    n = float(cnt[0] - cnt0[0])
    per = acc[0] / max(n, 1.0)
    tot = per[:len(PHASES)].sum()
    print(f"k_cnn_head_loss workgroup 0 over {int(n)} launches: {tot:8.0f} cyc = {tot / 2.4e3:6.2f} us at 2.4 GHz")
    for i, ph in enumerate(PHASES):
        print(f"    {ph:28s} {per[i]:8.0f} cyc  {per[i] / 2.4e3:6.2f} us")
    # k_cnn_head_wgrad: slot 1 its record workgroup, slot 2 main workgroup 0 (round 6)
    for k, kn, names in ((1, "k_cnn_head_wgrad record workgroup", ["loss-sum partials", "totals", "record"]),
                         (2, "k_cnn_head_wgrad workgroup 0", ["dz rows -> LDS", "dbf partials", "barrier",
                                                              "h loads + FMAs", "slice shuffles",
                                                              "wave partials + block out"])):
        nk = float(cnt[k] - cnt0[k])
        if nk <= 0:
            continue
        pk = acc[k] / nk
        print(f"{kn} over {int(nk)} launches: {pk[:len(names)].sum():8.0f} cyc = "
              f"{pk[:len(names)].sum() / 2.4e3:6.2f} us")
        for i, ph in enumerate(names):
            print(f"    {ph:28s} {pk[i]:8.0f} cyc  {pk[i] / 2.4e3:6.2f} us")
    if a.bf16 and hasattr(lib, "gs_debug_conv_stamps"):
        # k_conv1_wgrad_bf's unit loop (csrc/gs_conv.hip C1S_MARK), workgroup 0, per launch
        lib.gs_debug_conv_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        c_acc, c_cnt = np.zeros(40, np.uint64), np.zeros(5, np.uint64)
        lib.gs_debug_conv_stamps(c_acc.ctypes.data, c_cnt.ctypes.data)
        c_acc = c_acc.reshape(5, 8)
        sets = [("k_conv1_wgrad_bf", ["MFMAs (LDS operand reads)", "tiles landed + LDS stores", "barrier",
                                      "load issue", "prologue", "partial out"]),
                ("k_conv_wgrad conv2", ["bias + gathers + MFMAs", "staging burst + LDS stores", "barrier",
                                        "loop-top barrier", "prologue", "partial out"]),
                ("k_conv_wgrad conv3", ["bias + gathers + MFMAs", "staging burst + LDS stores", "barrier",
                                        "loop-top barrier", "prologue", "partial out"])]
        for k, (kn, names) in enumerate(sets):
            cn = max(float(c_cnt[k]), 1.0)
            cper = c_acc[k, :6].astype(np.float64) / cn
            print(f"{kn} workgroup 0 over {int(cn)} launches (all launches of the process): "
                  f"{cper.sum():8.0f} cyc = {cper.sum() / 2.4e3:6.2f} us")
            for nm, v in zip(names, cper):
                print(f"    {nm:28s} {v:8.0f} cyc  {v / 2.4e3:6.2f} us")


if __name__ == "__main__":
    main()
