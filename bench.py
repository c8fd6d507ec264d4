#!/usr/bin/env python3
"""bench.py — env-steps/s of the MI355X rollout + GAE + PPO-update path.

Workload (BASELINE.json configs[1], "C2"): CartPole-v1:ppo shapes — MLP 4->256->256->{2,1},
n_envs=4096 per GPU, n_steps=32, batch 256, 20 epochs (10 240 minibatch steps per rollout),
gamma 0.98, lambda 0.8, clip 0.1, Adam lr 1e-3, max_grad_norm 0.5 — on the synthetic
fixed-length-episode env (no gymnasium on the box).  A "step" is one
reference epoch: one rollout of 4096 x 32 env steps (policy forward + sample + env step
per vector step, bootstrap value, GAE) followed by the whole PPO update over it.

  python bench.py [--gpus N --steps K --warmup W]
  python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

Multi-GPU: weak scaling — every rank owns its own 4096 envs (global env ids offset by
rank), runs its own sampler stream, and the flat gradient is all-reduced (RCCL, mean)
once per minibatch step before the norm clip.  value = all ranks' env steps / max-rank time.
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, os.path.join(ROOT, "gymnasium-solver_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402

PEAK_F32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md: dense f32 MFMA (= f32 vector peak)
PEAK_HBM_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E spec
PEAK_BF16_MFMA_TFLOPS = 2500.0  # MI355X_MICROARCH.md: ~2.5 PF dense bf16 (no sparsity)
# CPU port vs the reference's own loop on the same 8-core container at C2 shapes: port / reference, re-derived in round 6 on the build container (tools/cpu_calibration.py: the
# reference's own C2 loop, imported from /root/reference, and the port alternated in 24 blocks of 50
# minibatches on the same 8 threads, medians; 4 runs gave 0.90 / 1.36 / 1.18 / 1.06 on this shared
# container, the last — the longest, 1 200 minibatches — is the constant).  Round 1's 2.006 predates
# the port's activation-statistics and grad-norm work (the reference records both every step).  It is
# applied cross-CPU: measured on the container's Intel Xeon, applied to the GPU box's EPYC host.
CPU_PORT_OVER_REFERENCE = 1.057
CALIBRATION_PROVENANCE = ("build container, 8-core Intel Xeon (1 thread/core), torch 2.10 CPU at 8 threads, C2 shapes, "
                          "round 6: tools/cpu_calibration.py (reference loop 6.18 ms vs port 5.85 ms per minibatch, "
                          "medians of 24 alternated blocks; collect 0.144 vs 0.113 s); applied cross-CPU to the GPU "
                          "box's host")


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return ""


def _log(*a):
    print(*a, file=sys.stderr, flush=True)


# workload id -> (env id, variant, envs per GPU)  (BASELINE.json configs)
WORKLOADS = {"C2": ("CartPole-v1", "ppo", 4096), "C3": ("LunarLander-v3", "ppo", 1024),
             "C4": ("ALE-Pong-v5", "rgb_ppo", 256), "C5": ("ALE-Breakout-v5", "rgb_ppo", 128)}
# BASELINE.json's metric is quoted on C2; the other workloads are labelled as what they are
METRICS = {"C2": "env steps/sec (rollout+PPO update), CartPole n_envs=4096, 1/2/4/8 MI355X",
           "C3": "env steps/sec (rollout+PPO update), LunarLander-v3 shapes n_envs={n}/GPU, MI355X",
           "C4": "env steps/sec (rollout+PPO update), ALE/Pong-v5 rgb_ppo NatureCNN n_envs={n}/GPU, MI355X",
           "C5": "env steps/sec (rollout+PPO update), ALE/Breakout-v5 rgb_ppo NatureCNN n_envs={n}/GPU, MI355X"}


def usable_cores() -> tuple:
    """(threads to use, cores in the affinity mask, cgroup CPU quota in cores or None): a GPU
    box shows the whole machine in sched_getaffinity while its cgroup grants a share of it, so
    the CPU baseline runs one thread per core of the quota (SURVEY §8d asks for the cores the
    process can use)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(-(-int(q) // int(period))))
    except (OSError, ValueError):
        pass
    use = min(aff, quota) if quota else aff
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:      # the box's per-GPU CPU share (16 on the GPU pool)
        use = min(use, int(omp))
    return use, aff, quota


def cnn_minibatch_flops(B, A):
    """NatureCNN minibatch step: forward (conv1..3, fc, heads) + backward (wgrad of every
    layer, dgrad of fc/conv3/conv2, none for conv1): 2 x MACs."""
    fwd = 400 * 32 * 256 + 81 * 64 * 512 + 49 * 64 * 576 + 3136 * 512 + 512 * (A + 1)
    bwd = 2 * (3136 * 512 + 49 * 64 * 576 + 81 * 64 * 512 + 512 * (A + 1)) + 400 * 32 * 256
    return 2.0 * B * (fwd + bwd)


def stage_flops_bytes(D, H1, H2, A, B, P, fused=True):
    """Algorithmic work per launch of each minibatch-step kernel; in the fused
    chain k_bwd also computes the loss rows (no k_loss launch)."""
    A1 = A + 1
    fwd = 2.0 * B * (D * H1 + H1 * H2 + H2 * A1)
    loss = 2.0 * B * A1 * (H2 // 16) + 30.0 * B
    bwd = 2.0 * B * H2 * A1 + 2.0 * B * H1 * H2 * 2 + 2.0 * B * H1 * (D + 1) + 2.0 * B * H2 * A1 + B * H2
    adam_bytes = 4.0 * P * 7      # read p, g, m, v; write p, m, v
    if fused:
        return {"fwd": ("mfma", fwd), "fwd_adam": ("mfma", fwd), "bwd": ("mfma", bwd + loss),
                "adam": ("hbm", adam_bytes)}
    return {"fwd": ("mfma", fwd), "loss": ("mfma", loss), "bwd": ("mfma", bwd), "adam": ("hbm", adam_bytes)}


def fwd_adam_hbm_bytes(D, H1, H2, A, B, P):
    """Algorithmic HBM bytes of one lagged forward (k_fwd_hidden<fused, adam>): the clip + Adam
    of the previous step (read p, g, m, v; write p, m, v: 28 B/param) + the dW1|db1 partials
    folded on the way (8 row blocks x H1(D+1) floats) + this minibatch's x rows, and the
    activations it writes for the backward (h1, h2, per-column-block head partials, relu' bits)."""
    nrb = (B + 31) // 32
    adam = 28.0 * P + 4.0 * nrb * H1 * (D + 1)
    acts = 4.0 * B * D + 4.0 * B * (H1 + H2) + 4.0 * (H2 // 16) * B * (A + 1) + 2.0 * B * (H2 // 16)
    return adam + acts


def time_stages(agent, reps: int):
    """Average device duration of each minibatch-step kernel: `reps` launches of one stage
    captured into a hipGraph (no host launch gaps) and replayed between HIP events recorded on
    the stream the kernels are launched on (the capture stream's replay target)."""
    from gsamd._lib import check, lib
    coll = agent.get_rollout_collector("train")
    idx = agent.prefetcher.device_buf
    pm = agent.policy_model
    args = lambda st: (st, pm.params.data_ptr(), agent.grads.data_ptr(), agent.adam_m.data_ptr(),  # noqa: E731
                       agent.adam_v.data_ptr(), pm.dims, agent.hparams(), coll.buffer.view(), idx.data_ptr(),
                       agent.batch_size, max(agent.adam_step, 1), agent.metrics_buf.data_ptr(),
                       agent.workspace.data_ptr(), torch.cuda.current_stream().cuda_stream)
    saved = [t.clone() for t in (pm.params, agent.grads, agent.adam_m, agent.adam_v)]
    out = {}
    # the fused chain (what gs_ppo_update runs for the compile-time shapes): gather once,
    # then k_fwd_hidden<fused>, k_bwd<fused> (loss rows inside), k_clip_adam.  The clip + Adam
    # step rides in the next minibatch's forward (stage 7, k_fwd_hidden<fused, adam>; with a
    # communicator after the exchange) and k_clip_adam runs once per update, so it is not a
    # per-minibatch stage.
    fused = lib.gs_ppo_stage(*args(6)) == 0
    lagged = fused and lib.gs_ppo_stage(*args(7)) == 0
    if lagged:
        stages = ((7, "fwd_adam"), (5, "bwd"))
    elif fused:
        stages = ((4, "fwd"), (5, "bwd"), (3, "adam"))
    else:
        stages = ((0, "fwd"), (1, "loss"), (2, "bwd"), (3, "adam"))
    for st, name in stages:
        for _ in range(3):
            check(lib.gs_ppo_stage(*args(st)), "gs_ppo_stage")
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            for _ in range(reps):
                check(lib.gs_ppo_stage(*args(st)), "gs_ppo_stage")
        g.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        out[name] = e0.elapsed_time(e1) / reps * 1e3   # microseconds per launch
        del g
    for t, s in zip((pm.params, agent.grads, agent.adam_m, agent.adam_v), saved):
        t.copy_(s)
    return out, fused


def time_gae(agent, reps: int):
    """Average device duration of the GAE scan (gs_gae_f32) on this workload's rollout buffer:
    `reps` launches captured into a hipGraph, replayed between HIP events on the launch
    stream; writes into scratch outputs (the inputs are the last rollout's)."""
    from gsamd.rollout import compute_batched_gae_advantages_and_returns as gae
    buf = agent.get_rollout_collector("train").buffer
    coll = agent.get_rollout_collector("train")
    adv, ret = torch.empty_like(buf.advantages), torch.empty_like(buf.returns)
    args = (buf.values, buf.rewards, buf.dones, buf.timeouts, buf.last_values, buf.bootstrapped_values,
            coll.gamma, coll.gae_lambda)
    gae(*args, adv_out=adv, ret_out=ret)
    torch.cuda.synchronize()
    if not (torch.equal(adv, buf.advantages) and torch.equal(ret, buf.returns)):
        raise RuntimeError("GAE replay differs from the rollout's own advantages")
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        for _ in range(reps):
            gae(*args, adv_out=adv, ret_out=ret)
    g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    e1.synchronize()
    T, N = buf.values.shape
    return e0.elapsed_time(e1) / reps * 1e3, int(T), int(N)


def roofline_entry(bound: str, amount: float, us: float, kernel: str, mfma_peak: float = None) -> dict:
    """mfma_peak: the dense MFMA peak of the operand type (f32 by default; the bf16 mode's lines use
    the bf16 peak)."""
    if bound == "mfma":
        pk = mfma_peak or PEAK_F32_MFMA_TFLOPS
        a = amount / (us * 1e-6) / 1e12
        return {"bound": "mfma", "achieved": round(a, 4), "peak": pk, "unit": "TFLOP/s",
                "frac": round(a / pk, 6), "kernel": kernel, "avg_us": round(us, 3),
                "work_per_launch": amount}
    a = amount / (us * 1e-6) / 1e9
    return {"bound": "hbm", "achieved": round(a, 2), "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": round(a / PEAK_HBM_GBS, 6), "kernel": kernel, "avg_us": round(us, 3), "work_per_launch": amount}


def time_exchange(comm, n: int, reps: int, device, barrier):
    """Average duration of one gradient exchange of n floats (all ranks replay a graph of
    `reps` exchanges together after a barrier; HIP events on this rank's stream)."""
    from gsamd._lib import check, lib
    buf = torch.zeros(n, dtype=torch.float32, device=device)
    run = lambda: check(lib.gs_comm_allreduce_mean_f32(comm, buf.data_ptr(), n,  # noqa: E731
                                                        torch.cuda.current_stream().cuda_stream), "exchange")
    for _ in range(3):
        run()
    barrier()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        for _ in range(reps):
            run()
    barrier()
    g.replay()
    barrier()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    e1.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    barrier()
    del g
    return us


def bf16_deviation(agent) -> dict:
    """Loss trajectory of one update (all its minibatches) in the fp32 parity path and in the bf16
    mode, from the same parameters / Adam state on the same rollout and index stream.  Each mode runs
    twice from that state and the second run is timed (`update_ms`): the MLP chain's update graph is
    then captured already (gs_ppo_update caches it), as in the bench line's own timed steps."""
    import numpy as np
    from gsamd._lib import GS_HP_BF16, check, lib, ptr, stream_handle
    pm, coll = agent.policy_model, agent.get_rollout_collector("train")
    idx = agent.prefetcher.device_buf
    state = [t.clone() for t in (pm.params, agent.adam_m, agent.adam_v)]
    res = {}
    for name, flags, rep in (("fp32", 0, 0), ("fp32", 0, 1), ("bf16", GS_HP_BF16, 0), ("bf16", GS_HP_BF16, 1)):
        for t, s0 in zip((pm.params, agent.adam_m, agent.adam_v), state):
            t.copy_(s0)
        hp = agent.hparams()
        hp.flags = flags
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        if agent.is_pixel:
            check(lib.gs_cnn_ppo_update(ptr(pm.params), ptr(agent.grads), ptr(agent.adam_m), ptr(agent.adam_v),
                                        pm.dims, hp, coll.buffer.view(), ptr(idx), agent.batch_size,
                                        agent.n_minibatches, agent.adam_step, ptr(agent.metrics_buf),
                                        ptr(agent.stop_flag), ptr(agent.workspace), None, stream_handle()),
                  "gs_cnn_ppo_update")
        else:     # the MLP's fused chain (the update the bench line times), as one captured graph
            check(lib.gs_ppo_update(ptr(pm.params), ptr(agent.grads), ptr(agent.adam_m), ptr(agent.adam_v), pm.dims,
                                    hp, coll.buffer.view(), ptr(idx), agent.batch_size, agent.n_minibatches,
                                    agent.adam_step, ptr(agent.metrics_buf), ptr(agent.stop_flag),
                                    ptr(agent.workspace), agent.workspace.numel(), None, 1, stream_handle()),
                  "gs_ppo_update")
        e1.record()
        e1.synchronize()
        if rep == 0:      # warm-up: the graph capture (MLP) and first-touch costs
            continue
        res[name] = (agent.metrics_buf[:, 0].cpu().numpy().astype(np.float64), pm.params.cpu().numpy().astype(np.float64),
                     e0.elapsed_time(e1))
    for t, s0 in zip((pm.params, agent.adam_m, agent.adam_v), state):
        t.copy_(s0)
    (l32, p32, t32), (l16, p16, t16) = res["fp32"], res["bf16"]
    scale = max(1.0, float(np.abs(l32).max()))
    return {"minibatches": int(l32.size), "loss_max_abs_dev": float(np.abs(l16 - l32).max()),
            "loss_max_dev_rel_to_scale": float(np.abs(l16 - l32).max() / scale),
            "loss_mean_abs_dev": float(np.abs(l16 - l32).mean()),
            "final_params_rel_l2": float(np.linalg.norm(p16 - p32) / np.linalg.norm(p32)),
            "update_ms": {"fp32": round(t32, 3), "bf16": round(t16, 3)}}


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])


def rank_environments(n: int, base: dict, port: int) -> list:
    """The torch.distributed.run-style environment of each of n local ranks (rank r on GPU r)."""
    envs = []
    for r in range(n):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0",
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        envs.append(e)
    return envs


def launch_ranks(n: int, argv, script: str = None, poll_s: float = 0.2) -> int:
    """`python bench.py --gpus N` without an external launcher: start N child processes of
    `script` (this file) with argv, one rank per GPU, and wait for them.  The parent never
    touches the GPU (children are fresh processes, not forks or execs of a GPU-initialised
    one).  Rank 0's stdout — the JSON line — is inherited; the other ranks' stdout goes to
    stderr.  If any rank fails, the rest are terminated (they would wait at a barrier) and
    the first failing exit code is returned."""
    import subprocess
    port = int(os.environ.get("MASTER_PORT") or 0) or _free_port()
    cmd = [sys.executable, "-u", os.path.abspath(script or __file__), *argv]
    procs = [subprocess.Popen(cmd, env=e, stdout=None if r == 0 else sys.stderr)
             for r, e in enumerate(rank_environments(n, os.environ, port))]
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]      # poll every rank (no short-circuit)
            if all(c is not None for c in codes):
                break
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                _log(f"[bench] a rank exited with {rc}; stopping the others")
                break
            time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    if rc == 0:
        rc = next((p.returncode for p in procs if p.returncode != 0), 0)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=tuple(WORKLOADS), default="C2",
                    help="C2: CartPole-v1:ppo (the metric's config); C3: LunarLander-v3:ppo shapes (T=2048, B=64); "
                         "C4/C5: ALE Pong/Breakout rgb_ppo (NatureCNN, Atari pixel pipeline)")
    ap.add_argument("--env-dynamics", choices=("synthetic", "cartpole"), default="synthetic",
                    help="MLP workloads: SURVEY §8d synthetic fixed-length episodes (default) or device CartPole-v1")
    ap.add_argument("--n-envs", type=int, default=None, help="envs per GPU (weak scaling; default per workload)")
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of the hipGraph")
    ap.add_argument("--local-comm", action="store_true",
                    help="N=1 only: run the multi-GPU chain through a one-rank communicator")
    ap.add_argument("--comm", choices=("xgmi", "rccl"), default="xgmi",
                    help="gradient-exchange transport for N>1 (and --local-comm): one-shot xGMI or RCCL")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal on a one-GPU box: all ranks share cuda:0 (gloo process group, "
                         "xGMI exchange through same-device IPC); throughput is not meaningful")
    ap.add_argument("--dtype", choices=("f32", "bf16"), default="f32",
                    help="f32: the fp32 parity path (default, the metric's line); bf16: bf16 MFMA operands in the "
                         "update (the MLP's fused chain, the NatureCNN's convolutions / GEMMs), reported as its own "
                         "line with its deviation from fp32 over one whole update")
    ap.add_argument("--dp-mode", choices=("local", "global"), default="local",
                    help="N>1: local (each rank's own minibatches, gradients averaged: the default) or global (the "
                         "reference's exact global minibatches split over the ranks, sums exchanged)")
    ap.add_argument("--stage-reps", type=int, default=200)
    ap.add_argument("--cpu-minibatches", type=int, default=-1,
                    help="minibatches timed in the CPU baseline (-1: the whole update, 0: no CPU baseline)")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher around us: start one rank per GPU ourselves (before any GPU call)
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"[bench] WORLD_SIZE={world} but --gpus {args.gpus}: they must agree")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dev_index = 0 if args.same_device else local_rank
    torch.cuda.set_device(dev_index)
    device = torch.device(f"cuda:{dev_index}")
    if world > 1:
        import torch.distributed as dist
        if args.same_device:          # rehearsal: every rank on cuda:0, host-side process group
            dist.init_process_group("gloo", rank=rank, world_size=world)
        else:
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=device)

    from gsamd.config import load_config
    from gsamd.ppo_agent import DevicePPOAgent
    torch.manual_seed(42)
    env_id, variant, n_default = WORKLOADS[args.workload]
    pixel = variant == "rgb_ppo"
    n_envs = args.n_envs or n_default
    # the benchmark's env is chosen explicitly: SURVEY §8d synthetic fixed-length episodes (or the
    # synthetic Atari frame source), or the device CartPole-v1 dynamics
    over = dict(n_envs=n_envs, env_dynamics="synthetic" if pixel else args.env_dynamics)
    if args.dtype == "bf16":
        over["precision"] = "bf16"
    if args.dp_mode == "global":
        over["dp_mode"] = "global"
    cfg = load_config(env_id, variant, overrides=over)
    agent = DevicePPOAgent(cfg, device=device, rank=rank, world_size=world,
                           use_graph=not args.no_graph, track_stats=False)
    comm = None
    if world > 1 or args.local_comm:      # sized to this policy's flat gradient
        from gsamd import distributed as gd
        n_params = agent.policy_model.n_params
        if world == 1:
            comm = gd.init_local_comm(args.comm, n_params)
        elif args.comm == "xgmi":
            try:
                # MLP: the in-backward exchange is checked on this job's shapes before the timed run
                comm = gd.init_xgmi_comm(rank, world, n_params, device,
                                         verify_shapes=None if pixel else (agent.policy_model.dims, cfg.batch_size,
                                                                           int(agent.hparams().flags)))
            except RuntimeError as e:     # every rank raises together: switch transport together
                _log(f"[bench] {e}; using RCCL for the gradient exchange")
                args.comm = "rccl (xgmi unavailable)"
                comm = gd.init_device_comm(rank, world, device)
        else:
            comm = gd.init_device_comm(rank, world, device)
        agent.comm = comm
    comm_info = None
    from gsamd.distributed import LAST_SELF_TEST as gd_self_test
    if comm is not None:
        from gsamd.distributed import comm_info as _comm_info
        comm_info = _comm_info(comm)
        if comm_info["nranks"] != world or comm_info["rank"] != rank:
            raise RuntimeError(f"communicator reports {comm_info}, launcher says rank {rank} of {world}")
    N, T = cfg.n_envs, cfg.n_steps

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()

    if args.warmup < 2 and not args.no_graph:
        _log("[bench] warning: --warmup < 2 times the rollout graph's capture (second collect)")
    tw = time.perf_counter()
    for _ in range(args.warmup):
        agent.train_epoch()
    barrier()
    _log(f"[bench] rank {rank}: warmup {args.warmup} steps {time.perf_counter() - tw:.2f}s")
    agent.phase_events = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        agent.train_epoch()
    barrier()
    elapsed = time.perf_counter() - t0
    phases = agent.phase_events
    agent.phase_events = None
    collect_ms = sum(e[0].elapsed_time(e[1]) for e in phases) / len(phases)
    update_ms = sum(e[1].elapsed_time(e[2]) for e in phases) / len(phases)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if args.same_device else device)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    losses = agent.minibatch_losses()
    if not (losses == losses).all():
        raise RuntimeError("non-finite loss in the timed region")
    total_env_steps = world * N * T * args.steps
    value = total_env_steps / elapsed
    ms_per_step = elapsed / args.steps * 1e3

    # ---- roofline of the dominant minibatch kernel (device time by events) ----
    pm = agent.policy_model
    stage_us = {}
    rooflines = {}
    if pixel:
        # the update is a chain of GEMMs + fused kernels per minibatch: price the whole
        # minibatch step (events around the update phase of the timed region) against MFMA
        amount = cnn_minibatch_flops(agent.batch_size, pm.n_actions)
        mb_us = update_ms * 1e3 / agent.n_minibatches
        achieved = amount / (mb_us * 1e-6) / 1e12
        peak = PEAK_BF16_MFMA_TFLOPS if args.dtype == "bf16" else PEAK_F32_MFMA_TFLOPS
        roofline = {"bound": "mfma", "achieved": round(achieved, 4), "peak": peak, "unit": "TFLOP/s",
                    "frac": round(achieved / peak, 6), "traffic": None,
                    "kernel": "cnn minibatch step (k_conv1_*, k_gemm, gs_cnn kernels)", "avg_us": round(mb_us, 3),
                    "work_per_launch": amount}
    else:
        stage_us, fused = time_stages(agent, args.stage_reps)
        work = stage_flops_bytes(pm.obs_dim, pm.hidden_dims[0], pm.hidden_dims[1], pm.n_actions, agent.batch_size,
                                 pm.n_params, fused)
        dom = max(stage_us, key=stage_us.get)
        kname = {"fwd": "k_fwd_hidden", "fwd_adam": "k_fwd_hidden", "loss": "k_loss", "bwd": "k_bwd", "adam": "k_clip_adam"}
        mpk = PEAK_BF16_MFMA_TFLOPS if args.dtype == "bf16" else PEAK_F32_MFMA_TFLOPS
        for st, us in stage_us.items():
            rooflines[st] = roofline_entry(work[st][0], work[st][1], us, kname[st], mpk)
        if "fwd_adam" in rooflines:
            # the lagged forward also streams the previous step's clip + Adam (28 B/param) and
            # writes the activations the backward reads: its HBM term beside the MFMA one; the
            # two fractions add (time shares of one launch)
            hb = fwd_adam_hbm_bytes(pm.obs_dim, pm.hidden_dims[0], pm.hidden_dims[1], pm.n_actions, agent.batch_size,
                                    pm.n_params)
            h = roofline_entry("hbm", hb, stage_us["fwd_adam"], "k_fwd_hidden")
            e = rooflines["fwd_adam"]
            e["hbm_term"] = {k: h[k] for k in ("achieved", "peak", "unit", "frac", "work_per_launch")}
            e["combined_frac"] = round(e["frac"] + h["frac"], 6)
        roofline = {k: v for k, v in rooflines[dom].items()}
        roofline["traffic"] = None
    # GAE scan on this workload's rollout buffer (HBM-bound; 22 B/element + 4 B/env)
    gae_us, gT, gN = time_gae(agent, args.stage_reps)
    rooflines["gae"] = roofline_entry("hbm", 22.0 * gT * gN + 4.0 * gN, gae_us,
                                      "k_gae_staged" if gN % 4 == 0 else "k_gae_f32")
    rooflines["gae"]["shape"] = [gT, gN]
    # the scan's own bound: T dependent steps of two VALU ops (24 cycles per step, the scanner's
    # in-kernel stamps) at 2.4 GHz — bit-exact parity forbids splitting T
    rooflines["gae"]["serial_bound_us"] = round(gT * 24 / 2.4e3, 3)
    rooflines["gae"]["serial_frac"] = round(gT * 24 / 2.4e3 / gae_us, 4) if gae_us > 0 else None
    in_bwd = None
    if comm is not None:       # every rank takes part (the exchange is collective)
        if not pixel:
            from gsamd.distributed import exchange_inside_bwd
            in_bwd = exchange_inside_bwd(comm, pm.dims, cfg.batch_size)
        # the exchange as its own launch (what the chain runs after k_bwd unless in_bwd)
        stage_us["exchange_launch" if in_bwd else "exchange"] = time_exchange(comm, pm.n_params, args.stage_reps,
                                                                               device, barrier)
    # PMC HBM traffic per launch (tools/pmc_run.py + tools/pmc_summarize.py), used only when it was
    # recorded from the kernel sources the LOADED library was compiled from: the library carries
    # its sources' hash (gs_build_source_hash, embedded by build_lib.py), and the sources on disk
    # must still hash to it (a stale prebuilt library is never labelled current)
    from gsamd.buildinfo import source_hash as _disk_hash
    from gsamd._lib import lib as _lib

    def source_hash(path):
        h = _lib.gs_build_source_hash(path.encode())
        h = h.decode() if h else None
        return h if h == _disk_hash(path) else f"{h} (library) != {_disk_hash(path)} (sources on disk)"
    pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    pmc = {}
    if os.path.exists(pmc_path):
        try:
            with open(pmc_path) as f:
                pmc = json.load(f)
        except (OSError, ValueError):
            pmc = {}
    traffic_src = {"file": "profiles/pmc_traffic.json", "recorded_source_hash": pmc.get("_source_hash"),
                   "library_source_hash": source_hash("mlp"), "sources": "mlp"}
    traffic_src["current"] = bool(pmc) and traffic_src["recorded_source_hash"] == traffic_src["library_source_hash"]
    if traffic_src["current"]:
        if args.workload == "C2":   # the committed minibatch-kernel PMC passes are C2-shaped
            roofline["traffic"] = pmc.get(roofline["kernel"], {}).get("hbm_bytes_per_launch")
            for st, ent in rooflines.items():
                if st != "gae":
                    ent["traffic"] = pmc.get(ent["kernel"], {}).get("hbm_bytes_per_launch")
        # the GAE passes are keyed by grid size (tools/pmc_run.py: C2 and C3 shapes)
        ew = 16 if gN % 16 == 0 else 8 if gN % 8 == 0 else 4
        grid = (gN // ew) * (8 if ew >= 8 else 4) * 64
        rooflines["gae"]["traffic"] = pmc.get(f"k_gae_staged[grid={grid}]", {}).get("hbm_bytes_per_launch")
    roofline["traffic_source"] = traffic_src
    if pixel and args.workload == "C4":
        # the C4 minibatch's HBM bytes: the per-kernel PMC passes (tools/cnn_kernel_summary.py over
        # tools/cnn_kernel_run.py, profiles/c4_kernels.json), again only from the current sources
        kname = "c4_kernels_bf16.json" if args.dtype == "bf16" else "c4_kernels.json"
        kpath = os.path.join(ROOT, "profiles", kname)
        kern = {}
        if os.path.exists(kpath):
            try:
                with open(kpath) as f:
                    kern = json.load(f)
            except (OSError, ValueError):
                kern = {}
        ksrc = {"file": "profiles/" + kname, "recorded_source_hash": kern.get("_source_hash"),
                "library_source_hash": source_hash("cnn"), "sources": "cnn", "operands": kern.get("operands")}
        ksrc["current"] = bool(kern) and ksrc["recorded_source_hash"] == ksrc["library_source_hash"] and \
            kern.get("operands") == ("bf16" if args.dtype == "bf16" else "f32")
        if ksrc["current"]:
            mb = kern.get("minibatch", {})
            roofline["traffic"] = mb.get("hbm_bytes")
            roofline["kernels"] = {k: {q: e.get(q) for q in ("avg_us", "mfma_frac", "hbm_frac", "traffic_over_alg")
                                       if e.get(q) is not None}
                                   for k, e in kern.get("kernels", {}).items()}
        roofline["traffic_source"] = ksrc

    # ---- bf16 mode: one whole update in fp32 and in bf16 from the same state, rollout and
    #      sampler order; the per-minibatch loss deviation is reported beside the line ----
    bf16_dev = bf16_deviation(agent) if args.dtype == "bf16" and rank == 0 else None

    # ---- CPU baseline (rank 0, N=1 only): oracle restatement on the host cores ----
    cpu = None
    if rank == 0 and world == 1 and args.cpu_minibatches != 0:
        import datetime
        import platform
        cores, aff, quota = usable_cores()
        host = {"cores": cores, "affinity_cores": aff, "cgroup_quota_cores": quota,
                "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "cpu_model": _cpu_model(),
                "measured_utc": datetime.datetime.now(datetime.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ"),
                "host": platform.node()}
    if cpu is None and rank == 0 and world == 1 and args.cpu_minibatches != 0 and pixel:
        from oracle.cpu_ppo import run_cpu_baseline_cnn
        r = run_cpu_baseline_cnn(n_envs=N, n_steps=T, batch=cfg.batch_size, n_epochs=cfg.n_epochs,
                                 in_shape=tuple(pm.in_shape), n_actions=pm.n_actions, valid=cfg.valid_actions,
                                 clip=cfg.clip_range, ent_coef=cfg.ent_coef, lr=cfg.policy_lr, threads=cores)
        cpu = {"value": round(r["env_steps_per_s"], 2), "unit": "env_steps/s", "cores": r["threads"], "kind": "port",
               "sample": (f"{r['sample_steps']} vector steps of the torch-CPU NatureCNN policy on {N} envs + "
                          f"{r['sample_minibatches']} of {r['minibatches_per_rollout']} minibatch steps "
                          f"(B={cfg.batch_size}), each after one untimed, extrapolated to the rollout / update; env "
                          f"emulation excluded; wall {r['wall_s']:.1f}s"),
               "step_ms": round(r["step_s"] * 1e3, 3), "minibatch_ms": round(r["minibatch_s"] * 1e3, 3),
               "window_minibatch_ms": [round(x * 1e3, 3) for x in r["window_minibatch_s"]], **host}
    elif cpu is None and rank == 0 and world == 1 and args.cpu_minibatches != 0:
        from oracle.cpu_ppo import run_cpu_baseline
        r = run_cpu_baseline(n_envs=N, n_steps=T, batch=cfg.batch_size, n_epochs=cfg.n_epochs,
                             obs_dim=pm.obs_dim, hidden=tuple(pm.hidden_dims), n_actions=pm.n_actions,
                             gamma=cfg.gamma, lam=cfg.gae_lambda, clip=cfg.clip_range, lr=cfg.policy_lr,
                             max_minibatches=args.cpu_minibatches if args.cpu_minibatches > 0 else None,
                             threads=cores)
        whole = r["minibatches_timed"] == r["minibatches_per_rollout"]
        cpu = {"value": round(r["env_steps_per_s"], 2), "unit": "env_steps/s", "cores": r["threads"], "kind": "port",
               "sample": (f"1 rollout of {N}x{T} env steps (torch-CPU policy, numpy synthetic env, numpy GAE) + "
                          f"{'all ' if whole else ''}{r['minibatches_timed']} of {r['minibatches_per_rollout']} "
                          f"minibatch steps (torch-CPU fwd/bwd/clip/Adam){'' if whole else ', update extrapolated'}; "
                          f"wall {r['wall_s']:.1f}s"),
               "collect_s": round(r["collect_s"], 4), "minibatch_ms": round(r["minibatch_s"] * 1e3, 4),
               # per-minibatch time of each tenth of the timed minibatches: their spread is how far an
               # extrapolation from a shorter sample (or a noisy neighbour) could move the value
               "window_minibatch_ms": [round(x * 1e3, 4) for x in r["window_minibatch_s"]],
               **host,
               # measured in the build container (tools/cpu_calibration.py), applied here
               "calibration_port_over_reference": CPU_PORT_OVER_REFERENCE,
               "calibration_provenance": CALIBRATION_PROVENANCE,
               "reference_equivalent_value": round(r["env_steps_per_s"] / CPU_PORT_OVER_REFERENCE, 2),
               "calibration": ("the port omits the reference's Lightning training_step, DataLoader collate and "
                               "metrics-recorder overheads; divided by the measured ratio it estimates the "
                               "reference loop on these cores")}

    if comm is not None:       # a timed-out exchange never yields a bench line
        from gsamd.distributed import comm_status
        comm_status(comm)
    if rank == 0:
        line = {
            "metric": METRICS[args.workload].format(n=N),
            "value": round(value, 2), "unit": "env_steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
            "data": "synthetic" if args.env_dynamics == "synthetic" else "device CartPole-v1 dynamics",
            "config": {"workload": (f"{env_id}:{variant} {args.workload} (rollout {N} envs x {T} steps + "
                                    f"{cfg.n_epochs}-epoch PPO update, B={cfg.batch_size})"),
                       "n_envs_per_gpu": N, "n_steps": T, "batch_size": cfg.batch_size, "n_epochs": cfg.n_epochs,
                       "minibatches_per_step": agent.n_minibatches, "policy": (f"NatureCNN {pm.in_shape} -> {pm.hidden} -> {{{pm.n_actions} masked to "
                                  f"{len(cfg.valid_actions or [])},1}}" if pixel else
                                  f"MLP {pm.obs_dim}-{pm.hidden_dims[0]}-{pm.hidden_dims[1]}-{{{pm.n_actions},1}}"),
                       "parallelism": f"dp{world}" if world > 1 else "single", "graph": not args.no_graph,
                       "grad_exchange": args.comm if comm is not None else None,
                       "exchange_in_bwd": in_bwd,
                       "exchange_self_test": dict(gd_self_test) if comm is not None else None,
                       "comm": comm_info, "same_device": bool(args.same_device),
                       "dp_mode": args.dp_mode,
                       # the reference's training_step diagnostics (opt/activations/*, per-step
                       # records) are a track_stats option; the timed region runs without them
                       "track_stats": False, "activation_stats_in_timed_region": False,
                       # the rollout's step graph is captured on the second collect (the first runs
                       # eagerly and allocates): with --warmup < 2 the capture is inside the timed region
                       "rollout_graph_capture_in_timed_region": (not args.no_graph) and args.warmup < 2},
            "roofline": roofline,
            "rooflines": rooflines,
            "stages_us": {k: round(v, 3) for k, v in stage_us.items()},
            "phases_ms": {"collect": round(collect_ms, 3), "update": round(update_ms, 3),
                          "update_us_per_minibatch": round(update_ms * 1e3 / agent.n_minibatches, 3)},
            "cpu_baseline": cpu,
        }
        if bf16_dev is not None:
            line["bf16_vs_fp32"] = bf16_dev
        print(json.dumps(line), flush=True)
    if comm is not None:
        from gsamd.distributed import destroy_comm
        del agent
        destroy_comm(comm)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
