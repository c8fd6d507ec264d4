"""Rank bodies for tests/test_multi_rank_cpu.py (spawned processes, gloo backend)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "gymnasium-solver_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)


def _init(rank, world, port):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    return dist


def _gather(dist, arr):
    import torch
    t = torch.as_tensor(np.ascontiguousarray(arr))
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [o.numpy() for o in out]


def dp_worker(rank, world, port, result_dir):
    """One rank of the data-parallel protocol the device path runs:
    unique-id exchange, env sharding by env_offset, per-rank minibatch gradients summed over
    ranks, scaled by 1/G, then an identical clip + Adam on every rank."""
    import torch
    dist = _init(rank, world, port)
    try:
        from gsamd.distributed import env_offset, exchange_unique_id
        from gsamd.samplers import index_stream
        from gsamd.synthetic_env import SyntheticVecEnv
        from oracle import ppo_ref as R

        # (1) the RCCL unique id made by rank 0 reaches every rank unchanged
        uid = np.frombuffer(exchange_unique_id(rank), np.uint8)
        uids = _gather(dist, uid)
        assert all(np.array_equal(u, uids[0]) for u in uids)
        assert uids[0].any()

        # (2) env shards: rank g's envs are global envs [g*N, (g+1)*N)
        N, D, A, T = 4, 4, 2, 9
        env = SyntheticVecEnv(n_envs=N, obs_dim=D, n_actions=A, episode_len=5, seed=42, truncate_every=2,
                              env_offset=env_offset(rank, N))
        obs = [env.reset()[0]]
        rew, done = [], []
        for t in range(T):
            o, r, te, tr, _ = env.step(np.zeros(N, np.int64))
            obs.append(o)
            rew.append(r)
            done.append(te | tr)
        shard = np.concatenate([np.asarray(obs).reshape(-1), np.asarray(rew, np.float32).reshape(-1),
                                np.asarray(done, np.float32).reshape(-1)]).astype(np.float32)
        shards = _gather(dist, shard)
        if rank == 0:
            whole = SyntheticVecEnv(n_envs=N * world, obs_dim=D, n_actions=A, episode_len=5, seed=42,
                                    truncate_every=2)
            wobs = [whole.reset()[0]]
            wr, wd = [], []
            for t in range(T):
                o, r, te, tr, _ = whole.step(np.zeros(N * world, np.int64))
                wobs.append(o)
                wr.append(r)
                wd.append(te | tr)
            wobs, wr, wd = np.asarray(wobs), np.asarray(wr, np.float32), np.asarray(wd, np.float32)
            for g in range(world):
                sl = slice(g * N, (g + 1) * N)
                ref = np.concatenate([wobs[:, sl].reshape(-1), wr[:, sl].reshape(-1),
                                      wd[:, sl].reshape(-1)]).astype(np.float32)
                assert np.array_equal(shards[g], ref), f"shard {g} differs from global envs"

        # (3) every rank draws its own sampler stream with the same seed (per-rank data differs)
        s = index_stream(64, 2, 42)
        ss = _gather(dist, s.astype(np.int64))
        assert all(np.array_equal(x, ss[0]) for x in ss)

        # (4) gradient exchange: sum over ranks, x 1/G, clip, Adam -> identical replicas that
        #     equal the mean-of-shard-gradients update computed in one process
        dims = (D, 32, 32, A)
        rng0 = np.random.default_rng(7)
        P = sum(int(np.prod(s)) for _, s in R.param_shapes(dims))
        p = (rng0.standard_normal(P) * 0.1).astype(np.float32)
        m = np.zeros(P, np.float32)
        v = np.zeros(P, np.float32)

        def batch(g, k):
            rng = np.random.default_rng(1000 * k + g)
            B = 16
            o = rng.uniform(-1, 1, (B, D)).astype(np.float32)
            a = rng.integers(0, A, B)
            olp = np.log(np.full(B, 0.5, np.float32)) + 0.01 * rng.standard_normal(B).astype(np.float32)
            ov = rng.standard_normal(B).astype(np.float32)
            adv = rng.standard_normal(B).astype(np.float32)
            return o, a, olp.astype(np.float32), ov, adv, (ov + adv).astype(np.float32)

        def grads(params, g, k):
            o, a, olp, ov, adv, ret = batch(g, k)
            return R.ppo_loss_and_grads(params, dims, o, a, olp, ov, adv, ret, clip=0.1, clip_vf=0.2,
                                        vf_coef=0.5, ent_coef=0.0)[2].astype(np.float32)

        p_loc, m_loc, v_loc = p.copy(), m.copy(), v.copy()
        for k in range(3):
            g = torch.as_tensor(grads(p, rank, k))
            dist.all_reduce(g)                                  # RCCL sum on the device path
            g = g.numpy() * np.float32(1.0 / world)
            gc, _ = R.clip_grad_norm(g, dims, 0.5)
            p, m, v = R.adam_step(p, gc.astype(np.float32), m, v, k + 1, 1e-3)
            # single-process restatement of the same update
            gl = np.zeros(P, np.float32)
            for r in range(world):
                gl = gl + grads(p_loc, r, k)
            gl = gl * np.float32(1.0 / world)
            glc, _ = R.clip_grad_norm(gl, dims, 0.5)
            p_loc, m_loc, v_loc = R.adam_step(p_loc, glc.astype(np.float32), m_loc, v_loc, k + 1, 1e-3)
        ps = _gather(dist, p)
        assert all(np.array_equal(x.view(np.uint32), ps[0].view(np.uint32)) for x in ps), "replicas diverged"
        assert np.array_equal(p.view(np.uint32), p_loc.view(np.uint32)), "DP update != mean-gradient update"
        # (5) per-epoch metric partial sums are summed over ranks (job-wide statistics)
        from gsamd.distributed import allreduce_sum_f64, world_active
        assert world_active()
        part = np.array([rank + 1.0, 10.0 * (rank + 1), 0.5], np.float64)
        tot = allreduce_sum_f64(part)
        assert np.array_equal(tot, np.array([sum(r + 1.0 for r in range(world)),
                                             sum(10.0 * (r + 1) for r in range(world)), 0.5 * world]))
        open(os.path.join(result_dir, f"ok{rank}"), "w").write("ok")
    finally:
        dist.destroy_process_group()


# --------------------------------------------------------------------------------------
# GPU ranks (tests/test_gpu_xgmi.py): every rank on cuda:0 of the one-GPU box, exchanging
# through IPC-mapped regions exactly as the ranks of a node do over xGMI.
# --------------------------------------------------------------------------------------
def exchange_values(rank, it, n):
    """Deterministic per-(rank, iteration) payload with mixed magnitudes and signs."""
    rng = np.random.default_rng(1 + 7919 * it + 104729 * rank)
    return (rng.standard_normal(n) * np.exp(rng.uniform(-6, 6, n))).astype(np.float32)


def xgmi_exchange_worker(rank, world, port, result_dir, n, iters, algo="", f64=False):
    """Back-to-back exchanges with no host sync in between (both parity slots reused many
    times), then the device result of every iteration is saved for the parent.  algo forces
    the exchange form (oneshot | rsag; default by rank count).  f64: gs_comm_allreduce_sum_f64
    on doubles (a communicator sized for n floats: n doubles take two pieces), interleaved with
    f32 mean exchanges on the same communicator."""
    os.environ.setdefault("GS_XGMI_TIMEOUT_S", "60")
    if algo:
        os.environ["GS_XGMI_ALGO"] = algo
    dist = _init(rank, world, port)
    try:
        import torch
        from gsamd._lib import check, lib
        from gsamd.distributed import comm_status, destroy_comm, init_xgmi_comm
        torch.cuda.set_device(0)
        h = init_xgmi_comm(rank, world, n)
        dt = np.float64 if f64 else np.float32
        bufs = [torch.from_numpy(exchange_values(rank, it, n).astype(dt) * (1.0 + 1e-9 * it) if f64 else
                                 exchange_values(rank, it, n)).cuda() for it in range(iters)]
        torch.cuda.synchronize()
        dist.barrier()
        s = torch.cuda.current_stream()
        for b in bufs:
            if f64:
                check(lib.gs_comm_allreduce_sum_f64(h, b.data_ptr(), n, s.cuda_stream), "allreduce f64")
                t = torch.ones(1000, device=b.device)      # an f32 mean exchange in between
                check(lib.gs_comm_allreduce_mean_f32(h, t.data_ptr(), 1000, s.cuda_stream), "allreduce")
            else:
                check(lib.gs_comm_allreduce_mean_f32(h, b.data_ptr(), n, s.cuda_stream), "allreduce")
        torch.cuda.synchronize()
        comm_status(h)
        np.save(os.path.join(result_dir, f"x{rank}.npy"), torch.stack(bufs).cpu().numpy())
        dist.barrier()
        destroy_comm(h)
        open(os.path.join(result_dir, f"ok{rank}"), "w").write("ok")
    finally:
        dist.destroy_process_group()


def xgmi_ppo_worker(rank, world, port, result_dir, use_graph, lagged="1", workload="mlp", algo="",
                    identical=False, bwd="1"):
    """Data-parallel PPO update over the xGMI transport: rank-sharded envs, one rollout and
    2 epochs; every rank saves its final parameters and per-minibatch losses.  lagged="0"
    selects the chain with a separate clip + Adam launch after each exchange.  workload="cnn":
    the C5 Breakout rgb_ppo shard (128 envs per rank, NatureCNN, B=1024, 4 epochs) over a
    32-step rollout, so the 1.69 M-float gradient exchange runs 16 times.  identical=True:
    every rank trains on rank 0's shard (same envs, sampler and seeds), so the exchanged mean
    of 2 ranks equals each rank's own gradient exactly.  bwd="0": the exchange runs as its
    own launch after the backward instead of inside it (GS_XGMI_BWD)."""
    os.environ.setdefault("GS_XGMI_TIMEOUT_S", "60")
    os.environ["GS_LAGGED_ADAM"] = lagged
    os.environ["GS_XGMI_BWD"] = bwd
    if algo:
        os.environ["GS_XGMI_ALGO"] = algo
    dist = _init(rank, world, port)
    try:
        import torch
        from gsamd.config import load_config
        from gsamd.distributed import comm_status, destroy_comm, init_xgmi_comm
        from gsamd.ppo_agent import DevicePPOAgent
        torch.cuda.set_device(0)
        dev = torch.device("cuda:0")
        torch.manual_seed(42)
        if workload == "cnn":
            cfg = load_config("ALE-Breakout-v5", "rgb_ppo", overrides=dict(env_dynamics="synthetic", n_envs=128, n_steps=32))
        elif workload == "lunar":     # C3's MLP shapes: a small backward grid (57 workgroups)
            cfg = load_config("LunarLander-v3", "ppo", overrides=dict(env_dynamics="synthetic", n_envs=64, n_steps=128, n_epochs=2))
        else:
            cfg = load_config("CartPole-v1", "ppo", overrides=dict(env_dynamics="synthetic", n_envs=256, n_epochs=2))
        agent = DevicePPOAgent(cfg, device=dev, rank=0 if identical else rank, world_size=1 if identical else world,
                               use_graph=use_graph, track_stats=False)
        agent.comm = init_xgmi_comm(rank, world, agent.policy_model.n_params)
        if workload != "cnn":      # which exchange the fused chain runs, for the parent's checks
            from gsamd.distributed import exchange_inside_bwd
            inside = exchange_inside_bwd(agent.comm, agent.policy_model.dims, agent.batch_size)
            open(os.path.join(result_dir, f"inside{rank}"), "w").write(str(int(inside)))
        agent.train_epoch()
        torch.cuda.synchronize()
        comm_status(agent.comm)
        np.save(os.path.join(result_dir, f"p{rank}.npy"), agent.policy_model.params.cpu().numpy())
        np.save(os.path.join(result_dir, f"l{rank}.npy"), np.asarray(agent.minibatch_losses(), np.float32))
        dist.barrier()
        comm = agent.comm
        del agent
        destroy_comm(comm)
        open(os.path.join(result_dir, f"ok{rank}"), "w").write("ok")
    finally:
        dist.destroy_process_group()


def xgmi_oracle_worker(rank, world, port, result_dir, transport="xgmi", algo="", bwd="1", n_steps=8):
    """One rank of the data-parallel C2-shaped update on its OWN env shard (env_offset = rank x
    256), for the parent's comparison with the numpy oracle's mean-gradient update: the fused
    lagged chain's first n_steps minibatches (gs_ppo_update over n_steps, the exchange inside
    k_bwd (bwd="1", forced also for ranks sharing the GPU) or as a launch after it (bwd="0"), or
    RCCL).  Saves the initial parameters, the rollout's env-major fields, the index stream, the
    per-minibatch losses and the final parameters."""
    os.environ.setdefault("GS_XGMI_TIMEOUT_S", "60")
    os.environ["GS_XGMI_BWD"] = bwd
    if algo:
        os.environ["GS_XGMI_ALGO"] = algo
    dist = _init(rank, world, port)
    try:
        import torch
        from gsamd._lib import check, lib
        from gsamd.config import load_config
        from gsamd.distributed import comm_status, destroy_comm, exchange_inside_bwd, init_device_comm, init_xgmi_comm
        from gsamd.ppo_agent import DevicePPOAgent
        torch.cuda.set_device(0)
        dev = torch.device("cuda:0")
        torch.manual_seed(42)
        cfg = load_config("CartPole-v1", "ppo", overrides=dict(env_dynamics="synthetic", n_envs=256, n_epochs=1))
        agent = DevicePPOAgent(cfg, device=dev, rank=rank, world_size=world, use_graph=False, track_stats=False)
        pm = agent.policy_model
        if transport == "xgmi":
            comm = init_xgmi_comm(rank, world, pm.n_params)
        else:
            try:
                comm = init_device_comm(rank, world, dev)
            except RuntimeError as e:        # RCCL refuses ranks that share one GPU
                open(os.path.join(result_dir, f"rccl_init_error{rank}"), "w").write(str(e))
                open(os.path.join(result_dir, f"ok{rank}"), "w").write("ok")
                return
        inside = exchange_inside_bwd(comm, pm.dims, agent.batch_size)
        agent.train_dataloader()
        traj = agent._trajectories
        idx = agent.prefetcher.upload(0)
        p0 = pm.params.cpu().numpy()
        torch.cuda.synchronize()
        dist.barrier()
        check(lib.gs_ppo_update(pm.params.data_ptr(), agent.grads.data_ptr(), agent.adam_m.data_ptr(),
                                agent.adam_v.data_ptr(), pm.dims, agent.hparams(), agent.get_rollout_collector("train")
                                .buffer.view(), idx.data_ptr(), agent.batch_size, n_steps, 0,
                                agent.metrics_buf.data_ptr(), agent.stop_flag.data_ptr(), agent.workspace.data_ptr(),
                                agent.workspace.numel(), comm, 0, torch.cuda.current_stream().cuda_stream),
              "gs_ppo_update")
        torch.cuda.synchronize()
        comm_status(comm)
        np.savez(os.path.join(result_dir, f"r{rank}.npz"), p0=p0, p1=pm.params.cpu().numpy(),
                 losses=agent.metrics_buf[:n_steps, 0].cpu().numpy(),
                 idx=idx[:n_steps * agent.batch_size].cpu().numpy(), obs=traj.observations.cpu().numpy(),
                 actions=traj.actions.cpu().numpy(), logp=traj.logprobs.cpu().numpy(),
                 values=traj.values.cpu().numpy(), adv=traj.advantages.cpu().numpy(),
                 ret=traj.returns.cpu().numpy(), inside=np.int32(inside))
        dist.barrier()
        del agent
        destroy_comm(comm)
        open(os.path.join(result_dir, f"ok{rank}"), "w").write("ok")
    finally:
        dist.destroy_process_group()


def xgmi_timeout_worker(rank, world, port, result_dir):
    """The designed failure: both ranks connect (self-test included), then rank 1 never runs its
    update.  Rank 0's train_epoch must raise GsError (the exchange's bounded wait, 2 s) naming
    the workgroup and the peer it waited for, and exit non-zero (3) — never return a trained
    model.  Rank 1 waits for rank 0's verdict file and exits 0."""
    import time
    os.environ["GS_XGMI_TIMEOUT_S"] = "2"
    dist = _init(rank, world, port)
    done = os.path.join(result_dir, "rank0_done")
    code = 0
    try:
        import torch
        from gsamd._lib import GsError
        from gsamd.config import load_config
        from gsamd.distributed import comm_error_record, init_xgmi_comm
        from gsamd.ppo_agent import DevicePPOAgent
        torch.cuda.set_device(0)
        dev = torch.device("cuda:0")
        torch.manual_seed(42)
        cfg = load_config("CartPole-v1", "ppo", overrides=dict(env_dynamics="synthetic", n_envs=64, n_epochs=1))
        agent = DevicePPOAgent(cfg, device=dev, rank=rank, world_size=world, use_graph=False, track_stats=False)
        agent.comm = init_xgmi_comm(rank, world, agent.policy_model.n_params)
        if rank == 1:
            t0 = time.time()
            while not os.path.exists(done) and time.time() - t0 < 90:
                time.sleep(0.1)
            return
        try:
            agent.train_epoch()
            open(os.path.join(result_dir, "outcome"), "w").write("returned")
        except GsError as e:
            import json
            rec = comm_error_record(agent.comm)
            json.dump({"message": str(e), **rec}, open(os.path.join(result_dir, "outcome"), "w"))
            code = 3
        open(done, "w").write("done")
    finally:
        if rank == 0 and not os.path.exists(done):
            open(done, "w").write("done")
    os._exit(code)


def global_trajectory_worker(rank, world, port, result_dir, fixture, transport="xgmi", bwd="1"):
    """dp_mode 'global' on the reference's trajectory fixture: the fixture's N envs split over
    `world` ranks (rank g steps global envs [g N/world, (g+1) N/world) of the same synthetic env),
    each replaying the reference's recorded actions of its envs; three rollouts + updates.  Saves
    every minibatch record and the final parameters."""
    os.environ.setdefault("GS_XGMI_TIMEOUT_S", "60")
    os.environ["GS_XGMI_BWD"] = bwd
    dist = _init(rank, world, port)
    try:
        import torch
        from gsamd.config import load_config
        from gsamd.distributed import comm_status, destroy_comm, init_device_comm, init_xgmi_comm
        from gsamd.ppo_agent import DevicePPOAgent
        torch.cuda.set_device(0)
        dev = torch.device("cuda:0")
        z = np.load(fixture)
        N, T, E, B, D, A = (int(x) for x in z["dims"])
        L, seed, trunc = (int(x) for x in z["env"])
        n = N // world
        torch.manual_seed(42)
        over = dict(env_dynamics="synthetic", episode_len=L, truncate_every=trunc, obs_dim=D, n_actions=A, n_envs=n,
                    dp_mode="global")
        if "target_kl" in z.files and float(z["target_kl"]) > 0:
            over["target_kl"] = float(z["target_kl"])
        cfg = load_config("CartPole-v1", "ppo", overrides=over)
        agent = DevicePPOAgent(cfg, device=dev, rank=rank, world_size=world, use_graph=False, track_stats=False)
        agent.policy_model.load_flat(z["params0"])
        if world > 1:
            agent.comm = (init_xgmi_comm(rank, world, agent.policy_model.n_params) if transport == "xgmi"
                          else init_device_comm(rank, world, dev))
        coll = agent.get_rollout_collector("train")
        recs = []
        for ep in range(3):
            acts = torch.as_tensor(z["actions"][ep].reshape(N, T).T[:, rank * n:(rank + 1) * n].copy()).to(dev)
            coll.collect(replay_actions=acts)
            agent.update_phase()
            recs.append(agent.metrics_buf.cpu().numpy().copy())
        torch.cuda.synchronize()
        np.savez(os.path.join(result_dir, f"g{rank}.npz"), rec=np.concatenate(recs),
                 p=agent.policy_model.params.cpu().numpy(), adam_step=np.int64(agent.adam_step))
        comm = agent.comm
        if comm:
            comm_status(comm)
            dist.barrier()
        del agent
        if comm:
            destroy_comm(comm)
        open(os.path.join(result_dir, f"ok{rank}"), "w").write("ok")
    finally:
        dist.destroy_process_group()


def kl_one_rank_worker(rank, world, port, result_dir):
    """Local data-parallel mode with target_kl set, where only rank 1's approx_kl trips the stop
    (its rollout's old log-probs are shifted by +1, so ratio = e^-1 at minibatch 0): the exchange
    ORs the stop bits, so rank 0 must skip the same optimizer steps, record them as skipped, and
    count the same Adam steps (replicas would otherwise drift through bias correction)."""
    os.environ.setdefault("GS_XGMI_TIMEOUT_S", "60")
    dist = _init(rank, world, port)
    try:
        import torch
        from gsamd._lib import M
        from gsamd.config import load_config
        from gsamd.distributed import comm_status, destroy_comm, init_xgmi_comm
        from gsamd.ppo_agent import DevicePPOAgent
        torch.cuda.set_device(0)
        dev = torch.device("cuda:0")
        torch.manual_seed(42)
        cfg = load_config("CartPole-v1", "ppo", overrides=dict(env_dynamics="synthetic", n_envs=64, n_epochs=2,
                                                               target_kl=0.05))
        agent = DevicePPOAgent(cfg, device=dev, rank=rank, world_size=world, use_graph=False, track_stats=False)
        agent.comm = init_xgmi_comm(rank, world, agent.policy_model.n_params)
        agent.train_dataloader()
        if rank == 1:
            agent.get_rollout_collector("train").buffer.logprobs.add_(1.0)
        step0 = agent.adam_step
        agent.update_phase()
        torch.cuda.synchronize()
        comm_status(agent.comm)
        rec = agent.metrics_buf.cpu().numpy()
        np.savez(os.path.join(result_dir, f"r{rank}.npz"), p=agent.policy_model.params.cpu().numpy(),
                 steps=np.int64(agent.adam_step - step0), skipped=rec[:, M["skipped"]], kl_stop=rec[:, M["kl_stop"]])
        dist.barrier()
        comm = agent.comm
        del agent
        destroy_comm(comm)
        open(os.path.join(result_dir, f"ok{rank}"), "w").write("ok")
    finally:
        dist.destroy_process_group()


def guard_worker(rank, world, port, result_dir, bwd="1"):
    """The multi-GPU guards (DESIGN §5 Failure surfacing): init_xgmi_comm with the job's MLP
    shapes runs the in-backward exchange self-test (GS_XGMI_BWD=1 forces that form for ranks
    sharing the one GPU; "" leaves it off there), then one update passes the per-epoch replica
    check, then rank 1 perturbs one parameter and the next train_epoch must raise GsError on
    EVERY rank.  Saves the self-test record and each rank's outcome."""
    import json
    os.environ.setdefault("GS_XGMI_TIMEOUT_S", "60")
    if bwd:
        os.environ["GS_XGMI_BWD"] = bwd
    else:
        os.environ.pop("GS_XGMI_BWD", None)
    dist = _init(rank, world, port)
    out = {}
    try:
        import torch
        from gsamd._lib import GsError
        from gsamd.config import load_config
        from gsamd import distributed as gd
        from gsamd.ppo_agent import DevicePPOAgent
        torch.cuda.set_device(0)
        dev = torch.device("cuda:0")
        torch.manual_seed(42)
        cfg = load_config("CartPole-v1", "ppo", overrides=dict(env_dynamics="synthetic", n_envs=64, n_epochs=1))
        agent = DevicePPOAgent(cfg, device=dev, rank=rank, world_size=world, use_graph=False, track_stats=False)
        pm = agent.policy_model
        agent.comm = gd.init_xgmi_comm(rank, world, pm.n_params, dev, verify_shapes=(pm.dims, agent.batch_size))
        out["self_test"] = dict(gd.LAST_SELF_TEST)
        out["inside"] = bool(gd.exchange_inside_bwd(agent.comm, pm.dims, agent.batch_size))
        agent.train_epoch()
        out["first_epoch"] = "ok"
        if rank == 1:
            with torch.no_grad():
                pm.params[123] += 1e-3
        try:
            agent.train_epoch()
            out["second_epoch"] = "returned"
        except GsError as e:
            out["second_epoch"] = "GsError"
            out["message"] = str(e)
        json.dump(out, open(os.path.join(result_dir, f"guard{rank}.json"), "w"))
        dist.barrier()
        comm = agent.comm
        del agent
        gd.destroy_comm(comm)
        open(os.path.join(result_dir, f"ok{rank}"), "w").write("ok")
    finally:
        dist.destroy_process_group()


def replica_check_cpu_worker(rank, world, port, result_dir):
    """CPU (gloo) half of the multi-GPU guards: check_replicas passes on identical parameters and
    raises GsError on EVERY rank once one rank's parameters differ in one element (also a swap of
    two elements, which keeps the plain sum); broadcast_int hands rank 0's sampler seed to all."""
    dist = _init(rank, world, port)
    try:
        import torch
        from gsamd._lib import GsError
        from gsamd.distributed import broadcast_int, check_replicas
        assert broadcast_int(42 + rank) == 42
        p = torch.linspace(-1.0, 1.0, 1001, dtype=torch.float32)
        check_replicas(p)
        outcomes = []
        for change in ("one", "swap"):
            q = p.clone()
            if rank == 1 and change == "one":
                q[500] += 1e-6
            if rank == 1 and change == "swap":
                q[[3, 7]] = q[[7, 3]]
            try:
                check_replicas(q)
                outcomes.append("passed")
            except GsError as e:
                outcomes.append("GsError" if "replica check failed" in str(e) else "other")
        open(os.path.join(result_dir, f"rc{rank}"), "w").write(",".join(outcomes))
        open(os.path.join(result_dir, f"ok{rank}"), "w").write("ok")
    finally:
        dist.destroy_process_group()


def cnn_global_tf_worker(rank, world, port, result_dir, ref_path, states_path):
    """Teacher-forced dp_mode 'global' for NatureCNN: the single-process run's envs split over
    `world` same-device ranks, replaying that run's actions; then, for every global minibatch k,
    every rank restarts from the single run's (params, adam_m, adam_v) before step k and runs that
    ONE minibatch through gs_cnn_ppo_update_global (its share of the rows, global advantage
    statistics, the ranks' gradient shares summed over xGMI), so each step's arithmetic is compared
    without Adam carrying earlier differences forward.  Rank 0 saves every step's clipped gradient
    and new parameters; every rank saves a digest of them (replicas must agree bit for bit); the
    records come from gs_ppo_global_records over all steps."""
    import ctypes
    import hashlib
    os.environ.setdefault("GS_XGMI_TIMEOUT_S", "60")
    dist = _init(rank, world, port)
    try:
        import torch
        from gsamd._lib import PPOGlobal, check, lib, ptr, stream_handle
        from gsamd.config import load_config
        from gsamd.distributed import comm_status, destroy_comm, init_xgmi_comm
        from gsamd.ppo_agent import DevicePPOAgent
        torch.cuda.set_device(0)
        dev = torch.device("cuda:0")
        z = np.load(ref_path)
        with np.load(states_path) as f:
            st = {k: f[k] for k in ("p", "m", "v")}
        N, T = (int(x) for x in z["NT"])
        n = N // world
        torch.manual_seed(42 + rank)
        cfg = load_config("ALE-Breakout-v5", "rgb_ppo", overrides=dict(
            env_dynamics="synthetic", n_envs=n, n_steps=T, batch_size=int(z["B"]), n_epochs=int(z["E"]),
            dp_mode="global"))
        agent = DevicePPOAgent(cfg, device=dev, rank=rank, world_size=world, use_graph=False, track_stats=False)
        agent.comm = init_xgmi_comm(rank, world, agent.policy_model.n_params)
        # the rollout's log-probs / values come from the single run's initial policy
        agent.policy_model.params.copy_(torch.from_numpy(np.ascontiguousarray(st["p"][0])).to(dev))
        coll = agent.get_rollout_collector("train")
        acts = torch.as_tensor(z["actions"][0][:, rank * n:(rank + 1) * n].copy()).to(dev)
        coll.collect(replay_actions=acts)
        pm, B, K = agent.policy_model, agent.batch_size, agent.n_minibatches
        buf = coll.buffer
        agent._gidx.copy_(torch.from_numpy(agent.global_shares(0)))
        torch.clamp(agent._gidx, min=0, out=agent._fidx)
        s = stream_handle()
        comm = agent.comm
        check(lib.gs_ppo_global_adv_stats(ptr(agent._gidx), K, B, B, ptr(buf.advantages), T, n, comm,
                                          ptr(agent._adv_sums), ptr(agent._adv_stats), s), "gs_ppo_global_adv_stats")
        hp = agent.hparams()
        grads, params, digests = [], [], []
        # every step's conv / fc ReLU decisions of this rank's padded row share (a1 / a2 / a3 / h > 0
        # in its workspace, NCHW), bit-packed per row: the parent assembles the global minibatch's
        # decisions from the ranks' shares for the oracle (the global run's arithmetic bars)
        act_shapes = [(20, 20, 32), (9, 9, 64), (7, 7, 64), (512,)]
        act_offs = [int(lib.gs_cnn_workspace_act_offset(pm.dims, B, layer)) for layer in (1, 2, 3, 4)]
        masks = [[] for _ in act_shapes]
        for k in range(K):
            for t, name in ((pm.params, "p"), (agent.adam_m, "m"), (agent.adam_v, "v")):
                t.copy_(torch.from_numpy(np.ascontiguousarray(st[name][k])).to(dev))
            glob = PPOGlobal(B, ptr(agent._adv_stats[k]), ptr(agent._gsums[k]))
            check(lib.gs_cnn_ppo_update_global(ptr(pm.params), ptr(agent.grads), ptr(agent.adam_m), ptr(agent.adam_v),
                                               pm.dims, hp, buf.view(), ptr(agent._gidx[k * B:]),
                                               ptr(agent._fidx[k * B:]), B, 1, k, ptr(agent.metrics_buf[k]),
                                               ptr(agent.stop_flag), ptr(agent.workspace), comm, ctypes.byref(glob), s),
                  "gs_cnn_ppo_update_global")
            g_k, p_k = agent.grads.cpu().numpy(), pm.params.cpu().numpy()
            digests.append(hashlib.sha256(g_k.tobytes() + p_k.tobytes()).hexdigest())
            for li, (off, sh) in enumerate(zip(act_offs, act_shapes)):
                nel = B * int(np.prod(sh))
                a = agent.workspace[off:off + 4 * nel].view(torch.float32).view(B, *sh) > 0
                a = a.permute(0, 3, 1, 2) if len(sh) == 3 else a
                masks[li].append(np.packbits(a.reshape(B, -1).cpu().numpy(), axis=1))
            if rank == 0:
                grads.append(g_k)
                params.append(p_k)
        check(lib.gs_ppo_global_records(ctypes.byref(hp), K, B, comm, ptr(agent._gsums), ptr(agent.metrics_buf), s),
              "gs_ppo_global_records")
        torch.cuda.synchronize()
        comm_status(comm)
        out = dict(rec=agent.metrics_buf.cpu().numpy(), digests=np.array(digests),
                   shares=agent._gidx.cpu().numpy(), **{f"mask{li}": np.stack(m) for li, m in enumerate(masks)})
        if rank == 0:
            out.update(g=np.stack(grads), p=np.stack(params))
        np.savez(os.path.join(result_dir, f"tf{rank}.npz"), **out)
        dist.barrier()
        del agent
        destroy_comm(comm)
    finally:
        dist.destroy_process_group()


def agent_selftest_worker(rank, world, port, result_dir, mode):
    """The agent's own exchange guards on ranks sharing the box's GPU (GS_XGMI_BWD=1 forces the
    in-backward form):
      mode "mlp":    init_xgmi_comm WITHOUT verify_shapes (the documented recipe may omit it): the
                     agent's first update runs bwd_exchange_self_test itself on its dims / batch /
                     flags; then two epochs pass the replica check and the per-epoch canary;
      mode "inject": as "mlp", but rank 1's first self-test chain raises before it exchanges
                     (a stand-in for a failed launch): rank 0's in-backward wait times out, every
                     rank still runs the same collectives (sentinel digest), resets the
                     communicator and switches to the exchange launch together, and training
                     continues on the launch form;
      mode "cnn":    a NatureCNN-sized communicator (1 693 875 floats): the vector self-test covers
                     the whole capacity, and a Breakout epoch passes the canary.
    Saves each rank's record."""
    import json
    os.environ["GS_XGMI_TIMEOUT_S"] = "5" if mode == "inject" else "60"
    os.environ["GS_XGMI_BWD"] = "1"
    dist = _init(rank, world, port)
    out = {}
    try:
        import torch
        from gsamd.config import load_config
        from gsamd import distributed as gd
        from gsamd.ppo_agent import DevicePPOAgent
        torch.cuda.set_device(0)
        dev = torch.device("cuda:0")
        torch.manual_seed(42)
        if mode == "cnn":
            cfg = load_config("ALE-Breakout-v5", "rgb_ppo", overrides=dict(env_dynamics="synthetic", n_envs=8,
                                                                           n_steps=32, batch_size=64, n_epochs=1))
        else:
            cfg = load_config("CartPole-v1", "ppo", overrides=dict(env_dynamics="synthetic", n_envs=64, n_epochs=1))
        agent = DevicePPOAgent(cfg, device=dev, rank=rank, world_size=world, use_graph=False, track_stats=False)
        pm = agent.policy_model
        if mode == "inject" and rank == 1:
            real = gd._chain_run
            calls = {"n": 0}

            def failing(*a, **k):
                calls["n"] += 1
                if calls["n"] == 1:
                    raise RuntimeError("injected failure before the exchange")
                return real(*a, **k)
            gd._chain_run = failing
        agent.comm = gd.init_xgmi_comm(rank, world, pm.n_params, dev)
        out["connect_self_test"] = dict(gd.LAST_SELF_TEST)
        out["n_params"] = int(pm.n_params)
        for ep in range(2):
            agent.train_epoch()
        torch.cuda.synchronize()
        out["epochs"] = "ok"
        out["agent_self_test"] = agent.exchange_self_test
        out["canary_rounds"] = int(getattr(agent, "_canary_round", 0))
        if not agent.is_pixel:
            out["inside"] = bool(gd.exchange_inside_bwd(agent.comm, pm.dims, agent.batch_size))
        out["params_sha"] = __import__("hashlib").sha256(pm.params.cpu().numpy().tobytes()).hexdigest()
        json.dump(out, open(os.path.join(result_dir, f"ast{rank}.json"), "w"))
        dist.barrier()
        comm = agent.comm
        del agent
        gd.destroy_comm(comm)
    finally:
        dist.destroy_process_group()


def no_comm_worker(rank, world, port, result_dir):
    """One rank of a data-parallel job whose agent has no communicator attached (CPU, gloo).
    Local mode as well as global mode: DevicePPOAgent.update_phase (train_epoch's update half) and
    training_step must raise ValueError on every rank before any device work, instead of each
    rank stepping its own replica on its own shard's gradient."""
    dist = _init(rank, world, port)
    try:
        from gsamd.ppo_agent import DevicePPOAgent
        out = []
        for mode in ("local", "global"):
            agent = object.__new__(DevicePPOAgent)       # no device: the check runs first
            agent.rank, agent.world_size, agent.comm = rank, world, None
            agent.global_mode = mode == "global"
            agent._early_stop_epoch = False
            for call in (lambda: agent.update_phase(), lambda: agent.training_step(None, 0)):
                try:
                    call()
                    out.append("returned")
                except ValueError as e:
                    assert f"world_size={world}" in str(e) and f"dp_mode '{mode}'" in str(e), str(e)
                    out.append("ValueError")
        dist.barrier()
        open(os.path.join(result_dir, f"nc{rank}"), "w").write(",".join(out))
    finally:
        dist.destroy_process_group()
