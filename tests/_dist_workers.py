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
        open(os.path.join(result_dir, f"ok{rank}"), "w").write("ok")
    finally:
        dist.destroy_process_group()
