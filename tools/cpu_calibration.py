"""CPU-baseline calibration, build container only (the reference never travels): the reference's
own C2 loop against the port (oracle/cpu_ppo.py, bench.py's cpu_baseline leg) on the same cores
and thread count, so bench.py's CPU_PORT_OVER_REFERENCE divisor is re-derived on the current
toolchain (SURVEY.md §6 measured the reference loop in round 1).

Reference loop (imported from /root/reference with tests/golden/make_golden.py's stubs for the
absent third-party packages): RolloutCollector over the synthetic fixed-length env at 4096 envs x
32 steps (compute_batched_gae_advantages_and_returns inside), the sampler + collate loader
(build_index_collate_loader_from_collector, B = 256, 20 passes), then per minibatch what
BaseAgent.training_step runs (agents/base_agent.py:330-366, 591-621): activation tracking around
PPOAgent.losses_for_batch, compute_activation_stats, backward, compute_grad_norms,
clip_grad_norm_(0.5), Adam — K minibatches timed after 5 untimed (the update extrapolated to its
10 240).  Lightning's own training loop overhead is not included (pytorch_lightning is absent), so
the reference figure is an upper bound of its throughput.
Usage: python tools/cpu_calibration.py [--threads 8] [--minibatches 400]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gymnasium-solver_amd"), os.path.join(ROOT, "tests", "golden")]


def main():
    threads = int(sys.argv[sys.argv.index("--threads") + 1]) if "--threads" in sys.argv else 8
    K = int(sys.argv[sys.argv.index("--minibatches") + 1]) if "--minibatches" in sys.argv else 400
    import torch
    torch.set_num_threads(threads)
    import make_golden as MG            # the stub finder + the reference's modules
    from utils.models import MLPActorCritic
    from utils.rollout_collector import RolloutCollector
    from utils.dataloaders import build_index_collate_loader_from_collector
    from utils.random import set_random_seed, get_global_torch_generator
    from gsamd.synthetic_env import SyntheticVecEnv
    N, T, B, E = 4096, 32, 256, 20
    set_random_seed(42)
    model = MLPActorCritic(input_shape=(4,), hidden_dims=(256, 256), output_shape=(2,), activation="relu")
    env = SyntheticVecEnv(n_envs=N, obs_dim=4, n_actions=2, episode_len=200, seed=42, truncate_every=3)
    coll = RolloutCollector(MG._RefVecEnvAdapter(env), model, n_steps=T, gamma=0.98, gae_lambda=0.8,
                            returns_type="gae:rtg", advantages_type="gae", normalize_advantages=False)
    agent, recs = MG._agent(model, dict(normalize="batch", clip=0.1, clip_vf=0.2, vf_coef=0.5, ent_coef=0.0))
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    coll.collect()                       # warm
    t0 = time.perf_counter()
    traj = coll.collect()
    t_collect = time.perf_counter() - t0
    holder = {"t": traj}
    loader = build_index_collate_loader_from_collector(collector=coll, trajectories_getter=lambda: holder["t"],
                                                       batch_size=B, num_passes=E,
                                                       generator=get_global_torch_generator(42))
    loader.sampler.set_epoch(0)
    it = iter(loader)

    def step():
        batch = next(it)
        opt.zero_grad()
        model._track_activations = True
        res = agent.losses_for_batch(batch, 0)
        model.compute_activation_stats()
        model._track_activations = False
        res["loss"].backward()
        model.compute_grad_norms()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 0.5)
        opt.step()
    for _ in range(5):
        step()
    # the reference and the port alternated in blocks (this container's cores are shared: a block
    # of either can land on a busy stretch), medians of the per-block minibatch times
    from oracle.cpu_ppo import run_cpu_baseline
    nb = max(4, K // 50)
    t_ref, t_port, c_port = [], [], []
    for b in range(nb):
        t0 = time.perf_counter()
        for _ in range(K // nb):
            step()
        t_ref.append((time.perf_counter() - t0) / (K // nb))
        r = run_cpu_baseline(n_envs=N, n_steps=T, batch=B, n_epochs=E, obs_dim=4, hidden=(256, 256), n_actions=2,
                             gamma=0.98, lam=0.8, clip=0.1, lr=1e-3, max_minibatches=K // nb, threads=threads)
        t_port.append(r["minibatch_s"])
        c_port.append(r["collect_s"])
    import numpy as np
    t_mb, p_mb, p_col = float(np.median(t_ref)), float(np.median(t_port)), float(np.median(c_port))
    n_mb = N * T // B * E
    ref = N * T / (t_collect + n_mb * t_mb)
    port = N * T / (p_col + n_mb * p_mb)
    import platform
    print(f"cpu: {platform.processor() or platform.machine()}, {threads} threads, torch {torch.__version__}")
    print(f"reference loop: collect {t_collect:.3f} s, minibatch {t_mb * 1e3:.3f} ms (blocks "
          f"{[round(x * 1e3, 2) for x in t_ref]}) -> {ref:.1f} env-steps/s")
    print(f"port:           collect {p_col:.3f} s, minibatch {p_mb * 1e3:.3f} ms (blocks "
          f"{[round(x * 1e3, 2) for x in t_port]}) -> {port:.1f} env-steps/s")
    print(f"port / reference = {port / ref:.3f}")

if __name__ == "__main__":
    main()
