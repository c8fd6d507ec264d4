"""GPU: the xGMI gradient exchange (csrc/gs_xgmi.hip: one-shot and reduce-scatter + all-gather
forms, as an exchange launch and inside the MLP backward, csrc/gs_xgmi_dev.h) with 2 to 4 ranks.  The box
has one MI355X, so every rank runs on cuda:0 and the peers' regions are opened through the
same IPC path the ranks of an 8-GPU node use; the cross-device link itself is
exercised only by the driver's multi-GPU bench.

Bar: bit-exact.  The exchange sums the ranks' vectors in rank order and scales by 1/world
in fp32, so numpy's ((x0 + x1) + x2) + ... then * float32(1/world) is the exact answer, and
replicas of a data-parallel PPO update end with bitwise-identical parameters."""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _run(target, world, tmp_path, *args, timeout=300):
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, str(tmp_path)) + args) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=timeout)
    for p in procs:
        if p.is_alive():
            p.kill()
            p.join()
    codes = [p.exitcode for p in procs]
    assert codes == [0] * world, codes


# 67 651: an MLP-sized vector with an odd tail; 1 693 875: the NatureCNN's parameter count —
# more chunks than the exchange has workgroups, so each workgroup loops over several chunks.
# algo: the one-shot form (default below 4 ranks) and the reduce-scatter + all-gather form
# (default from 4 ranks), each at 2 and 4 ranks
@pytest.mark.parametrize("world,n,iters,algo", [(2, 67_651, 24, ""), (4, 67_651, 24, ""), (2, 1_693_875, 6, ""),
                                                 (2, 67_651, 24, "rsag"), (4, 67_651, 24, "oneshot"),
                                                 (3, 1_693_875, 6, "rsag")])
def test_xgmi_exchange_bit_exact(tmp_path, world, n, iters, algo):
    from _dist_workers import exchange_values, xgmi_exchange_worker
    _run(xgmi_exchange_worker, world, tmp_path, n, iters, algo)
    outs = [np.load(tmp_path / f"x{r}.npy") for r in range(world)]
    for it in range(iters):
        acc = exchange_values(0, it, n)
        for r in range(1, world):
            acc = acc + exchange_values(r, it, n)
        want = acc * np.float32(1.0 / world)
        for r in range(world):
            assert np.array_equal(outs[r][it].view(np.uint32), want.view(np.uint32)), (world, it, r)


@pytest.mark.parametrize("world,algo", [(2, ""), (3, "rsag")])
def test_xgmi_sum_f64_bit_exact(tmp_path, world, algo):
    """gs_comm_allreduce_sum_f64 (the global mode's statistics exchange): doubles summed in rank
    order in double on both transport forms, in pieces of the communicator's capacity (n doubles
    on a communicator sized for n floats), interleaved with f32 exchanges: every element equals
    numpy's ((x0 + x1) + x2) in float64."""
    from _dist_workers import exchange_values, xgmi_exchange_worker
    n, iters = 5_000, 6
    _run(xgmi_exchange_worker, world, tmp_path, n, iters, algo, True)
    outs = [np.load(tmp_path / f"x{r}.npy") for r in range(world)]
    for it in range(iters):
        vals = [exchange_values(r, it, n).astype(np.float64) * (1.0 + 1e-9 * it) for r in range(world)]
        acc = vals[0]
        for r in range(1, world):
            acc = acc + vals[r]
        for r in range(world):
            assert outs[r].dtype == np.float64
            assert np.array_equal(outs[r][it].view(np.uint64), acc.view(np.uint64)), (world, it, r)


@pytest.mark.parametrize("use_graph", [False, True])
def test_xgmi_data_parallel_ppo_replicas_identical(tmp_path, use_graph):
    from _dist_workers import xgmi_ppo_worker
    world = 2
    _run(xgmi_ppo_worker, world, tmp_path, use_graph, timeout=400)
    p = [np.load(tmp_path / f"p{r}.npy") for r in range(world)]
    losses = [np.load(tmp_path / f"l{r}.npy") for r in range(world)]
    assert np.isfinite(p[0]).all() and all(np.isfinite(l).all() for l in losses)
    assert np.array_equal(p[0].view(np.uint32), p[1].view(np.uint32)), "replicas diverged"
    assert not np.array_equal(losses[0], losses[1])      # the ranks trained on different env shards


def test_xgmi_cnn_data_parallel_replicas_identical(tmp_path):
    """C5's sharded path: 2 ranks, each with its own 128 Breakout envs, NatureCNN update with the
    1.69 M-float gradient exchanged every minibatch; replicas end bitwise identical."""
    from _dist_workers import xgmi_ppo_worker
    world = 2
    _run(xgmi_ppo_worker, world, tmp_path, False, "1", "cnn", timeout=400)
    p = [np.load(tmp_path / f"p{r}.npy") for r in range(world)]
    losses = [np.load(tmp_path / f"l{r}.npy") for r in range(world)]
    assert p[0].size == 1_693_875 and np.isfinite(p[0]).all()
    assert np.array_equal(p[0].view(np.uint32), p[1].view(np.uint32)), "replicas diverged"
    assert not np.array_equal(losses[0], losses[1])


@pytest.mark.parametrize("world", [2, 4])
def test_xgmi_rsag_ppo_replicas_identical(tmp_path, world):
    """The reduce-scatter + all-gather exchange carrying the lagged data-parallel PPO update:
    replicas end bitwise identical (2 ranks forced, 4 ranks by default).  2 ranks exchange inside
    k_bwd; 4 ranks sharing the one GPU use the exchange launch (4 backward grids of 273
    workgroups do not fit on the GPU together, and the in-backward form would then wait on the
    scheduler's time slices — its rsag form is covered at 2 ranks here and in the oracle test)."""
    from _dist_workers import xgmi_ppo_worker
    _run(xgmi_ppo_worker, world, tmp_path, True, "1", "mlp", "rsag", False, "1" if world == 2 else "0", timeout=400)
    p = [np.load(tmp_path / f"p{r}.npy") for r in range(world)]
    assert np.isfinite(p[0]).all()
    for r in range(1, world):
        assert np.array_equal(p[0].view(np.uint32), p[r].view(np.uint32)), f"rank {r} diverged"


def test_xgmi_lagged_chain_equals_separate_chain(tmp_path):
    """2 ranks on the xGMI exchange: the lagged chain (each exchanged gradient's clip + Adam
    inside the next forward) ends with the parameters and losses of the chain with a separate
    clip + Adam launch, bit for bit, on every rank."""
    from _dist_workers import xgmi_ppo_worker
    world = 2
    runs = {}
    for lag in ("1", "0"):
        d = tmp_path / f"lag{lag}"
        d.mkdir()
        _run(xgmi_ppo_worker, world, d, True, lag, timeout=400)
        runs[lag] = [(np.load(d / f"p{r}.npy"), np.load(d / f"l{r}.npy")) for r in range(world)]
    for r in range(world):
        (p1, l1), (p0, l0) = runs["1"][r], runs["0"][r]
        assert np.array_equal(p1.view(np.uint32), p0.view(np.uint32)), f"rank {r}: params differ"
        assert np.array_equal(l1.view(np.uint32), l0.view(np.uint32)), f"rank {r}: losses differ"


@pytest.mark.parametrize("algo", ["oneshot", "rsag"])
def test_xgmi_bwd_exchange_identical_shards_equal_one_gpu(tmp_path, algo):
    """The exchange inside k_bwd (default for the fused MLP chain): 2 ranks training on the same
    shard exchange identical gradients, whose mean (g + g) * 0.5 is g exactly, so every rank must
    end bit-identical to the one-rank run — any slot, flag, parity or ordering error shows."""
    from _dist_workers import xgmi_ppo_worker
    runs = {}
    for world in (1, 2):
        d = tmp_path / f"w{world}"
        d.mkdir()
        _run(xgmi_ppo_worker, world, d, True, "1", "mlp", algo, True, timeout=400)
        runs[world] = [(np.load(d / f"p{r}.npy"), np.load(d / f"l{r}.npy")) for r in range(world)]
        assert all((d / f"inside{r}").read_text() == "1" for r in range(world)), "exchange not inside k_bwd"
    p1, l1 = runs[1][0]
    for r in range(2):
        p2, l2 = runs[2][r]
        assert np.array_equal(p2.view(np.uint32), p1.view(np.uint32)), f"rank {r}: params differ from one rank"
        assert np.array_equal(l2.view(np.uint32), l1.view(np.uint32)), f"rank {r}: losses differ from one rank"


def test_xgmi_bwd_exchange_matches_exchange_launch(tmp_path):
    """4 ranks on their own shards with C3's MLP shapes (a backward grid small enough for 4 ranks
    to share the GPU's workgroup slots), reduce-scatter + all-gather form: the exchange inside
    k_bwd and the separate exchange launch (GS_XGMI_BWD=0) compute the same mean gradient with
    the W1 partials folded after (inside k_bwd) or before (launch) the rank sum, so the final
    parameters agree to rounding; each run's replicas are bitwise identical."""
    from _dist_workers import xgmi_ppo_worker
    world = 4
    res = {}
    for bwd in ("1", "0"):
        d = tmp_path / f"bwd{bwd}"
        d.mkdir()
        _run(xgmi_ppo_worker, world, d, True, "1", "lunar", "", False, bwd, timeout=400)
        p = [np.load(d / f"p{r}.npy") for r in range(world)]
        for r in range(1, world):
            assert np.array_equal(p[0].view(np.uint32), p[r].view(np.uint32)), (bwd, r)
        assert all((d / f"inside{r}").read_text() == bwd for r in range(world)), "unexpected exchange placement"
        res[bwd] = p[0]
    assert not np.array_equal(res["1"].view(np.uint32), res["0"].view(np.uint32))   # two distinct paths ran
    np.testing.assert_allclose(res["1"], res["0"], rtol=1e-4, atol=1e-6)


def _oracle_mean_gradient_chain(runs, n_steps):
    """The numpy oracle's data-parallel update: at step k every rank's loss and
    gradient on its own minibatch rows (utils/torch.py:97-99 per-minibatch normalisation,
    agents/ppo/ppo_agent.py:21-152), the gradients summed in rank order and scaled by 1/world,
    then clip_grad_norm_ + Adam (agents/base_agent.py:591-621) on the shared parameters."""
    from oracle import ppo_ref as R
    world = len(runs)
    dims, B = (4, 256, 256, 2), 256
    p = runs[0]["p0"].copy()
    m, v = np.zeros_like(p), np.zeros_like(p)
    losses = np.zeros((world, n_steps))
    for k in range(n_steps):
        acc = None
        for g, z in enumerate(runs):
            rows = z["idx"][k * B:(k + 1) * B].astype(np.int64)
            loss, _, grad = R.ppo_loss_and_grads(p, dims, z["obs"][rows], z["actions"][rows], z["logp"][rows],
                                                 z["values"][rows], z["adv"][rows], z["ret"][rows], clip=0.1,
                                                 clip_vf=0.2, vf_coef=0.5, ent_coef=0.0)
            losses[g, k] = loss
            grad = grad.astype(np.float32)
            acc = grad if acc is None else (acc + grad).astype(np.float32)
        mean = (acc * np.float32(1.0 / world)).astype(np.float32)
        gc, _ = R.clip_grad_norm(mean, dims, 0.5)
        p, m, v = R.adam_step(p, gc.astype(np.float32), m, v, k + 1, 1e-3)
    return p, losses


@pytest.mark.parametrize("transport,algo,bwd,world", [("xgmi", "oneshot", "1", 2), ("xgmi", "rsag", "1", 2),
                                                      ("xgmi", "oneshot", "0", 2), ("xgmi", "rsag", "0", 3),
                                                      ("rccl", "", "0", 2)])
def test_multi_rank_update_vs_oracle_mean_gradient(tmp_path, transport, algo, bwd, world):
    """Parity of the multi-GPU update itself (not replica identity): ranks on DIFFERENT env shards
    (global envs [256 g, 256 (g + 1))) run the first 8 minibatches of the fused lagged chain with
    the gradient exchange — inside k_bwd (one-shot and reduce-scatter + all-gather forms, W1
    partials summed over ranks before their row-block fold), as a launch after it, or over RCCL —
    and every rank's per-minibatch losses and final parameters must match the oracle's
    mean-gradient update on the same rows.  Bars: loss 1e-5 relative, parameters 1e-5 relative
    L2 (Adam amplifies last-bit gradient differences of near-zero-gradient weights)."""
    from _dist_workers import xgmi_oracle_worker
    n_steps = 8
    _run(xgmi_oracle_worker, world, tmp_path, transport, algo, bwd, n_steps, timeout=400)
    refused = sorted(tmp_path.glob("rccl_init_error*"))
    if refused:     # only the communicator's creation may be refused, with RCCL's own message
        pytest.skip(f"RCCL refuses {world} ranks on one GPU: {refused[0].read_text()[:200]}")
    runs = [dict(np.load(tmp_path / f"r{r}.npz")) for r in range(world)]
    assert all(int(z["inside"]) == (1 if bwd == "1" else 0) for z in runs), "unexpected exchange placement"
    for g in range(1, world):
        assert np.array_equal(runs[g]["p0"], runs[0]["p0"])          # same initial replica
        assert not np.array_equal(runs[g]["obs"], runs[0]["obs"])    # different shards
    p_ref, l_ref = _oracle_mean_gradient_chain(runs, n_steps)
    for g, z in enumerate(runs):
        np.testing.assert_allclose(z["losses"], l_ref[g], rtol=1e-5, atol=1e-6, err_msg=f"rank {g} losses")
        p_dev = z["p1"].astype(np.float64)
        rel = np.linalg.norm(p_dev - p_ref) / np.linalg.norm(p_ref)
        assert rel < 1e-5, (g, rel)
        assert np.array_equal(z["p1"].view(np.uint32), runs[0]["p1"].view(np.uint32)), f"rank {g} diverged"
    # the oracle's update differs from any single rank's own-gradient update: the exchange mattered
    p_solo, _ = _oracle_mean_gradient_chain(runs[:1], n_steps)
    assert np.linalg.norm(p_solo - p_ref) / np.linalg.norm(p_ref) > 1e-4


def test_kl_stop_on_one_rank_skips_on_every_rank(tmp_path):
    """Only rank 1's approx_kl trips target_kl (local mode): the exchange ORs the stop bits, so
    both ranks skip the same optimizer steps — rank 0 records them as skipped too — count the same
    Adam steps and end with bit-identical parameters."""
    from _dist_workers import kl_one_rank_worker
    _run(kl_one_rank_worker, 2, tmp_path, timeout=300)
    r0, r1 = (dict(np.load(tmp_path / f"r{r}.npz")) for r in range(2))
    assert r1["kl_stop"][0] == 1 and r1["skipped"][0] == 1          # rank 1 tripped at minibatch 0
    assert r0["skipped"][0] == 1                                      # rank 0 took no step there either
    assert int(r0["steps"]) == int(r1["steps"]) == 0                  # sticky: no step this epoch
    assert np.array_equal(r0["p"].view(np.uint32), r1["p"].view(np.uint32))


def test_exchange_timeout_raises_from_train_epoch(tmp_path):
    """A peer that connects and then never runs its update: rank 0's train_epoch raises GsError
    after the exchange's bounded wait (GS_XGMI_TIMEOUT_S=2) — the message and
    gs_comm_error_record name the workgroup and the peer (rank 1) it waited for — and the
    process exits non-zero instead of returning a model trained on a non-mean gradient."""
    import json
    from _dist_workers import xgmi_timeout_worker
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=xgmi_timeout_worker, args=(r, 2, port, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    for p in procs:
        if p.is_alive():
            p.kill()
            p.join()
    assert [p.exitcode for p in procs] == [3, 0]
    out = json.load(open(tmp_path / "outcome"))
    assert out["timed_out"] and out["peer"] == 1 and out["workgroup"] >= 0 and out["site"] == 1, out
    assert "timed out" in out["message"] and "rank 1" in out["message"], out["message"]


@pytest.mark.parametrize("fixture,world,bwd", [("trajectory.npz", 2, "1"), ("trajectory.npz", 2, "0"),
                                               ("trajectory.npz", 1, "1"), ("trajectory_kl.npz", 2, "0")])
def test_global_mode_reproduces_single_gpu_reference(tmp_path, fixture, world, bwd):
    """dp_mode 'global' (SURVEY §8e exact-global option, gs_ppo_update_global): the reference
    trajectory's 8 envs split 4 + 4 over 2 same-device ranks, each replaying the reference's
    actions of its envs, reproduce the SINGLE-process reference run — the global sampler
    (utils/samplers.py:25-34 over all ranks' samples), advantage normalisation over the whole
    minibatch (utils/torch.py:97-99), the gradient as the sum of the ranks' shares (exchange inside
    k_bwd, or as a launch), and with target_kl the KL stop decided on the all-rank approx_kl
    (agents/ppo/ppo_agent.py:126-129): per-minibatch losses within 1e-4 of the fixture (the
    north-star bar), the evaluated / stepped pattern exact, replicas bitwise identical."""
    from _dist_workers import global_trajectory_worker
    from gsamd._lib import M
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", fixture)
    z = np.load(path)
    _run(global_trajectory_worker, world, tmp_path, path, "xgmi", bwd, timeout=400)
    runs = [np.load(tmp_path / f"g{r}.npz") for r in range(world)]
    rec = runs[0]["rec"]
    assert rec.shape[0] == z["losses"].shape[0]
    if "evaluated" in z.files:
        np.testing.assert_array_equal((rec[:, M["unevaluated"]] == 0).astype(np.uint8), z["evaluated"])
        np.testing.assert_array_equal((rec[:, M["skipped"]] == 0).astype(np.uint8), z["stepped"])
        ev = z["evaluated"].astype(bool)
    else:
        ev = np.ones(rec.shape[0], bool)
    np.testing.assert_allclose(rec[ev, M["loss"]], z["losses"][ev], atol=1e-4, rtol=0)
    p_ref = z["params_final"].astype(np.float64)
    for r in range(world):
        assert np.array_equal(runs[r]["p"].view(np.uint32), runs[0]["p"].view(np.uint32)), f"rank {r} diverged"
        np.testing.assert_array_equal(runs[r]["rec"][:, M["loss"]], rec[:, M["loss"]])
    p = runs[0]["p"].astype(np.float64)
    assert np.linalg.norm(p - p_ref) / np.linalg.norm(p_ref) < 1e-4


@pytest.mark.parametrize("bwd", ["1", ""])
def test_exchange_guards_self_test_and_replica_check(tmp_path, bwd):
    """Guards of the default multi-GPU path: (a) init_xgmi_comm(verify_shapes=…)
    runs the in-backward exchange itself on the job's shapes (fused-chain minibatches, replicas
    bit-identical, within rounding of the exchange launch) whenever the update would use it —
    forced here for ranks sharing the GPU (GS_XGMI_BWD=1); with the placement off (shared GPU, no
    force) it is skipped and the launch form is what runs; (b) train_epoch's per-epoch replica
    check passes on a clean update and raises GsError on every rank once one rank's parameters
    differ (a stand-in for a stale-but-finite exchange)."""
    import json
    from _dist_workers import guard_worker
    _run(guard_worker, 2, tmp_path, bwd, timeout=400)
    outs = [json.load(open(tmp_path / f"guard{r}.json")) for r in range(2)]
    for o in outs:
        st = o["self_test"]
        assert st["exchange_launch_ok"] is True
        if bwd == "1":
            assert st["in_bwd_checked"] and st["in_bwd_ok"] and st["launch_ok"], st
            assert 0.0 < st["rel_l2"] < 1e-4, st          # two distinct forms ran and agree to rounding
            assert o["inside"] is True                      # the checked form stays the job's form
        else:
            assert not st["in_bwd_checked"] and o["inside"] is False, st
        assert o["first_epoch"] == "ok"
        assert o["second_epoch"] == "GsError", o
        assert "replica check failed" in o["message"]


def test_cnn_global_mode_teacher_forced_vs_single_run_and_oracle(tmp_path, cuda):
    """dp_mode 'global' for NatureCNN (gs_cnn_ppo_update_global), teacher-forced at the production
    clip (Breakout rgb_ppo: clip 0.1, clip_vf 0.2): a single-process update of 8 envs x 32 steps,
    B = 64, 4 epochs = 16 minibatches (the local fused head + loss path: the reference's own
    single-process math, utils/samplers.py:25-34 + utils/torch.py:97-99) is stepped one minibatch
    at a time and its (params, adam_m, adam_v) kept before every step.  2 ranks x 4 envs in global
    mode replay its actions and, for every minibatch k, restart from the single run's state before
    k and run that one global minibatch (their row shares, the whole minibatch's advantage
    statistics and loss mean, the gradient shares summed over xGMI, the records rebuilt on the
    device from the ranks' summed loss sums).  So each step's arithmetic is compared on its own,
    without Adam carrying a reassociation-level difference into later steps.  Per step:
      * the global run against the single run: loss 1e-5 relative, every record field 1e-5 of its
        scale (the clip fractions at most one row apart), clipped gradient 1e-4 relative L2;
      * both against the oracle (oracle/cnn_ref.py on the whole global minibatch's rows from the
        same state, clip + Adam at step k + 1) under each run's OWN ReLU decisions — the single run's
        read from its workspace (gs_cnn_workspace_act_offset), the global run's assembled from the
        two ranks' workspaces in the global minibatch's row order: every decision that differs from
        the oracle's own undecidable (|u| <= 1e-5 of its terms' magnitudes, at most 32 per conv layer
        and 8 in the fc), then loss 1e-5 relative and the clipped gradient within 2e-5 relative L2,
        every entry within 1e-4 x max|g| and at most 1e-4 of them beyond 2e-5 x max|g| — the
        arithmetic alone, at every step whose clip decisions are not within rounding (a ReLU
        decision of a near-zero pre-activation flips with the summation order and moves the entries
        that unit feeds: one step of a round-5 run moved 3.6 K of 1.69 M entries under the oracle's
        own decisions; under the run's decisions none may move);
      * unforced, the relative L2 against the oracle stays below 1e-3 (a sanity bound);
      * replicas bitwise identical (gradient + parameters digest per step).
    A step where some row's policy ratio or value change sits within 1e-5 (relative) of a clip
    boundary in the oracle is decided by rounding: a z product summed in another order flips that
    row's clip and moves the gradient by a macroscopic 1/B share, so the 0.2 % entry count is not
    applied there (the relative L2 and max bars still are; at most 2 of the 16 steps may be such).
    The clip must actually fire: some minibatch has clip_fraction > 0."""
    import torch
    from gsamd._lib import M, check, lib, ptr, stream_handle
    from gsamd.config import load_config
    from gsamd.ppo_agent import DevicePPOAgent
    from oracle import cnn_ref as C
    from _dist_workers import cnn_global_tf_worker
    N, T, B, E = 8, 32, 64, 4
    torch.manual_seed(42)
    cfg = load_config("ALE-Breakout-v5", "rgb_ppo", overrides=dict(env_dynamics="synthetic", n_envs=N, n_steps=T,
                                                                   batch_size=B, n_epochs=E))
    assert cfg.clip_range == 0.1
    agent = DevicePPOAgent(cfg, device=cuda, use_graph=False, track_stats=False)
    pm = agent.policy_model
    coll = agent.get_rollout_collector("train")
    coll.collect()
    buf = coll.buffer
    K = agent.n_minibatches
    assert K == 16
    idx = agent.prefetcher.upload(0)
    hp = agent.hparams()
    st = {"p": [], "m": [], "v": []}
    g1, p1, dev_masks = [], [], []
    # the single run's ReLU decisions of each step (a1 / a2 / a3 / h > 0 in its workspace), which
    # the oracle takes over for the single-run comparison (test_gpu_cnn.py's 8-minibatch test)
    act_shapes = [(20, 20, 32), (9, 9, 64), (7, 7, 64), (512,)]
    act_offs = [int(lib.gs_cnn_workspace_act_offset(pm.dims, B, layer)) for layer in (1, 2, 3, 4)]

    def decisions():
        out = []
        for off, sh in zip(act_offs, act_shapes):
            n = B * int(np.prod(sh))
            assert off >= 0 and off % 4 == 0 and off + 4 * n <= agent.workspace.numel()
            a = agent.workspace[off:off + 4 * n].view(torch.float32).view(B, *sh) > 0
            out.append((a.permute(0, 3, 1, 2) if len(sh) == 3 else a).cpu().numpy())
        return out
    for k in range(K):
        for key, t in (("p", pm.params), ("m", agent.adam_m), ("v", agent.adam_v)):
            st[key].append(t.cpu().numpy())
        check(lib.gs_cnn_ppo_update(ptr(pm.params), ptr(agent.grads), ptr(agent.adam_m), ptr(agent.adam_v), pm.dims,
                                    hp, buf.view(), ptr(idx[k * B:]), B, 1, k, ptr(agent.metrics_buf[k]),
                                    ptr(agent.stop_flag), ptr(agent.workspace), None, stream_handle()),
              "gs_cnn_ppo_update")
        g1.append(agent.grads.cpu().numpy())
        p1.append(pm.params.cpu().numpy())
        dev_masks.append(decisions())
    torch.cuda.synchronize()
    rec1 = agent.metrics_buf.cpu().numpy()
    ii = idx.cpu().numpy().astype(np.int64)[:K * B]
    src = (ii % T) * N + ii // T
    flat = lambda x: x.reshape(T * N, *x.shape[2:]).cpu().numpy()  # noqa: E731
    rows = tuple(flat(x)[src] for x in (buf.obs, buf.actions, buf.logprobs, buf.values, buf.advantages, buf.returns))
    to_ref = lambda a: pm.flat_to_reference(torch.as_tensor(a))  # noqa: E731
    ref = tmp_path / "ref.npz"
    states = tmp_path / "states.npz"
    np.savez(ref, NT=np.array([N, T]), B=np.int64(B), E=np.int64(E), actions=buf.actions.cpu().numpy()[None])
    np.savez(states, **{k: np.stack(v) for k, v in st.items()})
    del agent
    _run(cnn_global_tf_worker, 2, tmp_path, str(ref), str(states), timeout=400)
    runs = [np.load(tmp_path / f"tf{r}.npz") for r in range(2)]
    np.testing.assert_array_equal(runs[0]["digests"], runs[1]["digests"])
    rec2, g2 = runs[0]["rec"], runs[0]["g"]
    assert rec2.shape == rec1.shape
    shapes = C.cnn_param_shapes()
    kw = dict(valid=cfg.valid_actions, clip=float(hp.clip_range), clip_vf=float(hp.clip_range_vf),
              vf_coef=float(hp.vf_coef), ent_coef=float(hp.ent_coef))
    rl = lambda a, b: float(np.linalg.norm(a.astype(np.float64) - b) / np.linalg.norm(b))  # noqa: E731
    worst = {}
    fails = []      # every step is evaluated and printed before the bars are applied

    def need(ok, what):
        if not ok:
            fails.append(what)
    ambiguous = []
    off_share = {}

    def clip_margin(logits, values, acts, olp, ov):
        # the oracle's distance of every row's ratio / value change from its clip boundaries
        lg = logits.astype(np.float64)
        lse = np.log(np.exp(lg - lg.max(1, keepdims=True)).sum(1)) + lg.max(1)
        r = np.exp(lg[np.arange(len(acts)), acts.astype(np.int64)] - lse - olp.astype(np.float64))
        c, cv = kw["clip"], kw["clip_vf"]
        mp = np.minimum(np.abs(r - (1 - c)), np.abs(r - (1 + c))).min()
        dv = values.astype(np.float64).reshape(-1) - ov.astype(np.float64)
        mv = (np.minimum(np.abs(dv - cv), np.abs(dv + cv)) / max(cv, 1e-12)).min()
        return min(mp, mv)
    for k in range(K):
        sl = slice(k * B, (k + 1) * B)
        p_ref = to_ref(st["p"][k])
        loss, _, g, lg, vals = C.loss_and_grads(p_ref, shapes, *(x[sl] for x in rows), **kw)
        amb = clip_margin(lg, vals, rows[1][sl], rows[2][sl], rows[3][sl]) < 1e-5
        if amb:
            ambiguous.append(k)
        _, _, _, gc, _ = C.clip_and_adam(p_ref, g, shapes, to_ref(st["m"][k]), to_ref(st["v"][k]), k + 1, float(hp.lr))
        gm = np.abs(gc).max()
        # the single run against the oracle under the single run's own ReLU decisions: every
        # differing decision undecidable (|u| <= 1e-5 of its terms' magnitudes), then the arithmetic
        # bars of test_gpu_cnn.py's 8-minibatch test (unless a clip decision sits within rounding)
        dm = dev_masks[k]
        dec = C.relu_decisions(p_ref, shapes, rows[0][sl], dm)
        worst.setdefault("relu_decisions_single", []).append([n_ for n_, _ in dec])
        for (n_, r_), cap, name in zip(dec, (32, 32, 32, 8), ("conv1", "conv2", "conv3", "fc")):
            need(n_ <= cap and r_ <= 1e-5, ("single relu decisions", k, name, n_, r_))
        _, _, gf, _, _ = C.loss_and_grads(p_ref, shapes, *(x[sl] for x in rows), conv_masks=dm[:3], fc_mask=dm[3],
                                          **kw)
        _, _, _, gcf, _ = C.clip_and_adam(p_ref, gf, shapes, to_ref(st["m"][k]), to_ref(st["v"][k]), k + 1,
                                          float(hp.lr))
        gr1 = to_ref(g1[k])
        dgf = np.abs(gr1.astype(np.float64) - gcf)
        gmf = np.abs(gcf).max()
        worst["single_forced"] = max(worst.get("single_forced", 0.0), rl(gr1, gcf))
        if not amb:
            need(rl(gr1, gcf) < 2e-5 and dgf.max() <= 1e-4 * gmf and (dgf > 2e-5 * gmf).sum() <= 1e-4 * dgf.size,
                 ("single forced", k, rl(gr1, gcf), float(dgf.max() / gmf), int((dgf > 2e-5 * gmf).sum())))
        # the GLOBAL run against the oracle under the global run's own ReLU decisions: each rank's
        # decisions of its row share, assembled in the global minibatch's row order (global row j is
        # the next row of rank env_j // n in stream order, gsamd.samplers.rank_share), the same
        # undecidability check, then the same arithmetic bars as the single run
        gmask = []
        ranks_j = (ii[sl] // T) // (N // 2)
        pos_j = np.array([int((ranks_j[:j] == ranks_j[j]).sum()) for j in range(B)])
        for li, shp in enumerate(((32, 20, 20), (64, 9, 9), (64, 7, 7), (512,))):
            nel = int(np.prod(shp))
            per = [np.unpackbits(runs[r][f"mask{li}"][k], axis=1)[:, :nel].astype(bool) for r in range(2)]
            gmask.append(np.stack([per[r_][p_] for r_, p_ in zip(ranks_j, pos_j)]).reshape(B, *shp))
        for r in range(2):      # each rank's padded share is exactly its rows of this minibatch
            sh_r = runs[r]["shares"][k * B:(k + 1) * B]
            assert (sh_r[:int((ranks_j == r).sum())] >= 0).all() and (sh_r[int((ranks_j == r).sum()):] < 0).all()
        decg = C.relu_decisions(p_ref, shapes, rows[0][sl], gmask)
        worst.setdefault("relu_decisions_global", []).append([n_ for n_, _ in decg])
        for (n_, r_), cap, name in zip(decg, (32, 32, 32, 8), ("conv1", "conv2", "conv3", "fc")):
            need(n_ <= cap and r_ <= 1e-5, ("global relu decisions", k, name, n_, r_))
        _, _, gg, _, _ = C.loss_and_grads(p_ref, shapes, *(x[sl] for x in rows), conv_masks=gmask[:3],
                                          fc_mask=gmask[3], **kw)
        _, _, _, gcg, _ = C.clip_and_adam(p_ref, gg, shapes, to_ref(st["m"][k]), to_ref(st["v"][k]), k + 1,
                                          float(hp.lr))
        gr2 = to_ref(g2[k])
        dgg = np.abs(gr2.astype(np.float64) - gcg)
        gmg = np.abs(gcg).max()
        worst["global_forced"] = max(worst.get("global_forced", 0.0), rl(gr2, gcg))
        worst["global_forced_off"] = max(worst.get("global_forced_off", 0), int((dgg > 2e-5 * gmg).sum()))
        if not amb:
            need(rl(gr2, gcg) < 2e-5 and dgg.max() <= 1e-4 * gmg and (dgg > 2e-5 * gmg).sum() <= 1e-4 * dgg.size,
                 ("global forced", k, rl(gr2, gcg), float(dgg.max() / gmg), int((dgg > 2e-5 * gmg).sum())))
        for tag, rec, gd in (("single", rec1, g1[k]), ("global", rec2, g2[k])):
            dl = abs(rec[k, M["loss"]] - loss) / max(1.0, abs(loss))
            need(dl < 1e-5, (tag, "loss", k, float(rec[k, M["loss"]]), loss))
            gr = to_ref(gd)
            dg = np.abs(gr.astype(np.float64) - gc)
            # unforced (the oracle's own ReLU decisions): information, plus a sanity bound — a
            # decision of a near-zero pre-activation flips with the summation order and moves the
            # entries that unit feeds; the arithmetic bars are the forced ones above
            off_share.setdefault(tag, []).append(float((dg > 2e-5 * gm).mean()))
            need(rl(gr, gc) < 1e-3, (tag, "grad rel L2 (unforced)", k, rl(gr, gc)))
            worst[tag] = max(worst.get(tag, 0.0), rl(gr, gc))
            worst[tag + "_off"] = max(worst.get(tag + "_off", 0), int((dg > 2e-5 * gm).sum()))
        worst["g_vs_s"] = max(worst.get("g_vs_s", 0.0), rl(g2[k], g1[k].astype(np.float64)))
        need(rl(g2[k], g1[k].astype(np.float64)) < 1e-4, ("global vs single grad", k))
    print(f"teacher-forced global mode: worst clipped-gradient rel L2 / entries off {worst}; "
          f"steps with a clip decision within rounding: {ambiguous}")
    assert not fails, fails
    assert len(ambiguous) <= 2, ambiguous
    np.testing.assert_allclose(rec2[:, M["loss"]], rec1[:, M["loss"]], atol=1e-5, rtol=1e-5)
    for key in ("policy_loss", "value_loss", "entropy", "approx_kl", "kl", "adv_norm_mean", "adv_norm_std",
                "explained_var"):
        scale = max(1.0, float(np.abs(rec1[:, M[key]]).max()))
        np.testing.assert_allclose(rec2[:, M[key]], rec1[:, M[key]], atol=1e-5 * scale, rtol=0, err_msg=key)
    for key in ("clip_fraction", "clip_fraction_vf"):
        assert np.abs(rec2[:, M[key]] - rec1[:, M[key]]).max() <= 1.0 / B + 1e-7, key
    assert (rec1[:, M["clip_fraction"]] > 0).any(), rec1[:, M["clip_fraction"]]


@pytest.mark.parametrize("mode", ["mlp", "inject", "cnn"])
def test_agent_attached_comm_self_tested(tmp_path, mode):
    """Multi-GPU guards run by the agent itself: with init_xgmi_comm
    called WITHOUT verify_shapes, the agent's first update self-tests the in-backward exchange on
    its own dims / batch / precision; every epoch passes the replica check and an exchange canary
    over the whole parameter count; a failure injected on one rank before its first self-test
    exchange leaves every rank in the same collective sequence, resets the communicator and moves
    every rank to the exchange launch, and training continues; the NatureCNN-sized communicator's
    vector self-test covers all 1 693 875 floats.  Replicas end bit-identical in every mode."""
    import json
    from _dist_workers import agent_selftest_worker
    _run(agent_selftest_worker, 2, tmp_path, mode, timeout=400)
    outs = [json.load(open(tmp_path / f"ast{r}.json")) for r in range(2)]
    assert outs[0]["params_sha"] == outs[1]["params_sha"]
    for o in outs:
        assert o["epochs"] == "ok" and o["canary_rounds"] == 2, o
        assert o["connect_self_test"]["exchange_launch_ok"] is True
        st = o["agent_self_test"]
        if mode == "cnn":
            assert o["n_params"] == 1_693_875 and st is None, o
            continue
        assert st["in_bwd_checked"] and st["launch_ok"] is True and st["flags"] == 0, st
        if mode == "mlp":
            assert st["in_bwd_ok"] is True and 0.0 < st["rel_l2"] < 1e-4 and o["inside"] is True, st
        else:
            assert st["in_bwd_ok"] is False and o["inside"] is False, st
