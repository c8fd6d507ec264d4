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
    replicas end bitwise identical (2 ranks forced, 4 ranks by default)."""
    from _dist_workers import xgmi_ppo_worker
    _run(xgmi_ppo_worker, world, tmp_path, True, "1", "mlp", "rsag", timeout=400)
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
