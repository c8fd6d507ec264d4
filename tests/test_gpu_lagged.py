"""The fused chain's lagged optimizer step: on one GPU, minibatch k's clip +
Adam runs inside the forward kernel of minibatch k+1, alternating between the caller's
parameter set and a workspace copy.  It must give bit for bit the update of the chain with a
separate k_clip_adam launch per minibatch.  GS_LAGGED_ADAM=0 selects the separate launch; these tests select
each chain explicitly."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _same(name, x, y):
    a, b = np.ascontiguousarray(x), np.ascontiguousarray(y)
    bad = np.flatnonzero(a.view(np.uint8) != b.view(np.uint8)) // a.itemsize
    assert bad.size == 0, f"{name}: {np.unique(bad).size} elements differ, first {np.unique(bad)[:8]}"


# eager; graph-replayed 512-step chunks + an eager tail with the last step landing in the
# workspace set (768 minibatches: copied back) and in the caller's set (767); and the
# multi-GPU chain (fwd(+Adam of k-1) -> bwd -> exchange of k) over a one-rank communicator
@pytest.mark.parametrize("use_graph,n_envs,n_epochs,drop,transport", [
    (False, 512, 2, 1, None), (True, 2048, 3, 0, None), (True, 2048, 3, 1, None),
    (False, 512, 2, 1, "xgmi"), (True, 2048, 3, 1, "xgmi"), (True, 2048, 3, 0, "rccl")])
def test_lagged_adam_matches_separate_adam(cuda, monkeypatch, use_graph, n_envs, n_epochs, drop, transport):
    """Parameters, Adam moments, the last step's clipped gradients and metric records
    bit-identical."""
    from gsamd._lib import check, lib
    from gsamd.config import load_config
    from gsamd.distributed import destroy_comm, init_local_comm
    from gsamd.ppo_agent import DevicePPOAgent
    out = []
    for lag in ("1", "0"):
        monkeypatch.setenv("GS_LAGGED_ADAM", lag)
        torch.manual_seed(7)
        cfg = load_config("CartPole-v1", "ppo", overrides=dict(env_dynamics="synthetic", n_envs=n_envs, n_epochs=n_epochs))
        comm = init_local_comm(transport, 70_000) if transport else None
        agent = DevicePPOAgent(cfg, device=cuda, use_graph=use_graph, track_stats=False, comm=comm)
        coll = agent.get_rollout_collector("train")
        coll.collect()
        idx = agent.prefetcher.upload(0)
        n = agent.n_minibatches - drop
        check(lib.gs_ppo_update(agent.policy_model.params.data_ptr(), agent.grads.data_ptr(), agent.adam_m.data_ptr(),
                                agent.adam_v.data_ptr(), agent.policy_model.dims, agent.hparams(), coll.buffer.view(),
                                idx.data_ptr(), agent.batch_size, n, 3, agent.metrics_buf.data_ptr(),
                                agent.stop_flag.data_ptr(), agent.workspace.data_ptr(), agent.workspace.numel(), comm,
                                1 if use_graph else 0, torch.cuda.current_stream().cuda_stream), "gs_ppo_update")
        torch.cuda.synchronize()
        out.append([t.cpu().numpy() for t in (agent.policy_model.params, agent.adam_m, agent.adam_v, agent.grads,
                                               agent.metrics_buf[:n])])
        del agent
        destroy_comm(comm)
    assert np.isfinite(out[0][0]).all()
    for name, x, y in zip(("params", "adam_m", "adam_v", "grads", "metrics"), out[0], out[1]):
        _same(name, x, y)


def test_lagged_stage_writes_workspace_set_only(cuda, monkeypatch):
    """gs_ppo_stage 7 (the lagged forward bench.py times) runs on the C2 shapes and leaves the
    caller's parameters alone (it writes the workspace's second set)."""
    from gsamd._lib import lib
    from gsamd.config import load_config
    from gsamd.ppo_agent import DevicePPOAgent
    monkeypatch.setenv("GS_LAGGED_ADAM", "1")
    torch.manual_seed(3)
    cfg = load_config("CartPole-v1", "ppo", overrides=dict(env_dynamics="synthetic", n_envs=512, n_epochs=1))
    agent = DevicePPOAgent(cfg, device=cuda, use_graph=False, track_stats=False)
    agent.train_epoch()
    pm = agent.policy_model
    args = lambda st: (st, pm.params.data_ptr(), agent.grads.data_ptr(), agent.adam_m.data_ptr(),  # noqa: E731
                       agent.adam_v.data_ptr(), pm.dims, agent.hparams(),
                       agent.get_rollout_collector("train").buffer.view(), agent.prefetcher.device_buf.data_ptr(),
                       agent.batch_size, 1, agent.metrics_buf.data_ptr(), agent.workspace.data_ptr(),
                       torch.cuda.current_stream().cuda_stream)
    before = [t.clone() for t in (pm.params, agent.adam_m, agent.adam_v)]
    assert lib.gs_ppo_stage(*args(6)) == 0
    assert lib.gs_ppo_stage(*args(7)) == 0
    torch.cuda.synchronize()
    for b, t in zip(before, (pm.params, agent.adam_m, agent.adam_v)):
        assert torch.equal(b, t)
