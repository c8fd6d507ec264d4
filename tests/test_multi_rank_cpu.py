"""CPU, world_size 2 (gloo): the multi-GPU protocol of the device path."""
import multiprocessing as mp
import os
import socket

import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("world", [2])
def test_data_parallel_protocol_gloo(tmp_path, world):
    from _dist_workers import dp_worker
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=dp_worker, args=(r, world, port, str(tmp_path))) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    for p in procs:
        if p.is_alive():
            p.kill()
    codes = [p.exitcode for p in procs]
    assert codes == [0] * world, codes
    assert sorted(os.listdir(tmp_path)) == [f"ok{r}" for r in range(world)]


def test_replica_check_and_seed_broadcast_gloo(tmp_path):
    """The per-epoch replica check of train_epoch (gsamd.distributed.check_replicas, DESIGN §5
    guards) and the global mode's sampler-seed agreement, on CPU ranks: identical parameters
    pass, one changed element or two swapped elements raise GsError on every rank."""
    from _dist_workers import replica_check_cpu_worker
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=replica_check_cpu_worker, args=(r, 2, port, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    for p in procs:
        if p.is_alive():
            p.kill()
    assert [p.exitcode for p in procs] == [0, 0]
    for r in range(2):
        assert (tmp_path / f"rc{r}").read_text() == "GsError,GsError"


def test_multi_rank_without_communicator_raises_gloo(tmp_path):
    """world_size 2 with no communicator attached: the agent's update (local and global mode) and
    training_step raise ValueError on every rank (DevicePPOAgent._require_exchange) — no rank
    trains a replica of its own silently."""
    from _dist_workers import no_comm_worker
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=no_comm_worker, args=(r, 2, port, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    for p in procs:
        if p.is_alive():
            p.kill()
    assert [p.exitcode for p in procs] == [0, 0]
    for r in range(2):
        assert (tmp_path / f"nc{r}").read_text() == ",".join(["ValueError"] * 4)
