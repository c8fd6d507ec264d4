"""Multi-GPU plumbing for the device path: one process per GPU, envs sharded
by rank, one communicator per process handed to DevicePPOAgent(comm=...) and used inside the
C-ABI for the per-minibatch gradient mean; nothing else crosses GPUs.

Two transports: the one-shot xGMI exchange (init_xgmi_comm: IPC handles of
each rank's exchange region all-gathered through torch.distributed; the default) and RCCL
(init_device_comm: a unique id that rank 0 makes and torch.distributed broadcasts)."""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from ._lib import check, lib

UNIQUE_ID_BYTES = 128


def world_active() -> bool:
    """True inside an initialised torch.distributed job of more than one rank."""
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def allreduce_sum_f64(values) -> "np.ndarray":
    """Sum a small host vector over ranks (float64; per-epoch metric partial sums).
    A no-op outside a multi-rank job."""
    import numpy as np
    v = np.asarray(values, dtype=np.float64)
    if not world_active():
        return v
    import torch.distributed as dist
    t = torch.from_numpy(v.copy())
    if dist.get_backend() == "nccl":
        t = t.to(torch.device("cuda", torch.cuda.current_device()))
    dist.all_reduce(t)
    return t.cpu().numpy()


def broadcast_int(value: int, src: int = 0) -> int:
    """Rank src's integer on every rank (int64 over torch.distributed); the value itself
    outside a multi-rank job."""
    if not world_active():
        return int(value)
    import torch.distributed as dist
    t = torch.tensor([int(value)], dtype=torch.int64)
    if dist.get_backend() == "nccl":
        t = t.to(torch.device("cuda", torch.cuda.current_device()))
    dist.broadcast(t, src)
    return int(t.item())


def env_offset(rank: int, n_envs_per_rank: int) -> int:
    """Global id of a rank's first env: rank g owns [g·N, (g+1)·N)."""
    return int(rank) * int(n_envs_per_rank)


def exchange_unique_id(rank: int, device: Optional[torch.device] = None) -> bytes:
    """Rank 0 creates the RCCL unique id; every rank returns the same 128 bytes.  Works over
    any initialised torch.distributed backend (nccl broadcasts from `device`, gloo from host)."""
    import torch.distributed as dist
    uid = torch.zeros(UNIQUE_ID_BYTES, dtype=torch.uint8)
    if rank == 0:
        check(lib.gs_comm_unique_id(uid.data_ptr()), "gs_comm_unique_id")
    if dist.get_backend() == "nccl":
        t = uid.to(device if device is not None else torch.device("cuda", torch.cuda.current_device()))
        dist.broadcast(t, 0)
        uid = t.cpu()
    else:
        dist.broadcast(uid, 0)
    return bytes(uid.contiguous().numpy().tobytes())


def init_device_comm(rank: int, world_size: int, device: Optional[torch.device] = None) -> int:
    """Exchange the id through torch.distributed and join the RCCL communicator; returns the
    opaque gs_comm handle (an integer address) for DevicePPOAgent / gs_ppo_update."""
    uid = exchange_unique_id(rank, device)
    buf = (ctypes.c_uint8 * UNIQUE_ID_BYTES).from_buffer_copy(uid)
    h = ctypes.c_void_p()
    check(lib.gs_comm_init(ctypes.addressof(buf), int(world_size), int(rank), ctypes.byref(h)), "gs_comm_init")
    return h.value


XGMI_HANDLE_BYTES = 64


def _all_gather_bytes(payload: bytes, device: Optional[torch.device] = None) -> bytes:
    """Concatenate every rank's fixed-size payload in rank order over torch.distributed."""
    import torch.distributed as dist
    t = torch.frombuffer(bytearray(payload), dtype=torch.uint8).clone()
    if dist.get_backend() == "nccl":
        t = t.to(device if device is not None else torch.device("cuda", torch.cuda.current_device()))
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    return b"".join(bytes(p.cpu().numpy().tobytes()) for p in parts)


def xgmi_create(rank: int, world_size: int, max_count: int):
    """Allocate and IPC-export this rank's exchange region: (handle, 64 handle bytes)."""
    hb = (ctypes.c_uint8 * XGMI_HANDLE_BYTES)()
    h = ctypes.c_void_p()
    check(lib.gs_comm_xgmi_create(int(world_size), int(rank), int(max_count), ctypes.addressof(hb), ctypes.byref(h)),
          "gs_comm_xgmi_create")
    return h.value, bytes(hb)


def xgmi_connect(handle: int, all_handles: bytes) -> None:
    buf = (ctypes.c_uint8 * len(all_handles)).from_buffer_copy(all_handles)
    check(lib.gs_comm_xgmi_connect(handle, ctypes.addressof(buf)), "gs_comm_xgmi_connect")


def _agree(ok: bool, device: Optional[torch.device]) -> bool:
    """True only if every rank passes ok=True."""
    import torch.distributed as dist
    t = torch.tensor([1 if ok else 0], dtype=torch.int32)
    if dist.get_backend() == "nccl":
        t = t.to(device if device is not None else torch.device("cuda", torch.cuda.current_device()))
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def _pattern(rank: int, it: int, n: int, device) -> torch.Tensor:
    """Rank `rank`'s exchange test vector of round `it`: small integers (exact in float32), a
    different value in every round and rank, so a stale slot from an earlier round shows."""
    idx = torch.arange(n, dtype=torch.int64, device=device)
    return ((rank + 1) * (it + 3) + (idx * (rank + 5) + it) % 11).to(torch.float32)


def xgmi_self_test(handle: int, rank: int, world_size: int, n: int, device: torch.device, rounds: int = 3,
                   salt: int = 0) -> bool:
    """Exchange known vectors `rounds` times through gs_comm_allreduce_mean_f32 and compare every
    element with the exact fixed-order answer ((x0 + x1) + ...) * f32(1 / world), computed on the
    device (also proves the peers' flags arrive).  n: the communicator's full capacity is what
    covers every exchange workgroup and chunk the job's gradient uses."""
    from ._lib import stream_handle
    for it in range(rounds):
        r_it = it + 7 * int(salt)
        buf = _pattern(rank, r_it, n, device)
        check(lib.gs_comm_allreduce_mean_f32(handle, buf.data_ptr(), n, stream_handle()), "gs_comm_allreduce_mean_f32")
        acc = _pattern(0, r_it, n, device)
        for r in range(1, world_size):
            acc = acc + _pattern(r, r_it, n, device)
        want = acc * torch.tensor(1.0 / world_size, dtype=torch.float32, device=device)
        same = torch.equal(buf.view(torch.int32), want.view(torch.int32))
        if lib.gs_comm_status(handle) != 0 or not same:
            return False
    return True


def xgmi_reset(handle: int, device: Optional[torch.device] = None) -> None:
    """Every rank back to the connect-time exchange state after a failed or timed-out exchange
    (gs_comm_xgmi_reset between two host barriers, after each rank's device work drained).
    Collective."""
    import torch.distributed as dist
    torch.cuda.synchronize(device)
    dist.barrier()
    check(lib.gs_comm_xgmi_reset(handle), "gs_comm_xgmi_reset")
    dist.barrier()


def _digest(t: torch.Tensor) -> bytes:
    import hashlib
    return hashlib.sha256(t.detach().cpu().numpy().tobytes()).digest()


_FAILED_DIGEST = bytes(32)          # sent by a rank whose chain raised: no real digest is all zeros


def _chain_run(handle: int, rank: int, dims, batch: int, steps: int, device: torch.device,
               flags: int = 0) -> torch.Tensor:
    """One fused-chain update of `steps` minibatches through gs_ppo_update on `handle`, from a
    fixed parameter state (identical on every rank) and a rank-specific synthetic batch set:
    the exchange the job's own update runs, on the job's shapes and precision (flags = the job's
    gs_ppo_hparams.flags: the bf16 chain exchanges from its own k_bwd instantiation).  Returns the
    new parameters."""
    import numpy as np
    from ._lib import PPOHparams, RolloutView, GS_NUM_METRICS, stream_handle
    D, H1, H2, A = int(dims.obs_dim), int(dims.hidden1), int(dims.hidden2), int(dims.n_actions)
    P = H1 * D + H1 + H2 * H1 + H2 + A * H2 + A + H2 + 1
    g = np.random.default_rng(20240917)
    p = torch.from_numpy((g.standard_normal(P) * 0.05).astype(np.float32)).to(device)
    r = np.random.default_rng(1009 + 7919 * int(rank))
    N = 2 * int(batch)                      # T = 1: sample index i is env i
    f32 = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(device)  # noqa: E731
    obs = f32(r.uniform(-1, 1, (1, N, D)))
    act = torch.from_numpy(r.integers(0, A, (1, N))).to(device)
    lp, val = f32(-r.uniform(0.1, 2.0, (1, N))), f32(r.standard_normal((1, N)))
    adv, ret = f32(r.standard_normal((1, N))), f32(r.standard_normal((1, N)))
    idx = torch.from_numpy(np.concatenate([r.permutation(N)[:batch] for _ in range(steps)]).astype(np.int32)).to(device)
    z = dict(dtype=torch.float32, device=device)
    grads, m, v = torch.zeros(P, **z), torch.zeros(P, **z), torch.zeros(P, **z)
    metrics = torch.zeros(steps, GS_NUM_METRICS, **z)
    stop = torch.zeros(1, dtype=torch.int32, device=device)
    ws = torch.zeros(int(lib.gs_ppo_update_workspace_bytes(dims, int(batch), steps)), dtype=torch.uint8, device=device)
    hp = PPOHparams(0.2, 0.2, 0.5, 0.01, 0.5, 1e-3, 0.9, 0.999, 1e-8, 0.0, 1, int(flags))
    view = RolloutView(obs.data_ptr(), act.data_ptr(), lp.data_ptr(), val.data_ptr(), adv.data_ptr(), ret.data_ptr(), 1, N)
    check(lib.gs_ppo_update(p.data_ptr(), grads.data_ptr(), m.data_ptr(), v.data_ptr(), dims, hp, view, idx.data_ptr(),
                            int(batch), steps, 0, metrics.data_ptr(), stop.data_ptr(), ws.data_ptr(), ws.numel(),
                            handle, 0, stream_handle()), "gs_ppo_update (exchange self-test)")
    torch.cuda.current_stream().synchronize()
    check(lib.gs_comm_status(handle), "gs_comm_status (exchange self-test)")
    if not bool(torch.isfinite(p).all()):
        raise RuntimeError("non-finite parameters after the exchange self-test chain")
    return p


def _chain_agreed(handle, rank, world_size, dims, batch, steps, dev, device, flags):
    """Run the chain, then ALWAYS all-gather a digest (a failing rank sends _FAILED_DIGEST), so every
    rank runs the same collective sequence whatever failed where.  -> (params or None, ok, why)."""
    try:
        p, why = _chain_run(handle, rank, dims, batch, steps, dev, flags), ""
    except RuntimeError as e:
        p, why = None, str(e)
    digests = _all_gather_bytes(_digest(p) if p is not None else _FAILED_DIGEST, device)
    parts = {digests[32 * r:32 * (r + 1)] for r in range(world_size)}
    ok = p is not None and len(parts) == 1 and _FAILED_DIGEST not in parts
    if p is not None and not ok:
        why = "a peer's chain failed" if _FAILED_DIGEST in parts else "replicas differ after the exchange"
    return p, ok, why


# what the last init_xgmi_comm's self-tests found (bench.py reports it beside its line)
LAST_SELF_TEST: dict = {}
# (handle, dims, batch, flags) whose in-backward exchange a self-test already verified
_VERIFIED: set = set()


def bwd_exchange_self_test(handle: int, rank: int, world_size: int, dims, batch: int,
                           device: Optional[torch.device] = None, steps: int = 4, flags: int = 0) -> dict:
    """The in-backward exchange (the fused MLP chain's default with one rank per GPU,
    csrc/gs_xgmi_dev.h bwd_exchange) checked on the job's own shapes and precision before the job
    trains: `steps` fused-chain minibatches from a fixed state, each rank on its own synthetic rows,
    (1) with the exchange inside k_bwd — every rank must end with the same parameter bits —
    and (2) with the separate exchange launch (the form init_xgmi_comm's vector self-test
    proved) — the two must agree to the rounding of their different W1-partial fold order
    (relative L2 < 1e-4, the bar of test_xgmi_bwd_exchange_matches_exchange_launch), and the
    launch form's replicas must be bit-identical too.  A stale or torn slot read on any rank
    breaks (1) or (2).  Every rank runs the same collectives whatever fails (a failing rank sends a
    sentinel digest); after a failure of (1) every rank resets the communicator (xgmi_reset: flags,
    sticky error, sequence counters) before (2) and then uses the launch form
    (gs_comm_xgmi_set_bwd_exchange(0)); if the launch form fails as well this raises on every rank
    (the caller falls back to RCCL).  Collective: every rank calls it together.
    Returns {"in_bwd_checked", "in_bwd_ok", "launch_ok", "rel_l2", "steps", "flags"}."""
    import sys
    import numpy as np
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    out = {"in_bwd_checked": False, "in_bwd_ok": None, "launch_ok": None, "rel_l2": None, "steps": int(steps),
           "flags": int(flags)}
    if world_size <= 1 or not exchange_inside_bwd(handle, dims, batch):
        return out
    out["in_bwd_checked"] = True
    pb, ok_b, why = _chain_agreed(handle, rank, world_size, dims, batch, steps, dev, device, flags)
    ok_b = _agree(ok_b, device)
    if not ok_b:
        xgmi_reset(handle, dev)          # a timed-out wait leaves flags / counters / the error word behind
    check(lib.gs_comm_xgmi_set_bwd_exchange(handle, 0), "gs_comm_xgmi_set_bwd_exchange")
    pl, ok_l, why_l = _chain_agreed(handle, rank, world_size, dims, batch, steps, dev, device, flags)
    why = why or why_l
    if ok_b and ok_l:
        a, b = pb.double().cpu().numpy(), pl.double().cpu().numpy()
        out["rel_l2"] = float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))
        if not out["rel_l2"] < 1e-4:
            ok_b, why = False, f"in-backward vs launch relative L2 {out['rel_l2']:.3e}"
    ok_b, ok_l = _agree(ok_b, device), _agree(ok_l, device)
    out["in_bwd_ok"], out["launch_ok"] = ok_b, ok_l
    if not ok_l:
        raise RuntimeError(f"xGMI exchange self-test: the exchange launch failed on the job's shapes: {why}")
    # restore the placement the job asked for (1: one rank per GPU; 2 where 1 would not place it
    # inside, i.e. GS_XGMI_BWD=1 on a shared GPU), or keep the launch form after a failure
    check(lib.gs_comm_xgmi_set_bwd_exchange(handle, 1 if ok_b else 0), "gs_comm_xgmi_set_bwd_exchange")
    if ok_b and not exchange_inside_bwd(handle, dims, batch):
        check(lib.gs_comm_xgmi_set_bwd_exchange(handle, 2), "gs_comm_xgmi_set_bwd_exchange")
    if ok_b:
        _VERIFIED.add(_verify_key(handle, dims, batch, flags))
    if rank == 0:
        print(f"[gsamd] xGMI in-backward exchange self-test ({world_size} ranks, {steps} minibatches, "
              f"dims {int(dims.obs_dim)}-{int(dims.hidden1)}-{int(dims.hidden2)}-{int(dims.n_actions)}, B={batch}, "
              f"flags {int(flags)}): "
              + ("replicas bit-identical, vs exchange launch rel L2 %.2e" % out["rel_l2"] if ok_b else
                 f"FAILED ({why or 'a peer failed'}); every rank uses the exchange launch"), file=sys.stderr, flush=True)
    return out


def _verify_key(handle, dims, batch, flags):
    return (int(handle), int(dims.obs_dim), int(dims.hidden1), int(dims.hidden2), int(dims.n_actions), int(batch),
            int(flags))


def verified(handle, dims, batch, flags) -> bool:
    """Whether bwd_exchange_self_test already verified this communicator on these shapes / flags."""
    return _verify_key(handle, dims, batch, flags) in _VERIFIED


def init_xgmi_comm(rank: int, world_size: int, max_count: int, device: Optional[torch.device] = None,
                   self_test: bool = True, verify_shapes=None) -> int:
    """One-shot xGMI communicator for exchanges of up to max_count floats (the policy's
    parameter count): create, all-gather the handles, open the peers, barrier, then (by
    default) a bit-exact self-test agreed on by every rank over the FULL max_count (every exchange
    workgroup and chunk the job's gradient will use: the NatureCNN's 1.69 M floats included).
    Raises RuntimeError on every rank if any rank fails (the caller may then choose RCCL
    instead).  verify_shapes = (gs_mlp_dims, batch[, flags]): also check the in-backward exchange
    on those shapes and that precision (bwd_exchange_self_test; it drops every rank to the exchange
    launch if that form fails).  DevicePPOAgent runs the same check itself on its first update with
    a communicator attached, so a launcher that passes no verify_shapes is still covered."""
    import torch.distributed as dist
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    h, ok, why = None, True, ""
    try:
        h, mine = xgmi_create(rank, world_size, max_count)
    except RuntimeError as e:
        ok, why = False, str(e)
    handles = _all_gather_bytes(mine if ok else bytes(XGMI_HANDLE_BYTES), device)
    if ok:
        try:
            xgmi_connect(h, handles)
        except RuntimeError as e:
            ok, why = False, str(e)
    ok = _agree(ok, device)
    if ok:
        # ranks sharing one GPU (same-device rehearsals): the exchange inside the backward
        # needs the peers' workgroups resident together (include/gsamd.h)
        pr = torch.cuda.get_device_properties(dev)
        ident = f"{pr.pci_domain_id:08x}:{pr.pci_bus_id:04x}:{pr.pci_device_id:04x}".encode()
        ids = _all_gather_bytes(ident.ljust(32, b"\0"), device)
        ids = [ids[32 * r:32 * (r + 1)] for r in range(world_size)]
        check(lib.gs_comm_xgmi_set_colocation(h, max(ids.count(i) for i in ids)), "gs_comm_xgmi_set_colocation")
    dist.barrier()
    if ok and self_test:
        try:
            ok = xgmi_self_test(h, rank, world_size, int(max_count), dev)
            why = "" if ok else "self-test mismatch or timeout"
        except RuntimeError as e:
            ok, why = False, str(e)
        ok = _agree(ok, device)
    LAST_SELF_TEST.clear()
    LAST_SELF_TEST["exchange_launch_ok"] = bool(ok) if self_test else None
    if ok and self_test and verify_shapes is not None:
        try:
            flags = int(verify_shapes[2]) if len(verify_shapes) > 2 else 0
            LAST_SELF_TEST.update(bwd_exchange_self_test(h, rank, world_size, verify_shapes[0], int(verify_shapes[1]),
                                                         dev, flags=flags))
        except RuntimeError as e:
            ok, why = False, str(e)
    if not ok:
        if h:
            destroy_comm(h)
        raise RuntimeError(f"xGMI exchange unavailable on rank {rank}: {why or 'a peer failed'}")
    return h


def replica_checksum(params: torch.Tensor) -> torch.Tensor:
    """Two float64 checksums of a flat parameter vector on its device: the plain sum and a
    position-weighted sum (a swapped or shifted element changes the second)."""
    p = params.detach().double()
    w = (torch.arange(p.numel(), device=p.device, dtype=torch.float64) % 1021) + 1.0
    return torch.stack([p.sum(), (p * w).sum()])


def check_replicas(params: torch.Tensor, what: str = "parameters") -> None:
    """Every rank's parameters must be bit-identical after an update (the exchange gives every
    rank the same mean gradient and every rank runs the same clip + Adam,
    agents/base_agent.py:591-621).  The checksums are all-reduced as MIN and MAX; any
    difference raises GsError on every rank, so a stale-but-finite exchange can never yield a
    trained model or a bench number.  A no-op outside a multi-rank job."""
    if not world_active():
        return
    import torch.distributed as dist
    from ._lib import GsError
    cs = replica_checksum(params)
    if dist.get_backend() != "nccl":
        cs = cs.cpu()
    lo, hi = cs.clone(), cs.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    lo, hi, mine = lo.cpu().numpy(), hi.cpu().numpy(), cs.cpu().numpy()
    if not (lo == hi).all():
        raise GsError(f"replica check failed on rank {dist.get_rank()}: the ranks' {what} differ after the update "
                      f"(checksums min {lo.tolist()}, max {hi.tolist()}, this rank {mine.tolist()}); the gradient "
                      f"exchange delivered different data to different ranks")


def exchange_inside_bwd(handle: int, dims, batch: int) -> bool:
    """Whether the fused MLP update exchanges gradients inside its backward kernel on this
    communicator (include/gsamd.h gs_ppo_exchange_inside_bwd)."""
    v = ctypes.c_int()
    check(lib.gs_ppo_exchange_inside_bwd(handle, dims, int(batch), ctypes.byref(v)), "gs_ppo_exchange_inside_bwd")
    return bool(v.value)


def comm_status(handle: Optional[int]) -> None:
    """Raise if an exchange on this communicator timed out waiting for a peer.  The current
    stream (the one the update ran on) is synchronised first: gs_comm_status reads the sticky
    error word with a host copy, which must come after the update's exchanges ran."""
    if handle:
        if torch.cuda.is_available():
            torch.cuda.current_stream().synchronize()
        check(lib.gs_comm_status(handle), "gs_comm_status")


def comm_error_record(handle: int) -> dict:
    """The first exchange timeout's record (include/gsamd.h gs_comm_error_record)."""
    t, w, p, site = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    check(lib.gs_comm_error_record(handle, ctypes.byref(t), ctypes.byref(w), ctypes.byref(p), ctypes.byref(site)),
          "gs_comm_error_record")
    return {"timed_out": bool(t.value), "workgroup": w.value, "peer": p.value, "site": site.value}


def init_local_comm(transport: str = "rccl", max_count: int = 1 << 20) -> int:
    """A one-rank communicator (no torch.distributed needed): exercises the multi-GPU kernel
    chain and the transport's call on a single GPU."""
    if transport == "xgmi":
        h, mine = xgmi_create(0, 1, max_count)
        xgmi_connect(h, mine)
        return h
    uid = (ctypes.c_uint8 * UNIQUE_ID_BYTES)()
    check(lib.gs_comm_unique_id(ctypes.addressof(uid)), "gs_comm_unique_id")
    h = ctypes.c_void_p()
    check(lib.gs_comm_init(ctypes.addressof(uid), 1, 0, ctypes.byref(h)), "gs_comm_init")
    return h.value


def comm_info(handle: int) -> dict:
    """{"nranks", "rank", "transport"} as the communicator itself reports them."""
    n, r, t = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    check(lib.gs_comm_info(handle, ctypes.byref(n), ctypes.byref(r), ctypes.byref(t)), "gs_comm_info")
    return {"nranks": n.value, "rank": r.value, "transport": "xgmi" if t.value == 1 else "rccl"}


def destroy_comm(handle: Optional[int]) -> None:
    if handle:
        check(lib.gs_comm_destroy(handle), "gs_comm_destroy")
