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


def xgmi_self_test(handle: int, rank: int, world_size: int, n: int, device: torch.device, rounds: int = 3) -> bool:
    """Exchange known vectors a few times and compare every element with the exact
    fixed-order answer (also proves the peers' flags arrive)."""
    import numpy as np
    from ._lib import stream_handle
    idx = np.arange(n, dtype=np.int64)
    for it in range(rounds):
        vals = [((r + 1) * (it + 3) + (idx * (r + 5) + it) % 11).astype(np.float32) for r in range(world_size)]
        buf = torch.from_numpy(vals[rank]).to(device)
        check(lib.gs_comm_allreduce_mean_f32(handle, buf.data_ptr(), n, stream_handle()), "gs_comm_allreduce_mean_f32")
        acc = vals[0]
        for r in range(1, world_size):
            acc = acc + vals[r]
        want = acc * np.float32(1.0 / world_size)
        got = buf.cpu().numpy()
        if lib.gs_comm_status(handle) != 0 or not np.array_equal(got.view(np.uint32), want.view(np.uint32)):
            return False
    return True


def init_xgmi_comm(rank: int, world_size: int, max_count: int, device: Optional[torch.device] = None,
                   self_test: bool = True) -> int:
    """One-shot xGMI communicator for exchanges of up to max_count floats (the policy's
    parameter count): create, all-gather the handles, open the peers, barrier, then (by
    default) a bit-exact self-test agreed on by every rank.  Raises RuntimeError on every
    rank if any rank fails (the caller may then choose RCCL instead)."""
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
            ok = xgmi_self_test(h, rank, world_size, min(int(max_count), 1 << 16), dev)
            why = "" if ok else "self-test mismatch or timeout"
        except RuntimeError as e:
            ok, why = False, str(e)
        ok = _agree(ok, device)
    if not ok:
        if h:
            destroy_comm(h)
        raise RuntimeError(f"xGMI exchange unavailable on rank {rank}: {why or 'a peer failed'}")
    return h


def exchange_inside_bwd(handle: int, dims, batch: int) -> bool:
    """Whether the fused MLP update exchanges gradients inside its backward kernel on this
    communicator (include/gsamd.h gs_ppo_exchange_inside_bwd)."""
    v = ctypes.c_int()
    check(lib.gs_ppo_exchange_inside_bwd(handle, dims, int(batch), ctypes.byref(v)), "gs_ppo_exchange_inside_bwd")
    return bool(v.value)


def comm_status(handle: Optional[int]) -> None:
    """Raise if an exchange on this communicator timed out waiting for a peer."""
    if handle:
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
