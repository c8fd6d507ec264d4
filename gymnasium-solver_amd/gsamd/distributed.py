"""Multi-GPU plumbing for the device path: one process per GPU, envs sharded
by rank, one RCCL communicator per process built from a unique id that rank 0 makes and
torch.distributed broadcasts.  The communicator is handed to DevicePPOAgent(comm=...) and used
inside the C-ABI for the per-minibatch gradient all-reduce; nothing else crosses GPUs."""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from ._lib import check, lib

UNIQUE_ID_BYTES = 128


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


def init_local_comm() -> int:
    """A one-rank communicator (no torch.distributed needed): exercises the multi-GPU kernel
    chain and the RCCL call on a single GPU."""
    uid = (ctypes.c_uint8 * UNIQUE_ID_BYTES)()
    check(lib.gs_comm_unique_id(ctypes.addressof(uid)), "gs_comm_unique_id")
    h = ctypes.c_void_p()
    check(lib.gs_comm_init(ctypes.addressof(uid), 1, 0, ctypes.byref(h)), "gs_comm_init")
    return h.value


def destroy_comm(handle: Optional[int]) -> None:
    if handle:
        check(lib.gs_comm_destroy(handle), "gs_comm_destroy")
