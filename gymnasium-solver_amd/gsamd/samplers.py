"""MultiPassRandomSampler with the reference's API and index stream
(utils/samplers.py:7-37), produced by libgsamd's host sampler (gs_sampler_stream_i32).

``set_epoch(e)`` re-seeds with ``base_seed + e`` (base_seed = torch.initial_seed() at
construction, as the reference reads it); Lightning calls it every epoch, and so does
the device agent.  Without a set_epoch call the reference draws from the passed
generator's running state; that stream is reproduced by delegating to the same torch
CPU calls (there is no state to re-seed from).

``IndexStreamPrefetcher`` computes the stream for the NEXT epoch on a worker thread
while the device runs the current update, and stages it through two pinned host buffers
into a device int32 buffer, so the host sampler never sits on the critical path.
"""
from __future__ import annotations

import os
import threading
from typing import Iterator, Optional

import numpy as np
import torch
from torch.utils.data import Sampler

from ._lib import check, lib


def index_stream(data_len: int, num_passes: int, seed: int, out: Optional[np.ndarray] = None,
                 n_threads: Optional[int] = None) -> np.ndarray:
    """int32 numpy array of num_passes concatenated permutations (the reference's order)."""
    if out is None:
        out = np.empty(int(data_len) * int(num_passes), np.int32)
    if n_threads is None:
        n_threads = max(1, min(int(num_passes), len(os.sched_getaffinity(0)), 16))
    check(lib.gs_sampler_stream_i32(int(data_len), int(num_passes), int(seed), out.ctypes.data, int(n_threads)),
          "gs_sampler_stream_i32")
    return out


class MultiPassRandomSampler(Sampler[int]):
    def __init__(self, data_len: int, num_passes: int, generator: Optional[torch.Generator] = None) -> None:
        if data_len <= 0:
            raise ValueError("data_len must be > 0")
        if num_passes <= 0:
            raise ValueError("num_passes must be > 0")
        self.data_len = int(data_len)
        self.num_passes = int(num_passes)
        self.generator = generator or torch.Generator()
        self._base_seed = int(torch.initial_seed())
        self._epoch_seed: Optional[int] = None

    def set_epoch(self, epoch: int) -> None:
        self._epoch_seed = self._base_seed + int(epoch)
        self.generator.manual_seed(self._epoch_seed)

    def stream(self) -> np.ndarray:
        if self._epoch_seed is not None:
            # set_epoch re-seeds before every pass over the data, so the generator's
            # state after a pass is never observed: it is not advanced here
            return index_stream(self.data_len, self.num_passes, self._epoch_seed)
        scores = torch.rand((self.num_passes, self.data_len), generator=self.generator)
        return torch.argsort(scores, dim=1).reshape(-1).numpy().astype(np.int32)

    def __iter__(self) -> Iterator[int]:
        return iter(self.stream().tolist())

    def __len__(self) -> int:
        return self.data_len * self.num_passes


class IndexStreamPrefetcher:
    """Epoch-e index streams computed ahead on a thread and uploaded to one device buffer."""

    def __init__(self, data_len: int, num_passes: int, base_seed: int, device):
        self.data_len, self.num_passes, self.base_seed = int(data_len), int(num_passes), int(base_seed)
        n = self.data_len * self.num_passes
        self.device_buf = torch.empty(n, dtype=torch.int32, device=device)
        self._host = [torch.empty(n, dtype=torch.int32).pin_memory() for _ in range(2)]
        self._events = [None, None]
        self._threads = {}

    def _work(self, epoch: int, slot: int):
        index_stream(self.data_len, self.num_passes, self.base_seed + epoch, out=self._host[slot].numpy())

    def prefetch(self, epoch: int) -> None:
        if epoch in self._threads:
            return
        slot = epoch % 2
        ev = self._events[slot]
        if ev is not None:
            ev.synchronize()          # the H2D copy that last read this pinned slot is done
        th = threading.Thread(target=self._work, args=(epoch, slot), daemon=True)
        th.start()
        self._threads[epoch] = th

    def upload(self, epoch: int, stream=None) -> torch.Tensor:
        """Stream-ordered H2D of epoch's indices into device_buf; returns device_buf."""
        self.prefetch(epoch)
        self._threads.pop(epoch).join()
        slot = epoch % 2
        s = stream or torch.cuda.current_stream()
        with torch.cuda.stream(s):
            self.device_buf.copy_(self._host[slot], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(s)
        self._events[slot] = ev
        return self.device_buf


def rank_share(stream: np.ndarray, batch: int, rank: int, samples_per_rank: int) -> np.ndarray:
    """Global-minibatch mode (include/gsamd.h gs_ppo_update_global): the global env-major index
    stream (global env g = rank * n_envs + local env, index g * T + t) cut into minibatches of
    `batch`; per minibatch, this rank's rows in stream order as local env-major indices, padded to
    `batch` entries with -1.  (n_minibatches * batch,) int32."""
    s = np.asarray(stream, np.int64).reshape(-1, int(batch))
    mine = (s // int(samples_per_rank)) == int(rank)
    order = np.argsort(~mine, axis=1, kind="stable")          # this rank's rows first, in order
    rows = np.take_along_axis(s - int(rank) * int(samples_per_rank), order, axis=1)
    keep = np.take_along_axis(mine, order, axis=1)
    return np.where(keep, rows, -1).astype(np.int32).reshape(-1)
