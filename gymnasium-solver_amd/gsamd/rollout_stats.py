"""Host-side episode window of the collector (the reference keeps its episode statistics in
utils/rollout_stats.py:6-31).

A fixed-capacity ring of the most recent values plus a running total.  The total is updated
with the same float operations, in the same order, as the reference's window — when full,
the evicted value is subtracted first, then the new value is added — so ``mean()`` agrees
with the reference's ``roll/ep_rew/mean`` / ``roll/ep_len/mean`` bit for bit.
"""
from __future__ import annotations


class RollingWindow:
    __slots__ = ("_ring", "_size", "_next", "_total")

    def __init__(self, capacity: int):
        capacity = int(capacity)
        if capacity < 1:
            raise ValueError(f"window capacity must be >= 1, got {capacity}")
        self._ring = [0.0] * capacity
        self._size = 0          # values held (<= capacity)
        self._next = 0          # slot the next value goes to (the oldest one once full)
        self._total = 0.0

    def append(self, value) -> None:
        if self._size == len(self._ring):
            self._total -= float(self._ring[self._next])
        else:
            self._size += 1
        self._ring[self._next] = value
        self._next = (self._next + 1) % len(self._ring)
        self._total += float(value)

    def mean(self) -> float:
        return self._total / self._size if self._size else 0.0

    def __len__(self) -> int:
        return self._size

    def __bool__(self) -> bool:
        return self._size > 0
