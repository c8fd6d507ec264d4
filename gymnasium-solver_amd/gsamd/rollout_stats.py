"""Host-side rolling window (utils/rollout_stats.py:6-31 RollingWindow semantics)."""
from collections import deque


class RollingWindow:
    def __init__(self, maxlen: int):
        if maxlen <= 0:
            raise ValueError("RollingWindow maxlen must be > 0")
        self._dq = deque(maxlen=int(maxlen))
        self._sum = 0.0

    def append(self, value: float) -> None:
        if len(self._dq) == self._dq.maxlen:
            self._sum -= float(self._dq[0])
        self._dq.append(value)
        self._sum += float(value)

    def mean(self) -> float:
        return self._sum / len(self._dq) if self._dq else 0.0

    def __len__(self) -> int:
        return len(self._dq)

    def __bool__(self) -> bool:
        return len(self._dq) > 0
