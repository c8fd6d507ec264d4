"""Identity of the kernel sources a measurement was taken with (no device import).

bench.py reports PMC traffic (profiles/pmc_traffic.json, tools/pmc_summarize.py) only when the
file was recorded from the same csrc/ sources as the library being benchmarked; otherwise the
traffic figure would describe another kernel and is reported as null."""
from __future__ import annotations

import hashlib
import os

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc")


def source_hash(csrc: str = CSRC) -> str:
    """sha256 (first 16 hex digits) over the names and bytes of csrc/*.{hip,h,cpp}, sorted."""
    h = hashlib.sha256()
    for name in sorted(os.listdir(csrc)):
        if name.endswith((".hip", ".h", ".cpp")):
            h.update(name.encode())
            with open(os.path.join(csrc, name), "rb") as f:
                h.update(f.read())
    return h.hexdigest()[:16]
