"""Identity of the kernel sources a measurement was taken with (no device import).

bench.py reports PMC traffic (profiles/pmc_traffic.json, tools/pmc_summarize.py) only when the
file was recorded from the same csrc/ sources as the library being benchmarked; otherwise the
traffic figure would describe another kernel and is reported as null."""
from __future__ import annotations

import hashlib
import os

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc")


# the sources each measured path is compiled from: the MLP minibatch chain + GAE (C2/C3 PMC
# passes, tools/pmc_run.py) and the NatureCNN update (C4 per-kernel passes, tools/cnn_kernel_run.py)
PATH_SOURCES = {
    "mlp": ("gs_mlp.hip", "gs_ppo.hip", "gs_gae.hip", "gs_common.h", "gs_xgmi_dev.h", "gs_synth_env.h"),
    "cnn": ("gs_cnn.hip", "gs_conv.hip", "gs_gemm.hip", "gs_fc.hip", "gs_common.h", "gs_conv.h", "gs_gemm.h"),
}


def source_hash(path: str = None, csrc: str = CSRC) -> str:
    """sha256 (first 16 hex digits) over the names and bytes of the kernel sources, sorted: of
    PATH_SOURCES[path] when given ("mlp" / "cnn"), else of every csrc/*.{hip,h,cpp}."""
    h = hashlib.sha256()
    names = PATH_SOURCES[path] if path else [n for n in os.listdir(csrc) if n.endswith((".hip", ".h", ".cpp"))]
    for name in sorted(names):
        h.update(name.encode())
        with open(os.path.join(csrc, name), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]
