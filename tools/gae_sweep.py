"""GAE scan throughput sweep on the GPU (gs_gae_f32 through the C-ABI).

For each (T, N): random inputs resident in HBM, `reps` launches captured into a hipGraph and
replayed between HIP events on the launch stream; reports µs per launch, algorithmic GB/s
(22 B/element + 4 B/env) and the fraction of the 8 TB/s HBM peak.  Every size
is also checked bit-exact against the C oracle (small sizes) or against the first-call result
(replays must be idempotent).

    python tools/gae_sweep.py [--reps 50] [--json gpurun_out/gae_sweep.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gymnasium-solver_amd")]

PEAK_HBM_GBS = 8000.0
SIZES = [(32, 4096), (32, 8192), (128, 1024), (256, 256), (128, 8192), (2048, 1024), (2048, 8192), (512, 32768)]


def gae_bytes(T: int, N: int) -> int:
    return 22 * T * N + 4 * N


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    from gsamd.rollout import compute_batched_gae_advantages_and_returns as gae
    dev = torch.device("cuda:0")
    out = []
    for T, N in SIZES:
        g = torch.Generator(device=dev).manual_seed(T * 31 + N)
        v = torch.randn(T, N, device=dev, generator=g)
        r = torch.randn(T, N, device=dev, generator=g)
        d = (torch.rand(T, N, device=dev, generator=g) < 0.05).to(torch.uint8)
        to = (d.bool() & (torch.rand(T, N, device=dev, generator=g) < 0.3)).to(torch.uint8)
        lv = torch.randn(N, device=dev, generator=g)
        b = torch.randn(T, N, device=dev, generator=g)
        adv = torch.empty(T, N, device=dev)
        ret = torch.empty(T, N, device=dev)
        gae(v, r, d, to, lv, b, 0.99, 0.95, adv_out=adv, ret_out=ret)
        torch.cuda.synchronize()
        first = adv.clone(), ret.clone()
        exact = None
        if T * N <= 1 << 18:
            import oracle
            a_ref, r_ref = oracle.gae_c(v.cpu().numpy(), r.cpu().numpy(), d.cpu().numpy(), to.cpu().numpy(),
                                        lv.cpu().numpy(), b.cpu().numpy(), 0.99, 0.95)
            exact = bool(np.array_equal(adv.cpu().numpy().view(np.uint32), a_ref.view(np.uint32))
                         and np.array_equal(ret.cpu().numpy().view(np.uint32), r_ref.view(np.uint32)))
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, capture_error_mode="thread_local"):
            for _ in range(args.reps):
                gae(v, r, d, to, lv, b, 0.99, 0.95, adv_out=adv, ret_out=ret)
        graph.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        graph.replay()
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) / args.reps * 1e3
        same = bool(torch.equal(adv, first[0]) and torch.equal(ret, first[1]))
        gbs = gae_bytes(T, N) / (us * 1e-6) / 1e9
        row = {"T": T, "N": N, "us": round(us, 3), "bytes": gae_bytes(T, N), "GBps": round(gbs, 1),
               "frac": round(gbs / PEAK_HBM_GBS, 4), "oracle_exact": exact, "replay_identical": same}
        print(json.dumps(row), flush=True)
        out.append(row)
        del graph
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)
    if not all(r["replay_identical"] and r["oracle_exact"] is not False for r in out):
        raise SystemExit("GAE mismatch")


if __name__ == "__main__":
    main()
