"""Diagnostic: per-phase cycle breakdown of the minibatch kernels (GS_STAMPS build).

Usage (on the GPU box):  python tools/stamp_run.py
Builds nothing; expects tools/libgsamd_stamps.so (made by `python tools/stamp_run.py --build` here).
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gymnasium-solver_amd")]
VARIANT = os.path.join(ROOT, "tools", "libgsamd_stamps.so")
SPANS = os.path.join(ROOT, "tools", "libgsamd_spans.so")     # timeline only: no per-phase atomics
SPANS_ONLY = "--spans" in sys.argv

if "--build" in sys.argv:
    import build_lib
    build_lib.build_variant(VARIANT, ["GS_STAMPS"])
    build_lib.build_variant(SPANS, ["GS_SPANS"])
    print("built", VARIANT, SPANS)
    sys.exit(0)
if SPANS_ONLY:
    VARIANT = SPANS
if "--lib" in sys.argv:      # an experiment variant (tools/ab_build.py)
    VARIANT = os.path.join(ROOT, sys.argv[sys.argv.index("--lib") + 1])

os.environ["GSAMD_LIB"] = VARIANT
import numpy as np  # noqa: E402
import torch  # noqa: E402
from gsamd import _lib  # noqa: E402
from gsamd.config import load_config  # noqa: E402
from gsamd.ppo_agent import DevicePPOAgent  # noqa: E402

if not SPANS_ONLY:
    _lib.lib.gs_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
torch.manual_seed(42)
cfg = load_config("CartPole-v1", "ppo", overrides=dict(env_dynamics="synthetic", n_envs=4096))
agent = DevicePPOAgent(cfg, device="cuda:0", use_graph=True, track_stats=False)
agent.train_epoch()
torch.cuda.synchronize()
acc0 = np.zeros(128, np.uint64)
cnt0 = np.zeros(8, np.uint64)
if not SPANS_ONLY:
    _lib.lib.gs_debug_stamps(acc0.ctypes.data, cnt0.ctypes.data)
_lib.lib.gs_debug_span_reset.argtypes = []
_lib.lib.gs_debug_span_read.argtypes = [ctypes.c_void_p]
_lib.lib.gs_debug_span_reset()
agent.train_epoch()
torch.cuda.synchronize()
span = np.zeros((2, 2048, 288, 9), np.uint32)   # start + up to 8 wave ends (0 = no such wave)
_lib.lib.gs_debug_span_read(span.ctypes.data)
acc = np.zeros(128, np.uint64)
cnt = np.zeros(8, np.uint64)
if not SPANS_ONLY:
    _lib.lib.gs_debug_stamps(acc.ctypes.data, cnt.ctypes.data)
acc = (acc - acc0).reshape(8, 16).astype(np.float64)
cnt = (cnt - cnt0).astype(np.float64)
names = {0: ("k_fwd_hidden<fused, adam> (0,0)", ["loads landed (waitcnt: stamp build only)", "W1 fold + norm",
                                                  "adam (W1, W2 rows, slices)", "operands in LDS", "h1", "mfma h2",
                                                  "h2 out + heads"]),
         1: ("k_loss", ["inputs + adv norm", "per-row loss/grad", "reduce", "metrics"]),
         2: ("k_bwd roleA blk0", ["load tiles", "dh2", "mfma dW2", "store + sumsq + db2"]),
         3: ("k_clip_adam blk0", ["own loads + LDS staging", "W1 fold + norm loops", "reduce", "adam"]),
         4: ("k_bwd roleB blk0", ["load slab", "dh2", "mfma dh1", "dW1 partial"]),
         5: ("k_bwd roleC blk0", ["load", "reduce + store"]),
         6: ("k_bwd roleB slab loads (wave 0, from role start)", ["landed"]),
         7: ("k_bwd roleB loss rows (wave 3, from role start)", ["done"])}
for k, (n, phases) in names.items():
    if cnt[k] == 0:
        continue
    per = acc[k] / cnt[k]
    tot = per[:len(phases)].sum()
    print(f"{n:18s} launches {int(cnt[k]):6d}  total {tot:8.0f} cyc = {tot / 2.4e3:6.2f} us")
    for i, ph in enumerate(phases):
        print(f"    {ph:24s} {per[i]:8.0f} cyc  {per[i] / 2.4e3:6.2f} us")

# chain timeline of the second update's first 2048 minibatches (100 MHz device clock -> us):
# kernel spans from the first workgroup start to the last wave end, and the gaps between kernels
n = min(agent.n_minibatches, 2048)
sp = span[:, :n].astype(np.int64)
ref = int(sp[0, 0, 0, 0])
rel = ((sp - ref + 2**31) % 2**32 - 2**31).astype(np.float64) / 100.0   # wrap-safe, us
live = span[:, :n, :, 0] != 0                                           # workgroups that ran
st = np.where(live, rel[..., 0], np.inf).min(axis=2)                     # (2, n) first start
wlive = live[..., None] & (span[:, :n, :, 1:] != 0)                     # waves that exist
en = np.where(wlive, rel[..., 1:], -np.inf).max(axis=(2, 3))            # (2, n) last wave end
wg_end = np.where(live, np.where(wlive, rel[..., 1:], -np.inf).max(axis=3), np.nan)   # per-workgroup end
pct = lambda x: f"mean {np.mean(x):6.2f}  p10 {np.percentile(x, 10):6.2f}  p50 {np.median(x):6.2f}  p90 {np.percentile(x, 90):6.2f}"
print(f"chain timeline over {n} minibatches (us)")
print("    fwd span (first WG start -> last wave end)", pct(en[0] - st[0]))
print("    fwd end -> bwd first WG start             ", pct(st[1] - en[0]))
print("    bwd span                                   ", pct(en[1] - st[1]))
print("    bwd end -> next fwd first WG start         ", pct(st[0, 1:] - en[1, :-1]))
print("    minibatch period (fwd start -> next)       ", pct(np.diff(st[0])))
# which workgroups end last: per kernel, the mean (end - kernel start) of each workgroup
for kern, name, nwg in ((0, "fwd", 256), (1, "bwd", 273)):
    e = np.nanmean(wg_end[kern, :, :nwg] - st[kern][:, None], axis=0)
    s0 = np.nanmean(rel[kern, :, :nwg, 0] - st[kern][:, None], axis=0)
    order = np.argsort(-e)[:6]
    print(f"    {name}: latest-ending workgroups " + ", ".join(f"#{w} start {s0[w]:.2f} end {e[w]:.2f}" for w in order))
    print(f"    {name}: workgroup start spread p50 {np.median(s0):.2f} max {s0.max():.2f}; end p50 {np.median(e):.2f}")
    if kern == 1:      # k_bwd dispatch order: role B, role A, role C (C2: 128 / 128 / 17 workgroups)
        nBw = nAw = 128
        for rname, lo, hi in (("B", 0, nBw), ("A", nBw, nBw + nAw), ("C", nBw + nAw, nwg)):
            r = e[lo:hi]
            print(f"    bwd role {rname}: end mean {r.mean():.2f} p90 {np.percentile(r, 90):.2f} max {r.max():.2f}")
