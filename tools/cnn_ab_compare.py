"""Side-by-side per-kernel C4 update times of tools/gpu/run_cnn_ab.sh runs.

Each run directory holds one rocprofv3 kernel trace of tools/cnn_kernel_run.py; the update's
minibatches are cut out of it with tools/cnn_kernel_summary.py's launch sequence, the first
--skip dropped, and every kernel's mean duration printed (us) with the minibatch's kernel sum.

    python tools/cnn_ab_compare.py gpurun_out/r05i/intree_bf_1 gpurun_out/r05i/hr4_bf_1
"""
import argparse
import glob
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import cnn_kernel_summary as S  # noqa: E402


def per_kernel(d, skip):
    rows = S.load_trace(S.one(os.path.join(d, "**", "*kernel_trace.csv")))
    if any(S.short(r["Kernel_Name"]) == "k_fc_sum" for r in rows):
        S.SEQ = S.SEQ_FC_SPLIT
    else:
        S.SEQ = S.SEQ_FC
    mbs = S.minibatches(rows)[skip:]
    if not mbs:
        raise SystemExit(f"{d}: no complete minibatch in the trace")
    out = {}
    for i, (label, _) in enumerate(S.SEQ):
        out[label] = statistics.mean((int(mb[i]["End_Timestamp"]) - int(mb[i]["Start_Timestamp"])) / 1e3 for mb in mbs)
    return out, len(mbs)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--skip", type=int, default=2, help="warm minibatches to drop")
    a = ap.parse_args()
    res = [per_kernel(d, a.skip) for d in a.dirs]
    labels = []
    for r, _ in res:
        labels += [k for k in r if k not in labels]
    print("%-22s" % "kernel" + "".join("%14s" % os.path.basename(d.rstrip("/"))[:13] for d in a.dirs))
    for k in labels:
        print("%-22s" % k + "".join("%14s" % ("%.2f" % r[k] if k in r else "-") for r, _ in res))
    print("%-22s" % "sum" + "".join("%14.2f" % sum(r.values()) for r, _ in res))
    print("%-22s" % "minibatches" + "".join("%14d" % n for _, n in res))


if __name__ == "__main__":
    main()
