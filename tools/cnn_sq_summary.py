#!/usr/bin/env python3
"""Per-kernel SQ counters of the NatureCNN minibatch step: one `rocprofv3 --pmc <SQ counters>`
pass over tools/cnn_kernel_run.py, each dispatch named by its position in the minibatch (as in
tools/cnn_kernel_summary.py), each counter averaged over the measured minibatches.

  python tools/cnn_sq_summary.py gpurun_out/X/cnn_sq [--skip 1]"""
import argparse
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import cnn_kernel_summary as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--skip", type=int, default=1)
    a = ap.parse_args()
    path = sorted(glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True))[0]
    names = sorted({r["Counter_Name"] for r in csv.DictReader(open(path))})
    table = {}
    for c in names:
        mbs = K.minibatches(K.load_pmc(path, c))[a.skip:]
        for mb in mbs:
            K.check_seq(mb)
        for j, (lab, _) in enumerate(K.SEQ):
            table.setdefault(lab, {})[c] = sum(float(mb[j]["Counter_Value"]) for mb in mbs) / max(len(mbs), 1)
    short = [c.replace("SQ_", "") for c in names]
    print(f"{'kernel':22s}" + "".join(f"{s[:14]:>15s}" for s in short))
    for lab, _ in K.SEQ:
        print(f"{lab:22s}" + "".join(f"{table[lab][c]:15.4g}" for c in names))
    if "SQ_WAVE_CYCLES" in names:
        print("\nfractions of SQ_WAVE_CYCLES")
        rest = [c for c in names if c not in ("SQ_WAVE_CYCLES", "SQ_WAVES", "SQ_BUSY_CYCLES")]
        print(f"{'kernel':22s}" + "".join(f"{c.replace('SQ_', '')[:14]:>15s}" for c in rest))
        for lab, _ in K.SEQ:
            wc = table[lab]["SQ_WAVE_CYCLES"] or 1.0
            print(f"{lab:22s}" + "".join(f"{table[lab][c] / wc:15.3f}" for c in rest))


if __name__ == "__main__":
    main()
