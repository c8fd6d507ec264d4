#!/usr/bin/env python3
"""Per-kernel rooflines of the NatureCNN minibatch step (C4 shapes) from three rocprofv3 runs of
tools/cnn_kernel_run.py: --kernel-trace (durations), --pmc FETCH_SIZE and --pmc WRITE_SIZE (HBM
bytes; separate passes).  Every minibatch dispatches the same kernels in the same order
(gs_cnn.hip cnn_step: forward, head + loss, head weight gradient, backward, the fused tail, clip + Adam), so each dispatch is named
by its position in the minibatch and the three runs line up position by position.

Per kernel: average duration over the measured minibatches, algorithmic FLOPs (2 x MACs of the
layer's product) and algorithmic bytes (each operand read once, each output written once, u8
frames; fp32 activations, or with --bf16 the bf16 update's storage: bf16 activations, dh and
weight operands), the HBM bytes the counters saw (2 x FETCH_SIZE + WRITE_SIZE, KB -> B:
the gfx950 FETCH_SIZE correction of MI355X_MICROARCH.md), the MFMA fraction against the dense
peak of the operand type and the HBM fraction against 8 TB/s.

  python tools/cnn_kernel_summary.py gpurun_out/r03 [--bf16] > profiles/r03_c4_kernels.json"""
import argparse
import csv
import glob
import json
import os
import re
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gymnasium-solver_amd"))
from gsamd.buildinfo import source_hash  # noqa: E402

PEAK_F32_MFMA = 157.3     # TFLOP/s, dense fp32 matrix (MI355X_MICROARCH.md)
PEAK_BF16_MFMA = 2500.0   # TFLOP/s, dense bf16 matrix
PEAK_HBM = 8000.0         # GB/s

# position in the minibatch -> (label, expected kernel): the update's dispatch sequence
# (gs_cnn.hip cnn_step): the fc layer's three products on the hand-written k_fc kernels
# (csrc/gs_fc.hip), the fused head + loss pair, the LDS-resident conv kernels
SEQ_FC = [("conv1_fwd", "k_conv1_fwd"), ("conv2_fwd", "k_conv_fwd"), ("conv3_fwd", "k_conv_fwd"),
          ("fc_fwd", "k_fc"), ("head_loss", "k_cnn_head_loss"), ("head_wgrad_metrics", "k_cnn_head_wgrad"),
          ("fc_wgrad", "k_fc"), ("fc_dgrad_relu_mask", "k_fc"),
          ("conv3_wgrad", "k_conv_wgrad"), ("conv3_wgrad_sum", "k_sum_parts"),
          ("conv3_dgrad", "k_conv_dgrad"), ("conv2_wgrad", "k_conv_wgrad"), ("conv2_wgrad_sum", "k_sum_parts"),
          ("conv2_dgrad", "k_conv_dgrad"), ("conv1_wgrad", "k_conv1_wgrad"),
          ("tail_conv1_sum_head_combine_norm", "k_conv1_sum_norm"), ("clip_adam", "k_clip_adam_flat")]
# (round 6: the head weight gradient's own kernel replaced k_cnn_head_wsum; the fused backward tail
# k_conv1_sum_norm sums conv1's weight-gradient partials, adds the head blocks and writes the norm
# partials, replacing the conv1 partial sum and k_norm_partials)
# the fp32 update (round 5): the fc forward as two K halves + k_fc_sum (the bias + ReLU epilogue)
SEQ_FC_SPLIT = SEQ_FC[:4] + [("fc_fwd_splitk_sum", "k_fc_sum")] + SEQ_FC[4:]
SEQ = SEQ_FC


def nature_work(B, A=18, C=4, H=84, W=84, store16=False):
    """(flops, bytes) per MFMA layer product of one minibatch of B rows.  store16: the bf16 update's
    storage (gs_cnn.hip trunk_bf16_storage) — the activations a1 / a2 / a3, dh and the weight
    operands cross HBM as bf16; gradients, h, z and biases stay fp32."""
    f = 4
    ea = ew = ed = 2 if store16 else f          # activation / weight-operand / dh element bytes
    h1, w1, c1, K1 = (H - 8) // 4 + 1, (W - 8) // 4 + 1, 32, C * 64
    h2, w2, c2, K2 = (h1 - 4) // 2 + 1, (w1 - 4) // 2 + 1, 64, c1 * 16
    h3, w3, c3, K3 = h2 - 2, w2 - 2, 64, c2 * 9
    F, HID, A1 = c3 * h3 * w3, 512, A + 1
    frames = B * C * H * W                     # u8
    n1, n2, n3 = B * h1 * w1 * c1, B * h2 * w2 * c2, B * F     # activation elements
    hb, zb = B * HID * f, B * A1 * f
    p1, p2, p3, pf, Wh = c1 * K1, c2 * K2, c3 * K3, HID * F, A1 * HID * f     # weight elements
    m1, m2, m3, mf, mh = B * h1 * w1 * c1 * K1, B * h2 * w2 * c2 * K2, B * h3 * w3 * c3 * K3, B * F * HID, B * HID * A1
    return {
        "conv1_fwd": (2 * m1, frames + p1 * ew + n1 * ea), "conv2_fwd": (2 * m2, n1 * ea + p2 * ew + n2 * ea),
        "conv3_fwd": (2 * m3, n2 * ea + p3 * ew + n3 * ea), "fc_fwd": (2 * mf, n3 * ea + pf * ew + hb),
        "heads_fwd": (2 * mh, hb + Wh + zb), "heads_wgrad": (2 * mh, zb + hb + Wh),
        "fc_wgrad": (2 * mf, B * HID * ed + n3 * ea + pf * f),
        "fc_dgrad": (2 * mf, B * HID * ed + pf * ew + n3 * f),
        "fc_dgrad_relu_mask": (2 * mf, B * HID * ed + pf * ew + n3 * f + n3 * ea),     # + the ReLU mask read
        "conv3_wgrad": (2 * m3, n2 * ea + n3 * f + p3 * f), "conv3_dgrad": (2 * m3, n3 * f + p3 * ew + n2 * f + n2 * ea),
        "conv2_wgrad": (2 * m2, n1 * ea + n2 * f + p2 * f), "conv2_dgrad": (2 * m2, n2 * f + p2 * ew + n1 * f + n1 * ea),
        "conv1_wgrad": (2 * m1, frames + n1 * f + p1 * f),
        "head_loss": (4 * mh, hb + Wh + zb + B * HID * ed),    # z = h Wh^T and dh = relu'(h) (dz Wh) (+ dh out)
        "head_wgrad_metrics": (2 * mh, hb + zb + Wh),          # [dWh | dbf] = dz^T [h | 1]
    }


def short(name):
    m = re.search(r"\b(k_\w+)", name)
    if m and m.group(1) == "k_conv1_wgrad_bf":    # the bf16 conv1 weight gradient (same position)
        return "k_conv1_wgrad"
    if m and m.group(1) in ("k_sum_parts_wb", "k_sum_partials", "k_sum_parts4", "k_sum_parts_tiles"):   # partial sums
        return "k_sum_parts"
    if m and m.group(1) == "k_fc16":      # the fp32 fc kernels on 16x16x4 MFMA blocks (same positions)
        return "k_fc"
    return m.group(1) if m else None


def minibatches(rows):
    """rows (dicts) in dispatch order -> list of per-minibatch dispatch lists (gs kernels only)."""
    gs = [r for r in rows if short(r["Kernel_Name"]) is not None]
    starts = [i for i, r in enumerate(gs) if short(r["Kernel_Name"]) == SEQ[0][1]]
    out = []
    for a, b in zip(starts, starts[1:] + [len(gs)]):
        mb = gs[a:b]
        if len(mb) >= len(SEQ):
            out.append(mb[:len(SEQ)])
    return out


def check_seq(mb):
    for (label, k), r in zip(SEQ, mb):
        got = short(r["Kernel_Name"])
        if got != k:
            raise SystemExit(f"dispatch order changed: position {label} expected {k}, got {got}")


def load_trace(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return rows


def load_pmc(path, counter):
    rows = [r for r in csv.DictReader(open(path)) if r.get("Counter_Name") == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return rows


def one(pattern):
    hits = sorted(glob.glob(pattern, recursive=True))
    if not hits:
        raise SystemExit(f"no file matches {pattern}")
    return hits[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir", help="directory holding cnn_stats/, cnn_fetch/, cnn_write/")
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--bf16", action="store_true", help="the run used GS_HP_BF16 (bf16 MFMA peak)")
    ap.add_argument("--skip", type=int, default=1, help="warm minibatches to drop")
    ap.add_argument("--prefix", default="cnn", help="run directories <prefix>_stats / _fetch / _write")
    a = ap.parse_args()
    global SEQ
    rows = load_trace(one(os.path.join(a.dir, a.prefix + "_stats", "**", "*kernel_trace.csv")))
    if any(short(r["Kernel_Name"]) == "k_fc_sum" for r in rows):
        SEQ = SEQ_FC_SPLIT
    trace = minibatches(rows)[a.skip:]
    fetch = minibatches(load_pmc(one(os.path.join(a.dir, a.prefix + "_fetch", "**", "*counter_collection.csv")),
                                 "FETCH_SIZE"))[a.skip:]
    write = minibatches(load_pmc(one(os.path.join(a.dir, a.prefix + "_write", "**", "*counter_collection.csv")),
                                 "WRITE_SIZE"))[a.skip:]
    for mb in trace + fetch + write:
        check_seq(mb)
    work = nature_work(a.batch, store16=a.bf16)
    peak = PEAK_BF16_MFMA if a.bf16 else PEAK_F32_MFMA
    kernels = {}
    tot_us = tot_bytes = tot_alg = 0.0
    for i, (label, k) in enumerate(SEQ):
        us = sum((int(mb[i]["End_Timestamp"]) - int(mb[i]["Start_Timestamp"])) / 1e3 for mb in trace) / len(trace)
        fb = 2.0 * 1024 * sum(float(mb[i]["Counter_Value"]) for mb in fetch) / len(fetch) if fetch else None
        wb = 1024 * sum(float(mb[i]["Counter_Value"]) for mb in write) / len(write) if write else None
        hbm = (fb or 0.0) + (wb or 0.0)
        e = {"kernel": k, "avg_us": round(us, 3), "hbm_bytes": round(hbm), "fetch_bytes": round(fb or 0),
             "write_bytes": round(wb or 0), "hbm_GBps": round(hbm / us / 1e3, 1),
             "hbm_frac": round(hbm / us / 1e3 / PEAK_HBM, 4)}
        if label in work:
            flops, alg = work[label]
            tf = flops / us / 1e6
            e.update({"bound": "mfma", "flops": flops, "TFLOPs": round(tf, 2), "mfma_frac": round(tf / peak, 4),
                      "alg_bytes": alg, "traffic_over_alg": round(hbm / alg, 3)})
            tot_alg += alg
        else:
            e["bound"] = "hbm"
        tot_us += us
        tot_bytes += hbm
        kernels[label] = e
    flops = sum(work[l][0] for l, _ in SEQ if l in work)
    out = {"_note": __doc__.split("\n\n")[1].replace("\n", " "),
           "_source_hash": source_hash("cnn"), "batch": a.batch, "operands": "bf16" if a.bf16 else "f32",
           "mfma_peak_TFLOPs": peak, "hbm_peak_GBps": PEAK_HBM, "minibatches_measured": len(trace),
           "minibatch": {"sum_kernel_us": round(tot_us, 2), "flops": flops,
                         "TFLOPs_over_kernel_time": round(flops / tot_us / 1e6, 2),
                         "mfma_frac": round(flops / tot_us / 1e6 / peak, 4), "hbm_bytes": round(tot_bytes),
                         "alg_bytes_mfma_kernels": tot_alg},
           "kernels": kernels}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
