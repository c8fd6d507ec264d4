#!/usr/bin/env python3
"""Reduce rocprofv3 counter_collection CSVs to per-launch HBM bytes per kernel.

gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE (KB, from TCC_EA0_RDREQ x 64 B)
reports half the bytes of wide coalesced reads -> x2; WRITE_SIZE (KB) is taken as is.  The two
counters come from separate passes (TCC slots: FETCH_SIZE costs 3, WRITE_SIZE 2).
  python tools/pmc_summarize.py FETCH.csv WRITE.csv > profiles/pmc_traffic.json"""
import csv
import json
import os
import re
import sys
from collections import defaultdict

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gymnasium-solver_amd"))
from gsamd.buildinfo import source_hash  # noqa: E402

SHORT = ("k_fwd_hidden", "k_loss", "k_bwd", "k_clip_adam", "k_heads_act", "k_gae_f32", "k_gae_staged", "k_env_step",
         "k_reduce_part1", "k_sumsq_flat")
BY_GRID = ("k_gae_staged", "k_gae_f32")   # one kernel at several shapes: keyed by grid size


def short(name):
    for s in SHORT:
        if re.search(r"\b" + s + r"\b", name):
            return s
    return None


def load(path, counter):
    per = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name") != counter:
                continue
            k = short(row.get("Kernel_Name", ""))
            if k in BY_GRID:
                k = f"{k}[grid={row.get('Grid_Size', '?')}]"
            if k:
                per[k].append(float(row["Counter_Value"]))
    return per


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    out = {"_note": "HBM-side bytes per launch = 2*FETCH_SIZE + WRITE_SIZE (KB->B, gfx950 FETCH_SIZE x2 "
                    "correction per MI355X_MICROARCH.md); Infinity-Cache hits are included by the counters",
           "_source_hash": source_hash("mlp")}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [])
        w = write.get(k, [])
        fb = 2.0 * 1024 * sum(f) / len(f) if f else None
        wb = 1024 * sum(w) / len(w) if w else None
        out[k] = {"launches_fetch": len(f), "launches_write": len(w),
                  "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
                  "hbm_bytes_per_launch": (fb or 0.0) + (wb or 0.0)}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
