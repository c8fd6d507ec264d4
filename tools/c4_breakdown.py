#!/usr/bin/env python3
"""Per-minibatch kernel breakdown of a C4 rocprofv3 --stats CSV (bench --steps 1 --warmup 1:
two updates of n_minibatches each)."""
import csv
import re
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/c4/prof/c4_kernel_stats.csv"
n_mb = int(sys.argv[2]) if len(sys.argv) > 2 else 1920
rows = list(csv.DictReader(open(path)))
tot = 0.0
for r in rows[:26]:
    m = re.search(r"(k_\w+)(<[^(]*)?", r["Name"])
    short = (m.group(1) + (m.group(2) or "")[:50]) if m else r["Name"][:60]
    per = float(r["TotalDurationNs"]) / n_mb / 1e3
    tot += per
    print(f"{short:70s} calls={r['Calls']:>6} avg={float(r['AverageNs']) / 1e3:8.1f}us per_mb={per:8.1f}us")
print(f"sum of listed per_mb: {tot:.1f} us")
