#!/usr/bin/env python3
"""Per-kernel mean of every counter in rocprofv3 --pmc csv outputs (one or more directories):
python tools/pmc_chain_summary.py DIR [DIR ...] -> JSON on stdout."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main(dirs):
    acc = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                k = row.get("Kernel_Name", "")
                short = k.split("(")[0].split("<")[0].replace("void ", "").replace("gs::", "")
                if "fwd_hidden" in k and "true, true" in k:
                    short = "k_fwd_hidden<fused,adam>"
                acc[short][row["Counter_Name"]].append(float(row["Counter_Value"]))
    out = {k: {c: sum(v[8:]) / max(1, len(v[8:])) for c, v in cs.items()} for k, cs in acc.items()}
    json.dump(out, sys.stdout, indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1:])
