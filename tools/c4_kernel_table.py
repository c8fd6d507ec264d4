"""Per-kernel table of a rocprofv3 --stats run of tools/cnn_kernel_run.py (the update's kernels:
those called once or twice per minibatch), with the per-minibatch kernel sum.
Usage: python tools/c4_kernel_table.py STATS.csv [MINIBATCHES=7]"""
import csv
import re
import sys


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("gs::", "")
    m = re.match(r"(void )?(\w+)(<[^(]*)?", n)
    return (m.group(2) + (m.group(3) or ""))[:72]


def main():
    path = sys.argv[1]
    mb = int(sys.argv[2]) if len(sys.argv) > 2 else 7
    rows = list(csv.DictReader(open(path)))
    tot = 0.0
    for r in sorted(rows, key=lambda r: -float(r["AverageNs"])):
        c, v = int(r["Calls"]), float(r["AverageNs"]) / 1e3
        if mb <= c <= 2 * mb and "Fill" not in r["Name"]:
            tot += v * c / mb
            print(f"{short(r['Name']):72s} {c:4d} {v:8.2f}")
    print(f"kernel sum per minibatch {tot:.1f} us")


if __name__ == "__main__":
    main()
