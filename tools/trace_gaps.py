"""Kernel durations and the idle gaps in front of each kernel from a rocprofv3 kernel trace
(`rocprofv3 --kernel-trace --output-format csv`): the trace's dispatches sorted by start time, the
gap = this start - the previous end, grouped by kernel name (short form).  Used on the C5 collect's
captured step graph (tools/collect_run.py) to price its launch gaps.
Usage: python tools/trace_gaps.py TRACE.csv [--skip N]"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    n = name.replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*$", "", n)
    n = re.sub(r"<.*$", "", n.replace("void ", ""))
    return n.split("::")[-1]


def main():
    path = sys.argv[1]
    skip = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 0
    rows = list(csv.DictReader(open(path)))
    ks = "Kernel_Name" if "Kernel_Name" in rows[0] else "Kernel-Name"
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r[ks])) for r in rows)[skip:]
    dur, gap = defaultdict(list), defaultdict(list)
    for (s0, e0, _), (s1, e1, n1) in zip(ev, ev[1:]):
        gap[n1].append(s1 - e0)
    for s, e, n in ev:
        dur[n].append(e - s)
    print(f"{'kernel':32s} {'calls':>6s} {'dur_us':>8s} {'gap_before_us(median)':>22s}")
    tot_d = tot_g = 0.0
    for n in sorted(dur, key=lambda k: -sum(dur[k])):
        d = sorted(dur[n])
        g = sorted(gap.get(n, [0]))
        md, mg = d[len(d) // 2] / 1e3, g[len(g) // 2] / 1e3
        tot_d += sum(d) / 1e3
        tot_g += sum(x for x in g if x < 1e6) / 1e3
        print(f"{n:32s} {len(d):6d} {md:8.2f} {mg:22.2f}")
    span = (ev[-1][1] - ev[0][0]) / 1e3
    print(f"span {span:.1f} us: kernels {tot_d:.1f} us, gaps {tot_g:.1f} us")


if __name__ == "__main__":
    main()
