"""Diagnostic A/B variants of the library for same-box comparisons (tools/stamp_run.py --lib).

Usage (here, on the CPU):  python tools/ab_build.py NAME [EXPERIMENT|DEFINE ...]
builds tools/libgsamd_NAME.so with GS_SPANS plus the named experiments (source substitutions from
tools/ab_experiments.py, applied to a copy of csrc/) and any other -D defines; tools/run_ab.sh then
times it against the plain spans variant alternately in one GPU call, so box-to-box variation does
not enter the comparison.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gymnasium-solver_amd")]
import build_lib  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "tools"))
from ab_experiments import EXPERIMENTS  # noqa: E402

name, args = sys.argv[1], sys.argv[2:]
patches = [p for a in args if a in EXPERIMENTS for p in EXPERIMENTS[a]]
defines = [a for a in args if a not in EXPERIMENTS]
out = os.path.join(ROOT, "tools", f"libgsamd_{name}.so")
build_lib.build_variant(out, ["GS_SPANS"] + defines, patches=patches, tag=name if patches else "")
print("built", out)
