"""Diagnostic A/B variants of the library for same-box comparisons (tools/stamp_run.py --lib).

Usage (here, on the CPU):  python tools/ab_build.py NAME DEFINE [DEFINE ...]
builds tools/libgsamd_NAME.so with GS_SPANS plus the given -D defines (experiment switches in the
sources, e.g. GS_EXP_SPLIT_STORES); tools/run_ab.sh then times it against the plain spans variant
alternately in one GPU call, so box-to-box variation does not enter the comparison.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gymnasium-solver_amd")]
import build_lib  # noqa: E402

name, defines = sys.argv[1], sys.argv[2:]
out = os.path.join(ROOT, "tools", f"libgsamd_{name}.so")
build_lib.build_variant(out, ["GS_SPANS"] + defines)
print("built", out)
