#!/bin/bash
# GPU box: alternate the spans variant and experiment variants (tools/libgsamd_<name>.so, built by
# tools/ab_build.py) three times each in one call and print their chain timelines, so box-to-box
# variation does not enter the comparison.  Usage: run_ab.sh NAME [NAME ...]
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab
for i in 1 2 3; do
  for v in spans "$@"; do
    timeout -k 10 200 python tools/stamp_run.py --spans --lib "tools/libgsamd_$v.so" > "gpurun_out/ab/$v.$i.log" 2>&1 || exit 1
    echo "$v run $i: $(grep -E 'minibatch period|fwd span|bwd span' gpurun_out/ab/$v.$i.log | awk '{printf "%s %s %s | ", $1, $2, $(NF-6)}')"
  done
done
