#!/bin/bash
# GPU-box: the xGMI test file (colocated exchange-launch grid cap), the C2 bench line + rocprof stats
# (run_r03d.sh), then the same-box pricing A/B of timing-only variants (tools/run_ab.sh, 2 rounds).
cd "$GRAFT_REPO_ROOT" || exit 1
PYTEST_SEL=${PYTEST_SEL:-tests/test_gpu_xgmi.py} bash tools/gpu/run_r03d.sh || exit 1
[ -n "$AB" ] || exit 0
mkdir -p gpurun_out/ab
for i in 1 2; do
  for v in spans $AB; do
    timeout -k 10 120 python tools/stamp_run.py --spans --lib "tools/libgsamd_$v.so" > "gpurun_out/ab/$v.$i.log" 2>&1 || exit 1
    echo "$v run $i: $(grep -E 'minibatch period|fwd span|bwd span' gpurun_out/ab/$v.$i.log | awk '{printf "%s %s %s | ", $1, $2, $(NF-6)}')"
  done
done
