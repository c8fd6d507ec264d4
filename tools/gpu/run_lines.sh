#!/bin/bash
# GPU box: the round's bench lines only (C2 default line, C2 bf16, C3, C4, C4 bf16, C5) with the
# committed profiles/ tables in place, so their traffic fields read the current PMC records.
# Warmup 2: the rollout graph is captured on the second collect, outside the timed steps.
# Outputs under gpurun_out/$TAG/.  Each step under its own limit; the chain stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-lines}; mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)" >&2; shift; "$@"; rc=$?; echo "rc=$rc" >&2; return $rc; }
step c2 timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
step c2bf16 timeout -k 10 400 python bench.py --dtype bf16 --cpu-minibatches 0 > $O/bench_c2_bf16.json 2> $O/bench_c2_bf16.err || exit 1
step c3 timeout -k 10 400 python bench.py --workload C3 --steps 3 --warmup 2 --cpu-minibatches 0 > $O/bench_C3.json 2> $O/bench_C3.err || exit 1
step c4 timeout -k 10 400 python bench.py --workload C4 --steps 3 --warmup 2 > $O/bench_C4.json 2> $O/bench_C4.err || exit 1
step c4bf16 timeout -k 10 400 python bench.py --workload C4 --dtype bf16 --steps 3 --warmup 2 --cpu-minibatches 0 > $O/bench_c4_bf16.json 2> $O/bench_c4_bf16.err || exit 1
step c5 timeout -k 10 400 python bench.py --workload C5 --steps 3 --warmup 2 > $O/bench_C5.json 2> $O/bench_C5.err || exit 1
exit 0
