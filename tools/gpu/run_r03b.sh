#!/bin/bash
# GPU-box evidence, round 3 (second script): bf16 per-kernel C4 passes, C3 / C5 bench lines.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03; mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)" >&2; shift; "$@"; rc=$?; echo "rc=$rc" >&2; return $rc; }
step cnn16-stats timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cnn16_stats -o cnn -- python tools/cnn_kernel_run.py --bf16 > $O/cnn16_stats.log 2>&1 &&
step cnn16-fetch timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/cnn16_fetch -o fetch -- python tools/cnn_kernel_run.py --bf16 > $O/cnn16_fetch.log 2>&1 &&
step cnn16-write timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/cnn16_write -o write -- python tools/cnn_kernel_run.py --bf16 > $O/cnn16_write.log 2>&1 &&
step c5 timeout -k 10 400 python bench.py --workload C5 --steps 1 --warmup 1 --cpu-minibatches 0 > $O/bench_c5.json 2> $O/bench_c5.err && cat $O/bench_c5.json &&
step c3 timeout -k 10 600 python bench.py --workload C3 --steps 1 --warmup 1 --cpu-minibatches 0 > $O/bench_c3.json 2> $O/bench_c3.err && cat $O/bench_c3.json
