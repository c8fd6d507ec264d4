#!/bin/bash
# GPU-box evidence run for round 3: selected tests, the C2 bench line and its rocprof stats, the
# per-kernel C4 passes (stats + FETCH_SIZE + WRITE_SIZE).  Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03; mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)" >&2; shift; "$@"; rc=$?; echo "rc=$rc" >&2; return $rc; }
if [ -n "$PYTEST_SEL" ]; then
  step pytest timeout -k 10 1000 python -u -m pytest $PYTEST_SEL -x -v -m gpu -p no:cacheprovider --timeout 300 \
      --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; grep -E "PASSED|FAILED|ERROR|SKIPPED|passed|failed" $O/pytest.log | tail -70; [ $rc -eq 0 ] || exit $rc
fi
[ -n "$NO_BENCH" ] && exit 0
if [ -z "$SKIP_C2" ]; then
  step bench timeout -k 10 400 python bench.py ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err && cat $O/bench.json || exit 1
fi
[ -n "$ONLY_C2" ] && exit 0
step cnn-stats timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cnn_stats -o cnn -- python tools/cnn_kernel_run.py > $O/cnn_stats.log 2>&1 &&
step cnn-fetch timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/cnn_fetch -o fetch -- python tools/cnn_kernel_run.py > $O/cnn_fetch.log 2>&1 &&
step cnn-write timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/cnn_write -o write -- python tools/cnn_kernel_run.py > $O/cnn_write.log 2>&1 &&
[ -n "$CNN_BF16" ] && {
  step cnn16-stats timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cnn16_stats -o cnn -- python tools/cnn_kernel_run.py --bf16 > $O/cnn16_stats.log 2>&1 &&
  step cnn16-fetch timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/cnn16_fetch -o fetch -- python tools/cnn_kernel_run.py --bf16 > $O/cnn16_fetch.log 2>&1 &&
  step cnn16-write timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/cnn16_write -o write -- python tools/cnn_kernel_run.py --bf16 > $O/cnn16_write.log 2>&1 || exit 1
}
step c4-f32 timeout -k 10 400 python bench.py --workload C4 --steps 1 --warmup 1 --cpu-minibatches 0 > $O/bench_c4.json 2> $O/bench_c4.err && cat $O/bench_c4.json &&
step c4-bf16 timeout -k 10 400 python bench.py --workload C4 --steps 1 --warmup 1 --cpu-minibatches 0 --dtype bf16 > $O/bench_c4_bf16.json 2> $O/bench_c4_bf16.err && cat $O/bench_c4_bf16.json
rc=$?
find $O -name "*.csv" | xargs ls -la
exit $rc
