#!/bin/bash
# GPU-box evidence, round 3 (re-entry): the whole GPU suite, the default C2 bench line and the
# same command under rocprofv3 kernel-trace stats.  Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r03d}; mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)" >&2; shift; "$@"; rc=$?; echo "rc=$rc" >&2; return $rc; }
if [ -z "$NO_TESTS" ]; then
  step pytest timeout -k 10 900 python -u -m pytest ${PYTEST_SEL:-tests} -x -v -m gpu -p no:cacheprovider --durations=0 --timeout 300 \
      --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/pytest.log | tail -30; [ $rc -eq 0 ] || exit $rc
fi
step bench timeout -k 10 300 python bench.py ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err && cat $O/bench.json &&
step bench-rocprof timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/stats -o bench --output-format csv -- python bench.py --cpu-minibatches 0 ${BENCH_ARGS} > $O/bench_prof.log 2>&1
rc=$?
rm -f $O/stats/*kernel_trace.csv
find $O -name "*.csv" | xargs ls -la
exit $rc
