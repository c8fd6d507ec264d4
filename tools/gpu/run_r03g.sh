#!/bin/bash
# GPU-box evidence for the final round-3 build: the whole GPU suite, the default C2 bench line
# and its rocprof kernel stats, the PMC passes (FETCH_SIZE / WRITE_SIZE, separate) over
# tools/pmc_run.py, the chain timeline, the C3 line.  Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r03g}; mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)" >&2; shift; "$@"; rc=$?; echo "rc=$rc" >&2; return $rc; }
if [ -z "$NO_TESTS" ]; then
  step pytest timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --durations=10 --timeout 170 \
      --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/pytest.log | tail -5; [ $rc -eq 0 ] || exit $rc
fi
step bench timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err && cat $O/bench.json &&
step bench-rocprof timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/stats -o bench --output-format csv -- python bench.py --cpu-minibatches 0 > $O/bench_prof.log 2>&1 &&
step pmc-fetch timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o pmc -- python tools/pmc_run.py > $O/pmc_fetch.log 2>&1 &&
step pmc-write timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write -o pmc -- python tools/pmc_run.py > $O/pmc_write.log 2>&1 &&
step spans timeout -k 10 200 python tools/stamp_run.py --spans > $O/spans_c2.log 2>&1 &&
step c3 timeout -k 10 400 python bench.py --workload C3 --steps 1 --warmup 1 --cpu-minibatches 0 > $O/bench_c3.json 2> $O/bench_c3.err && cat $O/bench_c3.json
rc=$?
if [ $rc -eq 0 ] && [ -n "$AB" ]; then
  mkdir -p $O/ab
  for i in 1 2; do
    for v in $AB; do
      timeout -k 10 120 python tools/stamp_run.py --spans --lib "tools/libgsamd_$v.so" > "$O/ab/$v.$i.log" 2>&1 || { rc=1; break 2; }
      echo "$v run $i: $(grep -E 'minibatch period|fwd span|bwd span' $O/ab/$v.$i.log | awk '{printf "%s %s %s | ", $1, $2, $(NF-6)}')"
    done
  done
fi
rm -f $O/stats/*kernel_trace.csv
find $O -name "*.csv" | xargs ls -la
exit $rc
