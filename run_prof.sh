#!/bin/bash
# GPU-box evidence run (profiles/): plain bench line, the same command under rocprofv3
# kernel-trace stats, two separate PMC passes (FETCH_SIZE / WRITE_SIZE), and the GAE sweep
# with its own kernel-trace stats.  Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${TAG:-r01}; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1"; shift; "$@"; rc=$?; echo "rc=$rc"; return $rc; }
step bench timeout -k 10 300 python bench.py ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err && cat $O/bench.json &&
step bench-rocprof timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/stats -o bench --output-format csv -- python bench.py ${BENCH_ARGS} > $O/bench_prof.log 2>&1 &&
step gae-sweep timeout -k 10 200 python tools/gae_sweep.py --json $O/gae_sweep.json > $O/gae_sweep.log 2>&1 &&
step gae-rocprof timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/gae_stats -o gae --output-format csv -- python tools/gae_sweep.py > $O/gae_prof.log 2>&1 &&
step pmc-fetch timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o pmc -- python tools/pmc_run.py > $O/pmc_fetch.log 2>&1 &&
step pmc-write timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write -o pmc -- python tools/pmc_run.py > $O/pmc_write.log 2>&1
rc=$?
rm -f $O/stats/*kernel_trace.csv $O/gae_stats/*kernel_trace.csv
find $O -name "*.csv" | xargs ls -la
exit $rc
