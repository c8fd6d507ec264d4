#!/bin/bash
# GPU-box: default bench under rocprofv3 kernel-trace stats, then two separate PMC passes.
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r01}; mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
O=gpurun_out/$TAG
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/stats -o bench --output-format csv -- python bench.py ${BENCH_ARGS} > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' $O/bench.log; tail -3 $O/bench.log
rm -f $O/stats/bench_kernel_trace.csv; cut -c1-60,200-400 $O/stats/bench_kernel_stats.csv | head -8
[ $rc -eq 0 ] || exit $rc
[ "${PMC:-1}" = 1 ] || exit 0
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o pmc -- python tools/pmc_run.py > $O/pmc_fetch.log 2>&1
rc=$?; echo "pmc fetch rc=$rc"; tail -2 $O/pmc_fetch.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write -o pmc -- python tools/pmc_run.py > $O/pmc_write.log 2>&1
rc=$?; echo "pmc write rc=$rc"; tail -2 $O/pmc_write.log
rm -f $O/stats/bench_kernel_trace.csv $O/pmc_*/pmc_kernel_trace.csv
find $O -name "*.csv" | xargs ls -la
exit $rc
