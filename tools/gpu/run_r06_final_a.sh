#!/bin/bash
# Round-6 closing evidence, part A: the whole -m gpu suite, the C2 kernels' FETCH_SIZE / WRITE_SIZE
# passes (tools/pmc_run.py) reduced to profiles/pmc_traffic.json on the box (so the C2 line below
# reads the current build's traffic; the file is copied back through gpurun_out/), the C2 bench
# line and its rocprofv3 --stats profile.  Each GPU step under its own limit; stops at a failure.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r06fa}; mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)" >&2; shift; "$@"; rc=$?; echo "rc=$rc" >&2; return $rc; }
step pytest timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --durations=10 \
    --timeout 170 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
step pmc-fetch timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o pmc \
    -- python tools/pmc_run.py > $O/pmc_fetch.log 2>&1 &&
step pmc-write timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write -o pmc \
    -- python tools/pmc_run.py > $O/pmc_write.log 2>&1 || exit 1
python tools/pmc_summarize.py $(ls $O/pmc_fetch/*counter_collection.csv) $(ls $O/pmc_write/*counter_collection.csv) \
    > $O/pmc_traffic.json && cp $O/pmc_traffic.json profiles/pmc_traffic.json || exit 1
step bench timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err && tail -c 400 $O/bench.json || exit 1
step bench-rocprof timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/stats -o bench --output-format csv \
    -- python bench.py --cpu-minibatches 0 > $O/bench_prof.log 2>&1 || exit 1
rm -f $O/stats/*kernel_trace.csv $O/pmc_*/*kernel_trace.csv
exit 0
