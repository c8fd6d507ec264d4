#!/bin/bash
# GPU-box evidence, round 3 (C2 final build): PMC passes (FETCH_SIZE, WRITE_SIZE, separate) over
# tools/pmc_run.py, the chain timeline, the GAE sweep.  Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03c; mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)" >&2; shift; "$@"; rc=$?; echo "rc=$rc" >&2; return $rc; }
step pmc-fetch timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o pmc -- python tools/pmc_run.py > $O/pmc_fetch.log 2>&1 &&
step pmc-write timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write -o pmc -- python tools/pmc_run.py > $O/pmc_write.log 2>&1 &&
step spans timeout -k 10 200 python tools/stamp_run.py --spans > $O/spans_c2.log 2>&1 &&
step gae-sweep timeout -k 10 200 python tools/gae_sweep.py --json $O/gae_sweep.json > $O/gae_sweep.log 2>&1
rc=$?
find $O -name "*.csv" | xargs ls -la
exit $rc
