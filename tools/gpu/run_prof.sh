#!/bin/bash
# GPU-box evidence run (profiles/): plain C2 bench line, the same command under rocprofv3
# kernel-trace stats, the GAE sweep (+ stats), separate FETCH_SIZE / WRITE_SIZE PMC passes, the
# C3/C4/C5 lines, and the multi-GPU rehearsals (one-rank comm chain; 2 and 4 self-launched ranks
# sharing the one GPU).  Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${TAG:-r02}; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; shift; "$@"; rc=$?; echo "rc=$rc"; return $rc; }
step bench timeout -k 10 300 python bench.py ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err && cat $O/bench.json &&
step bench-rocprof timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/stats -o bench --output-format csv -- python bench.py ${BENCH_ARGS} > $O/bench_prof.log 2>&1 &&
step spans timeout -k 10 200 python tools/stamp_run.py --spans > $O/spans_c2.log 2>&1 &&
step gae-sweep timeout -k 10 200 python tools/gae_sweep.py --json $O/gae_sweep.json > $O/gae_sweep.log 2>&1 &&
step gae-rocprof timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/gae_stats -o gae --output-format csv -- python tools/gae_sweep.py > $O/gae_prof.log 2>&1 &&
step pmc-fetch timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o pmc -- python tools/pmc_run.py > $O/pmc_fetch.log 2>&1 &&
step pmc-write timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write -o pmc -- python tools/pmc_run.py > $O/pmc_write.log 2>&1 &&
step c3 timeout -k 10 300 python bench.py --workload C3 --steps 3 --warmup 2 > $O/bench_c3.json 2> $O/bench_c3.err &&
step c4 timeout -k 10 300 python bench.py --workload C4 --steps 1 --warmup 1 > $O/bench_c4.json 2> $O/bench_c4.err &&
step c5 timeout -k 10 300 python bench.py --workload C5 --steps 2 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err &&
step localcomm timeout -k 10 300 python bench.py --local-comm --steps 3 --warmup 2 --cpu-minibatches 0 > $O/bench_localcomm.json 2> $O/bench_localcomm.err &&
step same2 timeout -k 10 300 python bench.py --gpus 2 --same-device --steps 2 --warmup 1 --cpu-minibatches 0 > $O/bench_same2.json 2> $O/bench_same2.err &&
step same4 timeout -k 10 300 python bench.py --gpus 4 --same-device --steps 2 --warmup 1 --cpu-minibatches 0 > $O/bench_same4.json 2> $O/bench_same4.err
rc=$?
rm -f $O/stats/*kernel_trace.csv $O/gae_stats/*kernel_trace.csv
find $O -name "*.csv" | xargs ls -la
exit $rc
