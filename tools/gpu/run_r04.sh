#!/bin/bash
# GPU-box driver for round 4.  Steps are chosen by env vars and chained: the first failure ends
# the call (no GPU step after a failed, killed or timed-out one).
#   SEL="tests/..."   pytest selection (default: the whole GPU suite); NO_TESTS=1 skips it
#   BENCH=1           default C2 bench line (+ C3=1, C4=1, C5=1, C4BF16=1, C2BF16=1 lines)
#   PROF=1            rocprofv3 --kernel-trace --stats of the C2 bench
#   PMC=1             FETCH_SIZE / WRITE_SIZE passes over tools/pmc_run.py (separate runs)
#   SPANS=1           chain timeline (needs tools/libgsamd_spans.so in the push)
#   CNNK=1            per-kernel C4 trace + PMC (tools/cnn_kernel_run.py)
#   EXTRA="cmd"       one more command at the end (under its own timeout)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r04}; mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)" >&2; shift; "$@"; rc=$?; echo "rc=$rc" >&2; return $rc; }
if [ -z "$NO_TESTS" ]; then
  step pytest timeout -k 10 1000 python -u -m pytest ${SEL:-tests} -x -v -m gpu -p no:cacheprovider --durations=15 \
      --timeout 170 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/pytest.log | tail -8; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$BENCH" ]; then
  step bench timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err && cat $O/bench.json || exit 1
fi
for w in C3 C4 C5; do
  if [ -n "${!w}" ]; then
    step bench-$w timeout -k 10 400 python bench.py --workload $w --steps ${WSTEPS:-2} --warmup 1 --cpu-minibatches 0 \
        > $O/bench_$w.json 2> $O/bench_$w.err && cat $O/bench_$w.json || exit 1
  fi
done
if [ -n "$C4BF16" ]; then
  step bench-c4bf16 timeout -k 10 400 python bench.py --workload C4 --dtype bf16 --steps 2 --warmup 1 --cpu-minibatches 0 \
      > $O/bench_c4_bf16.json 2> $O/bench_c4_bf16.err && cat $O/bench_c4_bf16.json || exit 1
fi
if [ -n "$C2BF16" ]; then
  step bench-c2bf16 timeout -k 10 400 python bench.py --dtype bf16 --cpu-minibatches 0 \
      > $O/bench_c2_bf16.json 2> $O/bench_c2_bf16.err && cat $O/bench_c2_bf16.json || exit 1
fi
if [ -n "$PROF" ]; then
  step bench-rocprof timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/stats -o bench --output-format csv \
      -- python bench.py --cpu-minibatches 0 > $O/bench_prof.log 2>&1 || exit 1
fi
if [ -n "$PMC" ]; then
  step pmc-fetch timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o pmc \
      -- python tools/pmc_run.py > $O/pmc_fetch.log 2>&1 &&
  step pmc-write timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write -o pmc \
      -- python tools/pmc_run.py > $O/pmc_write.log 2>&1 || exit 1
fi
if [ -n "$SPANS" ]; then
  step spans timeout -k 10 200 python tools/stamp_run.py --spans > $O/spans_c2.log 2>&1 || exit 1
fi
if [ -n "$CNNK" ]; then
  step cnn-trace timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/cnn_stats -o cnn --output-format csv \
      -- python tools/cnn_kernel_run.py ${CNNK_ARGS} > $O/cnn_trace.log 2>&1 &&
  step cnn-fetch timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/cnn_fetch -o pmc \
      -- python tools/cnn_kernel_run.py ${CNNK_ARGS} > $O/cnn_fetch.log 2>&1 &&
  step cnn-write timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/cnn_write -o pmc \
      -- python tools/cnn_kernel_run.py ${CNNK_ARGS} > $O/cnn_write.log 2>&1 || exit 1
fi
if [ -n "$EXTRA" ]; then
  step extra timeout -k 10 ${EXTRA_T:-300} bash -c "$EXTRA" > $O/extra.log 2>&1; rc=$?; tail -40 $O/extra.log; [ $rc -eq 0 ] || exit $rc
fi
rm -f $O/stats/*kernel_trace.csv
exit 0
