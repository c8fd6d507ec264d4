#!/bin/bash
# GPU box: the round's evidence on the final build, one call.  Each GPU step runs under its own
# limit and the chain stops at the first failure.  Outputs under gpurun_out/$TAG/ (copied into
# profiles/ by hand afterwards).  Steps by env var (all on by default; set to 0 to skip):
#   TESTS  the whole GPU suite            BENCH  C2 line + rocprof stats + PMC passes
#   LINES  C2 bf16, C3, C4, C4 bf16, C5   CNNK   C4 per-kernel trace + PMC passes (fp32, bf16)
#   ATARI  stack/render trace + PMC       SAME   2-rank same-device rehearsal, dp_mode global (C5)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r04ev}; mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)" >&2; shift; "$@"; rc=$?; echo "rc=$rc" >&2; return $rc; }
on() { [ "${!1:-1}" != 0 ]; }

if on TESTS; then
  step pytest timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --durations=10 \
      --timeout 170 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -3 $O/pytest.log
fi
if on BENCH; then
  step bench timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err && tail -c 300 $O/bench.json || exit 1
  step bench-rocprof timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/stats -o bench --output-format csv \
      -- python bench.py --cpu-minibatches 0 > $O/bench_prof.log 2>&1 || exit 1
  step pmc-fetch timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o pmc \
      -- python tools/pmc_run.py > $O/pmc_fetch.log 2>&1 &&
  step pmc-write timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write -o pmc \
      -- python tools/pmc_run.py > $O/pmc_write.log 2>&1 || exit 1
fi
if on LINES; then
  step bench-c2bf16 timeout -k 10 400 python bench.py --dtype bf16 --cpu-minibatches 0 \
      > $O/bench_c2_bf16.json 2> $O/bench_c2_bf16.err && tail -c 300 $O/bench_c2_bf16.json || exit 1
  for w in C3 C4 C5; do
    # the CPU port's bounded sample: C3's full update is 327 680 minibatches (no CPU leg here, it
    # would outrun the box's silence watchdog); C4 / C5 time 8 vector steps + 3 minibatch steps
    cm=${CPU_MB:-0}; [ $w = C3 ] && cm=0
    step bench-$w timeout -k 10 400 python bench.py --workload $w --steps 2 --warmup 1 --cpu-minibatches $cm \
        > $O/bench_$w.json 2> $O/bench_$w.err && tail -c 300 $O/bench_$w.json || exit 1
  done
  step bench-c4bf16 timeout -k 10 400 python bench.py --workload C4 --dtype bf16 --steps 2 --warmup 1 --cpu-minibatches 0 \
      > $O/bench_c4_bf16.json 2> $O/bench_c4_bf16.err && tail -c 300 $O/bench_c4_bf16.json || exit 1
fi
if on CNNK; then
  for v in "" "--bf16"; do
    d=cnn${v:+bf}
    step cnn-trace$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${d}_stats -o cnn --output-format csv \
        -- python tools/cnn_kernel_run.py $v > $O/${d}_trace.log 2>&1 &&
    step cnn-fetch$v timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/${d}_fetch \
        -o pmc -- python tools/cnn_kernel_run.py $v > $O/${d}_fetch.log 2>&1 &&
    step cnn-write$v timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/${d}_write \
        -o pmc -- python tools/cnn_kernel_run.py $v > $O/${d}_write.log 2>&1 || exit 1
  done
fi
if on ATARI; then
  step atari-trace timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/atari/stats -o atari --output-format csv \
      -- python tools/atari_run.py 256 > $O/atari.log 2>&1 &&
  step atari-fetch timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/atari/fetch -o pmc \
      -- python tools/atari_run.py 256 > $O/atari_fetch.log 2>&1 &&
  step atari-write timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/atari/write -o pmc \
      -- python tools/atari_run.py 256 > $O/atari_write.log 2>&1 || exit 1
  grep "env step" $O/atari.log
fi
if on SAME; then
  step same2-global timeout -k 10 400 python bench.py --gpus 2 --same-device --workload C5 --dp-mode global --steps 2 \
      --warmup 1 --cpu-minibatches 0 > $O/bench_same2_global_c5.json 2> $O/bench_same2_global_c5.err &&
      tail -c 300 $O/bench_same2_global_c5.json || exit 1
fi
rm -f $O/stats/*kernel_trace.csv $O/pmc_*/*kernel_trace.csv     # the C2 traces (10^5 rows); the CNN ones are read
exit 0
