#!/bin/bash
# GPU box: one bundle of round-4 evidence steps, each under its own time limit, chained so the
# first failure ends the call.  TAG names the gpurun_out/ subdirectory.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r04e}; mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)" >&2; shift; "$@"; rc=$?; echo "rc=$rc" >&2; return $rc; }
step tests timeout -k 10 300 python -u -m pytest ${SEL:-tests/test_gpu_atari.py} -x -q -m gpu -p no:cacheprovider \
    --timeout 170 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
step atari-prof timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/atari -o atari --output-format csv \
    -- python tools/atari_run.py 256 > $O/atari.log 2>&1 && grep "env step" $O/atari.log || exit 1
step c5-collect-prof timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/c5c -o c5c --output-format csv \
    -- python tools/collect_run.py C5 3 > $O/c5c.log 2>&1 && grep "collect" $O/c5c.log || exit 1
step fc-bench timeout -k 10 120 python tools/fc_bench.py > $O/fc_bench.log 2>&1 && cat $O/fc_bench.log || exit 1
if [ -n "$CNNK" ]; then
  step cnn-trace timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/cnn_stats -o cnn --output-format csv \
      -- python tools/cnn_kernel_run.py ${CNNK_ARGS} > $O/cnn_trace.log 2>&1 || exit 1
fi
[ -n "$C4B" ] || { rm -f $O/*/*kernel_trace.csv; exit 0; }
step bench-c4 timeout -k 10 300 python bench.py --workload C4 --steps 2 --warmup 1 --cpu-minibatches 0 \
    > $O/bench_c4.json 2> $O/bench_c4.err && tail -c 600 $O/bench_c4.json || exit 1
step bench-c4bf16 timeout -k 10 300 python bench.py --workload C4 --dtype bf16 --steps 2 --warmup 1 --cpu-minibatches 0 \
    > $O/bench_c4_bf16.json 2> $O/bench_c4_bf16.err && tail -c 600 $O/bench_c4_bf16.json || exit 1
if [ -n "$AB" ]; then
  step ab timeout -k 10 600 bash tools/run_ab_bench.sh $AB > $O/ab.log 2>&1; rc=$?; cat $O/ab.log; [ $rc -eq 0 ] || exit $rc
fi
rm -f $O/*/*kernel_trace.csv $O/*/*/*kernel_trace.csv
exit 0
