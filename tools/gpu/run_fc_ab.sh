#!/bin/bash
# GPU box: fc kernel parity tests, fc_bench over the in-tree library and ab_libs variants, then
# (optionally) the C2 bench A/B of AB variants.  Each step under its own limit, chained.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-fcab}; mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)" >&2; shift; "$@"; rc=$?; echo "rc=$rc" >&2; return $rc; }
step tests timeout -k 10 400 python -u -m pytest ${SEL:-tests/test_gpu_gemm.py tests/test_gpu_cnn.py} -x -q -m gpu \
    -p no:cacheprovider --timeout 170 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in intree $FCV; do
  if [ "$v" = intree ]; then lib=""; else lib="ab_libs/libgsamd_$v.so"; fi
  echo "-- $v"
  GSAMD_LIB=$lib step fc-$v timeout -k 10 120 python tools/fc_bench.py > $O/fc_$v.log 2>&1 && cat $O/fc_$v.log || exit 1
done
if [ -n "$ATARI" ]; then
  step atari-prof timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/atari -o atari --output-format csv \
      -- python tools/atari_run.py 256 > $O/atari.log 2>&1 && grep "env step" $O/atari.log || exit 1
  rm -f $O/atari/*kernel_trace.csv
fi
if [ -n "$FCPMC" ]; then
  step fc-fetch timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fc_fetch -o pmc \
      -- python tools/fc_bench.py > $O/fc_fetch.log 2>&1 &&
  step fc-write timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/fc_write -o pmc \
      -- python tools/fc_bench.py > $O/fc_write.log 2>&1 || exit 1
fi
if [ -n "$SQPMC" ]; then
  step fc-sq timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
      SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d $O/fc_sq -o pmc \
      -- python tools/fc_bench.py > $O/fc_sq.log 2>&1 || exit 1
fi
if [ -n "$C5C" ]; then
  step c5-collect-prof timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/c5c -o c5c --output-format csv \
      -- python tools/collect_run.py C5 3 > $O/c5c.log 2>&1 && grep "collect" $O/c5c.log || exit 1
  rm -f $O/c5c/*kernel_trace.csv
fi
if [ -n "$STAMPS" ]; then
  step cnn-stamps timeout -k 10 200 python tools/cnn_stamp_run.py > $O/stamps.log 2>&1 &&
  step cnn-stamps-bf16 timeout -k 10 200 python tools/cnn_stamp_run.py --bf16 >> $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
  grep -v "^W20" $O/stamps.log
fi
if [ -n "$C4B" ]; then
  step bench-c4 timeout -k 10 300 python bench.py --workload C4 --steps 2 --warmup 1 --cpu-minibatches 0 \
      > $O/bench_c4.json 2> $O/bench_c4.err && tail -c 400 $O/bench_c4.json || exit 1
  step bench-c4bf16 timeout -k 10 300 python bench.py --workload C4 --dtype bf16 --steps 2 --warmup 1 --cpu-minibatches 0 \
      > $O/bench_c4_bf16.json 2> $O/bench_c4_bf16.err && tail -c 400 $O/bench_c4_bf16.json || exit 1
fi
if [ -n "$AB" ]; then
  step ab timeout -k 10 600 bash tools/run_ab_bench.sh $AB > $O/ab.log 2>&1; rc=$?; cat $O/ab.log; [ $rc -eq 0 ] || exit $rc
fi
exit 0
