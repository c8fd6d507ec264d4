#!/bin/bash
# Round 6: same-box A/B of k_clip_adam_flat's float4 quads per thread (ab_libs/libgsamd_aq<q>.so:
# GS_ADAM_QUADS=<q>; round 6 ran 1, 2, then 6, 8) against the in-tree 4: the CNN update parity tests on each variant,
# then C4 bf16 bench update time alternated three times, and one per-kernel trace each.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r06u}; mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)" >&2; shift; "$@"; rc=$?; echo "rc=$rc" >&2; return $rc; }
step tests-window timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_agent.py -k "window" > $O/tests_window.log 2>&1 || { tail -30 $O/tests_window.log; exit 1; }
tail -1 $O/tests_window.log
step c2-collect timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/c2_collect -o c2 --output-format csv \
    -- python tools/collect_run.py C2 4 > $O/c2_collect.log 2>&1 || exit 1
rm -f $O/c2_collect/*kernel_trace.csv
for t in aq6 aq8; do
  GSAMD_LIB=ab_libs/libgsamd_$t.so step tests-$t timeout -k 10 400 python -u -m pytest -x -q --timeout 120 \
      --timeout-method thread -m gpu tests/test_gpu_cnn.py -k "bf16 or head or update" > $O/tests_$t.log 2>&1 || { tail -30 $O/tests_$t.log; exit 1; }
  tail -1 $O/tests_$t.log
done
for i in 1 2 3; do
  for t in cur aq6 aq8; do
    L=; [ $t != cur ] && L=ab_libs/libgsamd_$t.so
    GSAMD_LIB=$L step bench-$t-$i timeout -k 10 200 python bench.py --workload C4 --steps 2 --warmup 2 --dtype bf16 \
        --cpu-minibatches 0 > $O/bench_${t}_$i.json 2> $O/bench_${t}_$i.err || exit 1
    python -c "import json,sys;d=json.loads(open('$O/bench_${t}_$i.json').read().strip().splitlines()[-1]);print('$t $i',d['phases_ms'])"
  done
done
for t in cur aq6 aq8; do
  L=; [ $t != cur ] && L=ab_libs/libgsamd_$t.so
  GSAMD_LIB=$L step trace-$t timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/${t} -o cnn \
      --output-format csv -- python tools/cnn_kernel_run.py --bf16 > $O/${t}.log 2>&1 || exit 1
  rm -f $O/${t}/*kernel_trace.csv
done
exit 0
