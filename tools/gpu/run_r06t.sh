#!/bin/bash
# Round 6: same-box A/B of k_cnn_head_loss at 2 rows per workgroup (ab_libs/libgsamd_hr2.so,
# GS_HEAD_ROWS=2: 512 workgroups at B = 1024) against the in-tree 4: the bf16 CNN parity tests on the
# variant, then C4 bf16 bench update time and the per-kernel trace, alternated three times.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r06t}; mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)" >&2; shift; "$@"; rc=$?; echo "rc=$rc" >&2; return $rc; }
GSAMD_LIB=ab_libs/libgsamd_hr2.so step tests-hr2 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 \
    --timeout-method thread -m gpu tests/test_gpu_cnn.py -k "bf16 or head or update" > $O/tests_hr2.log 2>&1 || { tail -30 $O/tests_hr2.log; exit 1; }
tail -2 $O/tests_hr2.log
for i in 1 2 3; do
  for t in cur hr2; do
    L=; [ $t != cur ] && L=ab_libs/libgsamd_$t.so
    GSAMD_LIB=$L step bench-$t-$i timeout -k 10 200 python bench.py --workload C4 --steps 2 --warmup 2 --dtype bf16 \
        --cpu-minibatches 0 > $O/bench_${t}_$i.json 2> $O/bench_${t}_$i.err || exit 1
    python -c "import json,sys;d=json.loads(open('$O/bench_${t}_$i.json').read().strip().splitlines()[-1]);print('$t $i',d['phases_ms'])"
  done
done
for t in cur hr2; do
  L=; [ $t != cur ] && L=ab_libs/libgsamd_$t.so
  GSAMD_LIB=$L step trace-$t timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/${t} -o cnn \
      --output-format csv -- python tools/cnn_kernel_run.py --bf16 > $O/${t}.log 2>&1 || exit 1
  rm -f $O/${t}/*kernel_trace.csv
done
exit 0
