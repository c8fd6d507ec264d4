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
if [ -n "$AB" ]; then
  step ab timeout -k 10 600 bash tools/run_ab_bench.sh $AB > $O/ab.log 2>&1; rc=$?; cat $O/ab.log; [ $rc -eq 0 ] || exit $rc
fi
exit 0
