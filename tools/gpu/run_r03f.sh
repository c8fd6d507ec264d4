#!/bin/bash
# GPU-box: selected GPU tests (with durations), the C2 bench line, then a same-box A/B of spans
# variants (tools/libgsamd_<name>.so) alternated twice.  Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r03f}; mkdir -p $O/ab
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)" >&2; shift; "$@"; rc=$?; echo "rc=$rc" >&2; return $rc; }
if [ -n "$SEL" ]; then
  step pytest timeout -k 10 900 python -u -m pytest $SEL -x -v -m gpu -p no:cacheprovider --durations=25 --timeout 170 \
      --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; grep -E "FAILED|ERROR|passed|failed|^[0-9.]+s call" $O/pytest.log | head -40; [ $rc -eq 0 ] || exit $rc
fi
if [ -z "$NO_BENCH" ]; then
  step bench timeout -k 10 300 python bench.py --cpu-minibatches 0 ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err && cat $O/bench.json || exit 1
fi
for i in 1 2; do
  for v in $AB; do
    timeout -k 10 120 python tools/stamp_run.py --spans --lib "tools/libgsamd_$v.so" > "$O/ab/$v.$i.log" 2>&1 || exit 1
    echo "$v run $i: $(grep -E 'minibatch period|fwd span|bwd span' $O/ab/$v.$i.log | awk '{printf "%s %s %s | ", $1, $2, $(NF-6)}')"
  done
done
if [ -n "$STAMPS" ]; then
  timeout -k 10 120 python tools/stamp_run.py > $O/stamps.log 2>&1 || exit 1
  grep -v amdgpu.ids $O/stamps.log | head -40
fi
