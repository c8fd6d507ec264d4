#!/bin/bash
# GPU-box driver: parity tests, stamp timing, rocprof'd bench. Stops at the first GPU failure.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -m pytest tests -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
if [ -n "$STAMPS" ]; then
  timeout -k 10 200 python tools/stamp_run.py > gpurun_out/stamps.log 2>&1; rc=$?; echo "stamps rc=$rc"; cat gpurun_out/stamps.log | tail -40
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps ${BSTEPS:-3} --warmup 1 ${BENCH_ARGS} > gpurun_out/bench_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -3 gpurun_out/bench_prof.log
find gpurun_out/prof -name "*kernel_stats*" -exec head -12 {} \;
exit $rc
