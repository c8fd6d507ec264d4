#!/bin/bash
# GPU-box driver: parity tests, a plain bench line, the one-rank multi-GPU chain (--local-comm)
# and the same-device N-rank rehearsal of `bench.py --gpus N` (self-launched ranks).  Stops at
# the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $1"; shift; "$@"; rc=$?; echo "rc=$rc"; return $rc; }
PYTEST_SEL=${PYTEST_SEL:-tests}
step pytest timeout -k 10 900 python -u -m pytest $PYTEST_SEL -x -v -m gpu -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -60; [ $rc -eq 0 ] || exit $rc
[ -n "$NO_BENCH" ] && exit 0
step bench timeout -k 10 300 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err &&
cat gpurun_out/bench.json &&
step bench-localcomm timeout -k 10 300 python bench.py --local-comm --steps 3 --warmup 1 --cpu-minibatches 0 \
    > gpurun_out/bench_localcomm.json 2> gpurun_out/bench_localcomm.err && cat gpurun_out/bench_localcomm.json &&
step bench-same2 timeout -k 10 300 python bench.py --gpus 2 --same-device --steps 2 --warmup 1 --cpu-minibatches 0 \
    > gpurun_out/bench_same2.json 2> gpurun_out/bench_same2.err && cat gpurun_out/bench_same2.json
