#!/bin/bash
# GPU-box driver for the multi-GPU chain: xGMI / lagged / comm-parity tests, then the one-rank
# communicator bench and the same-device 2- and 4-rank rehearsals.  Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/mg; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest ${SEL:-tests/test_gpu_xgmi.py tests/test_gpu_lagged.py tests/test_gpu_parity.py} -x -v -m gpu \
    -p no:cacheprovider --timeout 450 --timeout-method thread > gpurun_out/mg/pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|Error" gpurun_out/mg/pytest.log | tail -40; [ $rc -eq 0 ] || exit $rc
[ -n "$NO_BENCH" ] && exit 0
summ() { python -c "
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'): d=json.loads(l); print(sys.argv[1], d['n_gpus'], d['value'], d['stages_us'], d['phases_ms'], d['config'].get('grad_exchange'))" "$1"; }
timeout -k 10 300 python bench.py --local-comm --steps 3 --warmup 1 --cpu-minibatches 0 \
    > gpurun_out/mg/bench_localcomm.json 2> gpurun_out/mg/bench_localcomm.err && summ gpurun_out/mg/bench_localcomm.json &&
timeout -k 10 300 python bench.py --gpus 2 --same-device --steps 2 --warmup 1 --cpu-minibatches 0 \
    > gpurun_out/mg/bench_same2.json 2> gpurun_out/mg/bench_same2.err && summ gpurun_out/mg/bench_same2.json &&
timeout -k 10 300 python bench.py --gpus 4 --same-device --steps 2 --warmup 1 --cpu-minibatches 0 \
    > gpurun_out/mg/bench_same4.json 2> gpurun_out/mg/bench_same4.err && summ gpurun_out/mg/bench_same4.json
