#!/bin/bash
# GPU-box quick loop: chain parity tests, phase stamps, one bench line.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/q; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${SEL:-tests/test_gpu_lagged.py tests/test_gpu_parity.py} -x -q -m gpu -p no:cacheprovider \
    --timeout 300 --timeout-method thread > gpurun_out/q/pytest.log 2>&1 || { tail -30 gpurun_out/q/pytest.log; exit 1; }
tail -1 gpurun_out/q/pytest.log
timeout -k 10 200 python tools/stamp_run.py ${STAMP_MODE:---spans} > gpurun_out/q/stamps.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/q/stamps.log
timeout -k 10 300 python bench.py --cpu-minibatches 0 ${BENCH_ARGS} > gpurun_out/q/bench.json 2> gpurun_out/q/bench.err || exit 1
python -c "
import json
for l in open('gpurun_out/q/bench.json'):
    if l.startswith('{'): d=json.loads(l); print(d['value'], d['stages_us'], d['phases_ms'])"
