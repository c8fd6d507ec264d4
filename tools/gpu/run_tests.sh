#!/bin/bash
# GPU-box test run: SEL (pytest selection, default the whole -m gpu suite) -> gpurun_out/$OUT/pytest.log
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-t}
mkdir -p gpurun_out/$OUT; export TMPDIR=/tmp
timeout -k 10 ${TMO:-1000} python -u -m pytest ${SEL:-tests} -x -v -m gpu -p no:cacheprovider -s \
    --timeout 300 --timeout-method thread > gpurun_out/$OUT/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|SKIPPED|passed|failed|^(fp32|bf16|teacher)" gpurun_out/$OUT/pytest.log | tail -60
exit $rc
