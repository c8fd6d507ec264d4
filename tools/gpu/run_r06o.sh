#!/bin/bash
# Round 6: fc / CNN GPU tests on the current build, the C4 bf16 per-kernel trace and bench line.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r06o}; mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)" >&2; shift; "$@"; rc=$?; echo "rc=$rc" >&2; return $rc; }
SEL="tests/test_gpu_gemm.py tests/test_gpu_cnn.py" OUT=${TAG:-r06o} TMO=400 \
    bash tools/gpu/run_tests.sh > $O/tests_summary.txt 2>&1 || { echo "tests failed" >&2; exit 1; }
step cnnbf-trace timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/cnnbf_stats -o cnn --output-format csv \
    -- python tools/cnn_kernel_run.py --bf16 > $O/cnnbf_trace.log 2>&1 || exit 1
rm -f $O/cnnbf_stats/*kernel_trace.csv
step c4bf timeout -k 10 200 python bench.py --workload C4 --steps 1 --warmup 1 --dtype bf16 > $O/c4bf.json 2> $O/c4bf.err || exit 1
