#!/bin/bash
# GPU-box: CNN/Atari parity tests, then the C4 bench under rocprofv3 kernel stats.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/c4
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_gpu_gemm.py tests/test_gpu_cnn.py tests/test_gpu_atari.py tests/test_gpu_agent.py -x -q -p no:cacheprovider > gpurun_out/c4/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/c4/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/c4/prof -o c4 --output-format csv -- python bench.py --workload ${WL:-C4} --steps 1 --warmup 1 > gpurun_out/c4/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep "^{" gpurun_out/c4/bench.log
rm -f gpurun_out/c4/prof/c4_kernel_trace.csv
exit $rc
