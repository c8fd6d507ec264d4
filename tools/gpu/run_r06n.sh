#!/bin/bash
# Round 6: GPU tests of the touched paths, the window kernel at C2 / C5, the act stamps, the C5
# collect time, the C4 bf16 per-kernel trace and bench line.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r06n}; mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)" >&2; shift; "$@"; rc=$?; echo "rc=$rc" >&2; return $rc; }
SEL="tests/test_gpu_agent.py tests/test_gpu_api.py tests/test_gpu_cnn.py tests/test_gpu_atari.py tests/test_gpu_gemm.py" OUT=${TAG:-r06n} TMO=500 \
    bash tools/gpu/run_tests.sh > $O/tests_summary.txt 2>&1 || { echo "tests failed" >&2; exit 1; }
for w in C2 C5; do
  step trace-$w timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/$w -o c --output-format csv \
      -- python tools/collect_run.py $w 4 > $O/$w.log 2>&1 || exit 1
  rm -f $O/$w/*kernel_trace.csv
done
grep -h "k_episode" $O/C2/c_kernel_stats.csv $O/C5/c_kernel_stats.csv
step act-stamps timeout -k 10 120 python tools/act_stamp_run.py 2 > $O/act_stamps.txt 2>&1 || exit 1
for i in 1 2 3; do timeout -k 10 150 python tools/collect_run.py C5 4 >> $O/collect.txt 2>&1 || exit 1; done
step cnnbf-trace timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/cnnbf_stats -o cnn --output-format csv \
    -- python tools/cnn_kernel_run.py --bf16 > $O/cnnbf_trace.log 2>&1 || exit 1
rm -f $O/cnnbf_stats/*kernel_trace.csv
step c4bf timeout -k 10 200 python bench.py --workload C4 --steps 1 --warmup 1 --dtype bf16 > $O/c4bf.json 2> $O/c4bf.err || exit 1
