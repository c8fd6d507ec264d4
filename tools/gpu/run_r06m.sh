#!/bin/bash
# Round 6: the episode-window rewrite — the collector / agent GPU tests, then per-kernel traces of
# the C2 and C5 rollouts (tools/collect_run.py) for k_episode_window's time at both shapes.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r06m}; mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)" >&2; shift; "$@"; rc=$?; echo "rc=$rc" >&2; return $rc; }
SEL="tests/test_gpu_agent.py tests/test_gpu_api.py" OUT=${TAG:-r06m} TMO=400 \
    bash tools/gpu/run_tests.sh > $O/tests_summary.txt 2>&1 || { echo "tests failed" >&2; exit 1; }
for w in C2 C5; do
  step trace-$w timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/$w -o c --output-format csv \
      -- python tools/collect_run.py $w 4 > $O/$w.log 2>&1 || exit 1
  rm -f $O/$w/*kernel_trace.csv
done
grep -h "k_episode_window" $O/C2/c_kernel_stats.csv $O/C5/c_kernel_stats.csv
step act-stamps timeout -k 10 120 python tools/act_stamp_run.py 2 > $O/act_stamps.txt 2>&1 || exit 1
