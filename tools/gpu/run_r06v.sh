#!/bin/bash
# Round 6: the rolling-window kernel (k_episode_window16) — its GPU tests, the untracked collector
# tests, and the C2 / C5 collect kernel traces (its duration per rollout).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r06v}; mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)" >&2; shift; "$@"; rc=$?; echo "rc=$rc" >&2; return $rc; }
step tests-window timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_agent.py -k "window or untracked or graph" > $O/tests_window.log 2>&1 || { tail -30 $O/tests_window.log; exit 1; }
tail -1 $O/tests_window.log
for w in C2 C5; do
  step collect-$w timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/${w}_collect -o c --output-format csv \
      -- python tools/collect_run.py $w 4 > $O/${w}_collect.log 2>&1 || exit 1
  rm -f $O/${w}_collect/*kernel_trace.csv
  grep -h "episode" $O/${w}_collect/*kernel_stats.csv | cut -c1-200
done
exit 0
