#!/bin/bash
# Round-6 evidence: the C5 collect's kernel trace (durations and the gaps between the captured step
# graph's kernels, tools/trace_gaps.py), the fc launch-shape sweep with the 128 x 128 split-K variants
# (sweeplibs/libgsamd_fcsweep.so, a GS_FC_SWEEP build), and the C4 per-kernel trace of the current
# build (fp32 and bf16, tools/cnn_kernel_run.py).  Each GPU step under its own limit, chained.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r06d}; mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)" >&2; shift; "$@"; rc=$?; echo "rc=$rc" >&2; return $rc; }
step c5-trace timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c5_trace -o c5 --output-format csv \
    -- python tools/collect_run.py C5 4 > $O/c5_trace.log 2>&1 &&
python tools/trace_gaps.py $(find $O/c5_trace -name "*kernel_trace.csv" | head -n 1) --skip 200 > $O/c5_gaps.txt 2>&1;
step fc-sweep timeout -k 10 300 env GSAMD_LIB=sweeplibs/libgsamd_fcsweep.so python tools/fc_sweep.py > $O/fc_sweep.txt 2>&1 &&
for v in "" "--bf16"; do
  d=cnn${v:+bf}
  step cnn-trace$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${d}_stats -o cnn --output-format csv \
      -- python tools/cnn_kernel_run.py $v > $O/${d}_trace.log 2>&1 || exit 1
done
rm -f $O/cnn_stats/*kernel_trace.csv $O/cnnbf_stats/*kernel_trace.csv 2>/dev/null
find $O -name "*kernel_trace.csv" -size +20M -delete
exit 0
