#!/bin/bash
# GPU box: the round's closing evidence in one call — the C4 per-kernel traces and separate
# FETCH_SIZE / WRITE_SIZE passes (fp32 and bf16), the per-kernel tables built from them on the box
# (tools/cnn_kernel_summary.py -> profiles/c4_kernels*.json, also under gpurun_out/$TAG/), then the
# bench lines (tools/gpu/run_lines.sh) reading those tables.  Each GPU step under its own limit;
# the chain stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-final}; mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)" >&2; shift; "$@"; rc=$?; echo "rc=$rc" >&2; return $rc; }
for v in "" "--bf16"; do
  d=cnn${v:+bf}
  step cnn-trace$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${d}_stats -o cnn --output-format csv \
      -- python tools/cnn_kernel_run.py $v > $O/${d}_trace.log 2>&1 &&
  step cnn-fetch$v timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/${d}_fetch \
      -o pmc -- python tools/cnn_kernel_run.py $v > $O/${d}_fetch.log 2>&1 &&
  step cnn-write$v timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/${d}_write \
      -o pmc -- python tools/cnn_kernel_run.py $v > $O/${d}_write.log 2>&1 || exit 1
done
# the tables (host-side reductions: a failure here leaves the old tables, whose source hash then
# does not match, and the lines report no C4 traffic rather than stopping)
python tools/cnn_kernel_summary.py $O > $O/c4_kernels.json 2> $O/c4_kernels.err &&
python tools/cnn_kernel_summary.py $O --bf16 --prefix cnnbf > $O/c4_kernels_bf16.json 2>> $O/c4_kernels.err &&
cp $O/c4_kernels.json profiles/c4_kernels.json && cp $O/c4_kernels_bf16.json profiles/c4_kernels_bf16.json ||
    echo "c4 kernel tables failed (see $O/c4_kernels.err)" >&2
TAG=${TAG:-final} bash tools/gpu/run_lines.sh
