#!/bin/bash
# Round 6: same-box A/B of the fused tail taking the conv2 / conv3 weight-gradient sums (current
# build) against GS_TAIL_CONV_SUMS=0 (sweeplibs/libgsamd_tail0.so): C4 bf16 bench update time and
# the per-kernel trace, alternated twice.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r06r}; mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)" >&2; shift; "$@"; rc=$?; echo "rc=$rc" >&2; return $rc; }
for i in 1 2; do
  for t in cur tail0; do
    L=; [ $t != cur ] && L=sweeplibs/libgsamd_$t.so
    GSAMD_LIB=$L step trace-$t-$i timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/${t}_$i -o cnn \
        --output-format csv -- python tools/cnn_kernel_run.py --bf16 > $O/${t}_$i.log 2>&1 || exit 1
    rm -f $O/${t}_$i/*kernel_trace.csv
    GSAMD_LIB=$L step bench-$t-$i timeout -k 10 200 python bench.py --workload C4 --steps 1 --warmup 1 --dtype bf16 \
        --cpu-minibatches 0 > $O/bench_${t}_$i.json 2> $O/bench_${t}_$i.err || exit 1
  done
done
