#!/bin/bash
# Round 6: the -m gpu suite on the current build, the C4 bf16 per-kernel trace and bench line,
# per-kernel C5 traces of the round-5 tree and the current build on the same box, and the C5
# collect A/B of the current build (tiny-batch conv FS = 4) against its FS = 2 variant.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r06f}; mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)" >&2; shift; "$@"; rc=$?; echo "rc=$rc" >&2; return $rc; }
OUT=${TAG:-r06f} TMO=600 bash tools/gpu/run_tests.sh > $O/tests_summary.txt 2>&1 || { echo "tests failed" >&2; exit 1; }
step cnnbf-trace timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/cnnbf_stats -o cnn --output-format csv \
    -- python tools/cnn_kernel_run.py --bf16 > $O/cnnbf_trace.log 2>&1 || exit 1
rm -f $O/cnnbf_stats/*kernel_trace.csv
# the conv2 / conv3 weight-gradient prefetch per layer (GS_WGRAD_PF: product 1 = conv2 only)
for i in 1 2; do
  for t in cur pf0 pf3; do
    L=; [ $t != cur ] && L=sweeplibs/libgsamd_$t.so
    GSAMD_LIB=$L step cnnab-$t-$i timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/cnnab_${t}_$i -o cnn \
        --output-format csv -- python tools/cnn_kernel_run.py --bf16 > $O/cnnab_${t}_$i.log 2>&1 || exit 1
    rm -f $O/cnnab_${t}_$i/*kernel_trace.csv
  done
done
step c4bf timeout -k 10 200 python bench.py --workload C4 --steps 1 --warmup 1 --dtype bf16 > $O/c4bf.json 2> $O/c4bf.err || exit 1
step c5-r05 bash -c "cd ab_libs/r05 && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d ../../$O/c5r05 -o c5 --output-format csv -- python tools/collect_run.py C5 2" > $O/c5r05.log 2>&1 || exit 1
step c5-cur timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/c5cur -o c5 --output-format csv -- python tools/collect_run.py C5 2 > $O/c5cur.log 2>&1 || exit 1
rm -f $O/c5r05/*kernel_trace.csv $O/c5cur/*kernel_trace.csv
for i in 1 2 3; do
  for t in cur fs2; do
    echo "== $t run $i" >> $O/collect_ab.txt
    if [ $t = cur ]; then timeout -k 10 150 python tools/collect_run.py C5 4 >> $O/collect_ab.txt 2>&1 || exit 1
    else GSAMD_LIB=sweeplibs/libgsamd_tinyfs2.so timeout -k 10 150 python tools/collect_run.py C5 4 >> $O/collect_ab.txt 2>&1 || exit 1; fi
  done
done
grep -E "^==|C5:" $O/collect_ab.txt
