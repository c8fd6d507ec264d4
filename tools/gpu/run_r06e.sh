#!/bin/bash
# Round 6: the head weight-gradient fix on the C4 bf16 per-kernel trace and bench line, and a
# same-box C5 collect A/B: the round-5 tree, the working build, and its GS_CONV_TINY_FS=4 variant
# (sweeplibs/libgsamd_tinyfs4.so), alternated three times.  Each GPU step under its own limit.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r06e}; mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)" >&2; shift; "$@"; rc=$?; echo "rc=$rc" >&2; return $rc; }
step cnnbf-trace timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/cnnbf_stats -o cnn --output-format csv \
    -- python tools/cnn_kernel_run.py --bf16 > $O/cnnbf_trace.log 2>&1 || exit 1
rm -f $O/cnnbf_stats/*kernel_trace.csv
step c4bf timeout -k 10 200 python bench.py --workload C4 --steps 1 --warmup 1 --dtype bf16 > $O/c4bf.json 2> $O/c4bf.err || exit 1
for i in 1 2 3; do
  for t in r05 cur fs4; do
    echo "== $t run $i" >> $O/collect_ab.txt
    case $t in
      r05) (cd ab_libs/r05 && timeout -k 10 150 python tools/collect_run.py C5 4) >> $O/collect_ab.txt 2>&1 || exit 1 ;;
      cur) timeout -k 10 150 python tools/collect_run.py C5 4 >> $O/collect_ab.txt 2>&1 || exit 1 ;;
      fs4) GSAMD_LIB=sweeplibs/libgsamd_tinyfs4.so timeout -k 10 150 python tools/collect_run.py C5 4 >> $O/collect_ab.txt 2>&1 || exit 1 ;;
    esac
  done
done
grep -E "^==|C5:" $O/collect_ab.txt
