#!/bin/bash
# GPU box: the fp32 conv weight-gradient slowdown across round-6 revisions — each tree under
# ab_libs/t_<rev> (git archive + its own build) and the working tree, fp32 C4 kernel traces of
# tools/cnn_kernel_run.py, alternated twice on one box.
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/${TAG:-r06bis}; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  for t in ab_libs/t_192cf1e ab_libs/t_8ad4511 ab_libs/t_6dcde4e ab_libs/t_1d5df87 .; do
    n=$(basename $t); [ "$t" = . ] && n=head
    echo "== $n run $i $(date +%T)"
    (cd $t && timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/${n}_$i -o cnn --output-format csv \
        -- python tools/cnn_kernel_run.py > $O/${n}_$i.log 2>&1) || { tail -20 $O/${n}_$i.log; exit 1; }
  done
done
