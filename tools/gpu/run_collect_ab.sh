#!/bin/bash
# Same-box A/B of the C5 rollout (collect) across source trees: the round-4 and round-5 trees
# (ab_libs/r04, ab_libs/r05: git archive of those revisions, built in the container) and the
# working tree, alternated three times; each run prints its mean collect ms per 128-step rollout.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-cab}; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3; do
  for t in ab_libs/r04 ab_libs/r05 .; do
    echo "== $t run $i" >> $O/collect_ab.txt
    (cd $t && timeout -k 10 150 python tools/collect_run.py C5 4) >> $O/collect_ab.txt 2>&1 || exit 1
  done
done
cat $O/collect_ab.txt
