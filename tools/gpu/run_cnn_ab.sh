#!/bin/bash
# GPU box: per-kernel C4 traces (rocprofv3 --kernel-trace --stats of tools/cnn_kernel_run.py, fp32
# and --bf16) of the in-tree library and of ab_libs/libgsamd_<name>.so variants, alternated REPS
# times on one box.  Usage: V="name ..." [REPS=2] [BF16_ONLY=1] bash tools/gpu/run_cnn_ab.sh
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-cnnab}; mkdir -p $O
export TMPDIR=/tmp
for i in $(seq 1 ${REPS:-2}); do
  for v in intree $V; do
    if [ "$v" = intree ]; then lib=""; else lib="ab_libs/libgsamd_$v.so"; fi
    if [ "${BF16_ONLY:-0}" = 1 ]; then FL=(--bf16); else FL=("" --bf16); fi
    for f in "${FL[@]}"; do
      d=$O/${v}${f:+_bf}_$i
      echo "== $v $f run $i $(date +%T)"
      GSAMD_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $d -o cnn --output-format csv \
          -- python tools/cnn_kernel_run.py $f > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
    done
  done
done
exit 0
