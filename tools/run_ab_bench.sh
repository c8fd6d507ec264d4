#!/bin/bash
# GPU box: the plain bench line of the in-tree library and of plain (non-diagnostic) variants
# tools/libgsamd_<name>.so alternated three times in one call (same box, so box-to-box variation
# does not enter the comparison).  Usage: run_ab_bench.sh NAME [NAME ...]
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/abb
for i in 1 2 3; do
  for v in intree "$@"; do
    if [ "$v" = intree ]; then lib=""; else lib="ab_libs/libgsamd_$v.so"; [ -f "$lib" ] || lib="tools/libgsamd_$v.so"; fi
    GSAMD_LIB=$lib timeout -k 10 200 python bench.py --cpu-minibatches 0 ${BENCH_ARGS} > "gpurun_out/abb/$v.$i.json" 2> "gpurun_out/abb/$v.$i.err" || exit 1
    python -c "
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]
print(sys.argv[2], round(d['value']), d['stages_us'], d['phases_ms'])" "gpurun_out/abb/$v.$i.json" "$v run $i"
  done
done
