#!/bin/bash
# Round-6: the C5 bench line's collect phase vs a back-to-back collect (tools/collect_phase_probe.py).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r06s}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/collect_phase_probe.py C5 4 > $O/probe_c5.txt 2>&1 && cat $O/probe_c5.txt &&
timeout -k 10 300 python -u bench.py --workload C5 --steps 6 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err && tail -c 400 $O/bench_c5.json
