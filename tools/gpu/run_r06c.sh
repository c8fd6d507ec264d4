#!/bin/bash
# Round-6 combined call: the -m gpu suite, the C4 fp32 / bf16 bench lines, the C4 eager-vs-graph
# timing, the same-box collect A/B (round-4 / round-5 / current trees), then run_r06d.sh's evidence.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r06c}; mkdir -p $O
OUT=${TAG:-r06c} TMO=800 bash tools/gpu/run_tests.sh > $O/tests_summary.txt 2>&1
echo "tests rc=$?" >> $O/tests_summary.txt
timeout -k 10 200 python bench.py --workload C4 --steps 1 --warmup 1 --dtype bf16 > $O/c4bf.json 2> $O/c4bf.err &&
timeout -k 10 200 python bench.py --workload C4 --steps 1 --warmup 1 > $O/c4.json 2> $O/c4.err &&
timeout -k 10 200 python tools/c4_graph_ab.py --bf16 > $O/c4_graph_ab.txt 2>&1 &&
TAG=${TAG:-r06c} bash tools/gpu/run_collect_ab.sh > /dev/null &&
TAG=${TAG:-r06c} bash tools/gpu/run_r06d.sh
