#!/bin/bash
# GPU box: the fp32 weight-gradient fix (round-5 staging form where the prefetch is off) — the CNN
# GPU tests, then same-box per-kernel traces against the previous build (ab_libs/libgsamd_head.so),
# then the C4 fp32 / bf16 bench lines.  Each step under its own limit; stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r06wg}; mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)" >&2; shift; "$@"; rc=$?; echo "rc=$rc" >&2; return $rc; }
step tests timeout -k 10 500 python -u -m pytest tests/test_gpu_cnn.py -x -q -m gpu -p no:cacheprovider \
    --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
TAG=${TAG:-r06wg} V=head REPS=2 bash tools/gpu/run_cnn_ab.sh > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
step c4 timeout -k 10 400 python bench.py --workload C4 --steps 3 --warmup 2 > $O/bench_C4.json 2> $O/bench_C4.err || exit 1
step c4bf16 timeout -k 10 400 python bench.py --workload C4 --dtype bf16 --steps 3 --warmup 2 --cpu-minibatches 0 > $O/bench_c4_bf16.json 2> $O/bench_c4_bf16.err || exit 1
cut -c1-300 $O/bench_C4.json $O/bench_c4_bf16.json
