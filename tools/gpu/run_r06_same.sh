#!/bin/bash
# GPU box: round-6 multi-rank rehearsals on the final build — two ranks sharing the one GPU,
# started by torch.distributed.run exactly as the driver starts an N-GPU bench (plus
# --same-device): C2 local mode (xGMI exchange inside k_bwd, self-tested) and C5 global mode.
# Protocol rehearsals: the throughput is not a scaling number.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r06same}; mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)" >&2; shift; "$@"; rc=$?; echo "rc=$rc" >&2; return $rc; }
run() { timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
          --master-port $1 bench.py --gpus 2 --same-device "${@:2}"; }
step c2 run 29511 --steps 3 --warmup 2 --cpu-minibatches 0 > $O/same2_c2.json 2> $O/same2_c2.err || exit 1
step c5g run 29512 --workload C5 --dp-mode global --steps 2 --warmup 2 --cpu-minibatches 0 \
    > $O/same2_global_c5.json 2> $O/same2_global_c5.err || exit 1
cat $O/same2_c2.json $O/same2_global_c5.json | cut -c1-400
