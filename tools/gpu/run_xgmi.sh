set -o pipefail
cd $GRAFT_REPO_ROOT
export GS_XGMI_TIMEOUT_S=30 TMPDIR=/tmp
timeout -k 10 420 python -m pytest tests/test_gpu_xgmi.py tests/test_gpu_parity.py -k "xgmi or comm" -x -q -p no:cacheprovider > gpurun_out/xgmi_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/xgmi_tests.log
[ $rc -eq 0 ] || exit $rc
for n in 2 4; do
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus $n --steps 2 --warmup 1 --same-device > gpurun_out/bench_same$n.log 2>&1; rc=$?; echo "bench same-device n=$n rc=$rc"; grep '^{' gpurun_out/bench_same$n.log | cut -c1-250; grep -o '"stages_us.*' gpurun_out/bench_same$n.log
[ $rc -eq 0 ] || { tail -20 gpurun_out/bench_same$n.log; exit $rc; }
done
