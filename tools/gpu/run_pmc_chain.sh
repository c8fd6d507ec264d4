cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmcc; export TMPDIR=/tmp
i=0
for C in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum" "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmcc/p$i -o p -- python tools/pmc_chain.py > gpurun_out/pmcc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmcc/p$i.log; exit 1; }
done
python tools/pmc_chain_summary.py gpurun_out/pmcc/p1 gpurun_out/pmcc/p2 gpurun_out/pmcc/p3 gpurun_out/pmcc/p4 > gpurun_out/pmcc/summary.json
cat gpurun_out/pmcc/summary.json
