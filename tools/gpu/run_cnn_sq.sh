#!/bin/bash
# GPU box: two SQ counter passes (stall / issue breakdown, LDS / instruction mix) over
# tools/cnn_kernel_run.py [$FLAGS] with the in-tree library; summarise with
#   python tools/cnn_sq_summary.py gpurun_out/$TAG/sq1 (and sq2)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-cnnsq}; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d $O/sq1 -o pmc \
    -- python tools/cnn_kernel_run.py $FLAGS > $O/sq1.log 2>&1 || { tail -5 $O/sq1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD \
    SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM_RD --kernel-trace --output-format csv -d $O/sq2 -o pmc \
    -- python tools/cnn_kernel_run.py $FLAGS > $O/sq2.log 2>&1 || { tail -5 $O/sq2.log; exit 1; }
exit 0
