#!/bin/bash
# PMC counters of the exact-split conv1 kernels (bench_f32 --only conv1, eager launches).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_c1
mkdir -p $OUT
B="python3 $GRAFT_REPO_ROOT/scripts/bench_f32.py --iters 3 --graph 0 --only conv1"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT -o p1 -- $B > $OUT/p1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE SQ_INSTS_SALU --output-format csv -d $OUT -o p2 -- $B > $OUT/p2.log 2>&1
rc=$?
echo "pmc rc=$rc"
exit $rc
