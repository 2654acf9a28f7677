#!/bin/bash
# PMC counters of the backward kernels (B=512), one rocprofv3 pass per counter group.
cd /tmp && export TMPDIR=/tmp && export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_bwd
mkdir -p $OUT
ONLY=${ONLY:-grad}
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_MFMA --output-format csv -d $OUT -o p1 -- python3 $GRAFT_REPO_ROOT/scripts/bench_conv.py --only $ONLY --iters 3 --graph 0 > $OUT/p1.log 2>&1; echo "p1 rc=$?"
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT -o p2 -- python3 $GRAFT_REPO_ROOT/scripts/bench_conv.py --only $ONLY --iters 3 --graph 0 > $OUT/p2.log 2>&1; echo "p2 rc=$?"
ls $OUT
