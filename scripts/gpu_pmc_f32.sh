#!/bin/bash
# PMC counters of the fp32 network kernels (scripts/bench_f32.py, eager launches), one
# rocprofv3 pass per counter group (block limits: 8 SQ, 4 TCC), each under its own limit.
# TAG names the output directory (pmc_f32$TAG); APEX_F32_STAGE_SPLIT set by the caller picks
# the GEMM forms (ops/csrc/f32_kernels.hip).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_f32${TAG}
mkdir -p $OUT
B="python3 $GRAFT_REPO_ROOT/scripts/bench_f32.py --iters 3 --graph 0"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT -o p1 -- $B > $OUT/p1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE TCC_HIT_sum --output-format csv -d $OUT -o p2 -- $B > $OUT/p2.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE TCC_MISS_sum --output-format csv -d $OUT -o p3 -- $B > $OUT/p3.log 2>&1
rc=$?
echo "pmc rc=$rc"
exit $rc
