#!/bin/bash
# Wave-state PMC passes (where the wave cycles go: waiting, issue-stalled, VALU / LDS / MFMA
# active) over the fp32 network kernels (scripts/bench_f32.py, eager), one rocprofv3 pass each.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_waits
mkdir -p $OUT
B="python3 $GRAFT_REPO_ROOT/scripts/bench_f32.py --iters 3 --graph 0 ${BENCH_F32_ARGS}"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES --output-format csv -d $OUT -o w1 -- $B > $OUT/w1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT -o w2 -- $B > $OUT/w2.log 2>&1
rc=$?
echo "pmc rc=$rc"
exit $rc
