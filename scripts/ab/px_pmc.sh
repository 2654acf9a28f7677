#!/bin/bash
# px forward microbench (fp32 body vs 6 / 8 term products, learner shapes) + PMC of the conv2
# forward launches (eager), one rocprofv3 pass per counter group.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
REPO=$(pwd)
mkdir -p gpurun_out/px_pmc
timeout -k 10 300 python -u -m pytest tests/test_gpu_px.py -x -v -s -rf --timeout 120 --timeout-method thread > gpurun_out/px_pmc/pytest_px.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed|errors" gpurun_out/px_pmc/pytest_px.log | tail -14
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python scripts/bench_px.py --iters 30 > gpurun_out/px_pmc/bench.txt 2>&1
rc=$?; cat gpurun_out/px_pmc/bench.txt; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
OUT=$REPO/gpurun_out/px_pmc
B="python3 $REPO/scripts/bench_px.py --iters 3 --graph 0 --only conv2"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT -o p1 -- $B > $OUT/p1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE TCC_HIT_sum --output-format csv -d $OUT -o p2 -- $B > $OUT/p2.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE TCC_MISS_sum --output-format csv -d $OUT -o p3 -- $B > $OUT/p3.log 2>&1
rc=$?
echo "pmc rc=$rc"; tail -3 $OUT/p2.log
exit $rc
