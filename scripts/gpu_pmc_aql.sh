#!/bin/bash
# PMC counters of the AQL learner kernels, one rocprofv3 pass per counter group.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_aql
mkdir -p $OUT
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d $OUT -o p1 -- python3 $GRAFT_REPO_ROOT/scripts/bench_aql.py --iters 5 --graph 0 > $OUT/p1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT -o p2 -- python3 $GRAFT_REPO_ROOT/scripts/bench_aql.py --iters 5 --graph 0 > $OUT/p2.log 2>&1 &&
timeout -k 10 90 python3 $GRAFT_REPO_ROOT/scripts/bench_aql.py --iters 200 > $OUT/bench.log 2>&1
rc=$?
cat $OUT/bench.log
exit $rc
