#!/bin/bash
# fp32 network kernels: per-launch timing + two PMC passes (each its own run).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/f32prof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 python3 $R/scripts/bench_f32.py > $O/time.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES \
  SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU --output-format csv -d $O -o p1 \
  -- python3 $R/scripts/bench_f32.py --graph 0 --iters 3 > $O/p1.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS \
  SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU --output-format csv -d $O -o p2 \
  -- python3 $R/scripts/bench_f32.py --graph 0 --iters 3 > $O/p2.log 2>&1
