#!/bin/bash
# PMC counters of the conv2 / conv3 forward, GEMM body (knob 25 = 0) vs sample-resident (25 = 1).
cd /tmp && export TMPDIR=/tmp && export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/direct_pmc
mkdir -p $OUT
for k in 1 2; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT -o a$k -- python3 $R/scripts/bench_f32.py --only conv --iters 3 --graph 0 --knobs 25=$k > $OUT/a$k.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT -o b$k -- python3 $R/scripts/bench_f32.py --only conv --iters 3 --graph 0 --knobs 25=$k > $OUT/b$k.log 2>&1 || exit 1
  echo "knob 25=$k"
  python3 $R/scripts/pmc_table.py --summary $(find $OUT -name "[ab]${k}_counter_collection.csv") | grep -v "conv1\|heads" || true
done
python3 $R/scripts/pmc_table.py $(find $OUT -name "*counter_collection.csv") > $OUT/raw.md 2>&1 || true
