cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 python scripts/bench_conv.py > gpurun_out/bench_conv.log 2>&1; rc=$?; cat gpurun_out/bench_conv.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/counters.txt 2>&1; echo "list rc=$?"
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_conv
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $OUT -o p1 -- python3 $GRAFT_REPO_ROOT/scripts/bench_conv.py --iters 5 > $OUT/p1.log 2>&1; echo "pmc1 rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --pmc SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS --output-format csv -d $OUT -o p2 -- python3 $GRAFT_REPO_ROOT/scripts/bench_conv.py --iters 5 > $OUT/p2.log 2>&1; echo "pmc2 rc=$?"
ls $OUT
