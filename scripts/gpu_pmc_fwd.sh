# PMC counters of the forward kernels at the learner's multi-problem size (1536 samples).
cd /tmp && export TMPDIR=/tmp && export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_fwd
mkdir -p $OUT
timeout -k 10 120 python3 $GRAFT_REPO_ROOT/scripts/bench_conv.py --B 1536 --only fwd > $OUT/time1536.log 2>&1; echo "time rc=$?"; cat $OUT/time1536.log
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $OUT -o p1 -- python3 $GRAFT_REPO_ROOT/scripts/bench_conv.py --B 1536 --only fwd --iters 3 --graph 0 > $OUT/p1.log 2>&1; echo "p1 rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS --output-format csv -d $OUT -o p2 -- python3 $GRAFT_REPO_ROOT/scripts/bench_conv.py --B 1536 --only fwd --iters 3 --graph 0 > $OUT/p2.log 2>&1; echo "p2 rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d $OUT -o p3 -- python3 $GRAFT_REPO_ROOT/scripts/bench_conv.py --B 1536 --only fwd --iters 3 --graph 0 > $OUT/p3.log 2>&1; echo "p3 rc=$?"
ls $OUT
