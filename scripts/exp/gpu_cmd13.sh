cd /tmp && export TMPDIR=/tmp && export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc2
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS --output-format csv -d $OUT -o a -- python3 $GRAFT_REPO_ROOT/scripts/bench_conv.py --iters 3 --graph 0 > $OUT/a.log 2>&1; echo "a rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR TA_BUSY SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT -o b -- python3 $GRAFT_REPO_ROOT/scripts/bench_conv.py --iters 3 --graph 0 > $OUT/b.log 2>&1; echo "b rc=$?"
ls $OUT
