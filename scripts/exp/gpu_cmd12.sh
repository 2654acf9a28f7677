cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 python scripts/bench_conv.py > gpurun_out/bench_conv3.log 2>&1; rc=$?; cat gpurun_out/bench_conv3.log; exit $rc
