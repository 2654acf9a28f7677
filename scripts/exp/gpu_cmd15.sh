cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests/test_gpu_fused_net.py tests/test_gpu_train_cli.py -q -rf -x > gpurun_out/pytest_fused.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_fused.log
if [ $rc -ne 0 ]; then tail -60 gpurun_out/pytest_fused.log; exit $rc; fi
timeout -k 10 120 python scripts/bench_conv.py > gpurun_out/bench_conv2.log 2>&1; rc=$?; cat gpurun_out/bench_conv2.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 300 --warmup 30 > gpurun_out/bench_hip9.log 2>&1; rc=$?; tail -1 gpurun_out/bench_hip9.log | cut -c1-250
exit $rc
