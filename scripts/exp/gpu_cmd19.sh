cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests/test_gpu_fused_net.py -q -rf -x > gpurun_out/pytest_c1.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_c1.log
if [ $rc -ne 0 ]; then tail -80 gpurun_out/pytest_c1.log; exit $rc; fi
timeout -k 10 120 python scripts/bench_conv.py --B 1536 --only conv1 > gpurun_out/bc_c1.log 2>&1; cat gpurun_out/bc_c1.log
timeout -k 10 120 python scripts/bench_conv.py --B 256 --only conv1 >> gpurun_out/bc_c1.log 2>&1; tail -2 gpurun_out/bc_c1.log
timeout -k 10 300 python bench.py --steps 2000 --warmup 50 --overlap > gpurun_out/bench_ovl_c1.log 2>&1; rc=$?; tail -1 gpurun_out/bench_ovl_c1.log | cut -c1-150
exit $rc
