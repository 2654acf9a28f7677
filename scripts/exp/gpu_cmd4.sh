cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -m pytest tests/test_gpu_fused_net.py -q -rf -x > gpurun_out/pytest_fused.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_fused.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python scripts/debug_hip_learner.py 512 256 > gpurun_out/debug5.log 2>&1; echo "debug rc=$?"; head -20 gpurun_out/debug5.log | cut -c1-200; tail -3 gpurun_out/debug5.log | cut -c1-400
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --forward hip > gpurun_out/bench_hip3.log 2>&1; rc=$?; tail -1 gpurun_out/bench_hip3.log
exit $rc
