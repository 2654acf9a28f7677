cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -m pytest tests -m gpu -q -rf -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 300 --warmup 30 > gpurun_out/bench_hip5.log 2>&1; rc=$?; tail -1 gpurun_out/bench_hip5.log | cut -c1-400
[ $rc -ne 0 ] && exit $rc
TAG=hip3 bash scripts/gpu_profile.sh
