cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -m pytest tests -m gpu -q -rf -x > gpurun_out/pytest_all.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_all.log
if [ $rc -ne 0 ]; then tail -80 gpurun_out/pytest_all.log; exit $rc; fi
bash scripts/gpu_bench_pair.sh
