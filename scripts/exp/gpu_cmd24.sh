cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests/test_gpu_overlap.py tests/test_gpu_train_cli.py -q -rf -x > gpurun_out/pytest_ovl.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_ovl.log
if [ $rc -ne 0 ]; then tail -60 gpurun_out/pytest_ovl.log; exit $rc; fi
BENCH_VARIANTS="ovl:" bash scripts/gpu_ab.sh || exit $?
TAG=ovl_h STEPS=300 bash scripts/gpu_profile.sh
