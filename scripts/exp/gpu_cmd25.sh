cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -m pytest tests -m gpu -q -rf -x > gpurun_out/pytest_all.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_all.log
if [ $rc -ne 0 ]; then tail -80 gpurun_out/pytest_all.log; exit $rc; fi
timeout -k 10 200 python scripts/bench_conv.py --only fc1_bwd > gpurun_out/bc_b.log 2>&1; timeout -k 10 200 python scripts/bench_conv.py --only finalize >> gpurun_out/bc_b.log 2>&1; grep " us" gpurun_out/bc_b.log
timeout -k 10 300 python scripts/host_probe.py || exit $?
BENCH_VARIANTS="ovl:" bash scripts/gpu_ab.sh
