#!/bin/bash
# One gpurun call: selected GPU tests (PYTEST_K) + a bench run.  Stops at the first crash/timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_quick.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_quick.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --steps ${STEPS:-1000} --warmup 50 ${BENCH_ARGS:-} > gpurun_out/bench_quick.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench_quick.log
exit $rc
