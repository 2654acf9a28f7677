#!/bin/bash
# Quick kernel loop: fp32-net numerics tests + the per-launch microbench (one gpurun call).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_f32_net.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_f32.log 2>&1
rc=$?; echo "== f32 tests rc=$rc"; tail -3 gpurun_out/pytest_f32.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/bench_f32.py ${BENCH_ARGS} > gpurun_out/bench_f32.log 2>&1
rc=$?; echo "== bench_f32 rc=$rc"; cat gpurun_out/bench_f32.log
exit $rc
