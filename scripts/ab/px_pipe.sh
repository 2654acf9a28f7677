#!/bin/bash
# px / pxb pipeline forms (knob 21) vs the fp32 bodies at the learner's shapes; px tests first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/px_pipe
export HSA_ENABLE_IPC_MODE_LEGACY=0
for pipe in 0 1; do
  APEX_F32_KNOBS="21=$pipe" timeout -k 10 300 python -u -m pytest tests/test_gpu_px.py -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/px_pipe/pytest_pipe$pipe.log 2>&1
  rc=$?; echo "pytest pipe=$pipe rc=$rc"; tail -2 gpurun_out/px_pipe/pytest_pipe$pipe.log
  [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 200 python scripts/bench_px.py --iters 30 --pipes 0,1 > gpurun_out/px_pipe/bench.txt 2>&1
rc=$?; cat gpurun_out/px_pipe/bench.txt; exit $rc
