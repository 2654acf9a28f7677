#!/bin/bash
# One gpurun call: GPU AQL trainer tests, then an AQL_dis CartPole-v0 learning run on the GPU
# env with greedy evaluations (profiles/r3_aql_learning_curve.jsonl).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/aql_run
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_train_aql.py tests/test_gpu_aql_engine.py -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_aql.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_aql.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 ${AQL_T:-600} python -u -m apex_amd.train_aql --env ${AQL_ENV:-CartPole-v0} --max-step ${AQL_ITERS:-8000} \
  --n-envs ${AQL_E:-256} --capacity 1000000 --save-interval 2000 --log-interval 100 --eval-interval ${AQL_EVAL:-500} \
  --save-dir gpurun_out/aql_run --log-dir gpurun_out/aql_run/tb --json-log gpurun_out/aql_learning.jsonl \
  > gpurun_out/aql_learning.log 2>&1
rc=$?; echo "train rc=$rc"; grep greedy gpurun_out/aql_learning.log | cut -c1-300 | tail -20
rm -f gpurun_out/aql_run/*.pth gpurun_out/aql_run/*.pt
exit $rc
