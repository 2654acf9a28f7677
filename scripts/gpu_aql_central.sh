#!/bin/bash
# Distributed AQL_dis over HIP IPC on one GPU (3 processes: learner + 2 actor ranks):
# the transition-completeness test, the central AQL bench, then a CartPole-v0 learning run
# with greedy evaluations (profiles/r4_aql_central_*).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/aql_central
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_central_aql.py -x -v --timeout 240 --timeout-method thread \
  > gpurun_out/pytest_central_aql.log 2>&1
rc=$?; echo "== test rc=$rc"; tail -4 gpurun_out/pytest_central_aql.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --algo aql --gpus 3 --same-device --backend gloo --steps 200 --warmup 20 \
  > gpurun_out/bench_aql_central3.log 2>&1
rc=$?; echo "== bench rc=$rc"; grep '^{' gpurun_out/bench_aql_central3.log | cut -c1-2500
[ $rc -ne 0 ] && exit $rc
[ -n "$SKIP_LEARN" ] && exit 0
timeout -k 10 ${AQL_T:-700} python -u -m apex_amd.train_aql --gpus 3 --same-device --env CartPole-v0 \
  --max-step ${AQL_ITERS:-4000} --n-envs 128 --capacity 1000000 --save-interval 100000 --log-interval 100 \
  --eval-interval ${AQL_EVAL:-250} --save-dir gpurun_out/aql_central --no-tb \
  --json-log gpurun_out/aql_central_learning.jsonl > gpurun_out/aql_central_learning.log 2>&1
rc=$?; echo "== train rc=$rc"; grep greedy gpurun_out/aql_central_learning.log | cut -c1-300 | tail -20
rm -f gpurun_out/aql_central/*.pth gpurun_out/aql_central/*.pt
exit $rc
