#!/bin/bash
# AQL: acting grid size, serial vs overlapped acting, fused sampling -- engine tests, then the bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/aql_actq
timeout -k 10 300 python -u -m pytest tests/test_gpu_aql_engine.py tests/test_gpu_train_aql.py -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/aql_actq/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/aql_actq/pytest.log; [ $rc -ne 0 ] && exit $rc
for cfg in "64 1 " "64 0 " "32 1 " "128 1 " "64 1 --no-overlap" "1024 1 --no-overlap" "64 1 "; do
  set -- $cfg
  APEX_AQL_ACT_BLOCKS=$1 APEX_AQL_FUSED_SAMPLE=$2 timeout -k 10 200 python bench.py --algo aql --steps 500 --warmup 20 $3 > gpurun_out/aql_actq/bench.log 2>&1
  rc=$?; echo "blocks=$1 fused=$2 $3 rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/aql_actq/bench.log) $(grep -o '"host_enqueue_ms_per_step": [0-9.]*' gpurun_out/aql_actq/bench.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/aql_actq/bench.log)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
