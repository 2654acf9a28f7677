#!/bin/bash
# AQL launch fusions (sampling in the forward, priority write in the noise-reset launch):
# engine tests, then the bench with each fusion on / off.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/aql_fuse
timeout -k 10 300 python -u -m pytest tests/test_gpu_aql_engine.py tests/test_gpu_train_aql.py tests/test_gpu_aql.py -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/aql_fuse/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/aql_fuse/pytest.log; [ $rc -ne 0 ] && exit $rc
for cfg in "1 1" "1 0" "0 0" "1 1"; do
  set -- $cfg
  APEX_AQL_FUSED_SAMPLE=$1 APEX_AQL_FUSED_TREE=$2 timeout -k 10 200 python bench.py --algo aql --steps 500 --warmup 20 > gpurun_out/aql_fuse/bench.log 2>&1
  rc=$?; echo "sample=$1 tree=$2 rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/aql_fuse/bench.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/aql_fuse/bench.log)"
  [ $rc -ne 0 ] && exit $rc
done
cp gpurun_out/aql_fuse/bench.log gpurun_out/aql_fuse/bench_final.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/aql_fuse/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --algo aql --steps 100 --warmup 10 > $GRAFT_REPO_ROOT/gpurun_out/aql_fuse/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
