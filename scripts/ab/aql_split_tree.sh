#!/bin/bash
# AQL priority write: own launch (default) vs folded into the noise reset (FUSED_TREE) vs split
# over the gradient contraction + noise reset (SPLIT_TREE), after the ILP level walk.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/aql_split
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_aql_engine.py tests/test_gpu_fused_bwd.py tests/test_gpu_replay.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
for v in base split fused base split fused; do
  case $v in base) E="APEX_AQL_SPLIT_TREE=0";; split) E="APEX_AQL_SPLIT_TREE=1";; fused) E="APEX_AQL_SPLIT_TREE=0 APEX_AQL_FUSED_TREE=1";; esac
  env $E timeout -k 10 200 python bench.py --algo aql --steps 500 --warmup 20 > $O/bench_$v.log 2>&1 || exit 1
  echo "$v: $(grep -o '"value": [0-9.]*' $O/bench_$v.log)"
done
