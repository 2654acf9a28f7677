#!/bin/bash
# multirank sharded-DP test with the FC1 DP weight gradient sliced (0) then in place (1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/mr
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in 0 1; do
  APEX_FC1_DP_INPLACE=$v timeout -k 10 280 python -u -m pytest tests/test_gpu_multirank.py -k sharded -x -v --timeout 250 --timeout-method thread > $O/t$v.log 2>&1
  rc=$?; echo "inplace=$v rc=$rc"; grep -E "passed|failed|PASSED|FAILED" $O/t$v.log | tail -3; [ $rc -ne 0 ] && exit $rc
done
exit 0
