#!/bin/bash
# One call: conv1 forward double-buffered vs single-buffered (bit-identity + interleaved timing),
# then the AQL A/B (scripts/ab/aql_bwd_tree.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for k in 1 2; do
  timeout -k 10 200 python scripts/bench_f32.py --only conv1_fwd --c1-db > gpurun_out/c1db_$k.log 2>&1
  rc=$?; cat gpurun_out/c1db_$k.log; [ $rc -ne 0 ] && exit $rc
done
bash scripts/ab/aql_bwd_tree.sh
