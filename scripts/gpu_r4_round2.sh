#!/bin/bash
# One call: AQL A/B (scripts/ab/aql_bwd_tree.sh), the learner bench kernel trace, and the conv1
# forward diagnostics microbench (interleaved twice).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/ab/aql_bwd_tree.sh || exit $?
for k in 1 2; do
  timeout -k 10 200 python scripts/bench_f32.py --only conv1_fwd --c1-diag > gpurun_out/c1diag_$k.log 2>&1
  rc=$?; cat gpurun_out/c1diag_$k.log; [ $rc -ne 0 ] && exit $rc
done
bash scripts/gpu_prof_bench.sh
