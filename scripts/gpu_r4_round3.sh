#!/bin/bash
# One call: fp32 net numerics tests, conv1 forward timing (+ diagnostics), the 1-GPU learner
# bench, then the AQL A/B (scripts/ab/aql_bwd_tree.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_f32_net.py tests/test_gpu_learning.py -x -q \
  --timeout 240 --timeout-method thread > gpurun_out/pytest_f32.log 2>&1
rc=$?; echo "== f32 tests rc=$rc"; tail -3 gpurun_out/pytest_f32.log
[ $rc -ne 0 ] && exit $rc
for k in 1 2; do
  timeout -k 10 200 python scripts/bench_f32.py --only conv1_fwd --c1-diag > gpurun_out/c1diag_$k.log 2>&1
  rc=$?; cat gpurun_out/c1diag_$k.log; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 python bench.py --steps 2000 --warmup 50 > gpurun_out/bench1.log 2>&1
rc=$?; echo "== bench rc=$rc"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/bench1.log | tr '\n' ' '; echo
[ $rc -ne 0 ] && exit $rc
bash scripts/ab/aql_bwd_tree.sh
