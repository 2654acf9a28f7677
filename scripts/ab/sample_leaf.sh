#!/bin/bash
# per_sample / fused AQL draw taking the leaf value from the descent + finalize load fixes:
# replay, learner, AQL and f32 tests, then both benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/sl
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_replay.py tests/test_gpu_aql_engine.py tests/test_gpu_learner.py tests/test_gpu_f32_net.py tests/test_gpu_fused_bwd.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 2000 --warmup 50 > $O/bench_$r.log 2>&1 || exit 1
  echo "bench: $(grep -o '"value": [0-9.]*' $O/bench_$r.log)"
  timeout -k 10 200 python bench.py --algo aql --steps 500 --warmup 20 > $O/aql_$r.log 2>&1 || exit 1
  echo "aql: $(grep -o '"value": [0-9.]*' $O/aql_$r.log)"
done
