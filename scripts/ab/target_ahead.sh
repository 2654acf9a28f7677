#!/bin/bash
# sampled-ahead batches with the target pass beside the previous step (--target-ahead 1) vs the
# 3-pass forward (default): tests, then interleaved 2000-step benches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/target_ahead
timeout -k 10 600 python -u -m pytest tests/test_gpu_learner.py tests/test_gpu_overlap.py -x -v -rf --timeout 120 --timeout-method thread > gpurun_out/target_ahead/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/target_ahead/pytest.log; [ $rc -ne 0 ] && exit $rc
for t in 0 1 2 0 1 2; do
  timeout -k 10 200 python bench.py --steps 2000 --warmup 50 $( [ $t = 2 ] && echo "--target-ahead 1 --target-pass fork" || echo "--target-ahead $t") > gpurun_out/target_ahead/bench_$t.log 2>&1
  rc=$?; echo "ahead=$t rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/target_ahead/bench_$t.log)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
