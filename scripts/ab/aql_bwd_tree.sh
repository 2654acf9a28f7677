#!/bin/bash
# AQL learner A/B: priority write in the backward launch (bwd_tree), the optimizers + noise +
# next draw as one launch (fused_update) vs the split write -- bit-identity tests, learner-step
# microbench with phase stamps, interleaved whole-engine benches, then a kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_aql_engine.py -x -q -k "fused_sampling or tile_groups or propose or acting" \
  --timeout 240 --timeout-method thread > gpurun_out/ab/test.log 2>&1
rc=$?; echo "== test rc=$rc"; tail -3 gpurun_out/ab/test.log
[ $rc -ne 0 ] && exit $rc
for v in "--fused-update 0" "--fused-update 1 --levels-in-grad 0" "--fused-update 1 --levels-in-grad 1"; do
  echo "== bench_aql $v"
  APEX_AQL_DBG=1 timeout -k 10 120 python scripts/bench_aql.py --fused-step 0 --iters 200 $v
  rc=$?; [ $rc -ne 0 ] && exit $rc
done
for k in 1 2; do
  for v in "--aql-fused-update 0" "--aql-fused-update 1 --aql-levels-in-grad 0" "--aql-fused-update 1 --aql-levels-in-grad 1"; do
    timeout -k 10 200 python bench.py --algo aql --steps 500 --warmup 20 $v > gpurun_out/ab/b.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "bench rc=$rc"; tail -5 gpurun_out/ab/b.log; exit $rc; }
    echo "$v: $(grep -o '"value": [0-9.]*' gpurun_out/ab/b.log)"
  done
done
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ab/prof -o run -- \
  python3 $R/bench.py --algo aql --steps 200 --warmup 10 --aql-fused-update 1 > $R/gpurun_out/ab/prof.log 2>&1
