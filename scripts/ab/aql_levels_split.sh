#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/ab
timeout -k 10 200 python scripts/diag/aql_variants.py || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_aql_engine.py tests/test_gpu_replay.py -x -q --timeout 240 \
  --timeout-method thread > gpurun_out/ab/test.log 2>&1
rc=$?; echo "== tests rc=$rc"; tail -2 gpurun_out/ab/test.log; [ $rc -ne 0 ] && exit $rc
for k in 1 2; do
  for v in 0 1 2; do
    timeout -k 10 200 python bench.py --algo aql --steps 500 --warmup 20 --aql-levels-in-bwd $v > gpurun_out/ab/b.log 2>&1 || exit $?
    echo "levels_in_bwd=$v: $(grep -o '"value": [0-9.]*' gpurun_out/ab/b.log)"
  done
done
