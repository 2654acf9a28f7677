#!/bin/bash
# One call: replay / AQL GPU tests (tree walks bit-identical), AQL engine bench interleaved
# (update launch vs separate launches), a kernel trace of the default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
timeout -k 10 200 python scripts/diag/aql_variants.py || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_aql_engine.py tests/test_gpu_replay.py tests/test_gpu_aql.py -x -q \
  --timeout 240 --timeout-method thread > gpurun_out/ab/test.log 2>&1
rc=$?; echo "== tests rc=$rc"; tail -3 gpurun_out/ab/test.log
[ $rc -ne 0 ] && exit $rc
APEX_AQL_DBG=1 timeout -k 10 120 python scripts/bench_aql.py --fused-step 0 --iters 200 || exit $?
for k in 1 2; do
  for v in "--aql-fused-update 0" "--aql-fused-update 1 --aql-levels-in-grad 1" "--aql-fused-update 1"; do
    timeout -k 10 200 python bench.py --algo aql --steps 500 --warmup 20 $v > gpurun_out/ab/b.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "bench rc=$rc"; tail -5 gpurun_out/ab/b.log; exit $rc; }
    echo "$v: $(grep -o '"value": [0-9.]*' gpurun_out/ab/b.log)"
  done
done
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ab/prof -o run -- \
  python3 $R/bench.py --algo aql --steps 200 --warmup 10 > $R/gpurun_out/ab/prof.log 2>&1
