#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests/test_gpu_aql_engine.py tests/test_gpu_aql.py -x -q --timeout 240 \
  --timeout-method thread > gpurun_out/ab/test.log 2>&1
rc=$?; echo "== tests rc=$rc"; tail -2 gpurun_out/ab/test.log; [ $rc -ne 0 ] && exit $rc
for k in 1 2; do
  timeout -k 10 200 python bench.py --algo aql --steps 500 --warmup 20 > gpurun_out/ab/b.log 2>&1 || exit $?
  echo "aql: $(grep -o '"value": [0-9.]*' gpurun_out/ab/b.log)"
done
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ab/prof -o run -- \
  python3 $R/bench.py --algo aql --steps 200 --warmup 10 > $R/gpurun_out/ab/prof.log 2>&1
