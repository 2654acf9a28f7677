#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/ab
for k in 1 2; do
  for v in "" "--aql-levels-in-grad 0" "--aql-levels-in-bwd 2" "--aql-levels-in-bwd 0"; do
    timeout -k 10 200 python bench.py --algo aql --steps 500 --warmup 20 $v > gpurun_out/ab/b.log 2>&1 || exit $?
    echo "[$v]: $(grep -o '"value": [0-9.]*' gpurun_out/ab/b.log)"
  done
done
