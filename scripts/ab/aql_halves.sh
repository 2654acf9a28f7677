#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/ab
for k in 1 2; do
  for v in 2 1; do
    timeout -k 10 200 python bench.py --algo aql --steps 500 --warmup 20 --aql-fwd-halves $v > gpurun_out/ab/b.log 2>&1 || exit $?
    echo "halves=$v: $(grep -o '"value": [0-9.]*' gpurun_out/ab/b.log)"
  done
done
