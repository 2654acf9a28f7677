#!/bin/bash
# AQL priority write: extra workgroup of the backward launch (bwd_tree) vs split over the
# gradient / noise-reset launches -- bit-identity test, then interleaved benches, then a
# kernel trace of the bwd_tree configuration.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_aql_engine.py -x -q -k fused_sampling --timeout 240 \
  --timeout-method thread > gpurun_out/ab/test.log 2>&1
rc=$?; echo "== test rc=$rc"; tail -3 gpurun_out/ab/test.log
[ $rc -ne 0 ] && exit $rc
for k in 1 2; do
  for t in 0 1; do
    timeout -k 10 200 python bench.py --algo aql --steps 500 --warmup 20 --aql-bwd-tree $t > gpurun_out/ab/b$t.$k.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "bench rc=$rc"; tail -5 gpurun_out/ab/b$t.$k.log; exit $rc; }
    echo "bwd_tree=$t: $(grep -o '"value": [0-9.]*' gpurun_out/ab/b$t.$k.log)"
  done
done
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ab/prof -o run -- \
  python3 $R/bench.py --algo aql --steps 200 --warmup 10 --aql-bwd-tree 1 > $R/gpurun_out/ab/prof.log 2>&1
