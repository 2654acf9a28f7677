#!/bin/bash
# One gpurun call: the fused AQL step tail -- engine tests (bit-identity vs the separate launches,
# fp64 reference), learner-step microbench A/B, the config-4 bench and a kernel-stats profile.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/aqlf
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_aql_engine.py \
  > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
for f in 0 1; do
  timeout -k 10 120 python -u scripts/bench_aql.py --iters 200 --fused-step $f >> $O/micro.log 2>&1 || exit $?
done
grep fused_step $O/micro.log | cut -c1-120
timeout -k 10 300 python -u bench.py --algo aql --steps 500 --warmup 20 > $O/bench.log 2>&1 || exit $?
grep '^{' $O/bench.log | cut -c1-400
timeout -k 10 300 python -u bench.py --algo aql --steps 500 --warmup 20 --aql-overlap > $O/bench_overlap.log 2>&1 || exit $?
grep -o '"value": [0-9.]*' $O/bench_overlap.log
[ -z "$PROF" ] && exit 0
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run \
   -- python3 $R/bench.py --algo aql --steps 100 --warmup 10 > $O/prof.log 2>&1
