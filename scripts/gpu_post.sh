#!/bin/bash
# Kernel microbench + the AQL engine bench (one gpurun call's second half).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 200 python scripts/bench_f32.py > gpurun_out/bench_f32.log 2>&1
rc=$?; echo "== bench_f32 rc=$rc"; cat gpurun_out/bench_f32.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --algo aql --steps 500 --warmup 20 > gpurun_out/bench_aql.log 2>&1
rc=$?; echo "== bench_aql rc=$rc"; grep '^{' gpurun_out/bench_aql.log | cut -c1-300
exit $rc
