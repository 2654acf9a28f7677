#!/bin/bash
# Round-4 end check: multirank + the whole GPU suite + smoke + 1-GPU bench x2 + AQL bench +
# the 3-rank same-device central bench, then a kernel-stats profile of the 1-GPU step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
SKIP_TRACE=1 bash scripts/gpu_r4_check.sh || exit $?
timeout -k 10 300 python bench.py --steps 2000 --warmup 50 > gpurun_out/bench1b.log 2>&1
rc=$?; echo "== bench1b rc=$rc"; grep '^{' gpurun_out/bench1b.log | cut -c1-400
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --algo aql --steps 1000 --warmup 20 > gpurun_out/bench_aql.log 2>&1
rc=$?; echo "== bench_aql rc=$rc"; grep '^{' gpurun_out/bench_aql.log | cut -c1-400
[ $rc -ne 0 ] && exit $rc
bash scripts/gpu_prof_bench.sh
