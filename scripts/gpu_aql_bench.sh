#!/bin/bash
# One gpurun call: GPU AQL engine bench (BASELINE config 4) + a rocprofv3 kernel-stats profile.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/aql
mkdir -p $O
cd $R
timeout -k 10 300 python -u bench.py --algo aql --steps ${STEPS:-500} --warmup 20 ${BENCH_ARGS} > $O/bench.log 2>&1 &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run \
   -- python3 $R/bench.py --algo aql --steps 100 --warmup 10 ${BENCH_ARGS} > $O/prof.log 2>&1)
rc=$?
grep '^{' $O/bench.log | cut -c1-600
exit $rc
