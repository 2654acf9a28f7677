#!/bin/bash
# Tree-write kernels: replay / fused-write tests, 2000-step bench, kernel-trace Gantt.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
REPO=$(pwd)
O=$REPO/gpurun_out/tree
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_replay.py tests/test_gpu_fused_bwd.py tests/test_gpu_learner.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 &&
timeout -k 10 200 python -u bench.py --steps 2000 --warmup 50 ${BENCH_ARGS:-} > $O/b.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 $REPO/bench.py --steps 100 --warmup 20 ${BENCH_ARGS:-} > $O/prof_stdout.log 2>&1
rc=$?
cd $REPO
tail -2 $O/t.log; grep '^{' $O/b.log | cut -c1-200
T=$(find $O/prof -name "*kernel_trace.csv" | head -1)
[ -n "$T" ] && python3 scripts/prof_timeline.py "$T" --dump-step > $O/timeline.txt 2>&1 && cat $O/timeline.txt
exit $rc
