#!/bin/bash
# rocprofv3 kernel trace of a short bench run (default args: fp32, overlap) -> gpurun_out/prof_bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof_bench${1:-}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O -o run -- python3 $R/bench.py --steps 200 --warmup 20 ${BENCH_ARGS} > $O/log.txt 2>&1
