#!/bin/bash
# kernel trace of the AQL engine with overlapped acting (queue placement of the acting kernels)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd); O=$R/gpurun_out/aql_ovl; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python3 $R/bench.py --algo aql --steps 100 --warmup 10 > $O/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
