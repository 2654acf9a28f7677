#!/bin/bash
# One gpurun call: fp32 + bf16 1-GPU benches, an fp32 rocprofv3 kernel-stats profile,
# then the GPU test suite.  Every GPU step has its own time limit; steps chained with &&.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u bench.py --steps 2000 --warmup 50 > $O/bench_fp32.log 2>&1 &&
timeout -k 10 300 python -u bench.py --dtype bf16 --steps 2000 --warmup 50 > $O/bench_bf16.log 2>&1 &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_fp32 -o run \
   -- python3 $R/bench.py --steps 200 --warmup 20 > $O/prof_fp32.log 2>&1) &&
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} \
   > $O/gputest.log 2>&1
