#!/bin/bash
# Row-state loaders: fp32 numerics tests, per-kernel microbench, full bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/rs
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_f32_net.py tests/test_gpu_learning.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 &&
timeout -k 10 200 python -u scripts/bench_f32.py > $O/k.log 2>&1 &&
timeout -k 10 200 python -u bench.py --steps 2000 --warmup 50 > $O/b.log 2>&1
rc=$?
tail -3 $O/t.log; grep -v amdgpu $O/k.log | tail -14; grep '^{' $O/b.log | cut -c1-300
exit $rc
