#!/bin/bash
# FC1 forward split-K count A/B: fp32 tests, microbench, bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/fcs
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_f32_net.py tests/test_gpu_learner.py tests/test_gpu_fused_bwd.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1
rc=$?; tail -3 $O/t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u scripts/bench_f32.py > $O/k.log 2>&1 &&
timeout -k 10 200 python -u bench.py --steps 2000 --warmup 50 > $O/b.log 2>&1
rc=$?
grep -v amdgpu $O/k.log
grep '^{' $O/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['host_launch_ms_per_step'])"
exit $rc
