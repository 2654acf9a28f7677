#!/bin/bash
# XCD-chunked tile order (knob 11) A/B: fp32 net tests, per-kernel microbench, bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/xcd
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_f32_net.py tests/test_gpu_learning.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1
rc=$?; tail -3 $O/t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u scripts/bench_f32.py > $O/k1.log 2>&1 &&
APEX_F32_KNOBS=11=0 timeout -k 10 200 python -u scripts/bench_f32.py > $O/k0.log 2>&1 &&
timeout -k 10 200 python -u bench.py --steps 2000 --warmup 50 > $O/b1.log 2>&1 &&
APEX_F32_KNOBS=11=0 timeout -k 10 200 python -u bench.py --steps 2000 --warmup 50 > $O/b0.log 2>&1
rc=$?
echo "== xcd chunked"; grep -v amdgpu $O/k1.log; echo "== identity"; grep -v amdgpu $O/k0.log
for f in b1 b0; do grep '^{' $O/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'])"; done
exit $rc
