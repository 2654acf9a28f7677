#!/bin/bash
# GEMM body: MFMA block fenced from the LDS store (knob 8 = 3) vs the default: microbench + bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/fence
mkdir -p $O
APEX_F32_KNOBS=8=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_f32_net.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1
rc=$?; tail -2 $O/t.log; [ $rc -ne 0 ] && exit $rc
APEX_F32_KNOBS=8=3 timeout -k 10 200 python -u scripts/bench_f32.py > $O/k3.log 2>&1 &&
timeout -k 10 200 python -u scripts/bench_f32.py > $O/k1.log 2>&1 &&
APEX_F32_KNOBS=8=3 timeout -k 10 200 python -u bench.py --steps 2000 --warmup 50 > $O/b3.log 2>&1 &&
timeout -k 10 200 python -u bench.py --steps 2000 --warmup 50 > $O/b1.log 2>&1
rc=$?
echo "== fenced"; grep -v amdgpu $O/k3.log; echo "== default"; grep -v amdgpu $O/k1.log
for f in b3 b1; do grep '^{' $O/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'])"; done
exit $rc
