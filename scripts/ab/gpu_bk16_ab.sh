#!/bin/bash
# conv2/conv3 forward BK = 16 tiles (knob 12) vs BK = 32: tests, microbench, bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/bk16
mkdir -p $O
APEX_F32_KNOBS=12=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_f32_net.py -x -q --timeout 120 --timeout-method thread > $O/t1.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_f32_net.py -x -q --timeout 120 --timeout-method thread > $O/t0.log 2>&1
rc=$?; tail -1 $O/t1.log; tail -1 $O/t0.log; [ $rc -ne 0 ] && exit $rc
APEX_F32_KNOBS=12=1 timeout -k 10 200 python -u scripts/bench_f32.py --only fwd > $O/k1.log 2>&1 &&
timeout -k 10 200 python -u scripts/bench_f32.py --only fwd > $O/k0.log 2>&1 &&
APEX_F32_KNOBS=12=1 timeout -k 10 200 python -u bench.py --steps 2000 --warmup 50 > $O/b1.log 2>&1 &&
timeout -k 10 200 python -u bench.py --steps 2000 --warmup 50 > $O/b0.log 2>&1
rc=$?
echo "== bk16"; grep -v amdgpu $O/k1.log; echo "== bk32"; grep -v amdgpu $O/k0.log
for f in b1 b0; do grep '^{' $O/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'])"; done
exit $rc
