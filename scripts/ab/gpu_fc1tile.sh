#!/bin/bash
# FC1 forward tile A/B (knob 13): fp32 numerics tests per tile, microbench, bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/fc1t
mkdir -p $O
for v in 1 2; do
  APEX_F32_KNOBS="13=$v" timeout -k 10 300 python -u -m pytest tests/test_gpu_f32_net.py -x -q --timeout 120 --timeout-method thread > $O/t$v.log 2>&1
  rc=$?; echo "tests tile $v rc=$rc"; tail -2 $O/t$v.log; [ $rc -ne 0 ] && exit $rc
done
for v in 0 1 2; do
  APEX_F32_KNOBS="13=$v" timeout -k 10 200 python -u scripts/bench_f32.py --only fc1_fwd > $O/k$v.log 2>&1 || exit 1
  echo "tile $v: $(grep fc1 $O/k$v.log)"
done
for v in 0 1 2 0 1 2; do
  APEX_F32_KNOBS="13=$v" timeout -k 10 200 python -u bench.py --steps 2000 --warmup 50 > $O/b$v.log 2>&1 || exit 1
  echo "bench tile $v: $(grep '^{' $O/b$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done
