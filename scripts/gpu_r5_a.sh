#!/bin/bash
# Round 5 call A: f32 kernel accuracy / identity tests (modes 0, 1, 2), per-launch and whole-step
# A/B of the register split (1) vs the staged split (2), then the tree / IPC / multirank / AQL /
# learning GPU tests.  Every GPU step has its own limit; the first failure ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5a
mkdir -p $O
export PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_f32_net.py \
  > $O/f32_test.log 2>&1; rc=$?; echo "== f32 tests rc=$rc"; grep -E "x6=|passed|failed|Error" $O/f32_test.log | head -30
[ $rc -ne 0 ] && exit $rc
for x in 1 2 1 2; do
  timeout -k 10 120 python scripts/bench_f32.py --x6 $x --tile2 > $O/bench_f32_x$x.log 2>&1 || exit $?
  echo "== bench_f32 x6=$x"; cat $O/bench_f32_x$x.log | grep -v amdgpu.ids
done
for x in 1 2 1 2; do
  timeout -k 10 200 python scripts/ab/x6_bench.py $x --steps 2000 --warmup 50 > $O/bench_x$x.log 2>&1 || exit $?
  echo "== bench x6=$x $(grep '^{' $O/bench_x$x.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done
timeout -k 10 800 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_gpu_replay.py \
  tests/test_gpu_fused_bwd.py tests/test_gpu_learner.py tests/test_gpu_overlap.py tests/test_gpu_ipc.py \
  tests/test_gpu_multirank.py tests/test_gpu_aql_engine.py tests/test_gpu_central_aql.py tests/test_gpu_learning.py \
  > $O/tests.log 2>&1; rc=$?; echo "== tests rc=$rc"; grep -E "passed|failed|FAILED|Error|median|^\| " $O/tests.log | tail -30
exit $rc
