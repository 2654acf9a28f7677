#!/bin/bash
# Round 5: exact-split bf16 GEMMs (X6) vs f32 MFMA -- accuracy test, per-launch timing, whole step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_f32_net.py \
  > gpurun_out/r5_x6_test.log 2>&1; rc=$?; echo "== f32 tests rc=$rc"; grep -E "x6=|passed|failed|Error" gpurun_out/r5_x6_test.log | head -30
[ $rc -ne 0 ] && exit $rc
for x in 0 1 0 1; do
  timeout -k 10 120 python scripts/bench_f32.py --x6 $x > gpurun_out/r5_bench_f32_x$x.log 2>&1 || exit $?
  echo "== bench_f32 x6=$x"; cat gpurun_out/r5_bench_f32_x$x.log
done
for x in 0 1 0 1; do
  timeout -k 10 200 python scripts/ab/x6_bench.py $x --steps 2000 --warmup 50 > gpurun_out/r5_bench_x$x.log 2>&1 || exit $?
  echo "== bench x6=$x"; grep '^{' gpurun_out/r5_bench_x$x.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
done
