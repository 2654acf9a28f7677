#!/bin/bash
# conv2 / conv3 weight-gradient tile width (knob 24): 0 = 64, 1 = 128 / 192, 2 = 256 / 192
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/wgrad_wide
for k in 1 2; do
  APEX_F32_KNOBS="24=$k" timeout -k 10 300 python -u -m pytest tests/test_gpu_f32_net.py tests/test_gpu_fused_bwd.py -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/wgrad_wide/pytest_$k.log 2>&1
  rc=$?; echo "pytest knob24=$k rc=$rc"; tail -2 gpurun_out/wgrad_wide/pytest_$k.log; [ $rc -ne 0 ] && exit $rc
done
for k in 0 1 2; do
  APEX_F32_KNOBS="24=$k" timeout -k 10 120 python scripts/bench_f32.py --only bwd --bwd-sweep --iters 30 > gpurun_out/wgrad_wide/micro_$k.txt 2>&1
  rc=$?; echo "knob24=$k"; cat gpurun_out/wgrad_wide/micro_$k.txt; [ $rc -ne 0 ] && exit $rc
done
for k in 0 1 2 0 1 2; do
  APEX_F32_KNOBS="24=$k" timeout -k 10 200 python bench.py --steps 2000 --warmup 50 > gpurun_out/wgrad_wide/bench.log 2>&1
  rc=$?; echo "bench knob24=$k rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/wgrad_wide/bench.log)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
