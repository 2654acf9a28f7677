#!/bin/bash
# learner conv forward tiles 128 x 64 (knob 14 = 3: 2 x 2 waves of 64 x 32) vs 64 x 64 (default 2)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/convtile3
APEX_F32_KNOBS="14=3" timeout -k 10 300 python -u -m pytest tests/test_gpu_f32_net.py -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/convtile3/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/convtile3/pytest.log; [ $rc -ne 0 ] && exit $rc
for k in 2 3; do
  APEX_F32_KNOBS="14=$k" timeout -k 10 120 python scripts/bench_px.py --iters 30 --terms 0 --bwd 0 > gpurun_out/convtile3/micro_$k.txt 2>&1
  rc=$?; echo "knob14=$k"; grep fwd gpurun_out/convtile3/micro_$k.txt; [ $rc -ne 0 ] && exit $rc
done
for k in 2 3 2 3; do
  APEX_F32_KNOBS="14=$k" timeout -k 10 200 python bench.py --steps 2000 --warmup 50 > gpurun_out/convtile3/bench.log 2>&1
  rc=$?; echo "bench knob14=$k rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/convtile3/bench.log)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
