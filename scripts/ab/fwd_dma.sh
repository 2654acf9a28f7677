#!/bin/bash
# fp32 forward GEMMs on the LDS-DMA ring body (knob 23 = ring stages): numerics tests, per-launch
# microbench, whole bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/fwd_dma
for S in 4 3; do
  APEX_F32_KNOBS="23=$S" timeout -k 10 300 python -u -m pytest tests/test_gpu_f32_net.py tests/test_gpu_fused_net.py -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/fwd_dma/pytest_$S.log 2>&1
  rc=$?; echo "pytest S=$S rc=$rc"; tail -2 gpurun_out/fwd_dma/pytest_$S.log; [ $rc -ne 0 ] && exit $rc
done
for S in 0 2 3 4; do
  APEX_F32_KNOBS="23=$S" timeout -k 10 120 python scripts/bench_px.py --iters 30 --terms 0 --bwd 0 > gpurun_out/fwd_dma/micro_$S.txt 2>&1
  rc=$?; echo "S=$S"; grep fwd gpurun_out/fwd_dma/micro_$S.txt; [ $rc -ne 0 ] && exit $rc
done
for S in 0 4 3 0 4 3; do
  APEX_F32_KNOBS="23=$S" timeout -k 10 200 python bench.py --steps 2000 --warmup 50 > gpurun_out/fwd_dma/bench.log 2>&1
  rc=$?; echo "bench S=$S rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/fwd_dma/bench.log)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
