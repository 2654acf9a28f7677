#!/bin/bash
# px plane-stride padding A/B (APEX_PX_PAD elements between the bf16 planes)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/px_pad
APEX_PX_PAD=2112 timeout -k 10 300 python -u -m pytest tests/test_gpu_px.py -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/px_pad/pytest.log 2>&1
rc=$?; echo "pytest pad rc=$rc"; tail -2 gpurun_out/px_pad/pytest.log; [ $rc -ne 0 ] && exit $rc
for pad in 0 2112 65600; do
  APEX_PX_PAD=$pad timeout -k 10 200 python scripts/bench_px.py --iters 30 --pipes 0,1 --terms 0,8 > gpurun_out/px_pad/bench_$pad.txt 2>&1
  rc=$?; echo "pad=$pad"; grep -v amdgpu.ids gpurun_out/px_pad/bench_$pad.txt; [ $rc -ne 0 ] && exit $rc
done
exit 0
