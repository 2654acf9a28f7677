#!/bin/bash
# px forward k-block depth 64 (full 128-byte plane rows; knob 22) x pipeline form (knob 21)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/px_bk
APEX_F32_KNOBS="22=64" timeout -k 10 300 python -u -m pytest tests/test_gpu_px.py -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/px_bk/pytest.log 2>&1
rc=$?; echo "pytest bk64 rc=$rc"; tail -2 gpurun_out/px_bk/pytest.log; [ $rc -ne 0 ] && exit $rc
APEX_F32_KNOBS="22=64" timeout -k 10 200 python scripts/bench_px.py --iters 30 --pipes 0,1 --terms 0,6,8 --bwd 0 > gpurun_out/px_bk/bench.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/px_bk/bench.txt; exit $rc
