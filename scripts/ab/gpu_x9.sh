#!/bin/bash
# Exact-split GEMM body (knob 10): numerics tests, per-kernel microbench x9 vs fp32 MFMA, bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/x9
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_f32_net.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1
rc=$?; tail -15 $O/t.log | grep -v "^$"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u scripts/bench_f32.py > $O/k1.log 2>&1 &&
APEX_F32_KNOBS=10=0 timeout -k 10 200 python -u scripts/bench_f32.py > $O/k0.log 2>&1 &&
timeout -k 10 200 python -u bench.py --steps 2000 --warmup 50 > $O/b.log 2>&1
rc=$?
echo "== x9"; grep -v amdgpu $O/k1.log; echo "== fp32 mfma"; grep -v amdgpu $O/k0.log; grep '^{' $O/b.log | cut -c1-180
exit $rc
