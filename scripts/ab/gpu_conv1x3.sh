#!/bin/bash
# Exact-split conv1: numerics tests, per-kernel microbench (variants 0 fp32-MFMA, 2 exact split), bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/c1x3
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_f32_net.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1
rc=$?; tail -15 $O/t.log | grep -v "^$"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u scripts/bench_f32.py --only conv1 --variants 0,2 > $O/k.log 2>&1 && APEX_F32_KNOBS=9=0 timeout -k 10 200 python -u scripts/bench_f32.py --only conv1_wgrad > $O/kw0.log 2>&1 &&
timeout -k 10 200 python -u scripts/bench_f32.py --B 256 --only conv1_fwd --variants 0,2 > $O/k256.log 2>&1 &&
timeout -k 10 200 python -u bench.py --steps 2000 --warmup 50 > $O/b.log 2>&1
rc=$?
grep -v amdgpu $O/k.log; grep -v amdgpu $O/kw0.log; grep -v amdgpu $O/k256.log; grep '^{' $O/b.log | cut -c1-180
exit $rc
