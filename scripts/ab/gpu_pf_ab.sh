#!/bin/bash
# A/B of the fp32 GEMM-body prefetch depth (APEX_F32_KNOBS=8=2): per-kernel microbench, then
# the full bench, for both depths.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pf
mkdir -p $O
cd $R
timeout -k 10 200 python -u scripts/bench_f32.py > $O/k_pf1.log 2>&1 &&
APEX_F32_KNOBS=8=2 timeout -k 10 200 python -u scripts/bench_f32.py > $O/k_pf2.log 2>&1 &&
timeout -k 10 200 python -u bench.py --steps 2000 --warmup 50 > $O/b_pf1.log 2>&1 &&
APEX_F32_KNOBS=8=2 timeout -k 10 200 python -u bench.py --steps 2000 --warmup 50 > $O/b_pf2.log 2>&1
rc=$?
for f in k_pf1 k_pf2; do echo "== $f"; grep -v amdgpu $O/$f.log | tail -12; done
for f in b_pf1 b_pf2; do echo "== $f"; grep '^{' $O/$f.log | cut -c1-300; done
exit $rc
