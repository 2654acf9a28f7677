#!/bin/bash
# conv1 fwd (exact split) with the next sample's frames prefetched: tests, microbench, bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/c1pf
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_f32_net.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1
rc=$?; tail -3 $O/t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u scripts/bench_f32.py --only conv1 > $O/k.log 2>&1 && APEX_F32_KNOBS=9=1 timeout -k 10 200 python -u scripts/bench_f32.py --only conv1_wgrad > $O/kw1.log 2>&1 &&
timeout -k 10 200 python -u scripts/bench_f32.py --B 256 --only conv1_fwd > $O/k256.log 2>&1 &&
timeout -k 10 200 python -u bench.py --steps 2000 --warmup 50 > $O/b.log 2>&1
rc=$?
grep -v amdgpu $O/k.log; grep -v amdgpu $O/kw1.log; grep -v amdgpu $O/k256.log
grep '^{' $O/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['host_enqueue_ms_per_step'], d['host_launch_ms_per_step'])"
exit $rc
