#!/bin/bash
# FC1 weight-gradient batch slices A/B (knob 15): fp32 tests at the default, bench per setting.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/fc1wg
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_f32_net.py tests/test_gpu_learner.py tests/test_gpu_learning.py tests/test_gpu_fused_bwd.py tests/test_gpu_overlap.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/t.log; [ $rc -ne 0 ] && exit $rc
for v in 0 1 2 4 0 2; do
  APEX_F32_KNOBS="15=$v" timeout -k 10 200 python -u bench.py --steps 2000 --warmup 50 > $O/b$v.log 2>&1 || exit 1
  echo "bench slices $v: $(grep '^{' $O/b$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done
