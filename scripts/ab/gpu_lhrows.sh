#!/bin/bash
# dqn_heads_bwd rows-per-workgroup A/B (knob 16 = 4 | 8): learner tests at 4, bench both.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/lhrows
mkdir -p $O
APEX_F32_KNOBS="16=4" timeout -k 10 300 python -u -m pytest tests/test_gpu_learner.py tests/test_gpu_fused_bwd.py tests/test_gpu_learning.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/t.log; [ $rc -ne 0 ] && exit $rc
for v in 8 4 8 4; do
  APEX_F32_KNOBS="16=$v" timeout -k 10 200 python -u bench.py --steps 2000 --warmup 50 > $O/b$v.log 2>&1 || exit 1
  echo "bench rows $v: $(grep '^{' $O/b$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done
