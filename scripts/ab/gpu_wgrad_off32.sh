#!/bin/bash
# conv wgrad 32-bit operand offsets A/B (knob 19): fp32 tests at 1, microbench, bench interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/woff
mkdir -p $O
APEX_F32_KNOBS="19=1" timeout -k 10 300 python -u -m pytest tests/test_gpu_f32_net.py tests/test_gpu_learner.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/t.log; [ $rc -ne 0 ] && exit $rc
for v in 0 1; do
  APEX_F32_KNOBS="19=$v" timeout -k 10 200 python -u scripts/bench_f32.py --only _bwd > $O/k$v.log 2>&1 || exit 1
  echo "off32 $v: $(grep -E "conv[23]_bwd" $O/k$v.log | tr -s ' ' | tr '\n' ';')"
done
for v in 0 1 0 1; do
  APEX_F32_KNOBS="19=$v" timeout -k 10 200 python -u bench.py --steps 3000 --warmup 50 > $O/b$v.log 2>&1 || exit 1
  echo "bench wgrad off32 $v: $(grep '^{' $O/b$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done
