#!/bin/bash
# conv2/conv3 forward tile A/B (knob 14 = 0 | 1 | 2), bench only, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/convt2
mkdir -p $O
for v in 0 2 1 0 2 1; do
  APEX_F32_KNOBS="14=$v" timeout -k 10 200 python -u bench.py --steps 3000 --warmup 50 > $O/b$v.log 2>&1 || exit 1
  echo "bench conv tile $v: $(grep '^{' $O/b$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done
