#!/bin/bash
# FC1 forward tile A/B (knob 13 = 1 | 3), bench only, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/fc1t2
mkdir -p $O
for v in 1 3 1 3; do
  APEX_F32_KNOBS="13=$v" timeout -k 10 200 python -u bench.py --steps 3000 --warmup 50 > $O/b$v.log 2>&1 || exit 1
  echo "bench fc1 tile $v: $(grep '^{' $O/b$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done
