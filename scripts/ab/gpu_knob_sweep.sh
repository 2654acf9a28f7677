#!/bin/bash
# Re-sweep of older kernel knobs on top of the current defaults (bench.py 3000 steps, interleaved).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/ks
mkdir -p $O
i=0
for k in "" "8=2" "7=2" "12=1" "11=0" "" "8=2" "7=2" "12=1" "11=0"; do
  i=$((i+1))
  APEX_F32_KNOBS="$k" timeout -k 10 200 python -u bench.py --steps 3000 --warmup 50 > $O/b$i.log 2>&1 || exit 1
  echo "knobs [$k]: $(grep '^{' $O/b$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done
