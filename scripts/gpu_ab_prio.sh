#!/bin/bash
# A/B (one box, interleaved): the DQN bench with the learner on a high-priority stream vs default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abprio
for r in 1 2; do
  for v in base prio; do
    f=""; [ $v = prio ] && f="--learner-priority"
    timeout -k 10 240 python bench.py --steps 2000 --warmup 50 $f > gpurun_out/abprio/$v$r.log 2>&1 || exit $?
    echo "$v$r $(grep -o '"value": [0-9.]*' gpurun_out/abprio/$v$r.log)"
  done
done
