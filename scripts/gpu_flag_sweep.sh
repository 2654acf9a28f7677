#!/bin/bash
# Engine scheduling flags re-swept on the current kernels: 2000-step bench per variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/sweep
mkdir -p $O
i=0
while IFS= read -r v; do
  i=$((i+1))
  timeout -k 10 180 python -u bench.py --steps 2000 --warmup 50 $v > $O/v$i.log 2>&1 || { echo "FAIL [$v]"; tail -3 $O/v$i.log; exit 1; }
  echo "[$v] $(grep '^{' $O/v$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["host_enqueue_ms_per_step"])')" | tee -a $O/summary.txt
done <<'V'

--late-join
--tree-write batch
--step-graph
--no-fork-late
--streams pool
--streams priority-learner
--streams priority-actor

V
