#!/bin/bash
# The learner's tree-branch join before the optimizer (default) vs after it (APEX_JOIN_AFTER_OPT=1).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/ab_join
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 150 python -u bench.py --steps 2000 --warmup 50 > $O/def_$i.log 2>&1 || exit $?
  APEX_JOIN_AFTER_OPT=1 timeout -k 10 150 python -u bench.py --steps 2000 --warmup 50 > $O/after_$i.log 2>&1 || exit $?
done
for f in $O/def_*.log $O/after_*.log; do echo "$f $(tail -n 1 $f | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"; done
