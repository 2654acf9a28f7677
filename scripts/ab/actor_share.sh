#!/bin/bash
# diagnostic: learner step with and without the concurrent actor step (actor-steps 0 is NOT a
# valid bench config -- it prices how much the actor's kernels slow the learner chain)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/actor_share
for a in 1 0 1 0; do
  APEX_DIAG_NO_ACTOR=$((1-a)) timeout -k 10 200 python bench.py --steps 2000 --warmup 50 > gpurun_out/actor_share/bench.log 2>&1
  rc=$?; echo "actor=$a rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/actor_share/bench.log)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
