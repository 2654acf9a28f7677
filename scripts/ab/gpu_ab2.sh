#!/bin/bash
# A/B of two bench configurations, interleaved on one box (3 rounds each).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for i in 1 2 3; do
  for arm in "$A" "$B"; do
    timeout -k 10 200 python bench.py --steps 2000 --warmup 50 $arm > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
    echo "[$arm] $(grep '^{' gpurun_out/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
