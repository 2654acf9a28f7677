#!/bin/bash
# Back-to-back bench variants: each argument is a flag string for bench.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
i=0
for flags in "$@"; do
  i=$((i+1))
  timeout -k 10 200 python bench.py --steps ${STEPS:-2000} --warmup 50 $flags > gpurun_out/ab_$i.log 2>&1 || { tail -20 gpurun_out/ab_$i.log; exit 1; }
  grep '^{' gpurun_out/ab_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('[$flags]', d['value'], d['ms_per_step'], d['host_enqueue_ms_per_step'])"
done
