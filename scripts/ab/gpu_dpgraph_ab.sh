#!/bin/bash
# Forced-DP (1-rank RCCL): three phase graphs + eager RCCL vs one graph with captured RCCL.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
summ() { grep '^{' "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', d['value'], d['ms_per_step'], d['host_enqueue_ms_per_step'])"; }
i=0
for flags in "--no-dp-graph" "" "--no-dp-graph" ""; do
  i=$((i+1))
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29519 bench.py --force-dp --steps ${STEPS:-1000} --warmup 50 $flags > gpurun_out/dpg_$i.log 2>&1 || { tail -30 gpurun_out/dpg_$i.log; exit 1; }
  summ gpurun_out/dpg_$i.log "forced-dp [$flags]"
done
