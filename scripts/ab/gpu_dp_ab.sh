#!/bin/bash
# Forced-DP (1-rank RCCL group) A/B of two bench argument sets, interleaved (3 rounds).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
P=29531
for i in 1 2 3; do
  for arm in "$A" "$B"; do
    P=$((P+1))
    timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port $P bench.py --force-dp --steps 2000 --warmup 50 $arm > gpurun_out/dpab.log 2>&1 || { tail -20 gpurun_out/dpab.log; exit 1; }
    echo "[dp $arm] $(grep '^{' gpurun_out/dpab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["dp_graph"])')"
  done
done
