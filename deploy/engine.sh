#!/bin/bash
# GPU-resident Ape-X on MI355X nodes: one rank per GPU (RCCL over xGMI inside a node).
# Run once per node with NODE_RANK set (0 on the MASTER_ADDR host):
#   NODE_RANK=0 NNODES=2 MASTER_ADDR=10.0.0.1 deploy/engine.sh --max-step 1000000
# TOPOLOGY=sharded: DP learner replica + replay shard + actor shard per GPU;
# TOPOLOGY=central: global rank 0 = learner + replay, every other GPU = actors.
source "$(dirname "$0")/_common.sh"
NODE_RANK=${NODE_RANK:-0}
cd "$REPO_ROOT" || exit 1
exec python -m torch.distributed.run --nnodes "$NNODES" --node-rank "$NODE_RANK" \
  --nproc-per-node "$GPUS_PER_NODE" --master-addr "$MASTER_ADDR" --master-port "$MASTER_PORT" \
  -m apex_amd.train --topology "$TOPOLOGY" "$@"
