#!/bin/bash
# fp32 data-parallel step on one GPU (1-rank RCCL communicator, sharded sampling, captured
# all-reduces) vs the plain single-GPU step: the DP structure's own cost per step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/forcedp
mkdir -p $O
cd $R
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u bench.py --steps 2000 --warmup 50 > $O/plain.log 2>&1 &&
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --force-dp --steps 2000 --warmup 50 > $O/forced.log 2>&1
rc=$?
grep -h '^{' $O/plain.log $O/forced.log | cut -c1-300
exit $rc
