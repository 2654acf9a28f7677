#!/bin/bash
# 2 ranks on the one GPU over gloo (host-staged collectives): exercises the sharded DP
# engine path (three phase graphs, async all-reduce slices, pipelined shard-mass
# all-gather) end to end with real multi-rank collectives.  RCCL itself needs one GPU
# per rank (the driver's 8-GPU run).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --backend gloo --same-device --steps ${STEPS:-100} --warmup 10 \
  --capacity 262144 --threshold 20000 ${BENCH_ARGS:-} > gpurun_out/dp_rehearsal.log 2>&1
rc=$?; echo "dp rehearsal rc=$rc"; grep -v amdgpu.ids gpurun_out/dp_rehearsal.log | tail -5
exit $rc
