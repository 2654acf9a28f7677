#!/bin/bash
# Refresh the recorded configs: 10M-transition replay (memory-pressure path, BASELINE config 5)
# and the 2-rank central-replay rehearsal (gloo, one GPU).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python bench.py --capacity 10000000 --steps 1000 --warmup 50 > gpurun_out/bench_10M.log 2>&1
rc=$?; echo "10M rc=$rc"; grep '^{' gpurun_out/bench_10M.log | cut -c1-220
[ $rc -ne 0 ] && { tail -20 gpurun_out/bench_10M.log; exit $rc; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29541 bench.py --gpus 2 --topology central --backend gloo --same-device --steps 100 --warmup 10 \
  --capacity 262144 --threshold 20000 > gpurun_out/central_2rank.log 2>&1
rc=$?; echo "central rc=$rc"; grep '^{' gpurun_out/central_2rank.log | cut -c1-220
exit $rc
